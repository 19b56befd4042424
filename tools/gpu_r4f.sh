#!/bin/bash
# GPU box, round 4 call F: SQ counters of the C3 host path (LDS bank conflicts after the lane
# kernel's slot swizzle), the stamps build's wave-kernel phase split, fragile voting throughput
mkdir -p gpurun_out/r4f
timeout -k 10 900 bash tools/pmc_sq.sh gpurun_out/r4f/sq c3 > gpurun_out/r4f/sq.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 5000000 > gpurun_out/r4f/phases_c3.txt 2> gpurun_out/r4f/phases_c3.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 1 > gpurun_out/r4f/fragile_gap1.json 2> gpurun_out/r4f/fragile_gap1.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 3 > gpurun_out/r4f/fragile_gap3.json 2> gpurun_out/r4f/fragile_gap3.err
