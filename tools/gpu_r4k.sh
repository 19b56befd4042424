#!/bin/bash
# GPU box, round 4 call K: the stamps build's wave-kernel phase split, fragile voting throughput,
# the host and HBM-resident entries' per-kernel times side by side (bucket-code index), SQ
# counters (raw rocprofv3 databases removed after the summary: gpurun_out must stay < 64 MiB),
# then the work-loop A/B of call L
mkdir -p gpurun_out/r4k
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 5000000 > gpurun_out/r4k/phases_c3.txt 2> gpurun_out/r4k/phases_c3.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 1 > gpurun_out/r4k/fragile_gap1.json 2> gpurun_out/r4k/fragile_gap1.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 3 > gpurun_out/r4k/fragile_gap3.json 2> gpurun_out/r4k/fragile_gap3.err && \
timeout -k 10 300 python -u tools/ab_images.py --config bcode: --rounds 4 --device --out gpurun_out/r4k/host_vs_device.json > gpurun_out/r4k/hvd.out 2> gpurun_out/r4k/hvd.err && \
timeout -k 10 600 bash tools/pmc_sq.sh /tmp/r4k_sq c3 > gpurun_out/r4k/sq.txt 2>&1 && \
mkdir -p gpurun_out/r4l && \
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_abF.so > gpurun_out/r4l/ab_preload_vs_F.txt 2>&1
rc=$?
rm -rf /tmp/r4k_sq
exit $rc
