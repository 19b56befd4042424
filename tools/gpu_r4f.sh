#!/bin/bash
# GPU box, round 4 call F: the wave kernel's deferred reads dealt out statically (three
# quarters) before the work counter -- parity tests, C3 bench line; then the SQ counters of the
# C3 host path (LDS bank conflicts after the lane kernel's slot swizzle), the stamps build's
# wave-kernel phase split, fragile voting throughput
mkdir -p gpurun_out/r4f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4f/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4f/c3_kernel_record_bench.json > gpurun_out/r4f/bench_c3.json 2> gpurun_out/r4f/bench_c3.err && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 5000000 > gpurun_out/r4f/phases_c3.txt 2> gpurun_out/r4f/phases_c3.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 1 > gpurun_out/r4f/fragile_gap1.json 2> gpurun_out/r4f/fragile_gap1.err && \
timeout -k 10 300 python -u tools/bench_fragile.py --gap 3 > gpurun_out/r4f/fragile_gap3.json 2> gpurun_out/r4f/fragile_gap3.err && \
timeout -k 10 600 bash tools/pmc_sq.sh gpurun_out/r4f/sq c3 > gpurun_out/r4f/sq.txt 2>&1
