#!/bin/bash
# GPU box, round 4 call Z: 16 slots per lane as the build default -- parity tests, C3 bench line
# (deferral count in it), and the A/B against a 20-slot build with the order swapped
mkdir -p gpurun_out/r4z
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4z/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4z/c3_kernel_record_bench.json > gpurun_out/r4z/bench_c3.json 2> gpurun_out/r4z/bench_c3.err && \
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd_k20.so subread_amd/lib/libsubread_amd.so > gpurun_out/r4z/ab_k20_vs_k16.txt 2>&1
