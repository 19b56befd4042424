#!/bin/bash
# GPU box, round 4 call AC: 16 lane slots for fused align only (subjunc and the gather path 20) --
# parity tests, C3, C5, C3g
mkdir -p gpurun_out/r4ac
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ac/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4ac/c3_kernel_record_bench.json > gpurun_out/r4ac/bench_c3.json 2> gpurun_out/r4ac/bench_c3.err || exit $?
for wl in c5 c3g; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 \
    > gpurun_out/r4ac/bench_$wl.json 2> gpurun_out/r4ac/bench_$wl.err || exit $?
done
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd_k12.so subread_amd/lib/libsubread_amd.so > gpurun_out/r4ac/ab_k12_vs_k16.txt 2>&1
