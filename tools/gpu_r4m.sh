#!/bin/bash
# GPU box, round 4 call M: host sub-batches ramped at both ends -- parity tests (the sub-batch
# schedule test among them), C3 bench line, ramp on/off interleaved
mkdir -p gpurun_out/r4m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4m/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4m/c3_kernel_record_bench.json > gpurun_out/r4m/bench_c3.json 2> gpurun_out/r4m/bench_c3.err && \
timeout -k 10 400 python -u tools/sweep_host.py c3 10 'flat:host_ramp=0' 'ramp:host_ramp=1' 'flat2:host_ramp=0' 'ramp2:host_ramp=1' > gpurun_out/r4m/sweep_ramp.txt 2>&1
