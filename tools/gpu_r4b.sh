#!/bin/bash
# GPU box, round 4 call B: the GPU test suite (inline key-hash image now the default probe image),
# then C3 with it (the bench line + kernel record) and without it (the option then named no_kinline; now kinline=1 is opt-in), then the
# serialised trace + HIP-event kernel record of the metric's path
mkdir -p gpurun_out/r4b
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4b/c3_kernel_record_bench.json > gpurun_out/r4b/bench_c3.json 2> gpurun_out/r4b/bench_c3.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --opt no_kinline=1 --no-cpu --ascii-reads 0 --long-reads 0 > gpurun_out/r4b/bench_c3_nokinline.json 2> gpurun_out/r4b/bench_c3_nokinline.err
