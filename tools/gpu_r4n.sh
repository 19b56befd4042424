#!/bin/bash
# GPU box, round 4 call N: three device slots in the host pipeline, ramped device-entry chunks --
# parity tests, C3 bench line, slots 2/3 interleaved
mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4n/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4n/c3_kernel_record_bench.json > gpurun_out/r4n/bench_c3.json 2> gpurun_out/r4n/bench_c3.err && \
timeout -k 10 400 python -u tools/sweep_host.py c3 10 's2:host_slots=2' 's3:host_slots=3' 's2b:host_slots=2' 's3b:host_slots=3' > gpurun_out/r4n/sweep_slots.txt 2>&1
