#!/bin/bash
# GPU box, round 4 call H: the bucket-code and key-hash probes with two probes in flight per
# thread and pass, the wave kernel's counters added where they happen -- parity tests of the vote
# paths, then C3 (bench line + HIP-event kernel record) and C3g (the key-hash image)
mkdir -p gpurun_out/r4h
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4h/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4h/c3_kernel_record_bench.json > gpurun_out/r4h/bench_c3.json 2> gpurun_out/r4h/bench_c3.err && \
timeout -k 10 400 python -u bench.py --workload c3g --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 > gpurun_out/r4h/bench_c3g.json 2> gpurun_out/r4h/bench_c3g.err
