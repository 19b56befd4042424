#!/bin/bash
# GPU box, round 4 call J: the wave kernel's static read indices preloaded in a lane register,
# 32-bit uniform positions -- parity tests, C3 bench line, the static share swept (eighths)
mkdir -p gpurun_out/r4j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_io.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4j/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --ascii-reads 0 --long-reads 0 --kernel-record gpurun_out/r4j/c3_kernel_record_bench.json > gpurun_out/r4j/bench_c3.json 2> gpurun_out/r4j/bench_c3.err && \
timeout -k 10 400 python -u tools/sweep_host.py c3 10 's4:wave_static=4' 's7:wave_static=7' 's8:wave_static=8' 's6:wave_static=6' > gpurun_out/r4j/sweep_static.txt 2>&1
