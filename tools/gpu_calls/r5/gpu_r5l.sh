#!/bin/bash
# GPU box, round 5 call L: quad_kernel (four single-end reads per wave) -- lane/quad parity tests,
# then an interleaved A/B against the wave kernel on the C3 host path (blocks per CU 2/3/4)
mkdir -p gpurun_out/r5l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lane.py > gpurun_out/r5l/tests.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_opts.py 4 "wave_quad=0" "wave_quad=1" "wave_quad=1,wave_cap=2" "wave_quad=1,wave_cap=4" "wave_quad=1,wave_cap=5" > gpurun_out/r5l/ab.txt 2> gpurun_out/r5l/ab.err
