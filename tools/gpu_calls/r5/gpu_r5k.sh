#!/bin/bash
# GPU box, round 5 call K: the wave kernel's compact slot pool -- pool-limit parity tests, the lane
# tests, then an interleaved A/B (pool off / on / with wave_cap 8) on the C3 host path
mkdir -p gpurun_out/r5k
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lane.py > gpurun_out/r5k/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_opts.py 5 "wave_pool=0" "wave_pool=1" "wave_pool=1,wave_cap=8" "wave_pool=1,wave_cap=10" > gpurun_out/r5k/ab.txt 2> gpurun_out/r5k/ab.err
