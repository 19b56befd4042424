#!/bin/bash
# GPU box, round 4 call X: deeper host ramp (1/8, 1/4, 1/2) and the single-end static share 5,
# interleaved at C3; then the sub-batch schedule tests
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u tools/sweep_host.py c3 10 'r2:host_ramp=2' 's5:wave_static=5' 'r1:host_ramp=1' 'r2b:host_ramp=2' 's6:wave_static=6' 'r1b:host_ramp=1' > gpurun_out/r4x/sweep.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_io.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4x/gpu_io_tests.log 2>&1
