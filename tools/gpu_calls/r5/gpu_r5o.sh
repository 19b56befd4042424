#!/bin/bash
# GPU box, round 5 call O: the wave kernel's hit values two chunks ahead -- lane / parity tests,
# interleaved A/B against the previous build (C3 host path)
mkdir -p gpurun_out/r5o
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lane.py tests/test_gpu_parity.py > gpurun_out/r5o/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py c3 6 subread_amd/lib/ab/lib_old.so subread_amd/lib/ab/lib_pf2.so > gpurun_out/r5o/ab.txt 2> gpurun_out/r5o/ab.err
