#!/bin/bash
# GPU box, round 6 call P: slot_of by a shuffle binary search (5 steps, not 29 readlanes), the
# candidate locate in fixed steps (no divergent loop), no division by the gap on the full index --
# vote-path parity tests, then an interleaved A/B on the C3 host step against fb3bc80 and d8e0940
out=gpurun_out/r6p
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_fragile.py > $out/tests.txt 2>&1 &&
timeout -k 10 900 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_fb3.so \
  subread_amd/lib_ab/libsubread_amd_d8e.so > $out/ab_c3.txt 2> $out/ab_c3.err
