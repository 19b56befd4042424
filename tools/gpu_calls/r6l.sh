#!/bin/bash
# GPU box, round 6 call L: the wave kernel's first-chunk prefetch (single end: strand 1's first 64
# hit values loaded when strand 0's replay starts, the next read's strand 0 when strand 1's starts)
# -- vote-path parity tests incl. the 50M C3 reference digest, then an interleaved A/B on the C3 host
# step against the build of d8e0940
out=gpurun_out/r6l
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py tests/test_gpu_fragile.py > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_d8e.so \
  > $out/ab_c3.txt 2> $out/ab_c3.err
