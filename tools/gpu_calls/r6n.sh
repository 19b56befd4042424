#!/bin/bash
# GPU box, round 6 call N: batch mode's chunk-neighbour test through a 32-entry LDS table of lane masks
# by kv bin (row masks through the same table) instead of all m x m comparisons, and its slot scan by
# row segment -- on top of the next-read index loaded a read ahead.  Vote-path parity tests incl. the
# 50M C3 reference digest, then an interleaved A/B on the C3 host step: this build, the index change
# alone (libsubread_amd_idx.so), the build of d8e0940
out=gpurun_out/r6n
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py > $out/tests.txt 2>&1 &&
timeout -k 10 900 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_idx.so \
  subread_amd/lib_ab/libsubread_amd_d8e.so > $out/ab_c3.txt 2> $out/ab_c3.err
