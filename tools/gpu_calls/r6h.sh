#!/bin/bash
# GPU box, round 6 call H: the wave kernel's top-3 insert made branch-free (the lambda's a/b/c had
# become a dynamically indexed private array: scratch 60 -> 48 B/lane single-end, 16 -> 0 long reads)
# -- vote-path parity tests, then an interleaved A/B on the C3 host step against the committed build
# (libsubread_amd_c231.so) and round 5's kernel (libsubread_amd_base.so), records compared
out=gpurun_out/r6h
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py tests/test_gpu_sublong.py > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_c231.so \
  subread_amd/lib/libsubread_amd_base.so > $out/ab.txt 2> $out/ab.err
