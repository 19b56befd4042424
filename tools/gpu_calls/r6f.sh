#!/bin/bash
# GPU box, round 6 call F: the wave kernel with the read's length and the table's max vote scalar too --
# vote-path parity tests, an interleaved A/B (current / _uni: round-6 call E's winner / _base: round 5),
# then the end-to-end runs of call D (C3 genome, 3M reads: BAM with 1 and 8 replicas, SAM)
out=gpurun_out/r6f
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_uni.so \
  subread_amd/lib/libsubread_amd_base.so > $out/ab.txt 2> $out/ab.err &&
bash tools/gpu_calls/r6d.sh
