#!/bin/bash
# GPU box, round 6 call U: batch mode's neighbour-member loop without branches inside (36 instead of
# ~48 instructions per member) and no division by the gap on the full index -- vote-path parity tests
# incl. the 50M C3 digest, then A/B against a848e07 in both orders
out=gpurun_out/r6u
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py > $out/tests.txt 2>&1 &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_bf.so subread_amd/lib_ab/libsubread_amd_a84.so > $out/ab_a.txt 2> $out/ab_a.err &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_a84.so subread_amd/lib_ab/libsubread_amd_bf.so > $out/ab_b.txt 2> $out/ab_b.err
