#!/bin/bash
# GPU box, round 6 call Q: batch mode's neighbour test with a row filter (bins in the vote table's
# pad slots, rows in btab: a lane tests only its bins' members whose row is within R of its own)
# -- vote-path parity tests incl. the 50M C3 digest, then an interleaved A/B on the C3 host step:
# this build, fb3bc80, fb3bc80 with the single-end wave kernel at 7 waves/SIMD (72 VGPRs), d8e0940;
# then the SQ counter passes of this build
out=gpurun_out/r6q
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py > $out/tests.txt 2>&1 &&
timeout -k 10 900 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_fb3.so \
  subread_amd/lib_ab/libsubread_amd_occ7.so subread_amd/lib_ab/libsubread_amd_d8e.so > $out/ab_c3.txt 2> $out/ab_c3.err &&
bash tools/pmc_sq.sh $out/sq c3 > $out/sq.txt 2>&1
rc=$?
rm -rf $out/sq/p*/
exit $rc
