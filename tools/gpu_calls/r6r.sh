#!/bin/bash
# GPU box, round 6 call R: the single-end wave kernel's register budget and grid after the batch-mode
# table -- this build (7 waves/SIMD budget, 72 VGPRs), 8 (64 VGPRs), 7 with the lane kernel at 5
# waves/SIMD (96 VGPRs), 7 with 8 wave-kernel blocks per CU beside the probe stream (cap 6), and
# fb3bc80 (80 VGPRs): vote-path parity tests of this build, then an interleaved A/B on the C3 host step
out=gpurun_out/r6r
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py > $out/tests.txt 2>&1 &&
timeout -k 10 1000 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_occ8.so \
  subread_amd/lib_ab/libsubread_amd_occ7_lw5.so subread_amd/lib_ab/libsubread_amd_occ7_cap8.so \
  subread_amd/lib_ab/libsubread_amd_fb3.so > $out/ab_c3.txt 2> $out/ab_c3.err
