#!/bin/bash
# GPU box, round 6 call S: the single-end wave kernel's register budget, 7 (72 VGPRs) against 6 (80,
# fb3bc80), in two processes with the libraries in opposite orders (the interleaved A/B's position in
# the process -- which index is built first -- moved results by several percent in calls Q and R)
out=gpurun_out/r6s
mkdir -p $out
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_occ7.so subread_amd/lib_ab/libsubread_amd_fb3.so \
  > $out/ab_c3_a.txt 2> $out/ab_c3_a.err &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_fb3.so subread_amd/lib_ab/libsubread_amd_occ7.so \
  > $out/ab_c3_b.txt 2> $out/ab_c3_b.err
