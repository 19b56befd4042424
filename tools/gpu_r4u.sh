#!/bin/bash
# GPU box, round 4 call U: the single-end wave kernel at 5 waves/SIMD (96 VGPRs) against 6 (80,
# spilling), interleaved in one process
mkdir -p gpurun_out/r4u
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_occ5.so > gpurun_out/r4u/ab_occ6_vs_occ5.txt 2>&1
