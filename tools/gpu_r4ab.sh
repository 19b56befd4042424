#!/bin/bash
# GPU box, round 4 call AB: 12 lane slots (6 KB LDS per wave) against 16, interleaved (C3)
mkdir -p gpurun_out/r4ab
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd_k12.so subread_amd/lib/libsubread_amd.so > gpurun_out/r4ab/ab_k12_vs_k16.txt 2>&1
