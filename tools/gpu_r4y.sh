#!/bin/bash
# GPU box, round 4 call Y: the lane kernel with 16 slots per lane (8 KB LDS per wave) against 20,
# interleaved in one process (C3)
mkdir -p gpurun_out/r4y
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_k16.so > gpurun_out/r4y/ab_k20_vs_k16.txt 2>&1
