#!/bin/bash
# GPU box, round 4 call L: interleaved A/B of the wave kernel's work loop -- A: static read indices
# preloaded in a lane register, 32-bit uniform positions (current); B: call F's loop
mkdir -p gpurun_out/r4l
timeout -k 10 400 python -u tools/ab_libs.py c3 10 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_abF.so > gpurun_out/r4l/ab_preload_vs_F.txt 2>&1
