#!/bin/bash
# GPU box, round 6 call E: interleaved A/B of the wave-kernel builds on the C3 host step (records compared):
#   libsubread_amd.so        single-pass top-3, the wave's read-loop state scalar (SGPRs), 6 waves/SIMD
#   libsubread_amd_top1.so   single-pass top-3 only
#   libsubread_amd_base.so   round 5's kernel
#   libsubread_amd_occ5.so   the current kernel at 5 waves/SIMD (96 VGPRs: no VGPR spills left)
# then the device path with / without host pacing (option dev_pace)
out=gpurun_out/r6e
mkdir -p $out
timeout -k 10 900 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_top1.so \
  subread_amd/lib/libsubread_amd_base.so subread_amd/lib/libsubread_amd_occ5.so > $out/ab.txt 2> $out/ab.err &&
SETTINGS="host;0,1;0,1,1" ROUNDS=3 timeout -k 10 400 python3 -u tools/device_sweep.py > $out/dev.txt 2> $out/dev.err
