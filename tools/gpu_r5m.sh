#!/bin/bash
# GPU box, round 5 call M: the wave kernel's per-phase cycles (stamps build, C3 deferred reads),
# then end to end at human scale with the round-5 loader (C3 genome, 3M reads: stock vs drop-in)
mkdir -p gpurun_out/r5m
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 400 python -u tools/phase_profile.py c3 5000000 > gpurun_out/r5m/phases_c3.txt 2> gpurun_out/r5m/phases_c3.err &&
timeout -k 10 1000 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5m/e2e_c3.json > gpurun_out/r5m/e2e.out 2> gpurun_out/r5m/e2e.err
