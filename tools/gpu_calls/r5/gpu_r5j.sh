#!/bin/bash
# GPU box, round 5 call J: the wave kernel's per-phase cycles on C3 deferred reads (stamps build),
# then an interleaved A/B of the wave kernel's blocks per CU and static share (C3 host path)
mkdir -p gpurun_out/r5j
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 400 python -u tools/phase_profile.py c3 5000000 > gpurun_out/r5j/phases_c3.txt 2> gpurun_out/r5j/phases_c3.err &&
timeout -k 10 400 python -u tools/ab_opts.py 4 "" "wave_cap=7" "wave_cap=8" "wave_static=4" "wave_static=7" > gpurun_out/r5j/ab.txt 2> gpurun_out/r5j/ab.err
