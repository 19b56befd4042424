#!/bin/bash
# GPU box, round 6 call T: the wave kernel's blocks per CU beside the probe stream (option wave_cap,
# default 6) after the batch-mode table and the 72-VGPR budget: 5 and 7 against 6, each pair in both
# orders, the same build under two file names
out=gpurun_out/r6t
mkdir -p $out
cp subread_amd/lib/libsubread_amd.so /tmp/libsvg_a.so && cp subread_amd/lib/libsubread_amd.so /tmp/libsvg_b.so &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 /tmp/libsvg_a.so /tmp/libsvg_b.so@wave_cap=5 > $out/ab_cap5_a.txt 2> $out/ab_cap5_a.err &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 /tmp/libsvg_b.so@wave_cap=5 /tmp/libsvg_a.so > $out/ab_cap5_b.txt 2> $out/ab_cap5_b.err &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 /tmp/libsvg_a.so /tmp/libsvg_b.so@wave_cap=7 > $out/ab_cap7_a.txt 2> $out/ab_cap7_a.err &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 /tmp/libsvg_b.so@wave_cap=7 /tmp/libsvg_a.so > $out/ab_cap7_b.txt 2> $out/ab_cap7_b.err
