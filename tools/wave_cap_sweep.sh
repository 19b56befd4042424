#!/bin/bash
# C3 with the wave kernel's blocks-per-CU capped while it overlaps the probe kernel
# (SVG_WAVE_CAP; 0 = uncapped, 10 blocks/CU for the SE align variant).  GPU box.
set -e
out=${1:-gpurun_out/wcap}; mkdir -p $out
for c in ${CAPS:-0 8 6 4 3}; do
  SVG_WAVE_CAP=$c timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-host > $out/cap$c.json 2> $out/cap$c.err
  python3 -c "import json,sys;d=json.load(open('$out/cap$c.json'));k=d['roofline']['kernels'];print('cap $c', d['value'], d['ms_per_step'], {n:k[n]['launch_ms'] for n in k})"
done
