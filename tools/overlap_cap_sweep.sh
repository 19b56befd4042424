#!/bin/bash
# PE (C4) and subjunc (C5) with the chunk pipeline forced on (SVG_OVERLAP=1) at several
# wave-kernel caps (SVG_WAVE_CAP blocks/CU; 0 = uncapped), against the default (overlap
# off for these variants).  GPU box.
set -e
out=${1:-gpurun_out/ovcap}; mkdir -p $out
for w in ${WORKLOADS:-c4 c5}; do
  for cfg in ${CFGS:-off 1:0 1:6 1:4}; do
    if [ "$cfg" = off ]; then ov=0; cap=0; else ov=${cfg%%:*}; cap=${cfg##*:}; fi
    f=$out/${w}_ov${ov}_cap${cap}
    SVG_OVERLAP=$ov SVG_WAVE_CAP=$cap timeout -k 10 300 python3 -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-host > $f.json 2> $f.err
    python3 -c "import json;d=json.load(open('$f.json'));k=d['roofline']['kernels'];print('$w overlap $ov cap $cap', d['value'], d['ms_per_step'], d['parity_check'], {n:k[n]['launch_ms'] for n in k})"
  done
done
