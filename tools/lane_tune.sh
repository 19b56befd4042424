#!/bin/bash
# lane-path tuning sweep at C3 (slot pool K, candidate cap). Usage: tools/lane_tune.sh OUTDIR
set -o pipefail
out=$1; mkdir -p $out
for v in "16_40" "20_40" "24_40" "20_48"; do
  k=${v%_*}; c=${v#*_}
  SVG_LANE_K=$k SVG_LANE_CAP=$c timeout -k 10 300 python -u bench.py --no-cpu --no-check --steps 3 > $out/$v.json 2> $out/$v.log || exit 1
done
