#!/bin/bash
# probe_kernel variants at C3 (bench --steps 3, no CPU leg): one-shot bucket window on/off,
# SoA thread mapping vs read-major threads.  Usage: tools/probe_sweep.sh OUTDIR
set -o pipefail
out=$1
mkdir -p $out
for v in "w" "w_sm" "nw"; do
  case $v in
    w) env="" ;;
    w_sm) env="SVG_PROBE_MAP=0" ;;
    w_rm) env="SVG_PROBE_MAP=1" ;;
    nw) env="SVG_NO_WINDOW=1" ;;
  esac
  env $env timeout -k 10 300 python -u bench.py --no-cpu --no-check --steps 3 > $out/$v.json 2> $out/$v.log || exit 1
done
