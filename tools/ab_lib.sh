#!/bin/bash
# GPU box: A/B of two library builds on one workload.  Usage: tools/ab_lib.sh WL LIB_B
set -o pipefail
mkdir -p gpurun_out/ab
wl=$1; lb=$2
for v in a b; do
  if [ $v = b ]; then export SVG_LIB=$lb; fi
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu --no-host --no-check --steps 3 > gpurun_out/ab/${wl}_$v.json 2> gpurun_out/ab/${wl}_$v.log || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],{k:v['launch_ms'] for k,v in d['roofline']['kernels'].items()})" gpurun_out/ab/${wl}_$v.json
done
