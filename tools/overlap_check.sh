#!/bin/bash
# GPU box: parity suite, then bench of the given workloads with the chunk pipeline on and off.
# Usage: tools/overlap_check.sh [workloads...]  (default c3)
set -o pipefail
mkdir -p gpurun_out/ov
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ov/tests.log 2>&1 || { tail -30 gpurun_out/ov/tests.log; exit 1; }
tail -2 gpurun_out/ov/tests.log
for wl in ${@:-c3}; do
  for ov in 1 0; do
    SVG_OVERLAP=$ov timeout -k 10 300 python -u bench.py --workload $wl --no-cpu --no-host --steps 3 > gpurun_out/ov/${wl}_$ov.json 2> gpurun_out/ov/${wl}_$ov.log || exit 1
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['parity_check'],{k:v['launch_ms'] for k,v in d['roofline']['kernels'].items()})" gpurun_out/ov/${wl}_$ov.json
  done
done
