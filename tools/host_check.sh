#!/bin/bash
# GPU box: pipeline parity tests, then C3 bench with the host-buffer measurement.
set -o pipefail
mkdir -p gpurun_out/hc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pipelines or split or empty" -x -q --timeout 120 --timeout-method thread > gpurun_out/hc/tests.log 2>&1 || { tail -30 gpurun_out/hc/tests.log; exit 1; }
tail -2 gpurun_out/hc/tests.log
for wl in ${@:-c3}; do
  timeout -k 10 400 python -u bench.py --workload $wl --no-cpu --steps 3 > gpurun_out/hc/$wl.json 2> gpurun_out/hc/$wl.log || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['parity_check'],d['host_path'])" gpurun_out/hc/$wl.json
done
