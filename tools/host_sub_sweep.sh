#!/bin/bash
# GPU box: host-buffer path rate vs sub-batch size (SVG_HOST_SUB), C3.
set -o pipefail
mkdir -p gpurun_out/hs
for sub in 1000000 2000000 4000000; do
  SVG_HOST_SUB=$sub timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-check --steps 1 --warmup 1 > gpurun_out/hs/$sub.json 2> gpurun_out/hs/$sub.log || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['host_path']['value'],d['host_path']['pageable_value'])" gpurun_out/hs/$sub.json
done
