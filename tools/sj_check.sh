#!/bin/bash
# GPU box: subjunc parity tests, then the C5 bench.
set -o pipefail
mkdir -p gpurun_out/sj
timeout -k 10 400 python -u -m pytest tests -m gpu -k "sj or subjunc or golden or pipelines" -x -q --timeout 120 --timeout-method thread > gpurun_out/sj/tests.log 2>&1 || { tail -30 gpurun_out/sj/tests.log; exit 1; }
tail -2 gpurun_out/sj/tests.log
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu --no-host --steps 3 > gpurun_out/sj/c5.json 2> gpurun_out/sj/c5.log || exit 1
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['parity_check'],{k:v['launch_ms'] for k,v in d['roofline']['kernels'].items()})" gpurun_out/sj/c5.json
