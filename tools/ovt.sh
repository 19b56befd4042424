set -o pipefail
mkdir -p gpurun_out/ovt
for ov in d 1 0; do
  if [ $ov = d ]; then unset SVG_OVERLAP; else export SVG_OVERLAP=$ov; fi
  SVG_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-host --no-check --steps 3 > gpurun_out/ovt/$ov.json 2> gpurun_out/ovt/$ov.log || exit 1
  grep -m2 "chunk pipeline" gpurun_out/ovt/$ov.log
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],{k:v['launch_ms'] for k,v in d['roofline']['kernels'].items()})" gpurun_out/ovt/$ov.json
done
