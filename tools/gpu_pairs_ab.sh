# GPU box: C5pe with the lane PE kernel's pair-loop bound at 96 (default) / 256 / 1024, then a C5pe parity check at 1024
mkdir -p gpurun_out
for v in 96 256 1024; do
  SVG_LANE_PAIRS=$v timeout -k 10 400 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_pairs_$v.json 2> gpurun_out/c5pe_pairs_$v.err || exit 1
done
SVG_LANE_PAIRS=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_pairs_tests.log 2>&1
