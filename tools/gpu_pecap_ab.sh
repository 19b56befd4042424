# GPU box: C5pe and C4 with the lane PE candidate cap at 40 (default) / 64 / 96 (pair bound 256)
mkdir -p gpurun_out
for v in 40 64 96; do
  SVG_LANE_PE_CAP=$v timeout -k 10 400 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_cap_$v.json 2> gpurun_out/c5pe_cap_$v.err || exit 1
done
for v in 40 64; do
  SVG_LANE_PE_CAP=$v timeout -k 10 400 python -u bench.py --workload c4 --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c4_cap_$v.json 2> gpurun_out/c4_cap_$v.err || exit 1
done
