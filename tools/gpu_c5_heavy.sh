# GPU box: C5 (subjunc SE) with the default lane path vs the heavy second lane pass (SVG_LANE=3)
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5_default.json 2> gpurun_out/c5_default.err && \
SVG_LANE=3 timeout -k 10 400 python -u bench.py --workload c5 --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5_lane3.json 2> gpurun_out/c5_lane3.err
