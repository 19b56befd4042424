# GPU box: C5pe bench with / without the chunk-pipeline overlap
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_base.json 2> gpurun_out/c5pe_base.err && \
SVG_OVERLAP=1 timeout -k 10 500 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_ovl.json 2> gpurun_out/c5pe_ovl.err
