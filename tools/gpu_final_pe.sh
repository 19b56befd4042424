# GPU box: final-build C4 and C5pe bench lines with their parity checks
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --workload c4 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c4_final.json 2> gpurun_out/c4_final.err && \
timeout -k 10 600 python -u bench.py --workload c5pe --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_final.json 2> gpurun_out/c5pe_final.err
