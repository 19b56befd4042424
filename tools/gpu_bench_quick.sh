# GPU box: a short bench.py run (fewer reads) to check the JSON line's figures
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --reads 5000000 --steps 2 --warmup 1 --no-cpu --ascii-reads 0 --device-steps 1 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
