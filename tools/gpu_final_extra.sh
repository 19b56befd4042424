# GPU box: extra round-end evidence -- C3g bench, sublong kernel trace of the final build
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --workload c3g --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c3g_final.json 2> gpurun_out/c3g_final.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long_final -o long -- python3 -u tools/bench_long.py --gap 1 --steps 2 --warmup 1 --check 0 --cpu-reads 0 > gpurun_out/prof_long_final.log 2>&1
