# GPU box: sublong voting -- chunk statistics, kernel trace of one step, the long-read bench (full
# and gapped), and the end-to-end drop-in comparison
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SVG_LONG_DEBUG=1 timeout -k 10 400 python -u tools/bench_long.py --gap 1 --steps 2 > gpurun_out/bench_long_full2.json 2> gpurun_out/bench_long_full2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long -o long -- python3 tools/bench_long.py --gap 1 --steps 1 --warmup 0 --check 0 --cpu-reads 0 > gpurun_out/prof_long.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_long.py --gap 3 --steps 2 > gpurun_out/bench_long_gapped.json 2> gpurun_out/bench_long_gapped.err && \
timeout -k 10 500 python -u tools/e2e_dropin.py --mbp 200 --reads 4000000 > gpurun_out/e2e2.json 2> gpurun_out/e2e2.err
