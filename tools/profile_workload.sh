#!/bin/bash
# rocprofv3 evidence for one bench.py workload (GPU box): kernel trace + FETCH_SIZE + WRITE_SIZE,
# each in its own run, summarised per kernel by tools/prof_kernels.py.
# Usage: tools/profile_workload.sh WORKLOAD READS_PER_STEP OUTDIR   (OUTDIR under gpurun_out/)
set -e
wl=$1; reads=$2; out=$3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 bench.py --workload $wl --no-cpu --no-host > $out/bench.json 2> $out/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu --no-host --no-check > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu --no-host --no-check > $out/write.log 2>&1
python3 tools/prof_kernels.py $out/summary --trace $out/trace --fetch $out/fetch --write $out/write --steps 5 --warmup 1 --reads $reads --workload $wl --bench-json $out/bench.json
