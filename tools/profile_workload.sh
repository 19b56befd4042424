#!/bin/bash
# rocprofv3 evidence for one workload (GPU box): kernel trace + FETCH_SIZE + WRITE_SIZE, each in
# its own run of tools/prof_run.py (device-resident vote path, 1 warmup + STEPS steps and nothing
# else on the GPU), summarised per kernel by tools/prof_kernels.py.
# Usage: tools/profile_workload.sh WORKLOAD READS_PER_STEP OUTDIR [STEPS]   (OUTDIR under gpurun_out/)
set -e
wl=$1; reads=$2; out=$3; steps=${4:-3}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 tools/prof_run.py $wl $steps > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- python3 tools/prof_run.py $wl 1 > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 tools/prof_run.py $wl 1 > $out/write.log 2>&1
python3 tools/prof_kernels.py $out/summary --trace $out/trace --fetch $out/fetch --write $out/write --steps $steps --warmup 1 --reads $reads --workload $wl
