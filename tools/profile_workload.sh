#!/bin/bash
# rocprofv3 evidence for one workload (GPU box): kernel trace + FETCH_SIZE + WRITE_SIZE, each in
# its own run of tools/prof_run.py (MODE host = the path bench.py's value measures, or device;
# 1 warmup + STEPS steps and nothing else on the GPU), summarised per kernel by tools/prof_kernels.py.
# Usage: tools/profile_workload.sh WORKLOAD READS_PER_STEP OUTDIR [STEPS] [MODE]   (OUTDIR under gpurun_out/)
set -e
wl=$1; reads=$2; out=$3; steps=${4:-3}; mode=${5:-host}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 tools/prof_run.py $wl $steps $mode > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- python3 tools/prof_run.py $wl 1 $mode > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- python3 tools/prof_run.py $wl 1 $mode > $out/write.log 2>&1
python3 tools/prof_kernels.py $out/summary --trace $out/trace --fetch $out/fetch --write $out/write --steps $steps --warmup 1 \
  --reads $reads --workload $wl --cmd "python3 tools/prof_run.py $wl STEPS $mode"
# the rocprofv3 databases exceed what gpurun copies back (64 MiB): keep the summary only
[ "${KEEP_DB:-0}" = 1 ] || rm -rf $out/trace $out/fetch $out/write
