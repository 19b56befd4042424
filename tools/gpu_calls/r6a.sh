#!/bin/bash
# GPU box, round 6 call A: kernel timelines (rocprofv3 --kernel-trace --memory-copy-trace, no counters) of
# bench.py's C3 host step, two-stream pipeline (the bench configuration) and single stream (overlap=0);
# each run also prints its own HIP-event kernel record and step times (tools/prof_run.py)
set -o pipefail
out=gpurun_out/r6a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $out/ovl -o run -- python3 tools/prof_run.py c3 3 host > $out/ovl.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $out/ser -o run -- python3 tools/prof_run.py c3 3 host overlap=0 > $out/ser.log 2>&1 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 host > $out/plain.log 2>&1
