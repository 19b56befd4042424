#!/bin/bash
# GPU box, round 6 call I: the final-build evidence after the container restart -- bench.py's default
# line, then the C3 host-path kernel trace + FETCH_SIZE / WRITE_SIZE passes and the SQ counter passes
out=gpurun_out/r6i
mkdir -p $out
timeout -k 10 500 python3 -u bench.py > $out/bench.json 2> $out/bench.err &&
bash tools/profile_workload.sh c3 50000000 $out/c3 3 host &&
bash tools/pmc_sq.sh $out/sq c3 > $out/sq.txt 2>&1
