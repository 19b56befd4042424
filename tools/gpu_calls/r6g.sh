#!/bin/bash
# GPU box, round 6 call G: the committed profile evidence of the final build, C3 host path (bench.py's
# metric): kernel trace + FETCH_SIZE + WRITE_SIZE passes (per-kernel HBM traffic), the SQ counter passes
# (issue, LDS bank conflicts), the single-stream trace and the untraced HIP-event kernel record
out=gpurun_out/r6g
mkdir -p $out
bash tools/profile_workload.sh c3 50000000 $out/c3 3 host &&
bash tools/pmc_sq.sh $out/sq c3 > $out/sq.txt 2>&1 &&
bash tools/profile_serial.sh c3 $out/serial 3 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 device > $out/device_record.log 2>&1 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 host > $out/host_record.log 2>&1
