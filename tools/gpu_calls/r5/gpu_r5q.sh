#!/bin/bash
# GPU box, round 5 call Q: rocprofv3 evidence of the metric's path on the final build -- kernel trace
# (--kernel-trace --stats) + FETCH_SIZE + WRITE_SIZE passes, each its own run; then the serialised
# single-stream trace and the HIP-event kernel record (tools/profile_serial.sh)
mkdir -p gpurun_out/r5q
bash tools/profile_workload.sh c3 50000000 gpurun_out/r5q/c3 3 host &&
bash tools/profile_serial.sh c3 gpurun_out/r5q/serial 3
