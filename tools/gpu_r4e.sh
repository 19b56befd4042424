#!/bin/bash
# GPU box, round 4 call E: the roofline's committed evidence for C3's metric path -- the
# serialised single-stream trace + the HIP-event kernel record (tools/profile_serial.sh), the
# kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile_workload.sh)
mkdir -p gpurun_out/r4e
timeout -k 10 700 bash tools/profile_serial.sh c3 gpurun_out/r4e/serial 3 && \
timeout -k 10 900 bash tools/profile_workload.sh c3 50000000 gpurun_out/r4e/work 3 host
