#!/bin/bash
# GPU box, round 4 call Q: the round-end build's roofline evidence (serialised single-stream trace,
# HIP-event record, kernel trace + FETCH_SIZE / WRITE_SIZE passes; raw databases kept small) and
# the end-to-end drop-in run
mkdir -p gpurun_out/r4q
timeout -k 10 700 bash tools/profile_serial.sh c3 gpurun_out/r4q/serial 3 && \
timeout -k 10 900 bash tools/profile_workload.sh c3 50000000 /tmp/r4q_work 3 host && \
cp /tmp/r4q_work/summary.json /tmp/r4q_work/summary.md gpurun_out/r4q/ && \
timeout -k 10 500 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r4q/e2e.json > gpurun_out/r4q/e2e.out 2> gpurun_out/r4q/e2e.err
rc=$?
rm -rf /tmp/r4q_work gpurun_out/r4q/serial/serial
exit $rc
