#!/bin/bash
# GPU box, round 4 call AE (final build): end to end, then the serialised trace + HIP-event record
mkdir -p gpurun_out/r4ae
timeout -k 10 500 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r4ae/e2e.json > gpurun_out/r4ae/e2e.out 2> gpurun_out/r4ae/e2e.err && \
timeout -k 10 700 bash tools/profile_serial.sh c3 gpurun_out/r4ae/serial 3
rc=$?
rm -rf gpurun_out/r4ae/serial/serial
exit $rc
