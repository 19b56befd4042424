#!/bin/bash
# GPU box: serialised (single-stream) kernel trace of the metric's host path + the HIP-event
# kernel record of the normal (two-stream) path, for the roofline's committed evidence.
# Usage: tools/profile_serial.sh WORKLOAD OUTDIR [STEPS]   (OUTDIR under gpurun_out/)
set -e
wl=$1; out=$2; steps=${3:-3}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/serial -o run -- python3 tools/prof_run.py $wl $steps host overlap=0 > $out/serial.log 2>&1
python3 tools/serial_trace.py $out/serial $out/serial.log $out/${wl}_serial_trace.json --steps $steps
timeout -k 10 400 python3 tools/prof_run.py $wl $steps host > $out/record.log 2>&1
grep kernel_record $out/record.log > $out/${wl}_kernel_record.json
