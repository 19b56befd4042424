#!/bin/bash
# GPU box, round 6 call W: the final build's committed profile evidence -- C3 host-path kernel trace +
# FETCH_SIZE / WRITE_SIZE passes, the single-stream trace and the HIP-event kernel record, the device
# path's kernel record, the SQ counter passes
out=gpurun_out/${OUT:-r6w}
mkdir -p $out
bash tools/profile_workload.sh c3 50000000 $out/c3 3 host &&
bash tools/profile_serial.sh c3 $out/serial 3 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 device > $out/device_record.log 2>&1 &&
bash tools/pmc_sq.sh $out/sq c3 > $out/sq.txt 2>&1
rc=$?
rm -rf $out/serial/serial $out/sq/p*/
exit $rc
