#!/bin/bash
# rocprofv3 evidence for the bench workloads, one after the other (GPU box).
# Usage: tools/profile_all.sh OUTDIR [workloads...]   (default: c3 c4 c5)
# READS is bench.py's n for the workload (pairs for the PE workload c4), so that
# traffic_bytes_per_read * n / launches_per_step in bench.py is the traffic of one launch.
set -e
out=$1; shift
wls=${@:-c3 c4 c5}
for wl in $wls; do
  case $wl in c2) n=10000000 ;; c4) n=25000000 ;; *) n=50000000 ;; esac
  bash tools/profile_workload.sh $wl $n $out/$wl
done
