#!/bin/bash
# GPU box, round 5 call I: vote-table sizes of C3 reads (oracle histogram) and the lane path's
# deferral reasons on the same workload
mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u tools/table_hist.py 400000 > gpurun_out/r5i/table_hist.txt 2> gpurun_out/r5i/table_hist.err &&
timeout -k 10 300 python -u tools/lane_defer.py c3 2000000 > gpurun_out/r5i/lane_defer.txt 2> gpurun_out/r5i/lane_defer.err
