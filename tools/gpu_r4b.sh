#!/bin/bash
# GPU box, round 4 call B: the C3 bench line (+ kernel record), the serialised trace and the HIP-event
# kernel record of the metric's path (profiles/ evidence for the roofline)
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4b/c3_kernel_record_bench.json > gpurun_out/r4b/bench_c3.json 2> gpurun_out/r4b/bench_c3.err && \
bash tools/profile_serial.sh c3 gpurun_out/r4b 3 > gpurun_out/r4b/profile_serial.log 2>&1
