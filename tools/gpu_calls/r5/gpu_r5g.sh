#!/bin/bash
# GPU box, round 5 call G: the HBM-resident entry's chunking against the host pipeline (C3, one
# process, interleaved), then the bench with the reference's CPU voting step timed in the same run
mkdir -p gpurun_out/r5g
timeout -k 10 400 python -u tools/device_sweep.py > gpurun_out/r5g/device_sweep.txt 2> gpurun_out/r5g/device_sweep.err &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5g/bench.json 2> gpurun_out/r5g/bench.err
