#!/bin/bash
# GPU box, round 5 call P: the whole GPU suite, then the bench line (default workload C3, with the
# reference's CPU voting step timed in the same run) and its per-kernel HIP-event record
mkdir -p gpurun_out/r5p
timeout -k 10 1100 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/ > gpurun_out/r5p/tests.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --kernel-record gpurun_out/r5p/c3_kernel_record_bench.json > gpurun_out/r5p/bench.json 2> gpurun_out/r5p/bench.err
