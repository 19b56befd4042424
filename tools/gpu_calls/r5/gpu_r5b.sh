#!/bin/bash
# GPU box, round 5 call B: the whole GPU suite after the option pruning (incl. the drop-in with two
# handles), then the default bench line
mkdir -p gpurun_out/r5b
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5b/gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5b/bench.json 2> gpurun_out/r5b/bench.err
