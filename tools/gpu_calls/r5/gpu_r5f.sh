#!/bin/bash
# GPU box, round 5 call F: the parallel bucket-chain walk of svg_index_open -- phase clocks on the
# C3 index files (18 GB .tab), then the GPU tests that open indexes from files
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u tools/index_open_time.py "${TMPDIR:-/tmp}/svg_open_c3" 2 > gpurun_out/r5f/open.json 2> gpurun_out/r5f/open.err &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_builder.py tests/test_gpu_dropin.py > gpurun_out/r5f/tests.txt 2>&1
