#!/bin/bash
# GPU box, round 5 call X: the .array read in parallel slices -- the builder / open tests, then the
# phase clocks of svg_index_open on the C3 files
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_builder.py > gpurun_out/r5x/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/index_open_time.py "${TMPDIR:-/tmp}/svg_open_c3" 3 > gpurun_out/r5x/open.json 2> gpurun_out/r5x/open.err
