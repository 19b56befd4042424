#!/bin/bash
# GPU box, round 6 call B: the drop-in tests (every stage asserted to be the library's; BAM through
# the library; the loader's error message), then the untraced single-stream C3 host step's HIP-event
# kernel record (the r05 serial figures were taken under the tracer)
out=gpurun_out/r6b
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_dropin.py \
  tests/test_gpu_builder.py -k "dropin or missing_array" > $out/tests.txt 2>&1 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 host overlap=0 > $out/serial_plain.log 2>&1
