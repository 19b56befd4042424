#!/bin/bash
# GPU box, round 4 call O (the build of the round's end): the whole GPU suite, smoke(), the default
# bench line (CPU baseline, ASCII entry, sublong figure included), end to end
mkdir -p gpurun_out/r4o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4o/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4o/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4o/c3_kernel_record_bench.json > gpurun_out/r4o/bench_c3.json 2> gpurun_out/r4o/bench_c3.err
