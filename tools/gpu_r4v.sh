#!/bin/bash
# GPU box, round 4 call V (final build): the whole GPU suite, smoke(), the default bench line
mkdir -p gpurun_out/r4v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4v/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4v/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4v/c3_kernel_record_bench.json > gpurun_out/r4v/bench_c3.json 2> gpurun_out/r4v/bench_c3.err
