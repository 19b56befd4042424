#!/bin/bash
# GPU box, round 4 call V2 (final build, after the CU-mask and ramp-option changes): the whole GPU suite, smoke(), the default bench line
mkdir -p gpurun_out/r4v2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4v2/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4v2/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4v2/c3_kernel_record_bench.json > gpurun_out/r4v2/bench_c3.json 2> gpurun_out/r4v2/bench_c3.err
