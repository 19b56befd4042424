#!/bin/bash
# GPU box, round 4 call AA (final build, 16 lane slots): the whole GPU suite, smoke(), the default
# bench line, C5 (single-end subjunc shares the lane kernel's slot count)
mkdir -p gpurun_out/r4aa
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4aa/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4aa/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --kernel-record gpurun_out/r4aa/c3_kernel_record_bench.json > gpurun_out/r4aa/bench_c3.json 2> gpurun_out/r4aa/bench_c3.err && \
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 > gpurun_out/r4aa/bench_c5.json 2> gpurun_out/r4aa/bench_c5.err
