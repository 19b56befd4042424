#!/bin/bash
# GPU box, round 4 call A: box facts, the GPU test suite + smoke, then the end-to-end phase split
# (stock vs drop-in, the reference's own phase clocks)
mkdir -p gpurun_out/r4a
(nproc; lscpu | grep -E "Model name|NUMA|Socket"; df -h /tmp . | cat; free -g) > gpurun_out/r4a/box.txt 2>&1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 && \
timeout -k 10 600 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r4a/e2e.json > gpurun_out/r4a/e2e.out 2> gpurun_out/r4a/e2e.err
