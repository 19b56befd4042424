#!/bin/bash
# GPU box, round 4 call AD (final build): the whole GPU suite and smoke()
mkdir -p gpurun_out/r4ad
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4ad/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ad/smoke.log 2>&1
