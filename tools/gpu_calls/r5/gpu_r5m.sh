#!/bin/bash
# GPU box, round 5 call M: the streamed index open against the built index (60 Mbp), the drop-in
# GPU tests (bulk FASTQ read, library anti-support scan), then end to end: C3 genome (3.0 Gbp)
# and the 200 Mbp genome, 3M reads each, stock vs drop-in
mkdir -p gpurun_out/r5m
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_builder.py tests/test_gpu_dropin.py > gpurun_out/r5m/tests.txt 2>&1 &&
timeout -k 10 900 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5m/e2e_c3.json > gpurun_out/r5m/e2e_c3.out 2> gpurun_out/r5m/e2e_c3.err &&
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --kinds dump,dropin,dropin_refit2 \
    --out gpurun_out/r5m/e2e_c200m.json > gpurun_out/r5m/e2e_c200m.out 2> gpurun_out/r5m/e2e_c200m.err
