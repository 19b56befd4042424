#!/bin/bash
# GPU box, round 5 call T: drop-in GPU tests (library remove_neighbour), end to end (C3 and 200 Mbp,
# 3M reads, stock vs drop-in), then the bench line with the reference's warm-up chunk
mkdir -p gpurun_out/r5t
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_dropin.py > gpurun_out/r5t/tests.txt 2>&1 &&
timeout -k 10 900 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5t/e2e_c3.json > gpurun_out/r5t/e2e_c3.out 2> gpurun_out/r5t/e2e_c3.err &&
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --kinds dump,dropin,dropin_refit2 \
    --out gpurun_out/r5t/e2e_c200m.json > gpurun_out/r5t/e2e_c200m.out 2> gpurun_out/r5t/e2e_c200m.err &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5t/bench.json 2> gpurun_out/r5t/bench.err
