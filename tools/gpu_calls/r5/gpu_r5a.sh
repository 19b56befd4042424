#!/bin/bash
# GPU box, round 5 call A: the drop-in with the library's iteration two (GPU vote) vs stock on the
# golden cases and 200k C2 reads, then end to end 3M reads (stock / library iteration two /
# reference iteration two)
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r5a/dropin_tests.txt 2>&1 && \
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r5a/e2e.json > gpurun_out/r5a/e2e.out 2> gpurun_out/r5a/e2e.err
