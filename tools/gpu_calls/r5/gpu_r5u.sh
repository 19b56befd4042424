#!/bin/bash
# GPU box, round 5 call U: where the time between the vote and iteration two goes (200 Mbp, 3M reads)
mkdir -p gpurun_out/r5u
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --kinds dump,dropin \
    --out gpurun_out/r5u/e2e_c200m.json > gpurun_out/r5u/e2e_c200m.out 2> gpurun_out/r5u/e2e_c200m.err
