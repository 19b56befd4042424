#!/bin/bash
# GPU box, round 5 call V: end to end on the final build, test dumps off: C3 genome (3.0 Gbp) and
# the 200 Mbp genome, 3M reads each, stock vs drop-in (and the drop-in with the reference's own
# iteration two)
mkdir -p gpurun_out/r5v
timeout -k 10 900 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5v/e2e_c3.json > gpurun_out/r5v/e2e_c3.out 2> gpurun_out/r5v/e2e_c3.err &&
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --kinds dump,dropin,dropin_refit2 \
    --out gpurun_out/r5v/e2e_c200m.json > gpurun_out/r5v/e2e_c200m.out 2> gpurun_out/r5v/e2e_c200m.err
