#!/bin/bash
# GPU box, round 5 call C: end to end 3M reads on the 200 Mbp genome: stock / drop-in with the
# library's iteration two / drop-in with the reference's iteration two
mkdir -p gpurun_out/r5c
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r5c/e2e.json > gpurun_out/r5c/e2e.out 2> gpurun_out/r5c/e2e.err
