#!/bin/bash
# GPU box, round 5 call D: end to end at human scale -- bench.py's C3 genome (3.0 Gbp), its full
# index written to files by the GPU builder, 3M x 100 bp reads: stock vs drop-in (GPU vote + the
# library's iteration two), outputs compared byte for byte; df first (the .tab is ~18 GB)
mkdir -p gpurun_out/r5d
df -h "${TMPDIR:-/tmp}" . > gpurun_out/r5d/df.txt 2>&1
timeout -k 10 1100 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5d/e2e_c3.json > gpurun_out/r5d/e2e.out 2> gpurun_out/r5d/e2e.err
