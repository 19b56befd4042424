#!/bin/bash
# GPU box, round 6: end to end on the final commit at human scale (C3 genome, 3.0 Gbp, 3M x 100 bp SE,
# the GPU builder's index files), stock subread-align vs the drop-in, the reference's default output
# (BAM, -T 16, unordered), outputs compared
out=gpurun_out/r6e2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --bam --kinds dump,dropin \
  --workdir /tmp/e2e_c3 --out $out/e2e_c3_bam.json > $out/e2e_c3_bam.log 2>&1
