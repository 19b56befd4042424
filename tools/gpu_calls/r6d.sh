#!/bin/bash
# GPU box, round 6 call D: end to end at human scale (C3 genome, 3.0 Gbp, 3M x 100 bp SE, the GPU
# builder's index files), stock subread-align vs the drop-in on this build: (1) the reference's
# default output, BAM (-T 16, unordered), incl. the drop-in with eight index replicas on this GPU
# (SVG_DEVICES=0,...,0: one read of the files, svg_index_open_devices); (2) SAM output
out=gpurun_out/r6d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --bam --kinds dump,dropin,dropin_dev \
  --devices 0,0,0,0,0,0,0,0 --workdir /tmp/e2e_c3 --out $out/e2e_c3_bam.json > $out/e2e_c3_bam.log 2>&1 &&
timeout -k 10 800 python3 -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
  --workdir /tmp/e2e_c3 --reuse --out $out/e2e_c3_sam.json > $out/e2e_c3_sam.log 2>&1
