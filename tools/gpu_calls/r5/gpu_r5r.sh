#!/bin/bash
# GPU box, round 5 call R: all 50M reads of the C3 bench workload, GPU records against the
# reference aligner's own (digests per 1M-read block, streamed through a pipe)
mkdir -p gpurun_out/r5r
df -h "${TMPDIR:-/tmp}" > gpurun_out/r5r/df.txt 2>&1
timeout -k 10 1500 python -u tools/c3_reference_digest.py 50000000 "${TMPDIR:-/tmp}/svg_c3dig" > gpurun_out/r5r/digest.json 2> gpurun_out/r5r/digest.err
