#!/bin/bash
# GPU box, round 4 call D: the GPU test suite (one shared stream set per device; the binding's
# plain-FASTQ parse), the probe-image A/B again (bucket code vs the key-hash beside it: with the
# shared streams the key-hash handle's 152 ms/step of call C should be gone), end to end
mkdir -p gpurun_out/r4d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4d/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_images.py --config bcode: --config khash:khash_probe=1 --rounds 6 --device --out gpurun_out/r4d/ab_images.json > gpurun_out/r4d/ab.out 2> gpurun_out/r4d/ab.err && \
timeout -k 10 500 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r4d/e2e.json > gpurun_out/r4d/e2e.out 2> gpurun_out/r4d/e2e.err
