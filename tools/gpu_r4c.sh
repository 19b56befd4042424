#!/bin/bash
# GPU box, round 4 call C: the interleaved A/B of the probe images at C3 (bucket code, key-hash
# beside it, inline key-hash), end to end with the full binding (stock vs drop-in, phase clocks),
# then the CPU-baseline calibration on this box's own CPU (reference voting step vs the
# restatement, C3 reads, index files written by the GPU builder)
mkdir -p gpurun_out/r4c
timeout -k 10 400 python -u tools/ab_images.py --config bcode: --config khash:khash_probe=1 --config kinline:kinline=1 --rounds 8 --device --out gpurun_out/r4c/ab_images.json > gpurun_out/r4c/ab.out 2> gpurun_out/r4c/ab.err && \
timeout -k 10 500 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --out gpurun_out/r4c/e2e.json > gpurun_out/r4c/e2e.out 2> gpurun_out/r4c/e2e.err && \
timeout -k 10 600 python -u tools/cpu_calibration.py --workload c3 --gpu-build --reads 1000000 --threads 16 --repeats 2 --workdir /tmp/svg_cal --out gpurun_out/r4c/r04_cpu_calibration.json > gpurun_out/r4c/cal.out 2> gpurun_out/r4c/cal.err
rc=$?
rm -rf /tmp/svg_cal
exit $rc
