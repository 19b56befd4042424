#!/bin/bash
# GPU box, round 4 call G: the secondary workloads on the current build (bench.py, parity-checked
# in the same runs): C3g (gapped index, the reference's default), C4 PE, C5 subjunc, C5pe
mkdir -p gpurun_out/r4g
for wl in c3g c4 c5 c5pe; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 \
    > gpurun_out/r4g/bench_$wl.json 2> gpurun_out/r4g/bench_$wl.err || exit $?
done
