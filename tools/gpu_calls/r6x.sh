#!/bin/bash
# GPU box, round 6 call X: the final build's secondary workloads (bench.py --workload, parity checked in
# each run): C4, C5, C5pe, C3g
out=gpurun_out/r6x
mkdir -p $out
for w in c4 c5 c5pe c3g; do
  timeout -k 10 400 python3 -u bench.py --workload $w --no-cpu > $out/bench_$w.json 2> $out/bench_$w.err || exit $?
done
