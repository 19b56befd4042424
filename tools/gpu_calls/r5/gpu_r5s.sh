#!/bin/bash
# GPU box, round 5 call S: the C3 50M digest test, then the secondary workloads' bench lines on the
# final build (no CPU leg): C3g (gapped index), C4 (PE 150 bp), C5 (subjunc), C5pe (subjunc PE)
mkdir -p gpurun_out/r5s
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread -m gpu tests/test_gpu_digest.py > gpurun_out/r5s/digest_tests.txt 2>&1 &&
for w in c3g c4 c5 c5pe; do
  timeout -k 10 600 python -u bench.py --workload $w --no-cpu --ascii-reads 0 --long-reads 0 > gpurun_out/r5s/bench_$w.json 2> gpurun_out/r5s/bench_$w.err || exit 1
done
