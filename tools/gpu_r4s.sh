#!/bin/bash
# GPU box, round 4 call S: pairs' deferred reads all from the work counter again -- parity tests,
# C4 and C5pe
mkdir -p gpurun_out/r4s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4s/gpu_tests.log 2>&1 || exit $?
for wl in c4 c5pe; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 \
    > gpurun_out/r4s/bench_$wl.json 2> gpurun_out/r4s/bench_$wl.err || exit $?
done
timeout -k 10 400 python -u tools/sweep_host.py c4 5 'pe6:wave_static=6' 'pe0:wave_static=0' 'pe4:wave_static=4' > gpurun_out/r4s/sweep_c4.txt 2>&1
