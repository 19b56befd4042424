#!/bin/bash
# GPU box, round 6 call M: the wave kernel's next-read index loaded a whole read ahead (lane 0, vector
# load; made scalar at the prefetch point) -- vote-path parity tests, interleaved A/B on the C3 host
# step against the build of d8e0940, then C5 / C3g bench lines of the build under test
out=gpurun_out/r6m
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_d8e.so \
  > $out/ab_c3.txt 2> $out/ab_c3.err &&
timeout -k 10 400 python3 -u bench.py --workload c5 --no-cpu > $out/bench_c5.json 2> $out/bench_c5.err &&
timeout -k 10 400 python3 -u bench.py --workload c3g --no-cpu > $out/bench_c3g.json 2> $out/bench_c3g.err
