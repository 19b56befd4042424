#!/bin/bash
# GPU box, round 6 call J: the vote kernel's PE / subjunc variants without scratch-resident wave state
# (topk / emit / run_read / vote_end inlined, per-end arrays read by value, the pair top-3 as scalars:
# PE subjunc scratch 920 -> 196 B/lane, PE align 20 -> 0) -- vote-path parity tests, an interleaved
# A/B on C5pe against the HEAD build, the bench line, C4 / C5pe bench lines, the SQ counter passes
out=gpurun_out/r6j
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_fragile.py > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c5pe 3 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_c314.so \
  > $out/ab_c5pe.txt 2> $out/ab_c5pe.err &&
timeout -k 10 500 python3 -u bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 400 python3 -u bench.py --workload c4 --no-cpu > $out/bench_c4.json 2> $out/bench_c4.err &&
timeout -k 10 400 python3 -u bench.py --workload c5pe --no-cpu > $out/bench_c5pe.json 2> $out/bench_c5pe.err &&
bash tools/pmc_sq.sh $out/sq c3 > $out/sq.txt 2>&1
rc=$?
rm -rf $out/sq/p*/
exit $rc
