#!/bin/bash
# GPU box, round 6 call K: the rest of the GPU suite on the build of d8e0940 (drop-in, io, builder,
# digest, prefill, shard, sublong, 2-rank bench), then the committed profile evidence of that build:
# C3 host-path kernel trace + FETCH_SIZE / WRITE_SIZE passes, the single-stream trace and the untraced
# HIP-event kernel record (host path), and the device path's HIP-event kernel record
out=gpurun_out/r6k
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_dropin.py \
  tests/test_gpu_io.py tests/test_gpu_builder.py tests/test_gpu_digest.py tests/test_gpu_prefill.py tests/test_gpu_shard.py \
  tests/test_gpu_sublong.py tests/test_gpu_bench_dist.py > $out/tests.txt 2>&1 &&
bash tools/profile_workload.sh c3 50000000 $out/c3 3 host &&
bash tools/profile_serial.sh c3 $out/serial 3 &&
timeout -k 10 300 python3 tools/prof_run.py c3 3 device > $out/device_record.log 2>&1
rc=$?
rm -rf $out/serial/serial
exit $rc
