#!/bin/bash
# GPU box, round 6 call C: the wave kernel's single-pass top-3 and the multi-device index open --
# vote-path parity tests with the new library, an interleaved A/B against the previous build
# (libsubread_amd_base.so; _top1: top-3 only, the current one also with the scalar loop state) on the
# C3 host step, and the device path with / without host pacing
out=gpurun_out/r6c
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_scale.py tests/test_gpu_digest.py tests/test_gpu_builder.py -k "not gpu_built_index_md5" > $out/tests.txt 2>&1 &&
timeout -k 10 700 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib/libsubread_amd_top1.so subread_amd/lib/libsubread_amd_base.so > $out/ab.txt 2> $out/ab.err &&
SETTINGS="host;0,1;0,1,1" ROUNDS=3 timeout -k 10 400 python3 -u tools/device_sweep.py > $out/dev.txt 2> $out/dev.err
