#!/bin/bash
# GPU box, round 6 call O: the chunk-neighbour table widened to 62 entries (btab + the vote table's
# unused 25th slot of each row), the next-read index change dropped -- vote-path parity tests incl. the
# 50M C3 digest, an interleaved A/B on the C3 host step against the 32-entry build of call N
# (libsubread_amd_t32.so) and d8e0940 (a PC-sampling pass after it was refused by the pool: not used)
out=gpurun_out/r6o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py > $out/tests.txt 2>&1 &&
timeout -k 10 900 python3 -u tools/ab_libs.py c3 5 subread_amd/lib/libsubread_amd.so subread_amd/lib_ab/libsubread_amd_t32.so \
  subread_amd/lib_ab/libsubread_amd_d8e.so > $out/ab_c3.txt 2> $out/ab_c3.err &&
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1000 --output-format csv -d $out/pcs -o run -- python3 tools/prof_run.py c3 1 host > $out/pcs.log 2>&1
rc=$?
python3 tools/pcs_summary.py $out/pcs $out/pcs_summary.txt > $out/pcs_summary.log 2>&1
find $out/pcs -name '*.csv' -size +20M -delete
exit $rc
