#!/bin/bash
# GPU box, round 5 call H: the wave kernel's packed 3-row lane map -- parity tests, an interleaved
# A/B against the previous build (C3 host path), and the LDS counters of the new build
mkdir -p gpurun_out/r5h
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lane.py > gpurun_out/r5h/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py c3 6 subread_amd/lib/ab/lib_old.so subread_amd/lib/ab/lib_new.so > gpurun_out/r5h/ab.txt 2> gpurun_out/r5h/ab.err &&
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/r5h/pmc -o run -- python3 tools/prof_run.py c3 1 host > gpurun_out/r5h/pmc.log 2>&1
