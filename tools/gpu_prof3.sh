# GPU box: rocprofv3 evidence of the host path (kernel trace + FETCH/WRITE), then SQ counters
mkdir -p gpurun_out
bash tools/profile_workload.sh c3 50000000 gpurun_out/r03prof 3 host > gpurun_out/r03prof.log 2>&1 && \
bash tools/pmc_sq.sh gpurun_out/r03sq c3 > gpurun_out/r03sq.txt 2>&1
