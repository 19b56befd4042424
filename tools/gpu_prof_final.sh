# GPU box: rocprofv3 evidence of the metric's path with the round's final build (C3 host path):
# kernel trace + FETCH_SIZE + WRITE_SIZE passes, summarised per kernel
cd $GRAFT_REPO_ROOT
bash tools/profile_workload.sh c3 50000000 gpurun_out/prof_c3_final 3 host
