# GPU box: SQ counters (three --pmc passes) of the C3 host path with the final build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc_sq.sh gpurun_out/sq_final c3 > gpurun_out/sq_final.txt 2>&1
