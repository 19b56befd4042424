# GPU box: the HBM-resident entry at two chunk sizes (1M reads = MALL-resident probe records,
# 6.29M = 1 GiB), plain timing then a kernel trace of each
mkdir -p gpurun_out/devchunk
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prof_run.py c3 3 device > gpurun_out/devchunk/plain_1m.txt 2>&1 && \
SVG_CHUNK=6291456 timeout -k 10 300 python3 tools/prof_run.py c3 3 device > gpurun_out/devchunk/plain_6m.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/devchunk/t1m -o run -- python3 tools/prof_run.py c3 2 device > gpurun_out/devchunk/t1m.log 2>&1 && \
SVG_CHUNK=6291456 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/devchunk/t6m -o run -- python3 tools/prof_run.py c3 2 device > gpurun_out/devchunk/t6m.log 2>&1
