# GPU box: interleaved A/B of two library builds (tools/ab_libs.py)
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_libs.py "$@" > gpurun_out/ab_libs.txt 2>&1
