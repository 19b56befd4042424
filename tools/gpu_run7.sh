# GPU box: lane parity subset + the bin-order sweep
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_digest.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests7.log 2>&1 && \
timeout -k 10 600 python3 -u tools/sweep_host.py c3 4 light:SVG_LANE_BIN=2 nobin:SVG_LANE_BIN=0 nowave:SVG_DIAG_NOWAVE=1 nowave_nobin:SVG_DIAG_NOWAVE=1,SVG_LANE_BIN=0 base2: > gpurun_out/sweep7.txt 2>&1
