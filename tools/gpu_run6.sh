# GPU box: lane-path parity (golden, lane edge cases, C3 scale, 10M digest), then the knob sweep
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_parity.py tests/test_gpu_digest.py tests/test_gpu_scale.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/tests6.log 2>&1 && \
timeout -k 10 600 python3 -u tools/sweep_host.py c3 4 nobin:SVG_LANE_BIN=0 nowave:SVG_DIAG_NOWAVE=1 base2: > gpurun_out/sweep6.txt 2>&1
