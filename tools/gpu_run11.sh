# GPU box: heavy lane bin -- parity with it on (C3 scale, lane tests, digest), then the sweep
mkdir -p gpurun_out
SVG_LANE_HEAVY=64 timeout -k 10 900 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_digest.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests11.log 2>&1 && \
timeout -k 10 700 python3 -u tools/sweep_host.py c3 4 heavy48:SVG_LANE_HEAVY=48 heavy56:SVG_LANE_HEAVY=56 heavy64:SVG_LANE_HEAVY=64 base2: > gpurun_out/sweep11.txt 2>&1
