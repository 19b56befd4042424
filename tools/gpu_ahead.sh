# GPU box: probe-ahead host pipeline -- parity (host-path tests, C3 scale, 10M-read digest) then C3 A/B (on vs SVG_PROBE_AHEAD=0)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_io.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_digest.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_ahead_tests.log 2>&1 && \
bash tools/gpu_ab.sh SVG_PROBE_AHEAD 0 --steps 10 --warmup 2
