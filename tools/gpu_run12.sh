# GPU box: probe-image refactor + image-backed key lookups -- parity (golden, probe images, C3/C3g
# scale, prefill vs the reference), then the keys/s benchmark
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prefill.py tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests12.log 2>&1 && \
timeout -k 10 600 python3 -u tools/bench_keys.py > gpurun_out/bench_keys.txt 2>&1
