# GPU box: vote-kernel parity (golden, lane/wave, C3 scale, 10M digest, drop-in), then C3 and C5pe benches
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_digest.py tests/test_gpu_scale.py tests/test_gpu_io.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests8.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu --no-check --ascii-reads 0 --device-steps 1 > gpurun_out/c3_8.json 2> gpurun_out/c3_8.err && \
timeout -k 10 600 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_8.json 2> gpurun_out/c5pe_8.err
