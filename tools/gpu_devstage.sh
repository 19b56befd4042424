# GPU box: device-path record staging -- parity (device-entry tests) then bench (device_path figure with and without staging)
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_io.py tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_devstage_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu --ascii-reads 0 --long-reads 0 --steps 3 --warmup 1 --device-steps 5 > gpurun_out/devstage_on.json 2> gpurun_out/devstage_on.err && \
SVG_DEV_STAGE=0 timeout -k 10 400 python -u bench.py --no-cpu --no-check --ascii-reads 0 --long-reads 0 --steps 3 --warmup 1 --device-steps 5 > gpurun_out/devstage_off.json 2> gpurun_out/devstage_off.err
