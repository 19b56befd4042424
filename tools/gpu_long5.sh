# GPU box: sublong parity (GPU tests) + long-read bench with the pipelined downloads (full, gapped)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sublong.py tests/test_gpu_dropin.py -k "sublong" -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_sublong5.log 2>&1 && \
SVG_LONG_DEBUG=1 timeout -k 10 400 python -u tools/bench_long.py --gap 1 --steps 3 > gpurun_out/bench_long_full5.json 2> gpurun_out/bench_long_full5.err && \
timeout -k 10 400 python -u tools/bench_long.py --gap 3 --steps 3 > gpurun_out/bench_long_gapped5.json 2> gpurun_out/bench_long_gapped5.err
