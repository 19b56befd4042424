# GPU box: sublong parity + live sublong drop-in + bench (full, gapped) + e2e subread-align
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sublong.py tests/test_gpu_dropin.py -k "sublong" -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_sublong3.log 2>&1 && \
SVG_LONG_DEBUG=1 timeout -k 10 400 python -u tools/bench_long.py --gap 1 --steps 3 > gpurun_out/bench_long_full3.json 2> gpurun_out/bench_long_full3.err && \
timeout -k 10 400 python -u tools/bench_long.py --gap 3 --steps 3 > gpurun_out/bench_long_gapped3.json 2> gpurun_out/bench_long_gapped3.err && \
timeout -k 10 600 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 > gpurun_out/e2e2.json 2> gpurun_out/e2e2.err
[ $? -eq 0 ] && bash tools/gpu_ab.sh SVG_STREAM_PRIO 1 --steps 10 --warmup 2
