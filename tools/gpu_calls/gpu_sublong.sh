# GPU box: sublong voting parity (reference fixtures, literal / chunked modes, oracle at scale)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sublong.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_sublong.log 2>&1
[ $? -eq 0 ] && timeout -k 10 500 python -u tools/bench_long.py --gap 1 > gpurun_out/bench_long_full.json 2> gpurun_out/bench_long_full.err
[ $? -eq 0 ] && timeout -k 10 400 python -u tools/e2e_dropin.py --mbp 200 --reads 2000000 > gpurun_out/e2e.json 2> gpurun_out/e2e.err
