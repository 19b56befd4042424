# GPU box: sublong voting parity (reference fixtures, literal / chunked modes, oracle at scale)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sublong.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_sublong.log 2>&1
