# GPU box: the whole -m gpu suite, then a short C3 bench line
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread --ignore=tests/test_gpu_digest.py > gpurun_out/gputests2.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
