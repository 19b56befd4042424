# GPU box: the live drop-in (stock subread-align / subjunc with the GPU voting step, GPU fragile
# windows) against the stock binaries, then the 10M-read C2 digest against the reference's records
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/dropin5.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/digest5.log 2>&1
