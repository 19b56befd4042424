# GPU box: fragile-voting parity (GPU windows vs the restatement, GPU windows -> reference events),
# then the wave kernel's phase shares on C3's deferred reads (stamps build)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fragile.py tests/test_events.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fragile4.log 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 5000000 se > gpurun_out/phase4.txt 2>&1
