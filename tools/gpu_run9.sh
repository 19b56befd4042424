# GPU box: wave-kernel parity subset, phase shares (stamps build), C3 sweep
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_digest.py tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests9.log 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 400 python -u tools/phase_profile.py c3 5000000 se > gpurun_out/phase_c3.txt 2>&1 && \
timeout -k 10 600 python3 -u tools/sweep_host.py c3 4 base2: > gpurun_out/sweep9.txt 2>&1
