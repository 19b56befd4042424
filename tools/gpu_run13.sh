# GPU box: batch-mode opener groups -- parity (golden, lane, scale, digest, io, events), phases, C3 and C5pe
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_digest.py tests/test_gpu_scale.py tests/test_gpu_io.py tests/test_events.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests13.log 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 2000000 sjpe > gpurun_out/phase_c5pe.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 5000000 se > gpurun_out/phase_c3.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: > gpurun_out/sweep13.txt 2>&1 && \
timeout -k 10 500 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_13.json 2> gpurun_out/c5pe_13.err
