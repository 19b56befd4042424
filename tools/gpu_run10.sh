# GPU box: parity (golden incl. PE / subjunc PE, lane, scale, io, events), C5pe phases and bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane.py tests/test_gpu_scale.py tests/test_gpu_io.py tests/test_events.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests10.log 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 400 python -u tools/phase_profile.py c3 2000000 sjpe > gpurun_out/phase_c5pe.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_10.json 2> gpurun_out/c5pe_10.err
