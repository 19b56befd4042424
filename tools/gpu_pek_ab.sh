# GPU box: lane PE kernel slot pool K=31 (default) vs K=47 (variant library): C5pe, C4, then PE parity with K=47
mkdir -p gpurun_out
for v in default pek47; do
  if [ $v = pek47 ]; then export SVG_LIB=subread_amd/lib_ab/libsubread_amd_pek47.so; fi
  timeout -k 10 400 python -u bench.py --workload c5pe --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c5pe_$v.json 2> gpurun_out/c5pe_$v.err || exit 1
  timeout -k 10 400 python -u bench.py --workload c4 --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 3 --warmup 1 > gpurun_out/c4_$v.json 2> gpurun_out/c4_$v.err || exit 1
done
SVG_LIB=subread_amd/lib_ab/libsubread_amd_pek47.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_pek47_tests.log 2>&1
