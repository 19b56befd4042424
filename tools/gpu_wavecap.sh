# GPU box: C3 with the overlapped wave kernel's blocks-per-CU cap at 5 / 6 (default) / 7
mkdir -p gpurun_out
for v in 6 5 7; do
  SVG_WAVE_CAP=$v timeout -k 10 400 python -u bench.py --no-cpu --no-check --ascii-reads 0 --long-reads 0 --device-steps 1 --steps 8 --warmup 2 > gpurun_out/c3_cap_$v.json 2> gpurun_out/c3_cap_$v.err || exit 1
done
