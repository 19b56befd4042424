# GPU box: long-read bench with per-phase chunk timings (full index), twice
mkdir -p gpurun_out
SVG_LONG_DEBUG=1 timeout -k 10 400 python -u tools/bench_long.py --gap 1 --steps 3 --check 0 --cpu-reads 0 > gpurun_out/bench_long_full4.json 2> gpurun_out/bench_long_full4.err
