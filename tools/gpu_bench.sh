# GPU box: one default bench.py run (C3), JSON line + log under gpurun_out/
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
