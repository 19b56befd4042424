# GPU box: bench.py (no CPU leg / parity / ASCII figure) with and without a library option
# usage: gpu_ab.sh OPTION VALUE [bench args]
mkdir -p gpurun_out
var=$1; val=$2; shift 2
timeout -k 10 400 python -u bench.py --no-cpu --no-check --ascii-reads 0 --device-steps 1 "$@" > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err && \
timeout -k 10 400 python -u bench.py --opt $var=$val --no-cpu --no-check --ascii-reads 0 --device-steps 1 "$@" > gpurun_out/ab_knob.json 2> gpurun_out/ab_knob.err
