# GPU box: kernel traces of the host path with an env knob off / on
# usage: gpu_trace_ab.sh VAR OFFVAL ONVAL
mkdir -p gpurun_out/tab
export TMPDIR=/tmp
var=$1
env $var=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tab/off -o run -- python3 tools/prof_run.py c3 2 host > gpurun_out/tab/off.log 2>&1 && \
env $var=$3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tab/on -o run -- python3 tools/prof_run.py c3 2 host > gpurun_out/tab/on.log 2>&1
