# GPU box: host-path knob sweep (tools/sweep_host.py), output in gpurun_out/sweep_<wl>.txt
mkdir -p gpurun_out
wl=$1; shift
timeout -k 10 900 python3 -u tools/sweep_host.py $wl "$@" > gpurun_out/sweep_$wl.txt 2>&1
