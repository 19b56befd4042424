set -o pipefail
mkdir -p gpurun_out
for cfg in "40 24" "64 24" "40 16" "96 24"; do
  set -- $cfg
  SVG_LANE_CAP=$1 SVG_LANE_K=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-check --steps 3 > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.log || exit 1
done
