#!/bin/bash
# GPU box, round 4 call W: CU masks on the library's streams (wave-kernel stream on K CUs; the
# probe / lane stream on all or on the rest) -- one bench process per configuration
mkdir -p gpurun_out/r4w
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 "$@" \
    > gpurun_out/r4w/bench_$name.json 2> gpurun_out/r4w/bench_$name.err
}
run base && run k64 --opt wave_cus=64 && run k128 --opt wave_cus=128 && run k64x --opt wave_cus=64 --opt lane_cus_excl=1 && \
run k96x --opt wave_cus=96 --opt lane_cus_excl=1 && run k192 --opt wave_cus=192
