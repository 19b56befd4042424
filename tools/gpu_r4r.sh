#!/bin/bash
# GPU box, round 4 call R: the HBM-resident entry's records array from torch's allocator vs
# hipMalloc (one process each, host path beside it), then the secondary workloads on the
# round-end build
mkdir -p gpurun_out/r4r
timeout -k 10 300 python -u tools/ab_images.py --config bcode: --rounds 4 --device --out gpurun_out/r4r/dev_torch.json > gpurun_out/r4r/dev_torch.out 2> gpurun_out/r4r/dev_torch.err && \
timeout -k 10 300 python -u tools/ab_images.py --config bcode: --rounds 4 --device --hipmalloc --out gpurun_out/r4r/dev_hipmalloc.json > gpurun_out/r4r/dev_hipmalloc.out 2> gpurun_out/r4r/dev_hipmalloc.err || exit $?
for wl in c3g c4 c5 c5pe; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu --ascii-reads 0 --long-reads 0 --device-steps 3 \
    > gpurun_out/r4r/bench_$wl.json 2> gpurun_out/r4r/bench_$wl.err || exit $?
done
