#!/bin/bash
# GPU box, round 5 call Y: verification of the final build -- the whole GPU suite (incl. the 60 Mbp
# open-vs-build test and the C3 50M digest), end to end at C3 and 200 Mbp (test dumps off; the
# index open now overlaps the first chunk's read), the bench line, and svg_index_open's clocks
mkdir -p gpurun_out/r5y
timeout -k 10 1200 python -u -m pytest -x -q --timeout 800 --timeout-method thread -m gpu tests/ > gpurun_out/r5y/tests.txt 2>&1 &&
timeout -k 10 900 python -u tools/e2e_dropin.py --genome c3 --gpu-build --reads 3000000 --kinds dump,dropin --no-startup \
    --out gpurun_out/r5y/e2e_c3.json > gpurun_out/r5y/e2e_c3.out 2> gpurun_out/r5y/e2e_c3.err &&
timeout -k 10 900 python -u tools/e2e_dropin.py --mbp 200 --reads 3000000 --kinds dump,dropin,dropin_refit2 \
    --out gpurun_out/r5y/e2e_c200m.json > gpurun_out/r5y/e2e_c200m.out 2> gpurun_out/r5y/e2e_c200m.err &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5y/bench.json 2> gpurun_out/r5y/bench.err &&
timeout -k 10 400 python -u tools/index_open_time.py "${TMPDIR:-/tmp}/svg_open_c3" 2 > gpurun_out/r5y/open.json 2> gpurun_out/r5y/open.err
