#!/bin/bash
# GPU box, round 6 call Z: the final build with the branch-free neighbour-member loop and the gap-1
# fast path (A/B in both orders: profiles/r06/r6y) -- the whole GPU suite, smoke(), bench.py's line
out=gpurun_out/r6z
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ > $out/gpu_tests.txt 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 &&
timeout -k 10 500 python3 -u bench.py > $out/bench.json 2> $out/bench.err
