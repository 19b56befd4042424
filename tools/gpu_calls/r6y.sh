#!/bin/bash
# GPU box, round 6 call Y: call U again on another box -- the branch-free neighbour-member loop + the
# gap-1 fast path against the final build, two libraries at a time in both orders (parity of this code
# was green in call U: 181 passed incl. the 50M C3 digest)
out=gpurun_out/r6y
mkdir -p $out
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_bf.so subread_amd/lib_ab/libsubread_amd_head.so > $out/ab_a.txt 2> $out/ab_a.err &&
timeout -k 10 500 python3 -u tools/ab_libs.py c3 5 subread_amd/lib_ab/libsubread_amd_head.so subread_amd/lib_ab/libsubread_amd_bf.so > $out/ab_b.txt 2> $out/ab_b.err
