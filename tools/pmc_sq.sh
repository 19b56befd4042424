#!/bin/bash
# SQ instruction/stall counters per kernel (three separate --pmc passes, no traces),
# bench.py on a reduced C3 read count.  Usage: tools/pmc_sq.sh OUTDIR [extra bench args]
set -e
out=$1; shift
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS"
C="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM"
i=0
for set in "$A" "$B" "$C"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $out/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-check "$@" > $out/p$i.log 2>&1
done
python3 - "$out" <<'PY'
import sqlite3, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
names = ("probe_kernel", "gather_kernel", "lane_kernel", "vote_kernel")
for d in sorted(glob.glob(out + "/p*/")):
    for db in glob.glob(d + "*results.db"):
        c = sqlite3.connect(db)
        for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            for kn in names:
                if kn in k:
                    tot[(kn, n)] += float(v)
for kn in names:
    rows = sorted((n, v) for (k, n), v in tot.items() if k == kn)
    if rows:
        print(kn)
        for n, v in rows:
            print("  %-26s %.4e" % (n, v))
PY
