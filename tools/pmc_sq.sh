#!/bin/bash
# SQ instruction/stall counters per kernel (three separate --pmc passes, no traces) of the
# host path bench.py times (tools/prof_run.py ... host: 1 warmup + 1 step).
# Usage: tools/pmc_sq.sh OUTDIR [WORKLOAD]
set -e
out=$1; wl=${2:-c3}
mkdir -p $out
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS"
C="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM"
i=0
for set in "$A" "$B" "$C"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set -d $out/p$i -o run -- python3 tools/prof_run.py $wl 1 host > $out/p$i.log 2>&1
done
python3 - "$out" <<'PY'
import sqlite3, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
names = ("probe_line_kernel", "probe_big_kernel", "probe_kernel", "gather_kernel", "lane_kernel", "vote_kernel",
         "compact_records", "unpack_reads")
def short(k):
    for kn in names:
        if kn in k:
            return kn
for d in sorted(glob.glob(out + "/p*/")):
    for db in glob.glob(d + "*results.db"):
        c = sqlite3.connect(db)
        for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            kn = short(k)
            if kn:
                tot[(kn, n)] += float(v)
for kn in names:
    rows = dict((n, v) for (k, n), v in tot.items() if k == kn)
    if not rows:
        continue
    print(kn)
    for n in sorted(rows):
        print("  %-26s %.4e" % (n, rows[n]))
    wc = rows.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print("  -> per wave-cycle: busy-issuing any %.3f, VALU %.3f, LDS %.3f, VMEM %.3f, waiting %.3f" % (
            rows.get("SQ_ACTIVE_INST_ANY", 0) / wc, rows.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            rows.get("SQ_ACTIVE_INST_LDS", 0) / wc, rows.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
            rows.get("SQ_WAIT_ANY", 0) / wc))
    if rows.get("SQ_INSTS"):
        print("  -> instructions %.3e: VALU %.2f, SALU %.2f, LDS %.2f, VMEM rd %.2f wr %.2f, branch %.2f" % (
            rows["SQ_INSTS"], rows.get("SQ_INSTS_VALU", 0) / rows["SQ_INSTS"], rows.get("SQ_INSTS_SALU", 0) / rows["SQ_INSTS"],
            rows.get("SQ_INSTS_LDS", 0) / rows["SQ_INSTS"], rows.get("SQ_INSTS_VMEM_RD", 0) / rows["SQ_INSTS"],
            rows.get("SQ_INSTS_VMEM_WR", 0) / rows["SQ_INSTS"], rows.get("SQ_INSTS_BRANCH", 0) / rows["SQ_INSTS"]))
PY
