#!/usr/bin/env python3
"""Aggregate a rocprofv3 PC-sampling CSV (host_trap) by code offset: the hottest instruction offsets of
each kernel, to be mapped onto the ISA of the same build (hipcc -S).  Usage: pcs_summary.py DIR OUT"""
import collections
import csv
import glob
import os
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    files = [f for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True) if "pc_sampl" in os.path.basename(f).lower()]
    with open(out, "w") as o:
        o.write("files: %s\n" % files)
        for f in files:
            with open(f, newline="") as fh:
                r = csv.reader(fh)
                hdr = next(r)
                o.write("header: %s\n" % hdr)
                low = [h.lower() for h in hdr]
                def col(*keys):
                    for k in keys:
                        for i, h in enumerate(low):
                            if k in h:
                                return i
                    return None
                ioff = col("offset", "pc")
                ikn = col("kernel_name", "kernel")
                icode = col("code_object_id")
                cnt = collections.Counter()
                tot = collections.Counter()
                n = 0
                for row in r:
                    n += 1
                    kn = row[ikn] if ikn is not None else "?"
                    key = (kn[:60], row[icode] if icode is not None else "", row[ioff] if ioff is not None else "")
                    cnt[key] += 1
                    tot[kn[:60]] += 1
                o.write("samples: %d\n" % n)
                for k, v in tot.most_common(20):
                    o.write("kernel %8d  %s\n" % (v, k))
                for k, v in cnt.most_common(400):
                    o.write("%8d  %s\n" % (v, "  ".join(k)))


if __name__ == "__main__":
    main()
