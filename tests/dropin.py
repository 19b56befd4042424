"""The drop-in harness: the reference's own subread-align / subjunc (oracle/_ref, built from
/root/reference/src by `make -C oracle dropin`) with integration/do_voting_gpu.c as its voting
step, run beside the stock reference binary on the same FASTQ; the outputs are compared byte
for byte (SAM except the @PG command line, .indel.vcf, .junction.bed, .breakpoint.vcf), plus
the reference's vote-record dump and event-table dump (oracle/ref_dump_hook.c), which both
binaries carry.

Binaries (test infrastructure, never part of the product):
  _ref/subread-align-dump, _ref/subjunc-dump      stock reference + dump hook
  _ref/subread-align-dropin, _ref/subjunc-dropin   the binding, votes on the GPU (libsubread_amd.so)
  _ref/*-oracle-dropin                             the binding, votes by the CPU restatement
"""
import glob
import os
import re
import subprocess

import numpy as np

from tests.common import ROOT

REFBIN = os.environ.get("SVG_TEST_REFBIN") or os.path.join(ROOT, "oracle", "_ref")


def binary(program, kind):
    return os.path.join(REFBIN, ("subjunc-" if program == 1 else "subread-align-") + kind)


def have(program, kind):
    return os.path.exists(binary(program, kind))


def write_fastq(path, batch):
    """FASTQ with varied (deterministic) qualities, so the text/quality orientation of the
    post-vote tail is exercised; the reads of a pair share their name."""
    with open(path, "wb") as f:
        for i in range(len(batch)):
            s = batch.read(i)
            q = bytes(33 + (i * 7 + k * 13) % 41 for k in range(len(s)))
            f.write(b"@r%d\n" % i + s + b"\n+\n" + q + b"\n")


def run(program, kind, index, f1, f2, out, threads=1, extra=(), env=None, timeout=900, sam=True):
    """One run of a reference binary (`kind`); the drop-ins run with SVG_REQUIRE_LIBRARY=1 unless
    `env` says otherwise, so that a stage falling back to the reference's own function fails the
    run instead of passing unnoticed (its output would be the stock program's by construction)."""
    args = [binary(program, kind), "-T", str(threads), "-i", index, "-r", f1, "-o", out] + (["--SAMoutput"] if sam else [])
    if program == 0:
        args += ["-t", "1"]
    if f2:
        args += ["-R", f2]
    args += list(extra)
    e = dict(os.environ, SVG_REF_DUMP=out + ".votes", SVG_REF_EVENTS=out + ".events")
    if kind.endswith("dropin"):
        e["SVG_REQUIRE_LIBRARY"] = "1"
    if env:
        e.update(env)
    for p in glob.glob(out + "*"):
        os.remove(p)
    r = subprocess.run(args, capture_output=True, text=True, env=e, timeout=timeout)
    assert r.returncode == 0, "%s failed (%d):\n%s\n%s" % (kind, r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return r


STAGES = ("vote", "fragile", "events", "anti_support", "remove_neighbour", "iteration_two")


def stages(stderr):
    """The drop-in's SVG_DROPIN_STAGES line: stage -> (runs by the library, runs by the reference's
    function)."""
    m = re.findall(r"^SVG_DROPIN_STAGES (.*)$", stderr, re.M)
    assert len(m) == 1, "no (or several) SVG_DROPIN_STAGES lines in the drop-in's stderr"
    d = {}
    for f in m[0].split():
        k, v = f.split("=")
        lib, ref = v.split(",")
        d[k] = (int(lib.split(":")[1]), int(ref.split(":")[1]))
    assert sorted(d) == sorted(STAGES), d
    return d


def assert_library(stderr, fragile=False):
    """Every stage of the drop-in run was the library's, each ran at least once (fragile voting only
    where the case has subjunc reads > 160 bp)."""
    st = stages(stderr)
    for k, (lib, ref) in st.items():
        assert ref == 0, "stage %s ran the reference's function %d times: %s" % (k, ref, st)
        if k != "fragile" or fragile:
            assert lib > 0, "stage %s never ran in the library: %s" % (k, st)
    return st


def outputs(out):
    """The files a run wrote: suffix -> bytes (SAM without its @PG line)."""
    res = {}
    for p in sorted(glob.glob(out + "*")):
        suf = p[len(out):]
        b = open(p, "rb").read()
        if suf == "":
            b = b"".join(l for l in b.splitlines(True) if not l.startswith(b"@PG"))
        res[suf] = b
    return res


def compare(stock_out, dropin_out):
    """Byte comparison of every output; returns a short report, raises on a difference."""
    a, b = outputs(stock_out), outputs(dropin_out)
    assert sorted(a) == sorted(b), (sorted(a), sorted(b))
    for suf in a:
        if a[suf] != b[suf]:
            la, lb = a[suf].splitlines(), b[suf].splitlines()
            bad = [i for i in range(min(len(la), len(lb))) if la[i] != lb[i]][:3]
            msg = "\n".join("line %d:\n  stock  %r\n  dropin %r" % (i, la[i][:300], lb[i][:300]) for i in bad)
            raise AssertionError("output %r differs (%d vs %d lines)\n%s" % (suf or ".sam", len(la), len(lb), msg))
    sam = a[""]
    recs = [l for l in sam.splitlines() if not l.startswith(b"@")]
    mapped = sum(1 for l in recs if not int(l.split(b"\t")[1]) & 4)
    return {"files": sorted(s or ".sam" for s in a), "sam_records": len(recs), "mapped": mapped}


def fastq_pair(tmp, name, r1, r2):
    f1 = os.path.join(tmp, name + "_1.fq")
    write_fastq(f1, r1)
    f2 = None
    if r2 is not None:
        f2 = os.path.join(tmp, name + "_2.fq")
        write_fastq(f2, r2)
    return f1, f2


def case_extra(case):
    over = case.meta["params_over"]
    extra = []
    if "total_subreads" in over:
        extra += ["-n", str(over["total_subreads"])]
    if "max_indel_length" in over:
        extra += ["-I", str(over["max_indel_length"])]
    return extra


def check_case(case, index, tmp, kind, threads=1, env=None, stock_env=None):
    """Stock reference vs the drop-in `kind` on a golden case's reads; identical outputs."""
    prog = case.meta["program"]
    f1, f2 = fastq_pair(tmp, case.name, case.r1, case.r2)
    so, do = os.path.join(tmp, case.name + ".stock.sam"), os.path.join(tmp, case.name + "." + kind + ".sam")
    run(prog, "dump", index, f1, f2, so, threads, case_extra(case), env=stock_env)
    r = run(prog, kind, index, f1, f2, do, threads, case_extra(case), env=env)
    rep = compare(so, do)
    long_sj = prog == 1 and max(int(case.r1.lens.max()), int(case.r2.lens.max()) if case.r2 is not None else 0) > 160
    rep["stages"] = assert_library(r.stderr, fragile=long_sj) if kind.endswith("dropin") else None
    # the dumped vote records are the golden records of the case (the reference dumps them
    # the same way when the fixtures are made)
    votes = np.fromfile(do + ".votes", dtype=np.uint8)
    assert votes.size == case.expected.size and (votes.reshape(case.expected.shape) == case.expected).all(), \
        "drop-in vote records differ from the golden records"
    return rep


# ---- sublong (src/longread-one): stock _ref/sublong vs _ref/sublong-dropin (GPU voting through
# integration/lrm_voting_gpu.c) or _ref/sublong-oracle-dropin (the restatement), same FASTQ

def sublong_binary(kind):
    return os.path.join(REFBIN, "sublong" if kind == "stock" else "sublong-" + kind)


def run_sublong(kind, index, fq, out, threads=1, timeout=900):
    args = [sublong_binary(kind), "-i", index, "-r", fq, "-o", out, "--SAMoutput", "-T", str(threads)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, "%s failed (%d):\n%s\n%s" % (kind, r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return r


def write_long_fastq(path, reads):
    """FASTQ of a LongReads batch (empty reads skipped: sublong's reader stops at one)."""
    with open(path, "wb") as f:
        for i in range(len(reads)):
            s = reads.read(i)
            if s:
                f.write(b"@r%d\n%s\n+\n%s\n" % (i, s, bytes(33 + (i * 7 + k * 13) % 41 for k in range(len(s)))))


def compare_sam(a_path, b_path, any_order=False):
    """Byte comparison of two SAM files without their @PG lines; any_order: as sorted line sets
    (sublong -T > 1 writes each thread's records in the order its reads were fetched)."""
    a = [l for l in open(a_path, "rb") if not l.startswith(b"@PG")]
    b = [l for l in open(b_path, "rb") if not l.startswith(b"@PG")]
    if any_order:
        a, b = sorted(a), sorted(b)
    bad = [i for i in range(min(len(a), len(b))) if a[i] != b[i]][:3]
    assert len(a) == len(b) and not bad, "SAM differs (%d vs %d lines): %s" % (
        len(a), len(b), "; ".join("line %d: %r / %r" % (i, a[i][:200], b[i][:200]) for i in bad))
    return len(a)
