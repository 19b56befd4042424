#!/usr/bin/env python3
"""Parity at bench scale against the reference itself (GPU box): all 50M reads of bench.py's C3
workload (3.0 Gbp genome with repeat families, full one-block index, 100 bp SE reads, seed
20261015) voted on the GPU through svg_vote_batch_packed (the metric's entry point), and the same
reads voted by the reference aligner built from its own sources (oracle/_ref/subread-align-votetime,
chunked mode: one index load, iteration two skipped), whose post-vote records its own dump hook
(oracle/ref_dump_hook.c, SVG_REF_DUMP) streams through a named pipe into SHA-256 digests per
1M-read block -- no 10 GB dump on disk.  Writes one JSON line: block digests of both sides, the
first differing block (if any), the timings.
Usage: c3_reference_digest.py [n_reads] [workdir]"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

BLOCK = 1_000_000
REC = 3 * 68


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def write_fastq_fast(path, rb, chunk=1_000_000):
    """Fixed-length reads: '@r<i>' names, constant 'I' qualities (bench.py's cpu_baseline FASTQ)."""
    n = len(rb)
    L = int(rb.lens[0])
    seq = rb.seq.reshape(n, L) if rb.seq.size == n * L else None
    assert seq is not None and (rb.lens == L).all()
    qual = b"I" * L
    with open(path, "wb", buffering=1 << 24) as f:
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            f.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, seq[i].tobytes(), qual) for i in range(a, b)))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    wd = sys.argv[2] if len(sys.argv) > 2 else tempfile.mkdtemp(prefix="svg_c3dig_")
    os.makedirs(wd, exist_ok=True)
    stop = threading.Event()

    def heartbeat():   # keep the GPU runner's log moving through the long silent steps
        t = time.time()
        while not stop.wait(30):
            log("[dig] ... %.0f s" % (time.time() - t))
    threading.Thread(target=heartbeat, daemon=True).start()
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import random_genome, simulate_reads, c3_lengths
    t0 = time.time()
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    pre = os.path.join(wd, "c3_full")
    ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0, save_prefix=pre)
    log("[dig] index in HBM and files in %.1f s" % (time.time() - t0))
    rb = simulate_reads(g, n, 100, seed=20261015, first=0, sub=0.01, indel=0.001)
    del g
    t1 = time.time()
    pk = sa.pack_reads(rb, 100, threads=16)
    out, _, _ = ix.vote_packed(default_params(), pk)
    t_gpu = time.time() - t1
    raw = out.view(np.uint8).reshape(n, -1)
    assert raw.shape[1] == REC
    gpu_blocks = [hashlib.sha256(raw[a:a + BLOCK].tobytes()).hexdigest() for a in range(0, n, BLOCK)]
    gpu_all = hashlib.sha256(raw.tobytes()).hexdigest()
    with_votes = int((out["selected_votes"][:, 0, 0] > 0).sum())
    del out, raw, pk
    ix.close()
    log("[dig] GPU vote of %d reads (incl. packing) %.1f s" % (n, t_gpu))
    fq = os.path.join(wd, "r.fq")
    t1 = time.time()
    write_fastq_fast(fq, rb)
    del rb
    log("[dig] FASTQ written in %.1f s (%.1f GB)" % (time.time() - t1, os.path.getsize(fq) / 1e9))
    fifo = os.path.join(wd, "votes.fifo")
    if os.path.exists(fifo):
        os.remove(fifo)
    os.mkfifo(fifo)
    ref_blocks, state = [], {"done": False, "bytes": 0, "err": None}
    h_all = hashlib.sha256()

    def reader():
        h, fill = hashlib.sha256(), 0
        try:
            while True:
                fd = os.open(fifo, os.O_RDONLY)   # blocks until the hook opens the pipe for a chunk
                with os.fdopen(fd, "rb", buffering=0) as f:
                    while True:
                        buf = f.read(1 << 22)
                        if not buf:
                            break
                        state["bytes"] += len(buf)
                        h_all.update(buf)
                        mv = memoryview(buf)
                        while len(mv):
                            take = min(len(mv), BLOCK * REC - fill)
                            h.update(mv[:take])
                            fill += take
                            mv = mv[take:]
                            if fill == BLOCK * REC:
                                ref_blocks.append(h.hexdigest())
                                h, fill = hashlib.sha256(), 0
                if state["done"]:
                    break
            if fill:
                ref_blocks.append(h.hexdigest())
        except Exception as ex:   # noqa: BLE001
            state["err"] = repr(ex)
    th = threading.Thread(target=reader, daemon=True)
    th.start()
    binp = os.path.join(ROOT, "oracle", "_ref", "subread-align-votetime")
    threads = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            threads = max(1, min(threads, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    t1 = time.time()
    env = dict(os.environ, SVG_REF_CHUNK=str(5 * BLOCK), SVG_REF_VOTETIME="1", SVG_REF_DUMP=fifo)
    with open(os.path.join(wd, "ref.err"), "w") as ferr:
        r = subprocess.run([binp, "-t", "1", "-T", str(threads), "-i", pre, "-r", fq, "-o", os.path.join(wd, "ref.sam"),
                            "--SAMoutput"], stdout=subprocess.DEVNULL, stderr=ferr, env=env, timeout=1800)
    t_ref = time.time() - t1
    state["done"] = True
    try:   # release a reader blocked in open()
        fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.close(fd)
    except OSError:
        pass
    th.join(60)
    err = open(os.path.join(wd, "ref.err")).read()
    import re
    chunks = [(float(a), int(b)) for _, a, b in re.findall(r"SVG_REF_CHUNK_VOTING_S (\d+) ([0-9.]+) (\d+)", err)]
    ref_reads = state["bytes"] // REC
    bad = [i for i, (a, b) in enumerate(zip(gpu_blocks, ref_blocks)) if a != b]
    res = {
        "workload": "C3: %d x 100 bp SE reads (seed 20261015) vs the 3.0 Gbp C3 genome, full one-block index" % n,
        "gpu": {"entry": "svg_vote_batch_packed", "seconds": round(t_gpu, 1), "sha256": gpu_all,
                "reads_with_votes": with_votes},
        "reference": {"binary": "oracle/_ref/subread-align-votetime (-t 1, -T %d, chunks of %d reads)" % (threads, 5 * BLOCK),
                      "exit": r.returncode, "seconds": round(t_ref, 1), "reads_dumped": ref_reads,
                      "sha256": h_all.hexdigest(), "voting_step_s": round(sum(c[0] for c in chunks), 2),
                      "reader_error": state["err"]},
        "block_reads": BLOCK, "blocks": len(gpu_blocks),
        "identical": r.returncode == 0 and ref_reads == n and not bad and h_all.hexdigest() == gpu_all,
        "first_differing_block": bad[0] if bad else None,
        "gpu_block_sha256": gpu_blocks, "reference_block_sha256": ref_blocks,
    }
    stop.set()
    print(json.dumps(res), flush=True)
    log("[dig] reference %.1f s (voting step %.1f s); records identical: %s" % (
        t_ref, res["reference"]["voting_step_s"], res["identical"]))
    for f in (fq, fifo):
        try:
            os.remove(f)
        except OSError:
            pass


if __name__ == "__main__":
    main()
