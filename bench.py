#!/usr/bin/env python3
"""bench.py -- throughput of the MI355X vote path (BASELINE.json metric).

A "step" = one pass of the vote path over one batch of synthetic reads, measured as
SURVEY.md §8(d) defines the metric: from 2-bit packed reads resident in host-pinned
memory to mapping_result_t[3] per read end in host memory (svg_vote_batch_packed:
PCIe both ways included; reads are packed once, before timing).  Secondary fields:
the same kernels with reads and records already in HBM (device_path,
svg_vote_batch_device) and the ASCII host entry point (svg_vote_batch).  Workloads
(SURVEY.md §8(d)):
  c3g: C3 with the gapped index (gap 3, the reference's default index type).
  c2: 10M x 100 bp SE reads per GPU vs a chr901-scale 1,000,000 bp
      i.i.d. genome (seed 901), full one-block index (subread-buildindex -F -B),
      1% substitutions, 0.1% reads with a 1-5 bp indel, read seed 20261015.
  c3 (default, the BASELINE.json metric): 50M x 100 bp SE reads per GPU vs a 3.0 Gbp 24-contig genome with repeat
      families, full one-block index.
  c4: 150 bp PE vs the C3 index, 25M pairs per GPU (400M reads over 8 GPUs); fragments N(300,50)
      clipped to [150,600], R2 reverse complement.  value counts reads (2 per pair).
  c5: subjunc mode, 50M x 100 bp RNA-seq-like reads per GPU vs the C3 index, 30% spanning one
      GT..AG intron (60 bp-50 kbp); outputs mapping + subjunc + big-margin records.
Multi-GPU (torchrun): one process per GPU, index replicated, reads sharded by
rank (disjoint read-stream ranges), no collective on the data path; the only
communication is the timing barrier / max.  scaling = "weak".
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mreads/s aligned, 100bp SE vs 3Gbp index; 1/2/4/8-GPU scaling + HBM GB/s"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
RANDOM_SECTOR_RATE = 26.4e9   # random 32-B sectors/s chip-wide, measured (profiles/r02_calib_random.txt)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(name):
    if name == "c2":
        return dict(lengths=[1_000_000], gseed=901, repeats=None, reads=10_000_000, read_len=100, kind="se",
                    desc="C2: 10M x 100bp SE reads vs chr901-scale 1 Mbp genome, full one-block index")
    from subread_amd.sim import c3_lengths
    c3 = dict(lengths=c3_lengths(), gseed=3000, repeats=(1_000_000, 300, 200, 0.12))
    if name == "c3":
        return dict(c3, reads=50_000_000, read_len=100, kind="se",
                    desc="C3: 50M x 100bp SE reads vs 3.0 Gbp 24-contig genome, full one-block index")
    if name == "c3g":
        # the reference's default index type: gapped (-M 8000 default budget, one block at 3 Gbp),
        # 3 probes per subread offset -> 60 probes per read
        return dict(c3, reads=50_000_000, read_len=100, kind="se", gap=3,
                    desc="C3g: 50M x 100bp SE reads vs the C3 genome, gapped index (subread-buildindex defaults)")
    if name == "c4":
        return dict(c3, reads=25_000_000, read_len=150, kind="pe",
                    desc="C4: 25M x 2 x 150bp PE pairs per GPU vs the C3 3.0 Gbp index (400M reads on 8 GPUs)")
    if name == "c5pe":
        # paired-end subjunc (SURVEY §8(d) lists C5 as SE; this is the PE shape of it)
        return dict(c3, reads=25_000_000, read_len=100, kind="sjpe",
                    desc="C5pe: subjunc PE, 25M x 2 x 100bp pairs per GPU (fragments N(300,50)) vs the C3 index")
    if name == "c5":
        return dict(c3, reads=50_000_000, read_len=100, kind="sj",
                    desc="C5: subjunc, 50M x 100bp spliced RNA-seq reads (30% span a GT..AG intron) vs the C3 index")
    raise SystemExit("unknown workload " + name)


def cpu_info():
    """Host CPU model, logical CPUs, and the CPUs this process may use (affinity, cgroup quota)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ncpu = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else ncpu
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    if quota:
        usable = min(usable, max(1, int(quota)))
    return {"model": model, "logical_cpus": ncpu, "usable_cpus": usable, "cgroup_quota_cpus": quota}


def ref_binary(kind):
    """The reference aligner built from its own sources with the voting-step clock (oracle/Makefile
    votetime; oracle/ref_votetime.c) -- git-ignored, travels with the tree like our own .so files."""
    return os.path.join(ROOT, "oracle", "_ref", "subjunc-votetime" if kind in ("sj", "sjpe") else "subread-align-votetime")


def reference_cpu_run(kind, prefix, rb, rb2, chunk, chunks, threads, wd):
    """The reference's own voting step on the CPU (SURVEY.md §8(d) cpu_baseline, kind "reference"):
    the first chunk*chunks reads (pairs) of the timed batch as FASTQ, one run of the reference
    aligner over the same index files with -T threads, the reads in `chunks` chunks of one process
    (one index load; SVG_REF_CHUNK), each chunk's voting step clocked from its first read handed
    out to its last (votes, bigtable writes, final-run tail; FASTQ parsing before the clock,
    iteration two not run).  Returns (per-chunk (seconds, reads), the vote records the reference
    dumped for the sample (raw bytes, read order), wall seconds)."""
    import re
    import subprocess
    from subread_amd.sim import write_fastq
    m = min(len(rb), chunk * chunks)
    f1 = os.path.join(wd, "cpu_r1.fq")
    write_fastq(f1, rb.slice(0, m))
    args = [ref_binary(kind), "-T", str(threads), "-i", prefix, "-r", f1, "-o", os.path.join(wd, "cpu.sam"),
            "--SAMoutput"]
    if kind not in ("sj", "sjpe"):
        args += ["-t", "1"]
    if rb2 is not None:
        f2 = os.path.join(wd, "cpu_r2.fq")
        write_fastq(f2, rb2.slice(0, m))
        args += ["-R", f2]
    dump = os.path.join(wd, "cpu.votes")
    if os.path.exists(dump):
        os.remove(dump)
    t = time.perf_counter()
    r = subprocess.run(args, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, SVG_REF_CHUNK=str(chunk), SVG_REF_VOTETIME="1", SVG_REF_DUMP=dump))
    wall = time.perf_counter() - t
    lines = re.findall(r"SVG_REF_CHUNK_VOTING_S (\d+) ([0-9.]+) (\d+)", r.stderr)
    if r.returncode != 0 or sum(int(x[2]) for x in lines) != m:
        raise RuntimeError("reference run failed (%d): %s" % (r.returncode, (r.stdout + r.stderr)[-1500:]))
    votes = np.fromfile(dump, dtype=np.uint8)
    for f in [f1, dump, os.path.join(wd, "cpu.sam")] + ([f2] if rb2 is not None else []):
        if os.path.exists(f):
            os.remove(f)
    return [(float(x[1]), int(x[2])) for x in lines], votes, wall


def committed_fracs(wl, kernel, bytes_per_launch):
    """The dominant kernel's roofline fraction recomputed from the committed evidence: the newest
    profiles/r*_<wl>_kernel_record.json (HIP events of a GPU run, per launch) and the newest
    profiles/r*_<wl>_serial_trace.json (rocprofv3 kernel trace of the single-stream pipeline)."""
    import glob
    out = {}
    for kind, pat in (("kernel_record", "r*_%s_kernel_record.json"), ("serial_trace", "r*_%s_serial_trace.json")):
        fs = sorted(glob.glob(os.path.join(ROOT, "profiles", pat % wl)))
        if not fs:
            continue
        d = json.load(open(fs[-1]))
        k = d.get("kernel_record", d.get("kernels", {})).get(kernel)
        if not k:
            continue
        ms = k["ms"] / k["launches"] if "launches" in k else k["avg_ms"]
        out[kind] = {"file": os.path.relpath(fs[-1], ROOT), "launch_ms": round(ms, 4),
                     "achieved": round(bytes_per_launch / (ms / 1e3) / 1e9, 2),
                     "frac": round(bytes_per_launch / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=os.environ.get("SVG_WORKLOAD", "c3"))
    ap.add_argument("--reads", type=int, default=0, help="reads per GPU per step (default: workload size)")
    ap.add_argument("--workdir", default=os.environ.get("SVG_BENCH_DIR", ""))
    ap.add_argument("--cpu-sample", type=int, default=20_000_000)
    ap.add_argument("--cpu-threads", type=int, default=0, help="default: the CPUs this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ref-chunk", type=int, default=600_000,
                    help="reads (pairs) per chunk of the reference's timed CPU run")
    ap.add_argument("--ref-chunks", type=int, default=4,
                    help="chunks of that run: the first warms the caches, the others are the repetitions")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--device-steps", type=int, default=5, help="timed steps of the HBM-resident secondary figure")
    ap.add_argument("--ascii-reads", type=int, default=8_000_000, help="reads of the ASCII host-entry figure (0: skip)")
    ap.add_argument("--long-reads", type=int, default=20_000,
                    help="ONT-like long reads of the sublong secondary figure on the same index (0: skip)")
    ap.add_argument("--opt", action="append", default=[],
                    help="library option name=value (svg_set_option; A/B runs -- none changes a record)")
    ap.add_argument("--kernel-record", default="",
                    help="also write the timing step's per-kernel HIP-event table and the step times here (JSON)")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share devices round-robin
    ndev = torch.cuda.device_count()
    device = local % ndev if ndev else local
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # the vote path has no exchange step: the process group only carries the timing barrier and
        # the max of one float, so it runs on gloo (host TCP) unless SVG_DIST_BACKEND asks for RCCL
        backend = os.environ.get("SVG_DIST_BACKEND", "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    import subread_amd as sa
    from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC, MAPPING_DTYPE, SUBJUNC_DTYPE, \
        BIG_MARGIN_WORDS
    from subread_amd.sim import random_genome, simulate_reads, simulate_pairs, simulate_spliced_reads

    for o in args.opt:
        k, v = o.split("=", 1)
        sa.set_option(k, int(v))
    cpu = cpu_info()
    threads = args.cpu_threads or cpu["usable_cpus"]
    W = workload(args.workload)
    n = args.reads or W["reads"]
    L = W["read_len"]
    wd = args.workdir or os.path.join(tempfile.gettempdir(), "svg_bench_%s" % args.workload)
    os.makedirs(wd, exist_ok=True)
    t0 = time.time()
    genome = random_genome(W["lengths"], W["gseed"], repeats=W["repeats"])
    log("[bench] genome %.3f Gbp in %.1fs" % (genome.length / 1e9, time.time() - t0))
    prefix = None
    prefix_cpu = None        # reference-format index files of this genome (the reference's CPU run)
    if args.workload == "c2":
        # the drop-in path: reference-format files written by our builder, loaded by svg_index_open
        prefix = os.path.join(wd, "genome_full")
        if rank == 0 and not os.path.exists(prefix + ".00.b.tab"):
            fa = os.path.join(wd, "genome.fa")
            genome.write_fasta(fa)
            sa.build_index(fa, prefix, gap=1, force_one_block=True)
            log("[bench] built index files in %.1fs" % (time.time() - t0))
        if dist is not None:
            dist.barrier()
        t1 = time.time()
        ix = sa.VoteIndex(prefix, device=device)
        prefix_cpu = prefix
    else:
        # 3 Gbp: build the same index straight into this GPU's HBM (replicated per rank); rank 0 of an
        # N=1 run also writes it to reference-format files for the reference's timed CPU run
        t1 = time.time()
        gap = W.get("gap", 1)
        if rank == 0 and world == 1 and not args.no_cpu and os.path.exists(ref_binary(W["kind"])):
            prefix_cpu = os.path.join(wd, "index_%s" % args.workload)
        ix = sa.VoteIndex.build_genome(genome, gap=gap, memory_mb=8000, force_one_block=gap == 1, device=device,
                                       save_prefix=prefix_cpu)
    log("[bench] index in HBM (%.1f GB, %d items) in %.1fs" % (ix.info.device_bytes / 1e9, ix.info.items,
                                                            time.time() - t1))

    placement = ix.host_placement()
    # this rank's shard of the read stream: reads (pairs) rank*n .. rank*n+n-1
    t1 = time.time()
    kind = W["kind"]
    rb2 = None
    if kind in ("pe", "sjpe"):
        rb, rb2 = simulate_pairs(genome, n, L, seed=4004, first=rank * n)
    elif kind == "sj":
        rb = simulate_spliced_reads(genome, n, L, seed=5005 + rank)
    else:
        rb = simulate_reads(genome, n, L, seed=20261015, first=rank * n, sub=0.01, indel=0.001)
    ends = 2 if rb2 is not None else 1
    log("[bench] simulated %d %s in %.1fs" % (n, "pairs" if ends == 2 else "reads", time.time() - t1))
    dev = torch.device("cuda", device)
    p = default_params(PROGRAM_SUBJUNC if kind in ("sj", "sjpe") else PROGRAM_ALIGN, ends == 2)
    mb = p.multi_best
    sj = kind in ("sj", "sjpe")

    # ---- host-pinned 2-bit packed reads and host-pinned output records
    keep = []

    def pinned(count, dt):
        # pinned pages on the NUMA node of this rank's GPU (svg_host_alloc), where the expansion
        # workers and the copy engines touch them
        a = ix.host_alloc(count, dt)
        keep.append(a)
        return a
    t1 = time.time()
    pk1 = sa.pack_reads(rb, L, threads=threads, alloc=pinned)
    pk2 = sa.pack_reads(rb2, L, threads=threads, alloc=pinned) if rb2 is not None else None
    pk1.lens = pinned(n, np.uint16)
    pk1.lens[:] = rb.lens
    if pk2 is not None:
        pk2.lens = pinned(n, np.uint16)
        pk2.lens[:] = rb2.lens
    out = pinned(n * ends * mb, MAPPING_DTYPE).reshape(n, ends, mb)
    jout = pinned(n * ends * mb, SUBJUNC_DTYPE).reshape(n, ends, mb) if sj else None
    bmo = pinned(n * ends * BIG_MARGIN_WORDS, np.uint16).reshape(n, ends, BIG_MARGIN_WORDS) if sj else None
    bufs = (out, jout, bmo)
    in_bytes_host = pk1.bases.nbytes + pk1.lens.nbytes + (pk2.bases.nbytes + pk2.lens.nbytes if pk2 else 0)
    log("[bench] packed reads (%.1f B/read) and pinned output in %.1fs" % (in_bytes_host / float(n * ends),
                                                                         time.time() - t1))
    rec_bytes = MAPPING_DTYPE.itemsize * mb * ends + (ends * (mb * 16 + BIG_MARGIN_WORDS * 2) if sj else 0)

    def host_step():
        ix.vote_packed(p, pk1, pk2, bufs=bufs)

    # ---- the metric: packed host reads -> host records, W warmup + K timed steps
    for _ in range(args.warmup):
        host_step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    step_ends = []
    for _ in range(args.steps):
        host_step()
        step_ends.append(time.perf_counter())   # host call returns when its records are in host memory
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    # per-kernel times: one more host step with per-launch HIP events (recorded by the library on
    # each launch's stream), outside the timed region -- folding the event ring synchronises
    ix.set_timing(True)
    host_step()
    kt = ix.kernel_timing()
    ix.set_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = [round((b - a) * 1e3, 1) for a, b in zip([t_start] + step_ends[:-1], step_ends)]
    log("[bench] packed host path: %.1f Mreads/s (%.1f ms/step; steps %s ms)" % (
        n * ends * args.steps / elapsed / 1e6, elapsed / args.steps * 1e3, step_ms))

    # ---- secondary: the same kernels with the same 2-bit packed reads and the records already in
    # HBM (svg_vote_batch_packed_device: no PCIe, no host expansion)
    from subread_amd.abi import SvgPackedReads

    def upload_packed(pk):
        t = [torch.from_numpy(pk.bases.view(np.uint8)).to(dev), torch.from_numpy(pk.lens.view(np.uint8)).to(dev)]
        if pk.xmask is not None:
            t.append(torch.from_numpy(pk.xmask.view(np.uint8)).to(dev))
        q = SvgPackedReads()
        q.bases, q.lens = t[0].data_ptr(), t[1].data_ptr()
        q.xmask = t[2].data_ptr() if pk.xmask is not None else None
        q.starts, q.stride, q.n_reads = None, pk.stride, n
        return q, t
    q1, t1k = upload_packed(pk1)
    q2, t2k = upload_packed(pk2) if pk2 is not None else (None, None)
    d_out = torch.empty(n * MAPPING_DTYPE.itemsize * mb * ends, dtype=torch.uint8, device=dev)
    d_jout = torch.empty(n * ends * mb * 16, dtype=torch.uint8, device=dev) if sj else None
    d_bm = torch.empty(n * ends * BIG_MARGIN_WORDS * 2, dtype=torch.uint8, device=dev) if sj else None
    ix.set_max_read_length(int(os.environ.get("SVG_BENCH_MAXLEN", L)))
    # the handle's own stream: a stream created now could share a hardware queue with the
    # library's second stream (HIP deals streams round-robin onto GPU_MAX_HW_QUEUES = 4 queues)

    def dev_step():
        ix.vote_packed_device(p, q1, q2, d_out.data_ptr(), d_jout.data_ptr() if d_jout is not None else None,
                              d_bm.data_ptr() if d_bm is not None else None)
    dev_step()
    torch.cuda.synchronize()
    ds = max(1, args.device_steps)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    td = time.perf_counter()
    for _ in range(ds):
        dev_step()
    torch.cuda.synchronize()
    td = time.perf_counter() - td
    ix.device_status()
    device_path = {"value": round(n * ends * ds / td / 1e6, 3), "unit": "Mreads/s", "steps": ds,
                   "ms_per_step": round(td / ds * 1e3, 3),
                   "entry": "svg_vote_batch_packed_device: the same 2-bit packed reads and the records resident in HBM "
                            "(no PCIe, no host expansion)"}

    # algorithmic bytes from the kernels' own counters, outside the timed region
    ix.set_stats(True)
    dev_step()
    torch.cuda.synchronize()
    st = ix.stats()
    dcs = ix.debug_counters()
    lane_hits = dcs[19] + dcs[24]       # candidates voted by the light and heavy lane passes
    ix.set_stats(False)
    in_bytes = in_bytes_host                         # 2-bit packed reads + lengths (the metric's input)
    probe_bytes = 8 * st["probes"] + 2 * st["bucket_items"] + 4 * st["hits"]
    out_bytes = n * rec_bytes
    algo_bytes = in_bytes + probe_bytes + out_bytes  # SURVEY §8(d) B_read summed over the step
    # per-kernel algorithmic bytes of one step (text read by the probe kernel: ASCII in HBM):
    #   probe_kernel  read text + bucket bounds (8 B) + bucket keys (2 B/item) + probe records out (8 B/probe)
    #   gather_kernel probe records in (8 B/probe) + hit values (4 B/hit) + candidates out (6 B/hit) + counts
    #   lane_kernel   fused: records 8 B/probe + hit values 4 B/hit of its reads + lengths + records out
    #   vote_kernel   (deferred reads only when the lane path runs) records in + hit values + records out
    lane_on = kt["lane_kernel"][1] > 0
    nd = st.get("deferred", 0) if lane_on else n                 # reads voted by vote_kernel
    dh = st["hits"] - lane_hits if lane_on else st["hits"]       # their hits
    dp = st["probes"] * nd / float(n)                           # their probes (same length)
    text_bytes = n * ends * (L + 8 + 2)
    kbytes = {
        "probe_kernel": text_bytes + 8 * st["probes"] + 2 * st["bucket_items"] + 8 * st["probes"],
        "gather_kernel": 8 * st["probes"] + 10 * st["hits"] + 4 * n,
        "lane_kernel": ((6 * lane_hits) if kt["gather_kernel"][1] else (8 * st["probes"] * (n - nd) / float(n) + 4 * lane_hits))
                       + 6 * n + out_bytes * (n - nd) / float(n),
        "vote_kernel": 8 * dp + 4 * dh + 2 * nd * ends + out_bytes * nd / float(n),
    }
    kernels = {}
    for k, (ms, nl) in kt.items():
        if not nl:
            continue
        per_step = nl                     # launches of the one timing step
        launch_s = ms / nl / 1e3
        kernels[k] = {"launch_ms": round(launch_s * 1e3, 3), "launches_per_step": per_step,
                      "algorithmic_bytes_per_read": round(kbytes[k] / n, 1),
                      "achieved": round(kbytes[k] / per_step / launch_s / 1e9, 2)}
    dom = max(kernels, key=lambda k: kernels[k]["launch_ms"] * kernels[k]["launches_per_step"])
    vote_achieved = kernels[dom]["achieved"]
    vote_launch_s = kernels[dom]["launch_ms"] / 1e3
    launches_per_step = kernels[dom]["launches_per_step"]
    vote_bytes = kbytes[dom]
    step_s = elapsed / args.steps
    achieved = algo_bytes / step_s / 1e9

    # HBM traffic per kernel from the committed PMC passes of this workload's host path (the path
    # `value` measures: tools/profile_workload.sh ... host -> profiles/r*_<workload>_kernels_host*.json;
    # rocprofv3 cannot run inside this process), per launch, scaled to this run's reads per launch
    traffic, traffic_src = None, None
    import glob
    tj = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_kernels_host*.json" % args.workload)))
    pmc = json.load(open(tj[-1])).get("kernels", {}) if tj else {}
    for k, kd in kernels.items():
        if k in pmc:
            per_read = pmc[k]["traffic_bytes_per_read"]
            kd["traffic_bytes_per_read"] = round(per_read, 1)
            # the HBM bandwidth the kernel really draws (counter bytes / its HIP-event launch time)
            kd["traffic_gbs"] = round(per_read * n / kd["launches_per_step"] / (kd["launch_ms"] / 1e3) / 1e9, 1)
    if dom in pmc:
        per_read = pmc[dom]["traffic_bytes_per_read"]
        traffic = round(per_read * n / launches_per_step / 1e9, 3)
        traffic_src = "%s (%s FETCH_SIZE+WRITE_SIZE, %.0f B/read, GB per launch)" % (
            os.path.relpath(tj[-1], ROOT), dom, per_read)
    # the probe kernels are bound by the HBM random-access rate, not by bytes: one random 32-B
    # sector per probe (bucket code / key-hash image) against the measured chip-wide ceiling
    if "probe_kernel" in kernels:
        kd = kernels["probe_kernel"]
        rate = st["probes"] / kd["launches_per_step"] / (kd["launch_ms"] / 1e3)
        kd["probes_per_s"] = round(rate / 1e9, 2)
        kd["random_sector_ceiling_per_s"] = RANDOM_SECTOR_RATE / 1e9
        kd["random_sector_frac"] = round(rate / RANDOM_SECTOR_RATE, 3)
    # the regime of each kernel from its own numbers
    for k, kd in kernels.items():
        bw = kd.get("traffic_gbs", kd["achieved"])
        if bw >= 0.5 * HBM_PEAK_GBS:
            kd["regime"] = "hbm-bandwidth"
        elif kd.get("random_sector_frac", 0) >= 0.6:
            kd["regime"] = "hbm-random-access-rate"
        else:
            kd["regime"] = "latency/issue-bound (%.0f GB/s of HBM traffic, %.1f%% of peak)" % (bw, 100 * bw / HBM_PEAK_GBS)

    # the roof the dominant kernel is actually against, from its own numbers: HBM bandwidth or the
    # HBM random-access rate (both "hbm"), else latency / issue (a serial state machine per read)
    reg = kernels[dom]["regime"]
    bound = "hbm" if reg in ("hbm-bandwidth", "hbm-random-access-rate") else "latency"
    # the same kernel's frac from the committed evidence under profiles/: the HIP-event kernel record
    # of a GPU run of this workload (tools/prof_run.py / --kernel-record) and the serialised
    # single-stream rocprofv3 trace summary (tools/profile_serial.sh)
    committed = committed_fracs(args.workload, dom, vote_bytes / launches_per_step)
    if args.kernel_record:
        json.dump({"workload": args.workload, "reads_per_step": n * ends, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                   "host_step_ms": [round((b - a) * 1e3, 1) for a, b in zip([t_start] + step_ends[:-1], step_ends)],
                   "kernel_record": {k: {"ms": round(ms, 4), "launches": nl} for k, (ms, nl) in kt.items() if nl},
                   "algorithmic_bytes_per_launch": {k: kbytes[k] / kernels[k]["launches_per_step"] for k in kernels}},
                  open(args.kernel_record, "w"), indent=1)
    check = None
    oi = None
    if rank == 0 and not (args.no_check and args.no_cpu):
        from oracle.pyoracle import OracleIndex
        oi = OracleIndex(prefix) if prefix else OracleIndex(arrays=ix.export())
    if rank == 0 and not args.no_check:
        # parity spot check against the oracle restatement (outside the timed region): the first and
        # the last 20k reads of the timed host-path output (first and last sub-batch / chunk)
        m = min(n, 20000)
        windows = [(0, m), (n - m, n)] if n > m else [(0, n)]
        check = True
        for a, b in windows:
            got = [out[a:b].view(np.uint8).reshape(b - a, -1)]
            if sj:
                got += [jout[a:b].view(np.uint8).reshape(b - a, -1), bmo[a:b].view(np.uint8).reshape(b - a, -1)]
            ref, rj, rbm, _ = oi.vote(p, rb.slice(a, b), rb2.slice(a, b) if rb2 is not None else None, threads=threads)
            want = [ref.view(np.uint8).reshape(b - a, -1)]
            if sj:
                want += [rj.view(np.uint8).reshape(b - a, -1), rbm.view(np.uint8).reshape(b - a, -1)]
            ok = bool(all((x == y).all() for x, y in zip(got, want)))
            # the HBM-resident run wrote the same records
            dv = d_out[a * mb * ends * 68:b * mb * ends * 68].cpu().numpy().reshape(b - a, -1)
            ok = ok and bool((dv == want[0]).all())
            check = check and ok
            log("[bench] parity check on reads %d..%d: %s" % (a, b, "IDENTICAL" if ok else "MISMATCH"))
    ascii_host = None
    if rank == 0 and world == 1 and args.ascii_reads:
        # the ASCII host entry point (svg_vote_batch, pageable numpy reads, pinned records)
        m = min(n, args.ascii_reads)
        h1, h2 = rb.slice(0, m), (rb2.slice(0, m) if rb2 is not None else None)
        sub = (out[:m], jout[:m] if sj else None, bmo[:m] if sj else None)
        ix.vote(p, h1, h2, bufs=sub)
        ta = time.perf_counter()
        ix.vote(p, h1, h2, bufs=sub)
        ta = time.perf_counter() - ta
        ascii_host = {"value": round(m * ends / ta / 1e6, 3), "unit": "Mreads/s", "reads": m * ends,
                      "entry": "svg_vote_batch: ASCII reads (pageable) in, records (pinned) out, PCIe both ways"}
    def sublong_figure():
        # secondary figure, f4 row: sublong's voting step (svg_long_vote_batch) on the same index --
        # host long reads in, vote-table slots + location order out (tools/bench_long.py's batch)
        from subread_amd.sim import simulate_long_reads
        lr = simulate_long_reads(genome, args.long_reads, mean_len=8000, seed=8000)
        lbases = int(lr.lens.astype(np.int64).sum())
        res = ix.long_vote(lr)
        del res
        lt = []
        for _ in range(3):
            t1 = time.perf_counter()
            res = ix.long_vote(lr)
            lt.append(time.perf_counter() - t1)
            if len(lt) < 3:
                del res
        vs_, lv_, lo_ = res
        fig = {"value": round(lbases / min(lt) / 1e6, 1), "unit": "Mbases/s", "reads": args.long_reads,
               "bases": lbases, "ms_per_batch": round(min(lt) * 1e3, 2), "slots": int(len(lv_)),
               "entry": "svg_long_vote_batch: sublong's LRMdo_one_voting_read + copy + location sort, host reads "
                        "in, host slots out (ONT-like reads, 3% sub / 2% ins / 2% del)"}
        if oi is not None:
            k = min(200, args.long_reads)
            want = oi.long_vote(lr.slice(0, k), threads=threads)
            kk = int(vs_[k])
            fig["parity_check"] = bool((want[0] == vs_[:k + 1]).all() and (want[1] == lv_[:kk]).all()
                                       and (want[2] == lo_[:kk]).all())
        log("[bench] sublong voting: %.1f Mbases/s (%.1f ms per %d reads), parity %s" % (
            fig["value"], fig["ms_per_batch"], args.long_reads, fig.get("parity_check")))
        return fig

    long_fig = None
    if rank == 0 and world == 1 and args.long_reads and args.workload != "c2":
        # a secondary figure never costs the metric's line
        try:
            long_fig = sublong_figure()
        except Exception as ex:   # noqa: BLE001
            long_fig = {"error": "%s: %s" % (type(ex).__name__, ex)}
            log("[bench] sublong figure failed: %s" % ex)
    cpu_base = None
    if rank == 0 and world == 1 and not args.no_cpu:   # the CPU baseline is an N=1 figure
        cpu_base = {"unit": "Mreads/s", "cores": threads, "cpu_model": cpu["model"],
                    "host_logical_cpus": cpu["logical_cpus"], "usable_cpus": cpu["usable_cpus"],
                    "cgroup_quota_cpus": cpu["cgroup_quota_cpus"]}
        # (1) the reference itself, timed in this run (oracle/_ref/*-votetime, same index and reads)
        if prefix_cpu and os.path.exists(ref_binary(kind)):
            try:
                per_all, votes, wall = reference_cpu_run(kind, prefix_cpu, rb, rb2, args.ref_chunk, args.ref_chunks,
                                                         threads, wd)
                per = per_all[1:] if len(per_all) > 1 else per_all   # chunk 0: warm-up
                rates = sorted(r_ * ends / s_ / 1e6 for s_, r_ in per)
                med = rates[len(rates) // 2] if len(rates) % 2 else 0.5 * (rates[len(rates) // 2 - 1] + rates[len(rates) // 2])
                m = sum(r_ for _, r_ in per_all)
                mine = [out[:m].view(np.uint8).reshape(m, -1)]
                if sj:
                    mine += [jout[:m].view(np.uint8).reshape(m, -1), bmo[:m].view(np.uint8).reshape(m, -1)]
                mine = np.concatenate(mine, 1).reshape(-1)
                cpu_base.update({
                    "value": round(med, 4), "kind": "reference",
                    "sample": "first %d %s of the timed batch in %d chunks of one run of the reference aligner (%s, "
                              "built from its sources, -T %d, same index files); value = median of the voting step's rate "
                              "over chunks 2..%d (chunk 1 warms the caches), FASTQ parsing and index loading outside the "
                              "clock" % (m, "pairs" if ends == 2 else "reads", len(per_all), os.path.basename(ref_binary(kind)),
                                         threads, len(per_all)),
                    "warmup_chunk": {"seconds": round(per_all[0][0], 4), "reads": per_all[0][1] * ends},
                    "reps": [{"seconds": round(s_, 4), "reads": r_ * ends, "value": round(r_ * ends / s_ / 1e6, 4)}
                             for s_, r_ in per],
                    "spread": {"min": round(rates[0], 4), "max": round(rates[-1], 4)},
                    "run_wall_s": round(wall, 1),
                    # the GPU host path's records of the same reads against the reference's own
                    # post-vote records (SVG_REF_DUMP, oracle/ref_dump_hook.c)
                    "records_identical_to_gpu": bool(votes.size == mine.size and (votes == mine).all())})
                log("[bench] reference CPU voting: %s Mreads/s per chunk (median %.3f), records vs GPU %s" % (
                    [round(x, 3) for x in rates], med, "IDENTICAL" if cpu_base["records_identical_to_gpu"] else "DIFFERENT"))
            except Exception as ex:   # noqa: BLE001
                cpu_base["reference_error"] = "%s: %s" % (type(ex).__name__, ex)
                log("[bench] reference CPU run failed: %s" % ex)
        # (2) the restatement (oracle/svoracle.c): chunks of the same reads until >= 10 s of CPU work
        done, cs, chunk = 0, 0.0, 200000
        while cs < 10.0 and done < min(n, args.cpu_sample):
            b = min(chunk, n - done)
            t1 = time.perf_counter()
            oi.vote(p, rb.slice(done, done + b), rb2.slice(done, done + b) if rb2 is not None else None,
                    threads=threads)
            cs += time.perf_counter() - t1
            done += b
        port = {"value": round(done * ends / cs / 1e6, 4), "kind": "port",
                "sample": "first %d reads of the timed batch, oracle/svoracle.c restatement, %d pthreads, %.1f s" % (
                    done, threads, cs)}
        if "value" in cpu_base:
            cpu_base["port"] = port
        else:
            cpu_base.update(port)
    total_reads = n * ends * world * args.steps
    value = total_reads / elapsed / 1e6
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mreads/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": W["desc"], "reads_per_gpu_per_step": n * ends, "read_len": L,
                       "mode": {"se": "subread-align SE", "pe": "subread-align PE", "sj": "subjunc SE",
                                "sjpe": "subjunc PE"}[kind],
                       "entry": "svg_vote_batch_packed: 2-bit packed reads in host-pinned memory -> mapping_result_t "
                                "in host-pinned memory (H2D + vote + compacted D2H + host expansion)",
                       "index": "%s one-block (gap %d), %d buckets, %d items, %s" % (
                           "full" if ix.info.index_gap == 1 else "gapped", ix.info.index_gap, ix.info.buckets, ix.info.items,
                           "reference-format files via svg_index_open" if prefix else "built in HBM by svg_index_build_mem"),
                       "parallelism": "reads sharded across %d GPU(s), index replicated, no collective" % world,
                       "host_threads_per_rank": int(sa.lib().svg_host_threads()),
                       "host_placement": {"gpu_numa_node": placement[0], "usable_cpus_on_node": placement[1],
                                          "pinned_pages": "svg_host_alloc: preferred node %d" % placement[0]
                                          if placement[0] >= 0 else "svg_host_alloc: node unknown (default policy)",
                                          "expansion_workers": "pinned to the node's CPUs" if placement[1] > 0
                                          else "unpinned (no usable CPU on the node)"}},
            "roofline": {"bound": bound, "regime": kernels[dom]["regime"], "kernel": dom, "achieved": round(vote_achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(vote_achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_unit": "GB per launch",
                         "traffic_source": traffic_src,
                         "launch_ms": round(vote_launch_s * 1e3, 3), "launches_per_step": launches_per_step,
                         "algorithmic_bytes_per_read": round(vote_bytes / n, 1),
                         "kernels": kernels,
                         "committed": committed,
                         "deferred_reads": st.get("deferred", 0),
                         "path": {"achieved": round(achieved, 2), "algorithmic_bytes_per_read": round(algo_bytes / n, 1),
                                  "step_ms": round(step_s * 1e3, 3), "frac": round(achieved / HBM_PEAK_GBS, 5)}},
            "host_step_ms": step_ms,
            "device_path": device_path,
            "ascii_host_path": ascii_host,
            "sublong_voting": long_fig,
            "cpu_baseline": cpu_base,
            "parity_check": check,
        }
        print(json.dumps(line), flush=True)
    del keep
    ix.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
