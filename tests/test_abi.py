"""CPU: the C-ABI library loads, exports every symbol include/subread_vote.h and
include/subread_events.h and include/subread_long.h declare, and its host-side pieces behave (no GPU compute here)."""
import ctypes
import re
import os

import numpy as np

import subread_amd as sa
from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC, MAPPING_DTYPE, SUBJUNC_DTYPE
from tests.common import ROOT, ensure_built

ensure_built()


def header_symbols():
    syms = set()
    for h in ("subread_vote.h", "subread_events.h", "subread_long.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(svg_[a-z0-9_]+)\s*\(", txt))
    return sorted(syms)


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(sa.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    assert set(sa.EXPORTS) == set(syms)
    assert L.svg_abi_version() == 2


def test_struct_sizes_match_reference():
    assert MAPPING_DTYPE.itemsize == 68      # sizeof(mapping_result_t), core.h:350-370
    assert SUBJUNC_DTYPE.itemsize == 16      # sizeof(subjunc_result_t), core.h:397-410
    assert MAPPING_DTYPE.fields["selected_indel_record"][1] == 16
    assert MAPPING_DTYPE.fields["confident_coverage_start"][1] == 60


def test_params_default_c_equals_python():
    for prog in (PROGRAM_ALIGN, PROGRAM_SUBJUNC):
        for paired in (False, True):
            assert sa.params_default(prog, paired).as_dict() == default_params(prog, paired).as_dict()
    p = default_params(PROGRAM_SUBJUNC, True)
    assert (p.total_subreads, p.min_votes_first, p.max_vote_simples, p.do_breakpoint_detection) == (14, 1, 64, 1)


def test_simulator_deterministic_across_threads():
    from subread_amd.sim import random_genome, simulate_reads
    g = random_genome([50000, 30000], 5)
    a = simulate_reads(g, 3000, 100, seed=9, threads=1)
    b = simulate_reads(g, 3000, 100, seed=9, threads=7)
    assert (a.seq == b.seq).all()
    c = simulate_reads(g, 1000, 100, seed=9, first=2000, threads=3)
    assert (c.seq == a.seq[2000 * 100:]).all()


def test_index_open_without_gpu_fails_loudly(tmp_path):
    # in the CPU container there is no HIP device: the product must refuse, not fall back
    import subprocess, sys
    code = ("import subread_amd as sa\n"
            "try:\n sa.VoteIndex('/nonexistent/x')\nexcept sa.SvgError as e:\n print('ERR', e)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert "ERR" in r.stdout


def _usable_cpus():
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def test_host_threads_follow_affinity_quota_and_ranks(monkeypatch, svgopt):
    """svg_host_threads: the host_threads option wins; else this process's usable CPUs (affinity capped by
    the cgroup quota) shared among LOCAL_WORLD_SIZE ranks, clamped to 2..12 (svg_io.hip)."""
    L = sa.lib()
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    u = _usable_cpus()
    assert L.svg_host_threads() == max(2, min(12, u))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert L.svg_host_threads() == max(2, min(12, u // 2))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "64")
    assert L.svg_host_threads() == 2
    svgopt.set("host_threads", 5)
    assert L.svg_host_threads() == 5
    svgopt.reset("host_threads")
    assert L.svg_host_threads() == 2
