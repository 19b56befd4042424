"""CPU: the C-ABI library loads, exports every symbol include/subread_vote.h and
include/subread_events.h and include/subread_long.h declare, and its host-side pieces behave (no GPU compute here)."""
import ctypes
import re
import os

import pytest
import numpy as np

import subread_amd as sa
from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC, MAPPING_DTYPE, SUBJUNC_DTYPE
from tests.common import ROOT, ensure_built

ensure_built()


def header_symbols():
    syms = set()
    for h in ("subread_vote.h", "subread_events.h", "subread_long.h", "subread_sam.h", "subread_realign.h"):
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


def test_cpulist_parse():
    """svg_cpulist_parse: the sysfs node cpulist format the NUMA placement reads
    (/sys/devices/system/node/nodeN/cpulist)."""
    import numpy as np
    L = sa.lib()
    for text, want in ((b"0-15,64-79\n", list(range(16)) + list(range(64, 80))), (b"3", [3]), (b"", []),
                       (b"0,2,4-6", [0, 2, 4, 5, 6]), (b"120-130", list(range(120, 128)))):
        m = np.zeros(128, np.uint8)
        n = L.svg_cpulist_parse(text, m.ctypes.data, 128)
        assert n == len(want) and list(np.nonzero(m)[0]) == want, (text, n)


@pytest.mark.gpu
def test_host_placement_reports_node_and_cpus():
    """svg_host_placement (GPU box): the NUMA node of device 0's PCIe function as sysfs gives it,
    and the CPUs of that node this process may use (the expansion workers' affinity); the node's
    pinned allocation (svg_host_alloc) comes back usable."""
    import ctypes
    import os
    import torch
    assert torch.cuda.is_available()
    node, ncpu = ctypes.c_int(-7), ctypes.c_int(-7)
    assert sa.lib().svg_host_placement(0, ctypes.byref(node), ctypes.byref(ncpu)) == 0
    assert node.value >= -1 and ncpu.value >= 0
    if node.value >= 0:
        cl = open("/sys/devices/system/node/node%d/cpulist" % node.value).read()
        import numpy as np
        m = np.zeros(4096, np.uint8)
        sa.lib().svg_cpulist_parse(cl.encode(), m.ctypes.data, 4096)
        want = len(set(np.nonzero(m)[0]) & os.sched_getaffinity(0))
        assert ncpu.value == want
    else:
        assert ncpu.value == 0