"""GPU multi-process path: two ranks (torch.distributed.run, gloo for the host gather) each
open an index replica on GPU 0 and vote a contiguous shard through the HIP library; the
records gathered on rank 0 in read order equal the reference's golden records byte for
byte (reads shard with no collective on the data path)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.common import Case, ROOT, ensure_built

ensure_built()
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("case", ["pe_full_errmut", "sj_se_full_junc", "se_gapped_mixed_n14_I16"])
def test_two_rank_hip_shards_match_golden(case, index_cache, tmp_path):
    c = Case(case)
    prefix = index_cache.get(c.index_key)
    out = str(tmp_path / "gathered.npy")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "tests", "shard_worker.py"), prefix, case, out],
                       capture_output=True, text=True, timeout=100, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = np.load(out)
    assert got.shape == c.expected.shape
    assert (got == c.expected).all()
