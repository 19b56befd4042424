"""GPU: bench.py's multi-rank path as the driver launches it (torch.distributed.run, one process per
GPU, reads sharded by rank, index replicated, gloo timing barrier + max; no collective on the data
path), rehearsed with 2 ranks on a 1-GPU box (ranks share device 0 round-robin).  The line must
count both ranks' reads and pass rank 0's parity check."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.common import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_bench_two_ranks(tmp_path):
    env = dict(os.environ, SVG_BENCH_DIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--workload", "c2",
           "--reads", "2000000", "--no-cpu", "--ascii-reads", "0", "--device-steps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=560, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step", "parity_check")}))
    assert line["n_gpus"] == 2
    assert line["config"]["reads_per_gpu_per_step"] == 2_000_000
    assert line["parity_check"] is True
    assert line["value"] > 0
