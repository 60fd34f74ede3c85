"""bench.py's N > 1 path on the GPU: the driver's first SCALE
run must not be where the multi-rank orchestration first breaks.

Two ranks on the one GPU of the box (the driver's 8-GPU launch has the same
shape), the exchange over the launcher's gloo group (RCCL refuses two ranks on
one device), a small C2 index: every form of the N > 1 line (hybrid value,
every-query doc-range shards, replica control), the max-over-ranks timing and
the oracle spot check.  A fresh child launcher, never an exec of this process.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo(built, tmp_path):
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--exchange", "gloo", "--workload", "c2",
           "--docs", "50000", "--vocab", "50000", "--queries", "20000", "--steps", "20", "--warmup", "2",
           "--no-extra", "--no-cpu", "--check", "64", "--index-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 20
    assert d["parity_checked_queries"] > 0
    forms = d["forms"]
    for f in ("docshard", "replica"):
        assert f in forms, forms.keys()
        assert forms[f]["value"] > 0 and forms[f]["hbm_per_rank"] > 0
    assert d["hbm_per_rank"]["total_bytes"] > 0
    assert d["config"]["parallelism"].startswith(("hybrid-docshard2", "docshard2"))
    assert "REHEARSAL" in d["exchange"]["kind"]


def test_bench_gpus2_spawns_its_launcher(built, tmp_path):
    """`bench.py --gpus 2` with no launcher around it starts one
    itself (a child torch.distributed.run) and reports n_gpus 2, not a silent
    one-rank measurement."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--exchange", "gloo",
           "--workload", "c2", "--docs", "50000", "--vocab", "50000", "--queries", "20000", "--steps", "20",
           "--warmup", "2", "--no-extra", "--no-cpu", "--check", "64", "--mode", "shard", "--heavy-blocks", "0",
           "--index-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["parity_checked_queries"] > 0
    assert d["config"]["parallelism"] == "docshard2"
