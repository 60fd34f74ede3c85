"""Host-side logic of bench.py's N > 1 path on the CPU (gloo, world size 4):
full-image loads are staggered two ranks at a time (bench.staggered), so at
most two host images exist at once on a node, and every rank gets its own
result back."""
import os
import socket
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def load():
        t0 = time.time()
        time.sleep(0.3)
        return (rank, t0, time.time())
    out = bench.staggered(dist, rank, world, load)
    q.put(out)
    dist.destroy_process_group()


def test_staggered_loads_two_at_a_time():
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r for r, _, _ in got) == list(range(world))
    spans = {r: (a, b) for r, a, b in got}
    for t in [a + 0.15 for a, _ in spans.values()]:
        assert sum(a <= t <= b for a, b in spans.values()) <= 2
    # ranks 2 and 3 start after ranks 0 and 1 have finished
    assert min(spans[2][0], spans[3][0]) >= max(spans[0][1], spans[1][1])


# ---- --gpus N: spawn a launcher or refuse ----
def test_check_world_rules():
    sys.path.insert(0, ROOT)
    import bench
    import pytest
    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(8, {}) == "spawn"
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == "run"
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) == "run"
    for gpus, ws in ((1, "2"), (8, "1"), (2, "8")):
        with pytest.raises(SystemExit):
            bench.check_world(gpus, {"WORLD_SIZE": ws})
    with pytest.raises(SystemExit):
        bench.check_world(0, {})
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "5"], 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_bench_refuses_world_mismatch():
    """A launcher of 2 ranks around `bench.py --gpus 1` exits non-zero before any
    HIP call (so this runs on the CPU)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_spawn_ranks_starts_n_ranks(tmp_path, capfd):
    """spawn_ranks runs torch.distributed.run as a child with N ranks and passes
    its exit code through (a stand-in script reports each rank's env)."""
    sys.path.insert(0, ROOT)
    import bench
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\n"
                      "print('RANK', os.environ['RANK'], os.environ['WORLD_SIZE'], *sys.argv[1:], flush=True)\n"
                      "sys.exit(3 if os.environ.get('FAIL_RANK') == os.environ['RANK'] else 0)\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    old = dict(os.environ)
    try:
        os.environ.clear()
        os.environ.update(env)
        rc = bench.spawn_ranks(3, ["--gpus", "3"], script=str(script))
        out = capfd.readouterr().out
        assert rc == 0, out
        got = sorted(l.split()[1:] for l in out.splitlines() if l.startswith("RANK"))
        assert got == [[str(r), "3", "--gpus", "3"] for r in range(3)]
        os.environ["FAIL_RANK"] = "1"
        assert bench.spawn_ranks(2, ["--gpus", "2"], script=str(script)) != 0
    finally:
        os.environ.clear()
        os.environ.update(old)
