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
