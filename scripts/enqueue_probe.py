#!/usr/bin/env python3
"""Diagnostics only: where the first timed steps of the headline loop go.

Opens the C3 stand-in as bench.py does (torch first, then the engine), uploads
the 25 batches of the log, runs each once, then STEPS steps of the replica
loop, timing every run() call on the host and, per window of WINDOW steps, the
wall time (a device sync at each window end only when --sync-windows).  Prints
per window: mean / max host enqueue ms, wall ms per step, and the cgroup's CPU
throttling counters (cpu.stat nr_throttled / throttled_usec) and the process's
thread count, before and after the loop.
usage: enqueue_probe.py [--steps N] [--window W] [--sync-windows]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_stat():
    for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"):
        try:
            d = dict(l.split() for l in open(p).read().splitlines())
            return {k: int(v) for k, v in d.items() if k in ("nr_throttled", "throttled_usec", "usage_usec",
                                                          "throttled_time", "nr_periods")}
        except OSError:
            continue
    return {}


def threads():
    for l in open("/proc/self/status"):
        if l.startswith("Threads:"):
            return int(l.split()[1])
    return -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--window", type=int, default=100)
    ap.add_argument("--sync-windows", action="store_true")
    ap.add_argument("--oracle-check", type=int, default=0, help="check this many queries of batch 0 "
                    "against the oracle first, as bench.py does")
    ap.add_argument("--warmup", type=int, default=0)
    args = ap.parse_args()
    import torch  # noqa: F401  (the bench's import order)
    import bench
    import wiser_amd as w
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    idx, qlog, _ = bench.ensure_index(a, 0, None)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    eng = bench.open_full(idx, 0, bench.HOST_THREADS, 0, 1, None)
    batches = []
    for s in range(0, len(lines), a.batch):
        b = w.ResidentBatch(eng, a.batch, a.k)
        b.upload(bench.resolve(eng, lines[s:s + a.batch], a.k))
        batches.append(b)
    if args.oracle_check:
        batches[0].run()
        hits, nh = batches[0].fetch()
        bench.check_against_oracle(idx, lines[:a.batch], hits, nh, a.k, args.oracle_check)
    for s in range(args.warmup):
        batches[s % len(batches)].run()
    w.sync(eng)
    for b in batches:
        b.run()
        b.fetch()
    w.sync(eng)
    nb = len(batches)
    print(f"batches {nb}; threads {threads()}; cpu.stat before {cpu_stat()}", flush=True)
    t_start = time.perf_counter()
    tw = t_start
    dts = []
    for s in range(args.steps):
        t0 = time.perf_counter()
        batches[s % nb].run()
        dts.append(time.perf_counter() - t0)
        if (s + 1) % args.window == 0:
            if args.sync_windows:
                w.sync(eng)
            now = time.perf_counter()
            win = dts[-args.window:]
            print(f"steps {s + 1 - args.window:5d}-{s:5d}: enqueue mean {1e3 * sum(win) / len(win):.3f} ms "
                  f"max {1e3 * max(win):.3f} ms; wall {1e3 * (now - tw) / args.window:.3f} ms/step; "
                  f"cpu.stat {cpu_stat()}", flush=True)
            tw = now
    w.sync(eng)
    el = time.perf_counter() - t_start
    print(f"total {args.steps} steps {el * 1e3 / args.steps:.4f} ms/step; threads {threads()}; "
          f"cpu.stat after {cpu_stat()}", flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
