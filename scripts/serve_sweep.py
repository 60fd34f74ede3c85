"""Serving sweep: the micro-batcher (wsr_server_*) under closed-loop load over
the headline index (C3 stand-in, or C2 with --c2), per dispatch depth
(WSR_SERVER_DEPTH), client count, per-client window and window_us; prints one
JSON line per point with the latency breakdown (queue / GPU / hand-off).
usage: serve_sweep.py [--c2] [seconds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import wiser_amd as w  # noqa: E402
from wiser_amd import _capi  # noqa: E402


def index(c2):
    if c2:
        idx = "/tmp/wiser_bench/c2_1000000_500000"
        build = lambda: w.build_synthetic(idx, threads=16)  # noqa: E731
    else:
        idx = "/tmp/wiser_bench/c3_wiki_5500000_1"
        build = lambda: w.build_wiki_standin(idx, n_docs=5_500_000, term_scale=1.0, threads=16)  # noqa: E731
    log = os.path.join(idx, "two_term_100000.log")
    if not os.path.exists(os.path.join(idx, "READY")):
        os.makedirs(idx, exist_ok=True)
        build()
        w.gen_two_term_log(idx, log, 100000, 7)
        open(os.path.join(idx, "READY"), "w").write("ok")
    return idx, log


def main():
    c2 = "--c2" in sys.argv
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    seconds = float(args[0]) if args else 2.0
    idx, log = index(c2)
    eng = w.VacuumEngine(idx, positions=False)
    eng.Load()
    lines = [l.split() for l in open(log).read().splitlines()]
    arr = (_capi.Query * len(lines))()
    for i, t in enumerate(lines):
        arr[i] = eng.resolve(w.SearchQuery(t, n_results=10))[0]
    points = [(2, 8, 512, 1000), (2, 10, 512, 1000), (2, 12, 448, 1000), (2, 16, 384, 1000),
              (2, 16, 320, 1000), (2, 12, 512, 1000), (3, 12, 512, 1000), (2, 8, 768, 1000),
              (2, 12, 512, 300), (2, 4, 64, 100)]
    if os.environ.get("SWEEP_POINTS"):   # "depth,clients,per,window;..."
        points = [tuple(int(x) for x in p.split(",")) for p in os.environ["SWEEP_POINTS"].split(";")]
    for depth, clients, per, win in points:
        os.environ["WSR_SERVER_DEPTH"] = str(depth)
        srv = w.Server(eng, max_batch=4096, window_us=win)
        st = srv.bench(arr, n_clients=clients, depth=per, seconds=seconds)
        srv.close()
        print(json.dumps({"index": os.path.basename(idx), "server_depth": depth, "clients": clients,
                          "in_flight": clients * per, "window_us": win, "qps": round(st.qps),
                          "p50_ms": round(st.p50_ms, 3), "p99_ms": round(st.p99_ms, 3),
                          "mean_batch": round(st.mean_batch, 1), "queue_ms": round(st.queue_ms, 3),
                          "gpu_ms": round(st.gpu_ms, 3), "handoff_ms": round(st.handoff_ms, 3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
