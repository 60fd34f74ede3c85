import os, sys, json
sys.path.insert(0, os.getcwd())
import wiser_amd as w
from wiser_amd import _capi
idx = "/tmp/wiser_bench/c2_1000000_500000"
if not os.path.exists(os.path.join(idx, "READY")):
    os.makedirs(idx, exist_ok=True)
    w.build_synthetic(idx, threads=16)
    w.gen_two_term_log(idx, os.path.join(idx, "two_term_100000.log"), 100000, 7)
    open(os.path.join(idx, "READY"), "w").write("ok")
eng = w.VacuumEngine(idx, positions=False); eng.Load()
lines = [l.split() for l in open(os.path.join(idx, "two_term_100000.log")).read().splitlines()]
arr = (_capi.Query * len(lines))()
for i, t in enumerate(lines):
    arr[i] = eng.resolve(w.SearchQuery(t, n_results=10))[0]
for c, d, win in [(4, 1024, 1000), (4, 1024, 500), (4, 1024, 250), (4, 1024, 100), (4, 2048, 250), (8, 512, 250), (4, 64, 100), (4, 64, 30)]:
    srv = w.Server(eng, max_batch=4096, window_us=win)
    st = srv.bench(arr, n_clients=c, depth=d, seconds=2.0)
    srv.close()
    print(f"clients={c} depth={d} window={win}: qps={st.qps:.0f} p50={st.p50_ms:.3f} p99={st.p99_ms:.3f} batch={st.mean_batch:.1f}", flush=True)
