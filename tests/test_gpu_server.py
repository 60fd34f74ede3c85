"""The micro-batching front end (wsr_server_*) on the GPU: concurrent single
queries from many threads are coalesced into batches and each caller gets the
oracle's exact result (the reference's gRPC workers share one engine,
grpc_server_impl.h:260-263,382-389)."""
import os
import random
import threading

import pytest

pytestmark = pytest.mark.gpu


def test_concurrent_search_matches_oracle(synth_small):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    eng = w.VacuumEngine(d)
    eng.Load()
    srv = w.Server(eng, max_batch=512, window_us=300)
    orc = OracleVacuum(d)
    log = os.path.join(d, "qsrv.log")
    w.gen_two_term_log(d, log, n_queries=1200, seed=5)
    qs = [l.split() for l in open(log).read().splitlines()]
    rng = random.Random(9)
    head = [f"t{i:07d}" for i in range(40)]
    qs += [rng.sample(head, rng.randint(1, 4)) for _ in range(300)]
    # k up to the batch limit (64 was the server's cap) and
    # queries past the 16 inline terms
    qs += [rng.sample(head, rng.randint(17, 30)) for _ in range(20)]
    items = [(q, i % 3 == 0 and 1 < len(q) <= 8, [1, 5, 10, 64, 100, 300][i % 6]) for i, q in enumerate(qs)]
    got = [None] * len(items)
    errors = []

    def worker(t):
        try:
            for i in range(t, len(items), 24):
                q, ph, k = items[i]
                r = srv.Search(w.SearchQuery(q, n_results=k, is_phrase=ph))
                got[i] = [(e.doc_id, e.doc_score) for e in r.entries]
        except Exception as e:   # noqa: BLE001 - surfaced below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors[:3]
    for (q, ph, k), g in zip(items, got):
        assert g == orc.search(q, k, phrase=ph)[0], (q, ph, k)
    srv.close()
    eng.close()


def test_closed_loop_bench(synth_small):
    import wiser_amd as w
    from wiser_amd import _capi
    d, _ = synth_small
    eng = w.VacuumEngine(d, positions=False)
    eng.Load()
    log = os.path.join(d, "qsrv2.log")
    w.gen_two_term_log(d, log, n_queries=2000, seed=6)
    qs = [l.split() for l in open(log).read().splitlines()]
    arr = (_capi.Query * len(qs))()
    for i, q in enumerate(qs):
        arr[i] = eng.resolve(w.SearchQuery(q, n_results=10))[0]
    srv = w.Server(eng, max_batch=1024, window_us=200)
    st = srv.bench(arr, n_clients=8, depth=64, seconds=1.0)
    assert st.queries > 1000 and st.qps > 0
    assert st.mean_batch > 1.0           # calls were coalesced
    assert 0 < st.p50_ms <= st.p99_ms
    srv.close()
    eng.close()


def test_bad_request_fails_alone(synth_small):
    """one caller's bad query (a phrase query on an engine opened
    without positions, an unknown flag, k over the limit) fails at submit and
    never takes the other callers' queries of the same batch down with it."""
    import ctypes as C
    import wiser_amd as w
    from wiser_amd import _capi
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    eng = w.VacuumEngine(d, positions=False)
    eng.Load()
    srv = w.Server(eng, max_batch=256, window_us=2000)
    orc = OracleVacuum(d)
    good = [[f"t{i:07d}", f"t{i + 1:07d}"] for i in range(0, 120, 2)]
    results, errors = {}, {}

    def good_worker(i):
        r = srv.Search(w.SearchQuery(good[i], n_results=10))
        results[i] = [(e.doc_id, e.doc_score) for e in r.entries]

    def bad_worker(kind):
        q = eng.resolve(w.SearchQuery(good[0], n_results=10, is_phrase=(kind == "phrase")))[0]
        if kind == "flags":
            q.flags = 6
        elif kind == "k":
            q.k = _capi.SERVER_MAX_K + 1   # (past the server's k limit)
        hits = (_capi.Hit * 1024)()
        nh = C.c_int32()
        errors[kind] = _capi.lib.wsr_server_search(srv._s, C.byref(q), hits, C.byref(nh))

    ts = [threading.Thread(target=good_worker, args=(i,)) for i in range(len(good))]
    ts += [threading.Thread(target=bad_worker, args=(k,)) for k in ("phrase", "flags", "k")]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert errors["phrase"] == _capi.E_INVALID and errors["flags"] == _capi.E_INVALID
    assert errors["k"] == _capi.E_LIMIT
    for i, q in enumerate(good):
        assert results[i] == orc.search(q, 10)[0], q
    srv.close()
    eng.close()
