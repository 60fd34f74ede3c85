"""Configs at their stated size on the GPU (C2 was only spot-checked
by bench.py, C3 never run):
  * C2 (BASELINE configs[1]): the 1M-doc synthetic Zipf index of bench.py and
    2,048 queries of its logged two-term workload, bit for bit against the oracle;
  * C3 stand-in (configs[2]): the en-Wikipedia-shaped corpus (df histogram of
    gen_synthetic_log.py:8-16) at 1/10 of its terms over 500k docs, its
    two-term log, bit for bit; and at its full size (5.5 M docs, 5.64 M terms,
    the bench's headline index): 2,048 queries spread over the whole 100k log,
    and 2,048 mixed 1-5 term queries (configs[3]'s mix), bit for bit;
  * the whole Search chain from query strings (wsr_search_text).
"""
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2_full(built, tmp_path_factory):
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("c2full"))
    st = w.build_synthetic(d, n_docs=1_000_000, vocab=500_000, threads=min(16, os.cpu_count()))
    log = os.path.join(d, "two_term_100000.log")
    w.gen_two_term_log(d, log, n_queries=100_000, seed=7)
    return d, log, st


@pytest.fixture(scope="module")
def c3_small(built, tmp_path_factory):
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("c3small"))
    st = w.build_wiki_standin(d, n_docs=500_000, term_scale=0.1, threads=min(16, os.cpu_count()))
    log = os.path.join(d, "two_term.log")
    w.gen_two_term_log(d, log, n_queries=20_000, seed=7)
    return d, log, st


@pytest.fixture(scope="module")
def c3_full(built, tmp_path_factory):
    """The bench's headline index: the stand-in at its full size (~35 s)."""
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("c3full"))
    st = w.build_wiki_standin(d, n_docs=5_500_000, term_scale=1.0, threads=min(16, os.cpu_count()))
    log = os.path.join(d, "two_term_100000.log")
    w.gen_two_term_log(d, log, n_queries=100_000, seed=7)
    return d, log, st


def _check_log(d, log, nq, k=10, stride=7, eng=None):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    lines = [l.split() for l in open(log).read().splitlines()]
    # spread over the whole log: every stride-th query
    qs = lines[::stride][:nq]
    own = eng is None
    if own:
        eng = w.VacuumEngine(d, positions=False)
        eng.Load()
    res = eng.SearchBatch([w.SearchQuery(q, n_results=k) for q in qs])
    orc = OracleVacuum(d)
    want = orc.search_lines(qs, k, threads=min(16, os.cpu_count()))
    bad = [(q, [(e.doc_id, e.doc_score) for e in r.entries][:3], x[:3])
           for q, r, x in zip(qs, res, want) if [(e.doc_id, e.doc_score) for e in r.entries] != x]
    if own:
        eng.close()
    orc.close()
    assert not bad, bad[:3]
    return sum(1 for x in want if x)


def test_c2_full_size_logged_queries(c2_full):
    d, log, st = c2_full
    assert st.n_docs == 1_000_000
    nonempty = _check_log(d, log, 2048)
    assert nonempty > 500


def test_c2_full_size_k64_other_slice(c2_full):
    # k = 64 (the largest) over another slice of the log
    d, log, _ = c2_full
    _check_log(d, log, 512, k=64, stride=97)


def test_c3_standin_logged_queries(c3_small):
    d, log, st = c3_small
    assert st.n_terms > 500_000
    _check_log(d, log, 2048, stride=5)


@pytest.fixture(scope="module")
def c3_full_engine(c3_full):
    import wiser_amd as w
    eng = w.VacuumEngine(c3_full[0], positions=False)
    eng.Load()
    yield eng
    eng.close()


def test_c3_full_size_logged_queries(c3_full, c3_full_engine):
    """configs[2] at the headline size: 2,048 queries, every 48th of the 100k
    log (so all of it is sampled), top-10, bit for bit against the oracle."""
    d, log, st = c3_full
    assert st.n_docs == 5_500_000 and st.n_terms > 5_000_000
    nonempty = _check_log(d, log, 2048, stride=48, eng=c3_full_engine)
    assert nonempty > 100


def test_c3_full_size_mixed_1to5(c3_full, c3_full_engine):
    """configs[3]'s query mix (1-5 AND terms, AOL shares) over the full-size
    stand-in, 2,048 queries, top-10, bit for bit."""
    import wiser_amd as w
    d, _, _ = c3_full
    mixed = os.path.join(d, "mixed_20000.log")
    w.gen_mixed_log(d, mixed, n_queries=20_000, seed=7)
    lens = [len(l.split()) for l in open(mixed).read().splitlines()]
    assert set(lens) == {1, 2, 3, 4, 5}
    _check_log(d, mixed, 2048, stride=9, eng=c3_full_engine)


def test_search_text_chain(c3_small):
    """wsr_search_text (strings -> host results) = per-query oracle, including
    unknown terms, phrase-quoted lines on a positions=0 engine being refused,
    and blank lines skipped."""
    import ctypes as C
    import wiser_amd as w
    from wiser_amd import _capi
    from oracle.oracle import OracleVacuum
    d, log, _ = c3_small
    lines = open(log).read().splitlines()[:300] + ["nosuchterm w00000001", "", "  w00000002  "]
    text = "\n".join(lines).encode()
    eng = w.VacuumEngine(d, positions=False)
    eng.Load()
    hits = (_capi.Hit * (len(lines) * 10))()
    nh = (C.c_int32 * len(lines))()
    nq = C.c_int32()
    _capi.check(_capi.lib.wsr_search_text(eng._h, text, len(text), 10, 10, len(lines), hits, nh,
                                           C.byref(nq)))
    qs = [l.split() for l in lines if l.strip()]
    assert nq.value == len(qs)
    orc = OracleVacuum(d)
    for i, q in enumerate(qs):
        got = [(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])]
        assert got == orc.search(q, 10)[0], q
    bad = b'"w00000001 w00000002"'
    rc = _capi.lib.wsr_search_text(eng._h, bad, len(bad), 10, 10, 4, hits, nh, C.byref(nq))
    assert rc == _capi.E_INVALID
    eng.close()
    orc.close()


def test_one_runtime():
    """The GPU suite runs the engine on the same runtime as bench.py: torch is
    imported first in both (conftest, bench.main), so libwiser_hip.so binds to
    the libamdhip64 / librccl torch mapped, and there is only that one.
    Printed so that the GPU log records it (bench.py prints it as "runtime")."""
    from wiser_amd import _capi
    info = _capi.runtime_info()
    print(info)
    hip = info.split("libamdhip64=")[1].split()[0]
    maps = open("/proc/self/maps").read()
    loaded = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert loaded == {os.path.realpath(hip)} or loaded == {hip}, (info, loaded)


def test_image_info(c3_small):
    """wsr_image_info_get: the per-buffer HBM bytes of an image add up, the
    blob holds at least the file's docid + tf spans, and dense lists exist."""
    import wiser_amd as w
    d, _, st = c3_small
    eng = w.VacuumEngine(d, positions=False)
    eng.Load()
    info = eng.image_info()
    eng.close()
    parts = ("blob_bytes", "dense_bytes", "tf8_bytes", "plen_bytes", "dir_bytes", "pos_bytes")
    assert info["total_bytes"] == sum(info[p] for p in parts)
    assert info["pos_bytes"] <= 8 * len(parts)   # positions off: only the 1-element placeholders
    assert 0 < info["dense_lists"] < info["n_lists"]
    assert info["blob_bytes"] < st.vacuum_bytes


def test_c5_full_size_phrases(c3_full):
    """configs[4]'s phrase queries over the full-size stand-in (its phrase
    pool, gen_synthetic_log.py:216-265 shape): 2,048 phrase queries, top-10,
    bit for bit against the oracle's PhraseQueryProcessor2 restatement, and a
    good share of them must find docs."""
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d, _, _ = c3_full
    log = os.path.join(d, "phrase_10000.log")
    w.gen_phrase_log(d, log, n_queries=10_000, seed=7)
    items = w.read_query_log(log)
    assert all(ph and len(t) == 2 for t, ph in items)
    qs = [t for t, _ in items][::4][:2048]
    eng = w.VacuumEngine(d, positions=True)
    eng.Load()
    res = eng.SearchBatch([w.SearchQuery(q, n_results=10, is_phrase=True) for q in qs])
    eng.close()
    orc = OracleVacuum(d)
    want = orc.search_lines(qs, 10, threads=min(16, os.cpu_count()), phrases=[True] * len(qs))
    orc.close()
    bad = [(q, [(e.doc_id, e.doc_score) for e in r.entries][:3], x[:3])
           for q, r, x in zip(qs, res, want) if [(e.doc_id, e.doc_score) for e in r.entries] != x]
    assert not bad, bad[:3]
    assert sum(1 for x in want if x) > len(qs) // 2


# ---- configs[3] / configs[4] in their stated form: doc-range sharded 8x ----
#  The full-size stand-in split into W = 8 doc-range shard
# engines on the one GPU (each holds its eighth of the blocks, with positions),
# driven through wsr_shard_step's device halves with the regions moved exactly
# as its ncclAllToAll moves them (tests/test_shard_gpu.py::_run_step_regions).
@pytest.fixture(scope="module")
def c3_shards8(c3_full):
    from test_shard_gpu import open_shards
    engs = open_shards(c3_full[0], 8, positions=True)
    yield engs
    for e in engs:
        e.close()


def _oracle_lines(d, qs, k, phrases=None):
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(d)
    try:
        return orc.search_lines(qs, k, threads=min(16, os.cpu_count()), phrases=phrases)
    finally:
        orc.close()


def test_c4_full_size_docshard8(c3_full, c3_shards8):
    """configs[3]: 2,048 mixed 1-5-term AND queries (AOL shares) over the
    5.5 M-doc stand-in, doc-range sharded 8x, top-10, bit for bit."""
    import wiser_amd as w
    from test_shard_gpu import _run_step_regions
    d, _, _ = c3_full
    mixed = os.path.join(d, "mixed_20000.log")
    if not os.path.exists(mixed):
        w.gen_mixed_log(d, mixed, n_queries=20_000, seed=7)
    qs = [l.split() for l in open(mixed).read().splitlines()][::9][:2048]
    qs2, got = _run_step_regions(d, qs, 10, 8, slot=None, engines=c3_shards8)
    want = _oracle_lines(d, qs2, 10)
    bad = [(q, g[:3], x[:3]) for q, g, x in zip(qs2, got, want) if g != x]
    assert not bad, bad[:3]
    assert sum(1 for x in want if x) > 500


def test_c5_full_size_docshard8(c3_full, c3_shards8):
    """configs[4]: 1,024 two-term phrase queries from the stand-in's phrase pool,
    doc-range sharded 8x (each shard keeps its lists' whole position boxes),
    top-10, bit for bit against the oracle's PhraseQueryProcessor2."""
    import wiser_amd as w
    from test_shard_gpu import _run_step_regions
    d, _, _ = c3_full
    log = os.path.join(d, "phrase_10000.log")
    if not os.path.exists(log):
        w.gen_phrase_log(d, log, n_queries=10_000, seed=7)
    qs = [t for t, _ in w.read_query_log(log)][1::8][:1024]
    qs2, got = _run_step_regions(d, qs, 10, 8, slot=None, phrase=True, engines=c3_shards8)
    want = _oracle_lines(d, qs2, 10, phrases=[True] * len(qs2))
    bad = [(q, g[:3], x[:3]) for q, g, x in zip(qs2, got, want) if g != x]
    assert not bad, bad[:3]
    assert sum(1 for x in want if x) > len(qs2) // 2


# ---- a topic-clustered corpus (terms co-occur by topic) ----
@pytest.fixture(scope="module")
def c3_topics(built, tmp_path_factory):
    """The full-size stand-in with topic-clustered doc ids (bench.py TOPICS)."""
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("c3topics"))
    st = w.build_wiki_standin(d, n_docs=5_500_000, term_scale=1.0, threads=min(16, os.cpu_count()),
                              topics=128, topics_per_term=2, affinity=0.6)
    log = os.path.join(d, "two_term_100000.log")
    w.gen_two_term_log(d, log, n_queries=100_000, seed=7)
    return d, log, st


def test_c3_topics_full_size_logged_queries(c3_topics):
    """2,048 queries spread over the clustered corpus's whole 100k log, top-10,
    bit for bit against the oracle."""
    d, log, st = c3_topics
    assert st.n_docs == 5_500_000
    nonempty = _check_log(d, log, 2048, stride=48)
    assert nonempty > 100


# ---- the reference's single-term workloads at size ----
def test_c3_full_size_single_terms(c3_full, c3_full_engine):
    """run_exp.py:116-117's type_single.docfreq_high / _low over the full-size
    stand-in (gen_synthetic_log.py:171-189: terms of the df >= 10^4 / < 10^4
    group, drawn with replacement): 256 of each, top-10, bit for bit against
    the oracle's SingleTermQueryProcessor (query_processing.h:620-642)."""
    import wiser_amd as w
    d, _, _ = c3_full
    for high in (True, False):
        log = os.path.join(d, f"single_{'high' if high else 'low'}_20000.log")
        w.gen_single_term_log(d, log, high, n_queries=20_000, seed=7)
        nonempty = _check_log(d, log, 256, stride=61, eng=c3_full_engine)
        assert nonempty == 256   # every term of the dictionary has postings


# ---- phrases and conjunctive queries in the same batches ----
def test_c3_full_size_realistic_mix(c3_full):
    """The reference's mixed log (query_pool.h:363-375: quoted phrase lines
    among plain ones): 10 % two-term phrases among the 1-5-term AND mix, 2,048
    queries in one batch (so the phrase and conjunctive classes share every
    launch), then the same queries from 16 threads through the serving front
    end, every result bit for bit against the oracle."""
    import threading
    import wiser_amd as w
    d, _, _ = c3_full
    log = os.path.join(d, "realistic_20000.log")
    w.gen_realistic_log(d, log, n_queries=20_000, phrase_share=0.1, seed=7)
    items = w.read_query_log(log)[::9][:2048]
    n_ph = sum(1 for _, ph in items if ph)
    assert 100 < n_ph < 400
    qs, phs = [t for t, _ in items], [ph for _, ph in items]
    want = _oracle_lines(d, qs, 10, phrases=phs)
    eng = w.VacuumEngine(d, positions=True)
    eng.Load()
    try:
        res = eng.SearchBatch([w.SearchQuery(q, n_results=10, is_phrase=ph) for q, ph in items])
        bad = [(q, ph) for q, ph, r, x in zip(qs, phs, res, want)
               if [(e.doc_id, e.doc_score) for e in r.entries] != x]
        assert not bad, bad[:3]
        srv = w.Server(eng, max_batch=1024, window_us=300)
        got = [None] * len(items)

        def worker(t):
            for i in range(t, len(items), 16):
                r = srv.Search(w.SearchQuery(qs[i], n_results=10, is_phrase=phs[i]))
                got[i] = [(e.doc_id, e.doc_score) for e in r.entries]
        ts = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        srv.close()
        assert got == want
    finally:
        eng.close()
