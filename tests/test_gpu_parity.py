"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bit-exact: doc ids, their order (including ties, reproduced through the
restated libstdc++ heap) and the f64 scores.  North-star tolerance for scores
is 1e-5 relative; these tests require exact equality, which is stricter.
"""
import os
import random

import pytest

from conftest import DATA, all_tokens

pytestmark = pytest.mark.gpu

SCORE_RTOL = 1e-5  # north_star tolerance; asserted only as a secondary check


# Other lists are probed either by decoding their blocks or through the rank
# bitmap of a dense list; both paths must give the reference's result.
#   blocks: no bitmaps; dense: the default thresholds; dense_all: every list
#   gets a bitmap and every other list is probed through it.
DENSE_MODES = {
    "blocks": {"WSR_DENSE_DIV": "0"},
    "dense": {},
    "dense_all": {"WSR_DENSE_DIV": "1000000000", "WSR_DENSE_RATIO": "0"},
}
ENGINE_ENV = ("WSR_DENSE_DIV", "WSR_DENSE_RATIO")


def _engine(d, mode="dense"):
    import wiser_amd as w
    saved = {k: os.environ.get(k) for k in ENGINE_ENV}
    try:
        for k in saved:
            os.environ.pop(k, None)
        os.environ.update(DENSE_MODES[mode])
        e = w.VacuumEngine(d)
        e.Load()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return e


def _check(eng, orc, queries, k):
    import wiser_amd as w
    res = eng.SearchBatch([w.SearchQuery(list(q), n_results=k) for q in queries])
    bad = []
    for q, r in zip(queries, res):
        want, dfs = orc.search(list(q), k)
        got = [(e.doc_id, e.doc_score) for e in r.entries]
        if got != want or (want and r.doc_freqs != dfs):
            bad.append((q, got[:3], want[:3]))
        for (gd, gs), (wd, ws) in zip(got, want):
            assert abs(gs - ws) <= SCORE_RTOL * max(1.0, abs(ws))
    assert not bad, f"{len(bad)}/{len(queries)} queries differ, first: {bad[:3]}"


@pytest.fixture(scope="module", params=sorted(DENSE_MODES))
def gpu_indexes(indexes, request):
    from oracle.oracle import OracleVacuum
    out = {}
    for name, (d, st, linedoc, fmt) in indexes.items():
        out[name] = (_engine(d, request.param), OracleVacuum(d), d)
    yield out
    for e, o, _ in out.values():
        e.close()
        o.close()


def test_three_doc_kat(gpu_indexes):
    """tests.cc:408-511 (scores produced by Elasticsearch, checked to 3 digits)."""
    import wiser_amd as w
    eng, orc, _ = gpu_indexes["three"]
    r = eng.Search(w.SearchQuery(["wisconsin"]))
    assert [e.doc_id for e in r.entries] == [1] and f"{r.entries[0].doc_score:.3g}" == "1.09"
    r = eng.Search(w.SearchQuery(["hello"]))
    assert [f"{e.doc_score:.3g}" for e in r.entries] == ["0.149", "0.149", "0.111"]
    r = eng.Search(w.SearchQuery(["hello", "world"]))
    assert [f"{e.doc_score:.3g}" for e in r.entries] == ["0.677", "0.672"]
    q = w.SearchQuery(["hello", "world"])
    q.n_results = 0
    assert eng.Search(q).Size() == 0
    _check(eng, orc, [["hello"], ["world"], ["hello", "world"], ["world", "hello"], ["big", "world"],
                      ["hello", "wisconsin", "world"], ["nothere"], ["hello", "nothere"]], 5)


def test_order_kat(gpu_indexes):
    """tests_5.cc:16-52: shorter docs rank first -> {4,3,2,1,0}; k=2 -> {4,3}."""
    import wiser_amd as w
    eng, orc, _ = gpu_indexes["order"]
    r = eng.Search(w.SearchQuery(["hello", "world"], n_results=5))
    assert [e.doc_id for e in r.entries] == [4, 3, 2, 1, 0]
    r = eng.Search(w.SearchQuery(["hello", "world"], n_results=2))
    assert [e.doc_id for e in r.entries] == [4, 3]
    r = eng.Search(w.SearchQuery(["hello", "world", "again"], n_results=2))
    assert [e.doc_id for e in r.entries] == [4, 3]


def test_iter3_kat(gpu_indexes):
    """tests_15.cc:11-116: sizes a:3 b:2 c:1; AND {a,b} -> {1,2}; d absent."""
    import wiser_amd as w
    eng, orc, _ = gpu_indexes["iter3"]
    assert eng.TermCount() == 3
    assert eng.PostinglistSizes(["a", "b", "c", "d"]) == {"a": 3, "b": 2, "c": 1}
    assert eng.Search(w.SearchQuery(["a"])).Size() == 3
    assert eng.Search(w.SearchQuery(["d"])).Size() == 0
    r = eng.Search(w.SearchQuery(["a", "b"]))
    assert sorted(e.doc_id for e in r.entries) == [1, 2]
    _check(eng, orc, [["a"], ["b"], ["c"], ["a", "b"], ["b", "a"], ["a", "b", "c"], ["c", "a"]], 5)


def test_one_word(gpu_indexes):
    """tests_14.cc:10-46: one list, one posting."""
    import wiser_amd as w
    eng, orc, _ = gpu_indexes["one_word"]
    r = eng.Search(w.SearchQuery(["a"]))
    assert [e.doc_id for e in r.entries] == [0]
    assert eng.Search(w.SearchQuery(["b"])).Size() == 0


def test_wiki5_all_tokens_single_term(gpu_indexes):
    """tests_15.cc:158-210: every token of all-tokens.txt, single-term, vs the oracle."""
    eng, orc, _ = gpu_indexes["wiki5"]
    toks = all_tokens()
    for k in (5, 10):
        _check(eng, orc, [[t] for t in toks], k)


def test_wiki5_multi_term(gpu_indexes):
    eng, orc, _ = gpu_indexes["wiki5"]
    toks = all_tokens()
    rng = random.Random(11)
    qs = []
    for n in (2, 2, 2, 3, 4, 5, 8):
        for _ in range(300):
            qs.append(rng.sample(toks, n))
    # frequent-term pairs (long lists, many survivors, many score ties)
    freq = sorted(toks, key=lambda t: -orc.df(t))[:40]
    for _ in range(300):
        qs.append(rng.sample(freq, 2))
    for _ in range(100):
        qs.append(rng.sample(freq, 3))
    for k in (1, 10, 64):
        _check(eng, orc, qs, k)


def test_duplicate_and_edge_terms(gpu_indexes):
    eng, orc, _ = gpu_indexes["wiki5"]
    _check(eng, orc, [["the", "the"], ["of", "the", "of"], ["the"] * 8, ["zzzmissing", "the"],
                      ["anarchist", "movement"]], 10)


def test_c1_tokenized_10k(gpu_indexes):
    """Config C1: test_doc_tokenized (9,999 docs, TOKEN_ONLY), single-term top-10,
    every distinct token plus 10k tokens sampled with seed 1."""
    eng, orc, d = gpu_indexes["tok10k"]
    from oracle.oracle import OracleQqMem
    qq = OracleQqMem(os.path.join(DATA, "test_doc_tokenized"), "TOKEN_ONLY")
    vocab = set()
    with open(os.path.join(DATA, "test_doc_tokenized")) as f:
        next(f)
        for line in f:
            cols = line.rstrip("\n").split("\t")
            vocab.update(cols[2].split())
    vocab = sorted(vocab)
    rng = random.Random(1)
    sample = [rng.choice(vocab) for _ in range(10000)]
    qs = [[t] for t in vocab[:20000]] + [[t] for t in sample]
    _check(eng, orc, qs, 10)
    # and the in-memory engine restatement agrees (Vacuum == QqMem, tests_15.cc:158-210)
    for t in vocab[:2000]:
        assert orc.search([t], 10)[0] == qq.search([t], 10)[0]
    # two-term queries over the same index
    pairs = [rng.sample(vocab[:3000], 2) for _ in range(3000)]
    _check(eng, orc, pairs, 10)


def test_device_block_decode(gpu_indexes):
    """Every block of a few long lists decoded on the device == the oracle iterator."""
    eng, orc, _ = gpu_indexes["tok10k"]
    for term in ["the", "of", "and", "a", "in", "to", "is"]:
        lid, df = eng.lookup(term)
        docs, tfs = orc.postings(term)
        assert len(docs) == df
        nblk = (df + 127) // 128
        got_d, got_t = [], []
        for b in range(nblk):
            got_d += eng.decode_block(lid, b, 0)
            got_t += eng.decode_block(lid, b, 1)
        assert got_d == docs and got_t == tfs, term


@pytest.mark.parametrize("mode", sorted(DENSE_MODES))
def test_synthetic_parity(synth_small, mode):
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    d, st = synth_small
    eng = _engine(d, mode)
    orc = OracleVacuum(d)
    log = os.path.join(d, "q.log")
    w.gen_two_term_log(d, log, n_queries=3000, seed=7)
    qs = [l.split() for l in open(log).read().splitlines()]
    _check(eng, orc, qs, 10)
    rng = random.Random(3)
    terms = [f"t{i:07d}" for i in range(0, 400)]
    multi = [rng.sample(terms, rng.randint(3, 5)) for _ in range(500)]
    singles = [[f"t{i:07d}"] for i in range(0, 3000, 7)]
    _check(eng, orc, multi + singles, 10)
    eng.close()
    orc.close()


def test_limits_fail_loudly(gpu_indexes):
    import wiser_amd as w
    eng, _, _ = gpu_indexes["three"]
    with pytest.raises(NotImplementedError):
        eng.Search(w.SearchQuery(["hello"], n_results=1025))
    with pytest.raises(NotImplementedError):
        eng.Search(w.SearchQuery(["hello"] * 1025))


@pytest.mark.parametrize("mode", sorted(DENSE_MODES))
def test_large_tf_dense_escape(tmp_path, mode):
    """tf >= 255 in a bitmap-probed list: the 1-byte tf escapes to the blob
    (pack blocks and the VInts tail)."""
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    ld = tmp_path / "big_tf.linedoc"
    rng = random.Random(5)
    with open(ld, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(300):
            toks = ["x"] * rng.choice([1, 2, 254, 255, 256, 600])
            if i % 2 == 0:
                toks += ["y"] * rng.randint(1, 3)
            if i % 7 == 0:
                toks += ["z"] * 300
            toks += [f"w{i}"]
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    d = tmp_path / "idx"
    d.mkdir()
    w.build_from_linedoc(str(ld), str(d), "TOKEN_ONLY")
    eng = _engine(str(d), mode)
    orc = OracleVacuum(str(d))
    _check(eng, orc, [["x"], ["y", "x"], ["x", "y"], ["z", "x"], ["y", "z", "x"], ["w7", "x"],
                      ["x", "w299"]], 64)
    eng.close()
    orc.close()


@pytest.mark.parametrize("mode", list(DENSE_MODES))
def test_wide_k(synth_small, mode):
    """k > 64 (refused before): every survivor of a wide query is
    an event and the replay keeps the libstdc++ heap in LDS; k = 65, 100, 500
    and the limit 1024, mixed with k = 10 queries in one batch."""
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    d, _ = synth_small
    eng = _engine(d, mode)
    orc = OracleVacuum(d)
    log = os.path.join(d, "qwide.log")
    w.gen_two_term_log(d, log, n_queries=300, seed=21)
    qs = [l.split() for l in open(log).read().splitlines()]
    head = [f"t{i:07d}" for i in range(12)]
    rng = random.Random(5)
    qs += [[h] for h in head] + [rng.sample(head, 2) for _ in range(40)]
    ks = [65, 100, 500, 1024, 10]
    items = [(q, ks[i % len(ks)]) for i, q in enumerate(qs)]
    res = eng.SearchBatch([w.SearchQuery(q, n_results=k) for q, k in items])
    for (q, k), r in zip(items, res):
        assert [(e.doc_id, e.doc_score) for e in r.entries] == orc.search(q, k)[0], (q, k)
    eng.close()


@pytest.mark.parametrize("mode", ["blocks", "dense", "dense_all"])
def test_many_terms(synth_small, mode):
    """Conjunctive queries of 9 to 16 terms inline, and of 17 to 40 terms
    through the batch's term table (the reference's processor
    has no term cap, query_processing.h:710-728,810-852); the phrase cap stays
    8 (query_processing.h:695) and a longer phrase is refused."""
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    from wiser_amd import _capi
    d, _ = synth_small
    eng = _engine(d, mode)
    orc = OracleVacuum(d)
    head = [f"t{i:07d}" for i in range(24)]
    rng = random.Random(6)
    head = [f"t{i:07d}" for i in range(48)]
    qs = [rng.sample(head[:24], n) for n in (9, 10, 12, 12, 14, 16, 16) for _ in range(6)]
    qs += [head[:12] + head[:4]]   # duplicates: each occurrence scores
    # past the inline 16: 17, 24 and 40 terms (the driver among the last ones
    # too), and a 40-term query of repeated head words
    qs += [rng.sample(head, n) for n in (17, 24, 24, 40) for _ in range(5)]
    qs += [head[:6] * 4, (head[:3] * 8) + head[40:42], head[:20] + head[:20]]
    for k in (10, 100):
        res = eng.SearchBatch([w.SearchQuery(q, n_results=k) for q in qs])
        for q, r in zip(qs, res):
            assert [(e.doc_id, e.doc_score) for e in r.entries] == orc.search(q, k)[0], (q, k)
    nonempty = sum(1 for r in eng.SearchBatch([w.SearchQuery(q) for q in qs]) if r.Size())
    assert nonempty > 10
    with pytest.raises(_capi.WiserError, match="LIMIT"):
        eng.SearchBatch([w.SearchQuery(head[:9], is_phrase=True)])
    # mixed with short queries in one batch, through the text path as well
    long_q = [q for q in qs if len(q) > 16]
    text = "\n".join(" ".join(q) for q in long_q + qs[:5]).encode()
    import ctypes as C
    n = len(long_q) + 5
    hits = (_capi.Hit * (n * 10))()
    nh = (C.c_int32 * n)()
    nq = C.c_int32()
    _capi.check(_capi.lib.wsr_search_text(eng._h, text, len(text), 10, 10, n, hits, nh, C.byref(nq)))
    assert nq.value == n
    for i, q in enumerate(long_q + qs[:5]):
        assert [(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])] == orc.search(q, 10)[0]
    eng.close()
