"""The round-2 reference KATs on the GPU (see test_ref_kats.py and
test_iter_kats.py for the CPU side): tests_18.cc:178-255 phrase engine with
bloom filters, tests_14.cc:163-219 tfs / decoded blocks, tests_16.cc:45-75
query-log parsing by the product's own text path (wsr_resolve_text), and the
doc-id iterator lists of tests_11.cc:218-424 / tests_12.cc:33-270."""
import ctypes as C
import os

import pytest

from conftest import DATA
from test_iter_kats import iter_indexes  # noqa: F401  (fixture)
from test_ref_kats import ref_phrases, toy_bloom  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def test_tests_18_on_gpu(toy_bloom):  # noqa: F811
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    eng = w.VacuumEngine(toy_bloom)
    eng.Load()
    assert eng.Search(w.SearchQuery(["prefix"])).Size() > 0
    assert eng.Search(w.SearchQuery(["close"])).Size() > 0
    assert eng.Search(w.SearchQuery(["solar", "body"], is_phrase=True)).Size() == 0
    phrases = ref_phrases()
    qs = [w.SearchQuery(p, n_results=5, is_phrase=True) for p in phrases]
    qs += [w.SearchQuery([p[0], "xxyxz3"], n_results=5, is_phrase=True) for p in phrases]
    res = eng.SearchBatch(qs)
    n = len(phrases)
    assert all(r.Size() > 0 for r in res[:n])
    assert all(r.Size() == 0 for r in res[n:])
    o = OracleVacuum(toy_bloom)
    for q, r in zip(qs[:n], res[:n]):
        assert [(e.doc_id, e.doc_score) for e in r.entries] == o.search(q.terms, 5, phrase=True)[0], q.terms
    eng.close()


def test_tests_14_on_gpu(built, tmp_path):
    import wiser_amd as w
    d = str(tmp_path / "i3tf")
    os.makedirs(d)
    w.build_from_linedoc(os.path.join(DATA, "iter_test_3_docs_tf"), d, "WITH_POSITIONS")
    eng = w.VacuumEngine(d)
    eng.Load()
    assert eng.TermCount() == 3
    lid, df = eng.lookup("a")
    assert df == 3
    assert (eng.decode_block(lid, 0, 0), eng.decode_block(lid, 0, 1)) == ([0, 1, 2], [1, 2, 1])
    # doc 1 holds "a a": the phrase "a a" matches only there
    r = eng.Search(w.SearchQuery(["a", "a"], is_phrase=True))
    assert [e.doc_id for e in r.entries] == [1]
    eng.close()


def test_tests_16_log_through_resolve_text(built, indexes):
    import wiser_amd as w
    from wiser_amd import _capi
    eng = w.VacuumEngine(indexes["wiki5"][0])
    eng.Load()
    text = open(os.path.join(DATA, "query_log_with_phrases"), "rb").read()
    q = (_capi.Query * 16)()
    nq = C.c_int32()
    _capi.check(_capi.lib.wsr_resolve_text(eng._h, text, len(text), 10, 16, q, C.byref(nq), None, 0))
    assert nq.value == 10
    assert q[0].n_terms == 2 and q[0].flags == _capi.QUERY_PHRASE
    assert q[1].n_terms == 3 and q[1].flags == 0
    assert [eng.lookup(t)[0] for t in ("nightt", "rain", "nashvil")] == list(q[1].list_ids[:3])
    # a query past WSR_MAX_TERMS terms: its ids past 16 land in the caller's
    # more_store (too small: WSR_E_LIMIT, nothing written there)
    toks = [f"nosuch{i}" for i in range(20)]
    long_text = (" ".join(["nightt"] * 17 + ["rain"] * 3) + "\n" + " ".join(toks)).encode()
    store = (C.c_int32 * 8)(*([-9] * 8))
    rc = _capi.lib.wsr_resolve_text(eng._h, long_text, len(long_text), 10, 4, q, C.byref(nq), store, 7)
    assert rc == _capi.E_LIMIT and list(store) == [-9] * 8
    _capi.check(_capi.lib.wsr_resolve_text(eng._h, long_text, len(long_text), 10, 4, q, C.byref(nq), store, 8))
    assert nq.value == 2 and q[0].n_terms == 20 and q[1].n_terms == 20
    night, rain = eng.lookup("nightt")[0], eng.lookup("rain")[0]
    assert [q[0].more_ids[i] for i in range(4)] == [night, rain, rain, rain]
    assert [q[1].more_ids[i] for i in range(4)] == [-1] * 4
    eng.close()


def test_iter_kat_lists_on_gpu(iter_indexes):  # noqa: F811
    """tests_11.cc:218-424 / tests_12.cc:33-270 lists (test_iter_kats.py) on the
    device: every block decoded equals the KAT values (the pack / VInts boundary
    at 127 / 128 included), and the intersections and single-term top-k with
    k up to the whole list (all ties) equal the oracle."""
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    from test_iter_kats import SPECS
    for name, (_, lists) in SPECS.items():
        d = iter_indexes[name]
        eng = w.VacuumEngine(d, positions=False)
        eng.Load()
        o = OracleVacuum(d)
        for t, docs in lists.items():
            lid, df = eng.lookup(t)
            assert df == len(docs)
            got = []
            for blk in range((df + 127) // 128):
                got += eng.decode_block(lid, blk, 0)
            assert got == docs, (name, t)
        terms = sorted(lists)
        qs = [[t] for t in terms] + [[a, b] for a in terms for b in terms if a != b]
        for k in (10, 1024):
            res = eng.SearchBatch([w.SearchQuery(q, n_results=k) for q in qs])
            for q, r in zip(qs, res):
                assert [(e.doc_id, e.doc_score) for e in r.entries] == o.search(q, k)[0], (name, q, k)
        o.close()
        eng.close()
