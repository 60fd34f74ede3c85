"""GPU end to end with SearchQuery::return_snippets: the HIP top-k followed by
the host snippet stage (wsr_snippet), against the oracle's
VacuumEngine::Search with snippets (vacuum_engine.h:201-258,286-296).
Doc ids, order, f64 scores and snippet strings must all be identical."""
import random

import pytest

from conftest import all_tokens, phrase_cases
from test_gpu_parity import _engine

pytestmark = pytest.mark.gpu


def _check_snippets(eng, orc, cases, k, n_passages):
    import wiser_amd as w
    qs = [w.SearchQuery(list(t), n_results=k, return_snippets=True, n_snippet_passages=n_passages,
                        is_phrase=ph) for t, ph in cases]
    res = eng.SearchBatch(qs)
    n = 0
    for (terms, ph), r in zip(cases, res):
        want = orc.search_snippets(list(terms), k, n_passages, phrase=ph)
        got = [(e.doc_id, e.doc_score, e.snippet) for e in r.entries]
        assert got == want, (terms, ph, got[:2], want[:2])
        n += len(got)
    return n


def test_snippet_kats_gpu(indexes):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d = indexes["iter3"][0]
    eng = _engine(d)
    r = eng.Search(w.SearchQuery(["a"], n_results=10, return_snippets=True))
    # tests_15.cc:22-60
    assert {e.doc_id: e.snippet for e in r.entries} == {0: "", 1: "<b>a <\\b>b\n", 2: "<b>a <\\b>b c\n"}
    assert eng.GetDocument(2) == "a b c"
    d3 = indexes["three"][0]
    eng3 = _engine(d3)
    r = eng3.Search(w.SearchQuery(["hello", "world"], n_results=5, return_snippets=True))
    # tests.cc:470-475
    assert [e.snippet for e in r.entries] == ["<b>hello<\\b> <b>world<\\b> big <b>world<\\b>\n",
                                              "<b>hello<\\b> <b>world<\\b>\n"]
    assert _check_snippets(eng3, OracleVacuum(d3), [(["hello"], False), (["wisconsin"], False)], 5, 3) == 4
    eng.close()
    eng3.close()


def test_snippets_wiki_gpu(indexes):
    from oracle.oracle import OracleVacuum
    d = indexes["wiki5"][0]
    eng = _engine(d)
    orc = OracleVacuum(d)
    toks = all_tokens()
    rng = random.Random(23)
    cases = [([t], False) for t in rng.sample(toks, 100)]
    cases += [(rng.sample(toks[:300], 2), False) for _ in range(100)]
    cases += [(["the", "of"], True), (["of", "the"], True), (["anarchist", "movement"], True)]
    assert _check_snippets(eng, orc, cases, 10, 3) > 300
    eng.close()


def test_snippets_phrase_gpu(positions_index):
    from oracle.oracle import OracleVacuum
    d, seqs = positions_index
    eng = _engine(d)
    orc = OracleVacuum(d)
    cases = [(c, True) for c in phrase_cases(seqs, 120, seed=31)]
    cases += [(c, False) for c in phrase_cases(seqs, 40, seed=32)]
    assert _check_snippets(eng, orc, cases, 10, 2) > 300
    eng.close()
