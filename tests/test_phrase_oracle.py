"""Phrase queries in the oracle (CPU only): PhraseQueryProcessor2 and the
position-bag iterator against the reference's known answers and against a
brute-force scan of the documents' token sequences.

Reference (paths under /root/reference/src/qq_mem/src):
  PhraseQueryProcessor2 ............ query_processing.h:170-382
  QueryProcessor::HandleTheFoundDoc  query_processing.h:854-912
  PositionPostingBagIterator ....... flash_iterators.h:458-634
  CozyBoxIterator .................. flash_iterators.h:280-412
KATs: tests_5.cc:447-581 (processor), tests_15.cc:96-155 (3-doc and 5-long-doc
engines), tests_18.cc:283-356 (the same phrases on iter_test_3_docs).
"""
import os
import random

import pytest

from conftest import DATA, has_phrase, phrase_cases
from oracle import oracle as O


def test_phrase_processor_kat():
    # tests_5.cc:448-490 "Simple": 3,4 is a match
    m, t = O.phrase_lists([[1, 3, 5], [4]])
    assert m == 1 and t[0] == [3] and t[1] == [4]
    # :492-503 two empty lists, :505-517 no matches, :519-532 same position,
    # :534-545 one list empty
    assert O.phrase_lists([[], []])[0] == 0
    assert O.phrase_lists([[1, 8, 20], [0, 7, 19]])[0] == 0
    assert O.phrase_lists([[0], [0]])[0] == 0
    assert O.phrase_lists([[10], []])[0] == 0
    # :547-569 multiple matches
    m, t = O.phrase_lists([[10, 20, 100, 1000], [11, 21, 88, 101]])
    assert m == 3
    assert t[0] == [10, 20, 100] and t[1] == [11, 21, 101]


def test_phrase_processor_general_matches_bruteforce():
    # ProcessGeneral (n >= 3) finds exactly the starts a with a + i in list i
    rng = random.Random(5)
    for _ in range(300):
        n = rng.randint(3, 6)
        lists = [sorted(rng.sample(range(40), rng.randint(0, 12))) for _ in range(n)]
        want = [a for a in range(40) if all(a + i in lists[i] for i in range(n))]
        m, t = O.phrase_lists(lists)
        assert m == len(want)
        assert t[0] == want


def test_engine_phrase_kat(indexes):
    # tests_15.cc:96-116 / tests_18.cc:334-352 on iter_test_3_docs
    d = indexes["iter3"][0]
    o = O.OracleVacuum(d)
    r, _ = o.search(["a", "b"], 10, phrase=True)
    assert sorted(x for x, _ in r) == [1, 2]
    r, _ = o.search(["a", "b", "c"], 10, phrase=True)
    assert [x for x, _ in r] == [2]
    r, _ = o.search(["b", "c"], 10, phrase=True)
    assert [x for x, _ in r] == [2]
    assert o.search(["b", "a"], 10, phrase=True)[0] == []
    assert o.search(["a", "c"], 10, phrase=True)[0] == []
    # a one-term phrase is a single-term query (ProcessQueryDelta :966-969)
    assert o.search(["a"], 10, phrase=True) == o.search(["a"], 10)
    # tests_15.cc:120-155 on line_doc_with_positions
    o = O.OracleVacuum(indexes["wiki5"][0])
    assert o.search(["a", "b"], 10, phrase=True)[0] == []
    assert len(o.search(["anarchist", "movement"], 10, phrase=True)[0]) == 1
    assert len(o.search(["1860"], 10, phrase=True)[0]) == 1


def _linedoc_positions(path):
    """{term: [(doc, [positions])]} straight from the linedoc's positions column"""
    out = {}
    with open(path) as f:
        f.readline()
        for doc, line in enumerate(f):
            cols = line.rstrip("\n").split("\t")
            toks = cols[2].split()
            groups = [g for g in cols[4].split(".") if g]
            for t, g in zip(toks, groups):
                out.setdefault(t, []).append((doc, [int(p) for p in g.split(";") if p]))
    return out


def test_position_bags_match_linedoc(indexes):
    d, _, linedoc, _ = indexes["wiki5"]
    want = _linedoc_positions(linedoc)
    o = O.OracleVacuum(d)
    n = 0
    for term, posts in want.items():
        for i, (_, pos) in enumerate(posts):
            assert o.positions(term, i) == pos, (term, i)
            n += 1
    assert n > 500


def test_phrase_search_matches_bruteforce(positions_index):
    d, seqs = positions_index
    o = O.OracleVacuum(d)
    checked = 0
    for terms in phrase_cases(seqs, 150, seed=3):
        docs = {i for i, s in enumerate(seqs) if has_phrase(s, terms)}
        got, _ = o.search(terms, 64, phrase=True)
        if len(docs) > 64:
            assert len(got) == 64 and {x for x, _ in got} <= docs
            continue
        assert {x for x, _ in got} == docs, terms
        # scored exactly as the conjunctive query scores those docs
        allr, _ = o.search(terms, 64, phrase=False) if len(docs) else ([], [])
        sc = dict(allr)
        for x, s in got:
            if x in sc:
                assert sc[x] == s
        checked += 1
    assert checked > 50
