"""Reference known-answer tests pinned in round 2 (CPU: the oracle over indexes
written by the product writer, and the product's own query-log parsing):

  tests_18.cc:178-255  the bloom phrase engine over wiki_linedoc.toy.pre-suf-bloom:
                       {prefix} and {close} are found, the phrase "solar body" is
                       not, every phrase listed in line_doc.with-bloom.toy-phrases
                       is found and none with its second term replaced by xxyxz3;
  tests_14.cc:163-219  iter_test_3_docs_tf: 3 terms, 'a' has docs 0,1,2 with tf
                       1,2,1 and doc 1's positions are {0, 1};
  tests_16.cc:45-75    query_log_with_phrases: "greek armi" is a phrase, the next
                       line three plain terms, ten queries.
The fixture files are the reference's own testdata, copied as data.
"""
import os

import pytest

from conftest import BLOOM_ENTRIES, BLOOM_RATIO, DATA


def ref_phrases():
    """GetPhrases (tests_18.cc:155-175): 'first:end end ...' -> [first, end] pairs."""
    out = []
    for line in open(os.path.join(DATA, "line_doc.with-bloom.toy-phrases")).read().splitlines():
        items = [x for x in line.split(":") if x]
        if len(items) > 1:
            out += [[items[0], e] for e in items[1].split(" ") if e]
    return out


@pytest.fixture(scope="module")
def toy_bloom(built, tmp_path_factory):
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("toybloom"))
    w.build_from_linedoc(os.path.join(DATA, "wiki_linedoc.toy.pre-suf-bloom"), d, "WITH_POSITIONS",
                         n_rows=10000, bloom=(BLOOM_RATIO, BLOOM_ENTRIES))
    return d


def test_tests_18_bloom_phrase_engine(toy_bloom):
    from oracle.oracle import OracleVacuum
    o = OracleVacuum(toy_bloom)
    assert o.has_bloom()
    assert o.term_count() > 0
    assert len(o.search(["prefix"], 5)[0]) > 0
    assert len(o.search(["close"], 5)[0]) > 0
    assert o.search(["solar", "body"], 5, phrase=True)[0] == []
    phrases = ref_phrases()
    assert len(phrases) > 1000
    for p in phrases:
        assert len(o.search(p, 5, phrase=True)[0]) > 0, p
        assert o.search([p[0], "xxyxz3"], 5, phrase=True)[0] == [], p
    o.close()


def test_tests_14_three_docs_tf(built, tmp_path):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d = str(tmp_path / "i3tf")
    os.makedirs(d)
    w.build_from_linedoc(os.path.join(DATA, "iter_test_3_docs_tf"), d, "WITH_POSITIONS")
    o = OracleVacuum(d)
    assert o.term_count() == 3
    assert o.postings("a") == ([0, 1, 2], [1, 2, 1])
    assert o.positions("a", 1) == [0, 1]
    assert o.positions("a", 0) == [0] and o.positions("a", 2) == [0]
    o.close()


def test_tests_16_query_log_with_phrases():
    import wiser_amd as w
    log = w.read_query_log(os.path.join(DATA, "query_log_with_phrases"))
    assert log[0] == (["greek", "armi"], True)
    assert log[1] == (["nightt", "rain", "nashvil"], False)
    assert len(log) == 10
