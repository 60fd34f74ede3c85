"""The en-Wikipedia-shaped stand-in writer (BASELINE configs[2], writer.h
WikiSpec) on the CPU: its df histogram is the reference's
(tools/gen_synthetic_log.py:8-16) times term_scale, its lists are readable by
the oracle, doc lengths are the sums of the docs' tfs, and it is deterministic."""
import math
import os
import struct

import pytest

DECADES = [4996891, 520675, 94721, 22139, 5717, 1434, 38]


@pytest.fixture(scope="module")
def tiny(built, tmp_path_factory):
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("wiki_tiny"))
    st = w.build_wiki_standin(d, n_docs=20_000, term_scale=0.002, threads=4)
    return d, st


def test_histogram_and_lists(tiny):
    from oracle.oracle import OracleVacuum
    d, st = tiny
    n = 20_000
    want = [round(c * 0.002) for e, c in enumerate(DECADES) if 10 ** e < n + 1]
    orc = OracleVacuum(d)
    assert orc.term_count() == st.n_terms == sum(want)
    assert orc.n_docs() == n
    per_dec = [0] * len(want)
    lens = [0] * n
    total = 0
    for i in range(st.n_terms):
        term = f"w{i:08d}"
        docs, tfs = orc.postings(term)
        assert len(docs) == orc.df(term) > 0
        assert docs == sorted(set(docs)) and all(0 <= x < n for x in docs)
        assert all(t >= 1 for t in tfs)
        per_dec[int(math.log10(len(docs)))] += 1
        for x, t in zip(docs, tfs):
            lens[x] += t
        total += len(docs)
    assert per_dec == want
    assert total == st.n_postings
    # my.doc_length holds Char4(sum of tfs) (DocLengthCharStore, doc_length_store.h:104-112)
    raw = open(os.path.join(d, "my.doc_length"), "rb").read()
    (cnt,) = struct.unpack("<i", raw[:4])
    assert cnt == n
    from oracle.oracle import lib
    for i in range(0, n, 97):
        assert raw[12 + 5 * i + 4] == lib.orc_char4_encode(lens[i])
    orc.close()


def test_deterministic(tiny, tmp_path):
    import wiser_amd as w
    d, _ = tiny
    d2 = str(tmp_path / "again")
    w.build_wiki_standin(d2, n_docs=20_000, term_scale=0.002, threads=2)
    for f in ("my.vacuum", "my.tip", "my.doc_length"):
        assert open(os.path.join(d, f), "rb").read() == open(os.path.join(d2, f), "rb").read(), f


def test_phrase_pool_and_positions(tiny):
    """The stand-in's phrase pool (gen_synthetic_log.py:216-252 shape: pairs,
    no term in two) and position bags: every bag is tf distinct sorted
    positions below the doc's length; a pair's second word follows its first
    in a share of the docs that hold both, so phrase queries find docs."""
    from oracle.oracle import OracleVacuum
    d, st = tiny
    pairs = [l.split() for l in open(os.path.join(d, "phrases.txt")).read().splitlines()]
    assert len(pairs) > 10
    flat = [t for p in pairs for t in p]
    assert len(flat) == len(set(flat)) and all(len(p) == 2 and p[0] != p[1] for p in pairs)
    orc = OracleVacuum(d)
    n = orc.n_docs()
    lens = [0] * n
    for i in range(st.n_terms):
        docs, tfs = orc.postings(f"w{i:08d}")
        for x, t in zip(docs, tfs):
            lens[x] += t
    both = adjacent = 0
    for a, b in pairs[:40]:
        da, _ = orc.postings(a)
        db, tb = orc.postings(b)
        assert orc.df(b) == len(db)
        pos_a = {}
        for j, x in enumerate(da):
            p = orc.positions(a, j)
            assert p == sorted(set(p)) and all(0 <= v < lens[x] for v in p)
            pos_a[x] = p
        for j, x in enumerate(db):
            p = orc.positions(b, j)
            assert len(p) == tb[j] and p == sorted(set(p)) and all(0 <= v < lens[x] for v in p)
            if x in pos_a:
                both += 1
                adjacent += any(v + 1 in p for v in pos_a[x])
        got, _ = orc.search([a, b], 10, phrase=True)
        assert all(x in pos_a for x, _ in got)
    # b's docs share half of the smaller list with a; 60 % of those are phrases
    assert both > 100 and 0.45 < adjacent / both < 0.8, (both, adjacent)
    orc.close()


def test_topic_clustered_variant(tiny, tmp_path):
    """The topic-clustered stand-in (WikiSpec::topics): the df of every term,
    and so the histogram, equals the uniform stand-in's; a term's doc ids
    gather in its home topics' ranges; two terms with a common home topic
    intersect far more often than two without; deterministic."""
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d0, st0 = tiny
    n, topics = 20_000, 16
    d = str(tmp_path / "topics")
    st = w.build_wiki_standin(d, n_docs=n, term_scale=0.002, threads=4, topics=topics, topics_per_term=1,
                              affinity=0.8)
    assert (st.n_terms, st.n_postings) == (st0.n_terms, st0.n_postings)
    o0, o = OracleVacuum(d0), OracleVacuum(d)
    width = n // topics
    home = {}
    # (a phrase pair's second word takes half its docs from the first word's)
    seconds = {l.split()[1] for l in open(os.path.join(d, "phrases.txt")).read().splitlines()}
    for i in range(st.n_terms):
        t = f"w{i:08d}"
        assert o.df(t) == o0.df(t), t
        docs, _ = o.postings(t)
        # (clustered while its home topic stays at most half full: df * 0.8 <= width / 2)
        if 50 <= len(docs) and len(docs) * 0.8 <= width / 2 and t not in seconds:
            top = max(range(topics), key=lambda k: sum(1 for x in docs if k * width <= x < (k + 1) * width))
            share = sum(1 for x in docs if top * width <= x < (top + 1) * width) / len(docs)
            assert share > 0.6, (t, share)   # 0.8 affinity + the uniform rest
            home[t] = (top, set(docs))
    same, diff = [], []
    terms = list(home)
    for i in range(len(terms)):
        for j in range(i + 1, min(len(terms), i + 40)):
            (ka, a), (kb, b) = home[terms[i]], home[terms[j]]
            r = len(a & b) / (len(a) * len(b) / n)   # intersection over the independent expectation
            (same if ka == kb else diff).append(r)
    assert same and diff and sum(same) / len(same) > 4 * sum(diff) / len(diff)
    d2 = str(tmp_path / "again")
    w.build_wiki_standin(d2, n_docs=n, term_scale=0.002, threads=2, topics=topics, topics_per_term=1,
                         affinity=0.8)
    for f in ("my.vacuum", "my.doc_length"):
        assert open(os.path.join(d, f), "rb").read() == open(os.path.join(d2, f), "rb").read(), f
    o0.close()
    o.close()
