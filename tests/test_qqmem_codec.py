"""The qq_mem engine's varint posting codec (A11; config 1's engine), restated
in the oracle and pinned by the reference's KATs:
  tests_4.cc:114-146  StandardPosting::Encode bytes (content size, doc delta, tf,
                      offset size, offset deltas);
  tests_4.cc:240-330  PostingListDelta skip index with span 3 (prev doc ids
                      {0,2,5,8}, offsets {0,12,24,36}), HasSkip / NextSpanDocId,
                      SkipForward one by one and two by two;
and round-tripped against the fixture postings: every list, its offsets and
positions read back through PostingListDeltaIterator equal the Vacuum index
built from the same linedoc (tests_15.cc:158-210 runs the same differential on
search results, now over these varint postings)."""
import os
import random

from conftest import DATA, all_tokens


def test_encode_kats():
    from oracle.oracle import posting_encode
    b = posting_encode(3, 4)
    assert list(b) == [3, 3, 4, 0]
    b = posting_encode(3, 4, [(i, i) for i in range(1, 11)])
    assert b[0] == 23 and b[1] == 3 and b[2] == 4 and b[3] == 20
    assert all(b[4 + 2 * i] == 1 and b[4 + 2 * i + 1] == 0 for i in range(10))
    assert len(b) == 24
    # positions: deltas from an imaginary 0 (posting.h:101-113)
    b = posting_encode(7, 3, [(0, 4), (10, 12), (300, 301)], [0, 5, 200])
    assert b[0] == len(b) - 1


def test_skip_list_kats():
    from oracle.oracle import pld_probe
    docs = list(range(10))
    tfs = [i + 1 for i in range(10)]
    prev, offs, has, span_doc, found = pld_probe(docs, tfs, 3, list(range(10)))
    assert prev == [0, 2, 5, 8]
    assert offs == [0, 12, 24, 36]
    assert [i for i in range(10) if has[i]] == [0, 3, 6]
    assert [span_doc[i] for i in range(10) if has[i]] == [2, 5, 8]
    assert found == list(range(10))
    assert pld_probe(docs, tfs, 3, list(range(0, 10, 2)))[4] == list(range(0, 10, 2))
    assert pld_probe(docs, tfs, 3, [9, 10])[4] == [9, -1]


def test_skip_forward_matches_lower_bound():
    from oracle.oracle import pld_probe
    rng = random.Random(3)
    docs = sorted(rng.sample(range(100000), 5000))
    tfs = [rng.randint(1, 9) for _ in docs]
    targets = sorted(rng.sample(range(100100), 700))
    found = pld_probe(docs, tfs, 100, targets)[4]
    import bisect
    for t, f in zip(targets, found):
        i = bisect.bisect_left(docs, t)
        assert f == (docs[i] if i < len(docs) else -1)


def test_varint_lists_equal_vacuum_lists(indexes):
    from oracle.oracle import OracleQqMem, OracleVacuum
    d, _, linedoc, fmt = indexes["wiki5"]
    q = OracleQqMem(linedoc, fmt)
    v = OracleVacuum(d)
    toks = all_tokens()
    for t in toks:
        assert q.postings(t) == v.postings(t), t
    rng = random.Random(4)
    for t in rng.sample(toks, 200):
        docs, _ = v.postings(t)
        i = rng.randrange(len(docs))
        doc, offs, pos = q.posting(t, i)
        assert doc == docs[i]
        assert pos == v.positions(t, i), t
        assert offs == v.offsets(t, i), t
    q.close()
    v.close()


def test_token_only_lists(indexes):
    from oracle.oracle import OracleQqMem, OracleVacuum
    d, _, linedoc, fmt = indexes["tok10k"]
    q = OracleQqMem(linedoc, fmt)
    v = OracleVacuum(d)
    rng = random.Random(5)
    toks = set()
    with open(linedoc) as f:
        next(f)
        for line in f:
            toks.update(line.rstrip("\n").split("\t")[2].split())
    for t in rng.sample(sorted(toks), 500):
        assert q.postings(t) == v.postings(t), t
    q.close()
    v.close()
