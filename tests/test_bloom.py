"""Two-way phrase bloom filters (CPU only): the writer's bloom sections against
the reference layout and semantics, read back by the oracle's restatement of
the reference reader.

Reference (paths under /root/reference/src/qq_mem/src):
  writer ........ FlashEngineDumper::DumpPostingListWithBloom / DumpBloomSection
                  (flash_engine_dumper.h:412-525,584-646), BloomBoxWriter /
                  BloomSkipListWriter (flash_containers.h:499-660), header (:288-316)
  filters ....... BloomFilterStore::Add (bloom_filter.h:277-300), libbloom
                  (libbloom/bloom.c:48-138), MurmurHash2
  reader ........ BloomFilterColumnReader / HasTerm (flash_iterators.h:776-823,994-1058)
  use ........... QueryProcessor::IsPossibleToPresent (query_processing.h:766-884)
KAT: tests_18.cc:283-356 (bi-bloom 3-doc engine: {a,b} and {b,c} found, {a,x}
and {x,c} not).
"""
import os
import random
import struct

import pytest

from conftest import BLOOM_RATIO as RATIO, BLOOM_ENTRIES as ENTRIES, DATA, phrase_cases
from oracle import oracle as O


def _neighbours(linedoc):
    """{(term, doc): (set of prior terms, set of next terms)} from positions"""
    out = {}
    with open(linedoc) as f:
        f.readline()
        for doc, line in enumerate(f):
            cols = line.rstrip("\n").split("\t")
            toks = cols[2].split()
            groups = [g for g in cols[4].split(".") if g]
            at = {}
            for t, g in zip(toks, groups):
                for p in g.split(";"):
                    if p:
                        at[int(p)] = t
            for p, t in at.items():
                pr, nx = out.setdefault((t, doc), (set(), set()))
                if p - 1 in at:
                    pr.add(at[p - 1])
                if p + 1 in at:
                    nx.add(at[p + 1])
    return out


def test_neighbours_match_the_fixture_columns():
    """The writer derives each posting's filter contents from positions; on the
    reference's bi-bloom fixture they equal its bloom / bloom_before columns."""
    path = os.path.join(DATA, "iter_test_3_docs_tf_bi-bloom")
    nb = _neighbours(path)
    with open(path) as f:
        f.readline()
        for doc, line in enumerate(f):
            cols = line.rstrip("\n").split("\t")
            toks = cols[2].split()
            ends = cols[5].split("!")[:-1]      # DocInfo::ParsePhraseElems (types.cc:42-49)
            begins = cols[6].split("!")[:-1]
            for t, e, b in zip(toks, ends, begins):
                assert set(e.split()) == nb[(t, doc)][1]
                assert set(b.split()) == nb[(t, doc)][0]


def test_header_and_sections(bloom_indexes):
    d = bloom_indexes["wiki5"][0]
    raw = open(os.path.join(d, "my.vacuum"), "rb").read(100)
    assert raw[0] == 0x88
    # twice: has_bloom = 1, bit array bytes, expected entries, f32 ratio
    import math
    bpe = -(math.log(struct.unpack("<f", struct.pack("<f", RATIO))[0]) / 0.480453013918201)
    bits = int(ENTRIES * bpe)
    nbytes = bits // 8 + (1 if bits % 8 else 0)
    i = 1
    for _ in range(2):
        assert raw[i] == 1 and raw[i + 1] == nbytes and raw[i + 2] == ENTRIES
        assert struct.unpack_from("<f", raw, i + 3)[0] == struct.unpack("<f", struct.pack("<f", RATIO))[0]
        i += 7
    o = O.OracleVacuum(d)
    assert o.has_bloom()
    assert not O.OracleVacuum(bloom_indexes["wiki5"][1]).has_bloom()


@pytest.mark.parametrize("name", ["wiki5", "pos"])
def test_filters_have_no_false_negatives(bloom_indexes, indexes, name):
    """Every true neighbour is 'may be present'; a posting with no neighbour on
    a side has no filter there (HasTerm answers not present)."""
    d = bloom_indexes[name][0]
    src = indexes["wiki5"][2] if name == "wiki5" else os.path.join(
        os.path.dirname(bloom_indexes["pos"][1]), "pos.linedoc")
    nb = _neighbours(src)
    o = O.OracleVacuum(d)
    per_term = {}
    for (t, doc) in sorted(nb, key=lambda x: (x[0], x[1])):
        per_term.setdefault(t, []).append(doc)
    rng = random.Random(1)
    terms = sorted(per_term)
    n = 0
    for t in rng.sample(terms, min(len(terms), 60)):
        for posting, doc in enumerate(per_term[t][:300]):
            prior, nxt = nb[(t, doc)]
            for side, want in ((0, prior), (1, nxt)):
                for e in want:
                    assert o.bloom_check(t, posting, side, e) == 1, (t, doc, side, e)
                    n += 1
                if not want:
                    assert o.bloom_check(t, posting, side, "x-never-a-term") == 0
    assert n > 200


def test_bloom_kat_tests_18(bloom_indexes):
    d = bloom_indexes["bi3"][0]
    o = O.OracleVacuum(d)
    assert o.search(["a"], 10)[0]
    assert o.search(["z"], 10)[0] == []
    for ph in (["a", "b"], ["b", "c"]):
        assert o.search(ph, 10, phrase=True)[0], ph
    for ph in (["a", "x"], ["x", "c"]):
        assert o.search(ph, 10, phrase=True)[0] == [], ph


@pytest.mark.parametrize("factor", [1, 2, 1000])
def test_bloom_prunes_but_never_changes_results(bloom_indexes, factor):
    """With bloom filters the reference prunes found docs before the position
    check; the filters have no false negatives, so the results are those of the
    index without filters (and of the exact position check)."""
    d, plain = bloom_indexes["pos"]
    ob = O.OracleVacuum(d, bloom_factor=factor)
    op = O.OracleVacuum(plain)
    seqs_src = os.path.join(os.path.dirname(plain), "pos.linedoc")
    seqs = [l.rstrip("\n").split("\t")[1].split() for l in open(seqs_src).readlines()[1:]]
    c0, p0 = O.bloom_stats()
    qs = phrase_cases(seqs, 300, seed=41) + [["w0", "w1"], ["w1", "w0"], ["w2", "w2"],
                                              ["w3", "w7", "w1"]]
    for q in qs:
        got = ob.search(q, 10, phrase=True)
        assert got == op.search(q, 10, phrase=True), q
        # non-phrase queries never consult the filters
        assert ob.search(q, 10) == op.search(q, 10)
    c1, p1 = O.bloom_stats()
    assert c1 > c0 and p1 > p0   # the bloom path did run and prune


def test_non_phrase_layout_unchanged(bloom_indexes):
    """Doc ids, tfs and positions read through the skip rows are those of the
    index written without filters (the bloom sections only shift the position
    and offset boxes)."""
    d, plain = bloom_indexes["wiki5"]
    ob, op = O.OracleVacuum(d), O.OracleVacuum(plain)
    assert ob.term_count() == op.term_count()
    toks = open(os.path.join(DATA, "all-tokens.txt")).readline().split()
    for t in toks[::3]:
        assert ob.postings(t) == op.postings(t)
        for i in range(min(3, ob.df(t))):
            assert ob.positions(t, i) == op.positions(t, i)
