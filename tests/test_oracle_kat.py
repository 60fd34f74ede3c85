"""The oracle against the reference's own known-answer tests (CPU only).

Every expectation below is copied from a reference test (path:line under
/root/reference/src/qq_mem/src); these pin the CPU restatement that every GPU
parity test compares against.
"""
import os
import random

import pytest

from conftest import DATA, all_tokens
from oracle import oracle as O

lib = O.lib


def fmt3(x):
    """utils::format_double(x, 3) == std::setprecision(3)"""
    return f"{x:.3g}"


def test_num_bits_kat():
    # tests_8.cc:13-22
    for v, n in [(0, 0), (1, 1), (8, 4), (12, 4), (0xff, 8), (0x7f, 7), (0x7fffffff, 31),
                 (0xffffffff, 32)]:
        assert lib.orc_num_bits(v) == n


def test_char4_kat():
    # tests_8.cc:24-48
    for v, c in [(0, 0), (1, 1), (7, 7), (8, 0x08), (0x80, 0x28)]:
        assert lib.orc_char4_encode(v) == c
    assert lib.orc_char4_encode(0xffffffff) == ((29 << 3) | 0x07) & 0xff
    for c, v in [(0, 0), (1, 1), (7, 7), (8, 8), (0x28, 0x80)]:
        assert lib.orc_char4_decode(c) == v
    assert lib.orc_char4_decode(((29 << 3) | 0x07) & 0xff) == 0xf0000000
    for c in (240, 248, 252):  # shift >= 29 loses the leading bit
        assert lib.orc_char4_decode(c) == 0
    # tests_8.cc:50-61: the 4 leading bits survive the round trip
    for i in range(0, 0x0fffffff, 777777):
        d = lib.orc_char4_decode(lib.orc_char4_encode(i))
        assert lib.orc_num_bits(d) == lib.orc_num_bits(i)
        sh = lib.orc_num_bits(d) - 4
        if sh > 0:
            assert d >> sh == i >> sh
        else:
            assert d == i


def test_bm25_kat():
    # tests_8.cc:65-122 (values from Elasticsearch runs)
    assert fmt3(lib.orc_es_idf(1, 1)) == "0.288"
    assert fmt3(lib.orc_es_idf(3, 1)) == "0.981"
    assert lib.orc_es_tfnorm(1, 3, 3.0) == 1.0
    assert lib.orc_es_tfnorm(1, 7, 7.0) == 1.0
    assert fmt3(lib.orc_es_tfnorm(1, 2, 8 / 3.0)) == "1.11"
    # lossy: lengths 3, 7 and 2 are exact in Char4
    assert lib.orc_tfnorm_lossy(3.0, 1, lib.orc_char4_encode(3)) == 1.0
    assert lib.orc_tfnorm_lossy(7.0, 1, lib.orc_char4_encode(7)) == 1.0
    assert fmt3(lib.orc_tfnorm_lossy(8 / 3.0, 1, lib.orc_char4_encode(2))) == "1.11"


def test_score_terms_in_doc_kat():
    """tests_2.cc:162-245: CalcDocScoreForOneQuery over the 3-doc engine
    (avg length 8/3): wisconsin on a 2-token doc 1.09, hello 0.149,
    hello + world 0.672 (idf summed in query order)."""
    avg = (2 + 2 + 4) / 3.0
    s1 = 0.0 + lib.orc_es_idf(3, 1) * lib.orc_es_tfnorm(1, 2, avg)
    assert fmt3(s1) == "1.09"
    s2 = 0.0 + lib.orc_es_idf(3, 3) * lib.orc_es_tfnorm(1, 2, avg)
    assert fmt3(s2) == "0.149"
    s3 = (0.0 + lib.orc_es_idf(3, 3) * lib.orc_es_tfnorm(1, 2, avg)) + \
        lib.orc_es_idf(3, 2) * lib.orc_es_tfnorm(1, 2, avg)
    assert fmt3(s3) == "0.672"


def test_varint_kat():
    # tests_15.cc:311-324 (64-bit varint round trip)
    b = O.varint_encode(3748449232)
    assert O.varint_decode(b) == (3748449232, len(b))
    # tests_4.cc-style small values
    for v in [0, 1, 127, 128, 255, 300, 2 ** 32 - 1, 2 ** 63]:
        b = O.varint_encode(v)
        assert O.varint_decode(b) == (v, len(b))
    assert O.varint_encode(0) == b"\x00" and O.varint_encode(300) == b"\xac\x02"


def test_pack_kat():
    # tests_16.cc:83-174
    vals = list(range(128))
    data = O.pack128(vals)
    assert len(data) == 112 + 2 and data[0] == 0xD6 and data[1] == 7
    assert O.unpack128(data) == (vals, 7)
    assert O.unpack128(O.pack128([0] * 128)) == ([0] * 128, 1)   # width 0 forced to 1
    assert O.unpack128(O.pack128([1] * 128)) == ([1] * 128, 1)
    rng = random.Random(0)
    r = [rng.randrange(10000000) for _ in range(128)]
    assert O.unpack128(O.pack128(r))[0] == r
    # layout: value j at bits [j*b, j*b+b) of an LSB-first stream
    d = O.pack128([1] + [0] * 127)
    assert d[2] == 1 and not any(d[3:])
    d = O.pack128([0, 1] + [0] * 126)
    assert d[2] == 1 << 1  # b = 1: value 1 at bit 1


def test_three_doc_engine_kat(indexes):
    # tests.cc:408-511: Elasticsearch-produced scores
    d, st, linedoc, fmt = indexes["three"]
    for eng in (O.OracleVacuum(d), O.OracleQqMem(linedoc, fmt)):
        r, _ = eng.search(["wisconsin"], 5)
        assert [x[0] for x in r] == [1] and fmt3(r[0][1]) == "1.09"
        r, _ = eng.search(["hello"], 5)
        assert [fmt3(x[1]) for x in r] == ["0.149", "0.149", "0.111"]
        r, _ = eng.search(["hello", "world"], 5)
        assert [fmt3(x[1]) for x in r] == ["0.677", "0.672"]
        assert eng.search(["hello", "world"], 0)[0] == []
    assert st.n_docs == 3 and st.n_terms == 4


def test_processor_order_kat(indexes):
    # tests_5.cc:16-52 (shorter docs first; k caps the result)
    d, _, linedoc, fmt = indexes["order"]
    o = O.OracleVacuum(d)
    assert [x[0] for x in o.search(["hello", "world"], 5)[0]] == [4, 3, 2, 1, 0]
    assert [x[0] for x in o.search(["hello", "world"], 2)[0]] == [4, 3]


def test_vacuum_three_docs_kat(indexes):
    # tests_15.cc:11-116 and tests_14.cc:62-120
    d, _, _, _ = indexes["iter3"]
    o = O.OracleVacuum(d)
    assert o.term_count() == 3
    assert (o.df("a"), o.df("b"), o.df("c"), o.df("d")) == (3, 2, 1, 0)
    assert o.postings("a") == ([0, 1, 2], [1, 1, 1])
    assert o.postings("b") == ([1, 2], [1, 1])
    assert sorted(x[0] for x in o.search(["a", "b"], 5)[0]) == [1, 2]
    assert o.search(["d"], 5)[0] == []


def test_differential_vacuum_vs_qqmem(indexes):
    # tests_15.cc:158-210: Vacuum engine == QqMem engine for every token
    d, _, linedoc, fmt = indexes["wiki5"]
    v = O.OracleVacuum(d)
    q = O.OracleQqMem(linedoc, fmt)
    assert v.term_count() == q.term_count()
    for t in all_tokens():
        rv, fv = v.search([t], 5)
        rq, fq = q.search([t], 5)
        assert rv and rv == rq and fv == fq, t
    rng = random.Random(5)
    toks = all_tokens()
    for _ in range(500):
        qs = rng.sample(toks, rng.randint(2, 4))
        assert v.search(qs, 10) == q.search(qs, 10), qs


def test_differential_tokenized_10k(indexes):
    d, _, linedoc, fmt = indexes["tok10k"]
    v = O.OracleVacuum(d)
    q = O.OracleQqMem(linedoc, fmt)
    assert v.term_count() == q.term_count() and v.n_docs() == 9999
    rng = random.Random(1)
    vocab = sorted({t for line in open(linedoc).read().splitlines()[1:]
                    for t in line.split("\t")[2].split()})
    for t in rng.sample(vocab, 800):
        assert v.search([t], 10) == q.search([t], 10), t
    for _ in range(300):
        qs = rng.sample(vocab[:500], 2)
        assert v.search(qs, 10) == q.search(qs, 10), qs


def test_ub_negative_index_not_hit(indexes):
    """Lengths >= 2^18 would index the reference's cache with a negative char
    (scoring.h:65-69, undefined behaviour); none of the fixtures hit it."""
    assert lib.orc_ub_negative_char_index() == 0
