"""The product's Vacuum writer against the reference layout (CPU only).

Byte layout checks restate flash_engine_dumper.h:288-411, flash_containers.h:
282-299/354-391, packed_value.h:87-128/372-397, file_dumper.h:82-86; the
posting contents are compared with postings computed here in plain Python from
the linedoc (engine_loader.h:53-96, qq_mem_engine.h:217-239).
"""
import os
import random
import struct

import numpy as np
import pytest

from conftest import DATA
from oracle import oracle as O


def read_tip(d):
    out = {}
    b = open(os.path.join(d, "my.tip"), "rb").read()
    i = 0
    while i < len(b):
        (n,) = struct.unpack_from("<I", b, i)
        i += 4
        t = b[i:i + n].decode()
        i += n
        (v,) = struct.unpack_from("<q", b, i)
        i += 8
        out[t] = (v & ((1 << 48) - 1), v >> 48)
    return out


def varint(b, i):
    v, s = 0, 0
    while True:
        c = b[i]
        v |= (c & 0x7F) << s
        s += 7
        i += 1
        if not c & 0x80:
            return v, i


def parse_list(vac, off):
    assert vac[off] == 0xF4
    df, i = varint(vac, off + 1)
    reserved = vac[i:i + 8]
    i += 8
    assert vac[i] == 0xA3
    n, i = varint(vac, i + 1)
    rows, prev = [], [0] * 7
    for _ in range(n):
        f = []
        for _ in range(7):
            v, i = varint(vac, i)
            f.append(v)
        row = [f[0] + prev[0], f[1] + prev[1], f[2] + prev[2], f[3] + prev[3], f[4],
               f[5] + prev[5], f[6]]
        rows.append(row)
        prev = row
    return df, reserved, rows, i


def test_header_and_first_list(indexes):
    # tests_14.cc:10-30: a one-term index puts its list at offset 100
    d, _, _, _ = indexes["one_word"]
    vac = open(os.path.join(d, "my.vacuum"), "rb").read()
    assert vac[0] == 0x88
    # has_bloom=0, bytes=0, entries=0, f32 0.0, twice; zero padding to 100
    assert vac[1:1 + 7] == b"\x00\x00\x00" + b"\x00" * 4
    assert vac[8:15] == b"\x00\x00\x00" + b"\x00" * 4
    assert not any(vac[15:100])
    tip = read_tip(d)
    assert list(tip) == ["a"] and tip["a"][0] == 100


def test_vints_blob_kat(indexes):
    # tests_14.cc:49-60: a VInts blob of two 1s is 4 bytes; list "b" of
    # iter_test_3_docs holds doc ids {1, 2} = deltas (1, 1)
    d, _, _, _ = indexes["iter3"]
    vac = open(os.path.join(d, "my.vacuum"), "rb").read()
    off, _ = read_tip(d)["b"]
    df, reserved, rows, end = parse_list(vac, off)
    assert df == 2 and reserved == b"\x00\x00" + b"\x00" * 6 and len(rows) == 1
    doc_off = rows[0][1]
    assert vac[doc_off:doc_off + 4] == b"\x9b\x02\x01\x01"
    tf_off = rows[0][2]
    assert vac[tf_off:tf_off + 4] == b"\x9b\x02\x01\x01"
    # the skip list ends where the data begins (modulo the estimate gap of zeros)
    assert doc_off >= end and not any(vac[end:doc_off])


def expected_postings(linedoc, fmt):
    post = {}
    rows = open(linedoc).read().split("\n")[1:]
    lengths = []
    for doc, line in enumerate(r for r in rows if r != "" or False):
        cols = line.split("\t")
        if fmt == "TOKEN_ONLY":
            toks = [t for t in cols[2].split(" ") if t]
            cnt = {}
            for t in toks:
                cnt[t] = cnt.get(t, 0) + 1
            for t, c in cnt.items():
                post.setdefault(t, []).append((doc, c))
            lengths.append(len(toks))
        else:
            toks = [t for t in cols[2].split(" ") if t]
            groups = [g for g in cols[3].split(".") if g]
            for t, g in zip(toks, groups):
                post.setdefault(t, []).append((doc, g.count(";")))
            lengths.append(len([t for t in cols[1].split(" ") if t]))
    return post, lengths


@pytest.mark.parametrize("name", ["iter3", "wiki5", "tok10k", "three"])
def test_postings_round_trip(indexes, name):
    d, st, linedoc, fmt = indexes[name]
    post, lengths = expected_postings(linedoc, fmt)
    o = O.OracleVacuum(d)
    assert o.term_count() == len(post) == st.n_terms
    vac = open(os.path.join(d, "my.vacuum"), "rb").read()
    tip = read_tip(d)
    terms = sorted(post)
    if len(terms) > 3000:
        terms = random.Random(2).sample(terms, 3000)
    for t in terms:
        docs, tfs = o.postings(t)
        assert list(zip(docs, tfs)) == post[t], t
        df, _, rows, _ = parse_list(vac, tip[t][0])
        assert df == len(post[t]) and len(rows) == (df + 127) // 128
        for r, row in enumerate(rows):   # prev_doc_id = doc of posting 128*r - 1
            assert row[0] == (0 if r == 0 else post[t][128 * r - 1][0])
            assert vac[row[1]] in (0xD6, 0x9B) and vac[row[2]] in (0xD6, 0x9B)
            assert (vac[row[1]] == 0x9B) == (r == len(rows) - 1 and df % 128 != 0)
        # prefetch zone pages = (tf end - list start) / 4096
        last = rows[-1][2]
        if vac[last] == 0xD6:
            tf_end = last + 2 + 16 * vac[last + 1]
        else:
            nb, j = varint(vac, last + 1)
            tf_end = j + nb
        assert tip[t][1] == (tf_end - tip[t][0]) // 4096


@pytest.mark.parametrize("name", ["wiki5", "tok10k"])
def test_doc_lengths(indexes, name):
    d, st, linedoc, fmt = indexes[name]
    _, lengths = expected_postings(linedoc, fmt)
    raw = open(os.path.join(d, "my.doc_length"), "rb").read()
    n, avg = struct.unpack_from("<id", raw, 0)
    assert n == len(lengths)
    rec = np.frombuffer(raw[12:], dtype=np.dtype([("id", "<i4"), ("c", "u1")]))
    assert (rec["id"] == np.arange(n)).all()
    assert [int(c) for c in rec["c"]] == [O.lib.orc_char4_encode(x) for x in lengths]
    # doc_length_store.h:108 incremental mean, bit for bit
    a = 0.0
    for i, x in enumerate(lengths):
        a = a + (x - a) / (i + 1)
    assert avg == a


def test_synthetic_index(synth_small):
    d, st = synth_small
    o = O.OracleVacuum(d)
    assert o.n_docs() == 20000 and st.n_docs == 20000
    assert st.docs_char4_ge_0x80 == 0
    # Zipf: the head terms are long, every list decodes to increasing doc ids
    dfs = [o.df(f"t{i:07d}") for i in range(50)]
    assert dfs[0] > dfs[10] > dfs[49] > 0
    for i in (0, 3, 77, 1000):
        docs, tfs = o.postings(f"t{i:07d}")
        assert docs == sorted(set(docs)) and min(tfs) >= 1


def test_two_term_log_rule(synth_small, tmp_path):
    import wiser_amd as w
    d, _ = synth_small
    p = str(tmp_path / "q.log")
    assert w.gen_two_term_log(d, p, n_queries=500, seed=7) == 500
    o = O.OracleVacuum(d)
    lines = open(p).read().splitlines()
    assert len(set(lines)) == 500
    for line in lines[:200]:
        a, b = line.split(" ")
        assert a < b                      # sorted pair, t1 != t2
        for t in (a, b):
            df = o.df(t)
            assert 1 <= df < 10 ** 7       # low = [1, 1e4), high = [1e4, 1e7)
    # deterministic
    p2 = str(tmp_path / "q2.log")
    w.gen_two_term_log(d, p2, n_queries=500, seed=7)
    assert open(p2).read() == open(p).read()
