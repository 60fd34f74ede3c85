"""Host-side check of the dense-list image (rank bitmap + 1-byte tf array).

The segment kernel probes long "other" lists through these bitmaps; this test
restates the probe on the host (wsr_debug_dense_lookup, no GPU) and checks,
for every doc id of the index and several doc-range shards, that the bitmap
holds exactly the list's postings in the range and returns the oracle's tf,
including tf >= 255 (escape to the tf blob) in pack blocks and VInts tails.
"""
import ctypes as C
import os
import random

import pytest

from conftest import DATA


def _lookup(d, term, lo, hi, div, n_docs):
    from wiser_amd._capi import check, lib
    docs = (C.c_uint32 * n_docs)(*range(n_docs))
    out = (C.c_int32 * n_docs)()
    dense = C.c_int32(0)
    check(lib.wsr_debug_dense_lookup(d.encode(), lo, hi, div, term.encode(), docs, n_docs, out,
                                     C.byref(dense)))
    return bool(dense.value), list(out)


def _expect(orc, term, lo, hi, n_docs):
    docs, tfs = orc.postings(term)
    exp = [-1] * n_docs
    for dd, tt in zip(docs, tfs):
        if lo <= dd < hi:
            exp[dd] = tt
    return exp


@pytest.fixture(scope="module")
def big_tf_index(built, tmp_path_factory):
    import wiser_amd as w
    root = tmp_path_factory.mktemp("bigtf")
    ld = root / "big_tf.linedoc"
    rng = random.Random(5)
    with open(ld, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(300):
            toks = ["x"] * rng.choice([1, 2, 254, 255, 256, 600])
            if i % 2 == 0:
                toks += ["y"] * rng.randint(1, 3)
            toks += [f"w{i}"]
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    d = root / "idx"
    d.mkdir()
    w.build_from_linedoc(str(ld), str(d), "TOKEN_ONLY")
    return str(d)


def _shards(n):
    return [(0, 0), (0, n // 2), (n // 2, 0), (n // 3, 2 * n // 3), (n - 1, n)]


def test_dense_bitmap_big_tf(big_tf_index):
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(big_tf_index)
    n = orc.n_docs()
    for term in ("x", "y", "w7"):
        for lo, hi in _shards(n):
            dense, got = _lookup(big_tf_index, term, lo, hi, 1 << 30, n)
            exp = _expect(orc, term, lo, hi if hi else n, n)
            assert dense or set(exp) == {-1}, (term, lo, hi)  # no postings in the shard
            assert got == exp, (term, lo, hi)
    orc.close()


def test_dense_bitmap_tok10k(indexes):
    from oracle.oracle import OracleVacuum
    d = indexes["tok10k"][0]
    orc = OracleVacuum(d)
    n = orc.n_docs()
    for term in ("the", "of", "a", "zero", "anarchism"):
        if orc.df(term) == 0:
            continue
        for lo, hi in _shards(n)[:4]:
            dense, got = _lookup(d, term, lo, hi, 1 << 30, n)
            exp = _expect(orc, term, lo, hi if hi else n, n)
            assert dense or set(exp) == {-1}, (term, lo, hi)
            assert got == exp, (term, lo, hi)
    # threshold: a rare term gets no bitmap at the default divisor
    rare = [t for t in ("anarchism", "zero", "wikipedia") if 0 < orc.df(t) < n // 128]
    for t in rare:
        dense, got = _lookup(d, t, 0, 0, 128, n)
        assert not dense and set(got) == {-1}
    orc.close()


def test_image_size_host_only(synth_small):
    """wsr_image_size (no device): the per-buffer sizes add up; doc-range shard
    images hold about 1/W of the blocks and of the bitmaps each, so the W
    shards together stay within a few percent of the whole image plus the
    per-shard directory heads; with positions the position boxes are added."""
    import wiser_amd as w
    d, st = synth_small
    full = w.image_size(d, threads=4)
    parts = ("blob_bytes", "dense_bytes", "tf8_bytes", "plen_bytes", "dir_bytes", "pos_bytes")
    assert full["total_bytes"] == sum(full[p] for p in parts)
    assert full["dense_lists"] > 0 and full["pos_bytes"] == 0
    from wiser_amd.shard import shard_range
    for world in (2, 4, 8):
        sh = [w.image_size(d, doc_range=shard_range(st.n_docs, r, world), threads=4) for r in range(world)]
        assert all(s["n_lists"] == full["n_lists"] for s in sh)
        # bitmaps and buckets cover the shard's doc range only: W of them ~ one
        # whole one; the buckets' offset bytes, like tf8, are one per posting
        # of the shard's blocks, whose edge blocks also hold postings outside
        # the range (a one-block list is in every shard it reaches)
        edge = sum(s["tf8_bytes"] for s in sh) - full["tf8_bytes"]
        assert sum(s["dense_bytes"] for s in sh) <= (1.15 * full["dense_bytes"] + edge +
                                                     world * 64 * full["dense_lists"])
        # every shard keeps the blocks that can hold its docs: ~1/W of a list's
        # blocks, plus at most one block per list at each shard edge
        assert sum(s["plen_bytes"] for s in sh) <= full["plen_bytes"] + world * 128 * full["n_lists"]
        assert max(s["total_bytes"] for s in sh) < full["total_bytes"]


@pytest.fixture(scope="module")
def bucket_index(built, tmp_path_factory):
    from bucket_corpus import build_bucket_index
    return build_bucket_index(tmp_path_factory.mktemp("buckets"))


def test_dense_buckets(bucket_index):
    """Offset buckets (sparse dense lists) answer every doc id exactly as the
    oracle, whole image and doc-range shards, crowded buckets included."""
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(bucket_index)
    n = orc.n_docs()
    for term in ("g", "s", "z", "y", "u77"):
        for lo, hi in _shards(n) + [(6400, 6464), (6410, 20000), (12801, 30000)]:
            dense, got = _lookup(bucket_index, term, lo, hi, 1 << 30, n)
            exp = _expect(orc, term, lo, hi if hi else n, n)
            assert dense or set(exp) == {-1}, (term, lo, hi)
            assert got == exp, (term, lo, hi)
    orc.close()
