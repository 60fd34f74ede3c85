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
