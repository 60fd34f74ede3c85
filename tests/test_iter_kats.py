"""The reference's doc-id iterator KATs, on lists whose doc ids are
the KATs' own value sequences, written as Vacuum indexes by the product writer:

  tests_11.cc:218-424  DocIdIterator over 200 ids 0..199 (one pack + 72 VInts),
                       exactly one pack (0..127) and 10 packs + 20 (0..1299):
                       SkipTo one by one, Advance to the end, SkipForward simple,
                       backwards (a no-op), into the VInts tail at 127 / 128 / 150,
                       and beyond the end;
  tests_12.cc:33-270   the delta-encoded pack (0..127 and PsudoIncreasingRandom,
                       test_helpers.h:34-38) and delta-encoded VInts (88 values)
                       iterators: Advance / SkipTo with strides, SkipForward to
                       the first, the last, past the end and backwards.

The oracle's DocIdIter restatement is driven op by op (orc_vacuum_docid_ops)
and must give the KATs' Value / PostingIndex / IsEnd; test_gpu_kats.py checks
the device decode and intersection of the same lists."""
import os

import pytest

PACK = 128


def psudo_increasing_random(i):
    """test_helpers.h:34-38"""
    return 1 + i * 30 + (i * 6263 + 12345) % 23


def write_lists_linedoc(path, n_docs, lists):
    """TOKEN_ONLY linedoc of n_docs docs; term t occurs once in each doc of
    lists[t]; every doc also holds 'filler' (no doc is empty)."""
    per_doc = [["filler"] for _ in range(n_docs)]
    for t, docs in lists.items():
        for d in docs:
            per_doc[d].append(t)
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for toks in per_doc:
            s = " ".join(toks)
            f.write(f"t\t{s}\t{s}\n")


# index name -> (n_docs, {term: doc ids})
SIMPLE200 = list(range(200))
ONE_PACK = list(range(PACK))
LARGE = list(range(PACK * 10 + 20))
PSEUDO_PACK = [psudo_increasing_random(i) for i in range(PACK)]
VINTS88 = list(range(88))
PSEUDO_VINTS = [psudo_increasing_random(i) for i in range(88)]
PROBE = [0, 10, 126, 127, 128, 129, 150, 198, 199]   # pack / VInts boundaries
SPECS = {
    "simple200": (200, {"a": SIMPLE200, "b": PROBE}),
    "onepack": (PACK, {"a": ONE_PACK, "b": [0, 63, 64, 126, 127]}),
    "large": (len(LARGE), {"a": LARGE, "b": [0, 127, 128, 255, 256, 1279, 1280, 1299]}),
    "pseudo": (PSEUDO_PACK[-1] + 1, {"p": PSEUDO_PACK, "v": PSEUDO_VINTS, "s": VINTS88,
                                     "b": PSEUDO_PACK[::9] + [PSEUDO_PACK[-1]]}),
}


@pytest.fixture(scope="module")
def iter_indexes(built, tmp_path_factory):
    import wiser_amd as w
    root = str(tmp_path_factory.mktemp("iterkats"))
    out = {}
    for name, (n, lists) in SPECS.items():
        ld = os.path.join(root, name + ".linedoc")
        write_lists_linedoc(ld, n, lists)
        d = os.path.join(root, name)
        os.makedirs(d)
        w.build_from_linedoc(ld, d, "TOKEN_ONLY")
        out[name] = d
    return out


def ops_of(o, d, term, ops):
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(d)
    r = orc.docid_ops(term, ops)
    orc.close()
    return r


def test_lists_are_the_kat_values(iter_indexes):
    from oracle.oracle import OracleVacuum
    for name, (_, lists) in SPECS.items():
        o = OracleVacuum(iter_indexes[name])
        for t, docs in lists.items():
            assert o.postings(t)[0] == docs, (name, t)
        o.close()


def test_tests_11_simple_200(iter_indexes):
    d = iter_indexes["simple200"]
    n = 200
    # Skip one by one
    r = ops_of(None, d, "a", [("skip_to", i) for i in range(n)])
    assert [x[1] for x in r] == list(range(n))
    # Advance(): Value == i before each advance, IsEnd after the last
    r = ops_of(None, d, "a", [("skip_to", 0)] + [("advance",)] * n)
    assert [x[1] for x in r[:n]] == list(range(n)) and not any(x[2] for x in r[:n])
    assert r[n][2]
    # SkipForward() simple and backwards
    r = ops_of(None, d, "a", [("skip_forward", 10), ("skip_forward", 8)])
    assert r[0][:2] == (10, 10) and r[1][:2] == (10, 10)
    # SkipForward() into VInts: end of pack, start of VInts, inside VInts
    r = ops_of(None, d, "a", [("skip_forward", 127), ("skip_forward", 128), ("skip_forward", 150)])
    assert [x[:2] for x in r] == [(127, 127), (128, 128), (150, 150)]
    # SkipForward() beyond the end
    r = ops_of(None, d, "a", [("skip_forward", 199), ("skip_forward", 10000)])
    assert r[0][1] == 199 and not r[0][2] and r[1][2]


def test_tests_11_exact_one_pack(iter_indexes):
    d = iter_indexes["onepack"]
    r = ops_of(None, d, "a", [("skip_to", i) for i in range(PACK)])
    assert [x[1] for x in r] == ONE_PACK
    r = ops_of(None, d, "a", [("skip_to", 0)] + [("advance",)] * PACK)
    assert [x[1] for x in r[:PACK]] == ONE_PACK and r[PACK][2]
    r = ops_of(None, d, "a", [("skip_forward", 10), ("skip_forward", 8)])
    assert r[1][:2] == (10, 10)
    r = ops_of(None, d, "a", [("skip_forward", 199)])   # pointing to the end: not found
    assert r[0][2]


def test_tests_11_large(iter_indexes):
    d = iter_indexes["large"]
    n = len(LARGE)
    r = ops_of(None, d, "a", [("skip_to", 0)] + [("advance",)] * n)
    assert [x[:2] for x in r[:n]] == [(i, i) for i in range(n)] and r[n][2]
    assert ops_of(None, d, "a", [("skip_forward", n + 10)])[0][2]
    assert ops_of(None, d, "a", [("skip_forward", n - 1)])[0] == (n - 1, n - 1, False)


def test_tests_12_delta_pack(iter_indexes):
    # the simple sequence is the one-pack list 0..127
    d = iter_indexes["onepack"]
    r = ops_of(None, d, "a", [("skip_to", i) for i in range(0, PACK, 3)] + [("skip_to", PACK)])
    assert [x[:2] for x in r[:-1]] == [(i, i) for i in range(0, PACK, 3)] and r[-1][2]
    r = ops_of(None, d, "a", [("skip_forward", 0), ("skip_forward", 100), ("skip_forward", 1000)])
    assert r[0] == (0, 0, False) and r[1] == (100, 100, False) and r[2][2]
    assert ops_of(None, d, "a", [("skip_forward", PACK - 1)])[0] == (PACK - 1, PACK - 1, False)
    r = ops_of(None, d, "a", [("skip_forward", 50), ("skip_forward", 0)])
    assert r[0][:2] == (50, 50) and r[1][:2] == (50, 50)
    # pseudo-random increasing values in one pack
    d = iter_indexes["pseudo"]
    v = PSEUDO_PACK
    r = ops_of(None, d, "p", [("skip_to", 0)] + [("advance",)] * PACK)
    assert [x[:2] for x in r[:PACK]] == [(i, v[i]) for i in range(PACK)] and r[PACK][2]
    r = ops_of(None, d, "p", [("skip_to", i) for i in range(0, PACK, 3)] + [("skip_to", PACK)])
    assert [x[:2] for x in r[:-1]] == [(i, v[i]) for i in range(0, PACK, 3)] and r[-1][2]
    r = ops_of(None, d, "p", [("skip_forward", v[10]), ("skip_forward", v[15] - 1)])
    assert r[0] == (10, v[10], False) and r[1] == (15, v[15], False)


def test_tests_12_delta_vints(iter_indexes):
    d = iter_indexes["pseudo"]
    cnt = 88
    # simple numbers 0..87 (a VInts-only list)
    r = ops_of(None, d, "s", [("skip_to", 0)] + [("advance",)] * cnt)
    assert [x[:2] for x in r[:cnt]] == [(i, i) for i in range(cnt)] and r[cnt][2]
    r = ops_of(None, d, "s", [("skip_to", i) for i in range(0, cnt, 3)] + [("skip_to", cnt)])
    assert [x[:2] for x in r[:-1]] == [(i, i) for i in range(0, cnt, 3)] and r[-1][2]
    r = ops_of(None, d, "s", [("skip_forward", 19), ("skip_forward", 1), ("skip_forward", 100)])
    assert r[0][:2] == (19, 19) and r[1][:2] == (19, 19) and r[2][2]
    assert ops_of(None, d, "s", [("skip_forward", 0)])[0] == (0, 0, False)
    r = ops_of(None, d, "s", [("skip_forward", cnt - 1), ("skip_forward", 100)])
    assert r[0] == (cnt - 1, cnt - 1, False) and r[1][2]
    # increasing pseudo-random numbers
    v = PSEUDO_VINTS
    r = ops_of(None, d, "v", [("skip_to", 0)] + [("advance",)] * cnt)
    assert [x[:2] for x in r[:cnt]] == [(i, v[i]) for i in range(cnt)] and r[cnt][2]
    r = ops_of(None, d, "v", [("skip_to", i) for i in range(0, cnt, 3)] + [("skip_to", cnt)])
    assert [x[:2] for x in r[:-1]] == [(i, v[i]) for i in range(0, cnt, 3)] and r[-1][2]
