"""GPU parity of the lean kernel's pre-probe pruning (a driver posting whose
score bound is <= the threshold known so far is dropped before its bitmap
probe; kernels.hip `lean_segment`).

The corpus is built for ties: doc lengths from four values and tfs 1..3, so
thousands of postings share a score, many of them exactly the running k-th
best or the floor handed on from a query's earlier items (the reference heap
inserts only a strictly larger score, query_processing.h:595-602, so a tie at
the threshold is never an event and must never be pruned as one either).
Lists of 20k postings span several work items per query, so item floors are
exercised.  One term carries a tf above the 1-byte escape (a loose bound).
Results must be bit-identical to the oracle in every dense mode.
"""
import os
import random

import pytest

from test_gpu_parity import DENSE_MODES, _check, _engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tie_index(built, tmp_path_factory):
    import wiser_amd as w
    root = str(tmp_path_factory.mktemp("ties"))
    path = os.path.join(root, "ties.linedoc")
    rng = random.Random(5)
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(20000):
            toks = ["a"] * rng.choice([1, 1, 1, 2, 3])
            if rng.random() < 0.8:
                toks += ["b"] * rng.choice([1, 1, 2])
            if rng.random() < 0.5:
                toks += ["c"] * rng.choice([1, 2, 3])
            if rng.random() < 0.3:
                toks += ["d"]
            if i == 7777:
                toks += ["c"] * 300   # above the tf8 escape: c's tf bound is 303
            n = rng.choice([8, 16, 24, 64])
            toks += [f"f{j}" for j in range(max(0, n - len(toks)))]
            rng.shuffle(toks)
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    d = os.path.join(root, "idx")
    os.makedirs(d)
    w.build_from_linedoc(path, d, "TOKEN_ONLY")
    return d


@pytest.mark.parametrize("mode", sorted(DENSE_MODES))
def test_prune_ties(tie_index, mode):
    from oracle.oracle import OracleVacuum
    eng = _engine(tie_index, mode)
    orc = OracleVacuum(tie_index)
    try:
        queries = [["a"], ["b"], ["c"], ["a", "b"], ["b", "a"], ["a", "c"], ["c", "b"], ["d", "a"],
                   ["a", "b", "c"], ["c", "b", "a", "d"], ["a", "a"], ["b", "c", "b"]]
        for k in (1, 3, 10, 64, 100):
            _check(eng, orc, queries, k)
    finally:
        eng.close()
        orc.close()


@pytest.fixture(scope="module")
def tie_index_long(built, tmp_path_factory):
    """Single-term ties across several single-term items: 80k docs, "a" in
    every doc (625 blocks: two items of single_segment's 8 windows at the
    default item length), "b" in most, four doc lengths, tfs 1..3."""
    import wiser_amd as w
    root = str(tmp_path_factory.mktemp("ties_long"))
    path = os.path.join(root, "ties.linedoc")
    rng = random.Random(11)
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(80000):
            toks = ["a"] * rng.choice([1, 1, 1, 2, 3])
            if rng.random() < 0.8:
                toks += ["b"] * rng.choice([1, 1, 2])
            n = rng.choice([8, 16, 24, 64])
            toks += [f"f{j}" for j in range(max(0, n - len(toks)))]
            rng.shuffle(toks)
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    d = os.path.join(root, "idx")
    os.makedirs(d)
    w.build_from_linedoc(path, d, "TOKEN_ONLY")
    return d


@pytest.mark.parametrize("item_blocks", [63, 8, 1])
def test_single_term_ties_items(tie_index_long, item_blocks):
    """Block skipping and the floor seed of single-term items (kernels.hip
    single_segment) on tie-heavy lists: thousands of postings score exactly
    the k-th best, items of 8 windows (the default) down to 8 blocks (short
    items: many items per query, each seeded from the blocks before it),
    k from 1 to 100 (64 < k: every survivor an event, no skipping)."""
    import wiser_amd as w
    from wiser_amd import _capi
    from oracle.oracle import OracleVacuum
    eng = w.VacuumEngine(tie_index_long)
    eng.Load()
    orc = OracleVacuum(tie_index_long)
    try:
        queries = [["a"], ["b"], ["a", "b"]]
        for k in (1, 3, 10, 64, 100):
            b = w.ResidentBatch(eng, len(queries), k)
            try:
                _capi.check(_capi.lib.wsr_batch_set_item_blocks(eng._h, b._b, item_blocks))
                b.upload((_capi.Query * len(queries))(*[eng.resolve(w.SearchQuery(q, n_results=k))[0]
                                                       for q in queries]))
                b.run()
                hits, nh = b.fetch()
                for i, q in enumerate(queries):
                    got = [(hits[i * k + j].doc_id, hits[i * k + j].score) for j in range(nh[i])]
                    assert got == orc.search(q, k)[0], (q, k, item_blocks)
            finally:
                b.close()
    finally:
        eng.close()
        orc.close()
