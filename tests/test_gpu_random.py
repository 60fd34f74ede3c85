"""Randomised GPU parity: small corpora with skewed shapes (lists of exactly
127 / 128 / 129 postings, one-posting lists, tf >= 255, empty-ish docs,
repeated terms) and random queries (1-6 terms, conjunctive or phrase,
k = 1..64) in every dense-probe mode, all against the oracle bit for bit."""
import os
import random

import pytest

from test_gpu_parity import DENSE_MODES, _engine

pytestmark = pytest.mark.gpu


def _corpus(path, seed):
    """WITH_POSITIONS linedoc; returns the vocabulary."""
    rng = random.Random(seed)
    vocab = [f"v{i}" for i in range(rng.choice([5, 30, 300]))]
    fixed = {f"x{n}": n for n in (1, 2, 127, 128, 129, 255, 256, 300)}   # term -> df
    n_docs = rng.choice([300, 700, 1500])
    docs = [[] for _ in range(n_docs)]
    for t, df in fixed.items():
        for d in rng.sample(range(n_docs), min(df, n_docs)):
            docs[d].append(t)
    weights = [1.0 / (i + 1) for i in range(len(vocab))]
    for d in range(n_docs):
        docs[d] += rng.choices(vocab, weights, k=rng.choice([0, 1, 3, 20, 80]))
        if d % 97 == 0:
            docs[d] += ["heavy"] * 300          # tf >= 255
        rng.shuffle(docs[d])
        if not docs[d]:
            docs[d] = ["lonely"]
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\toffsets\tpositions\n")
        for seq in docs:
            occ, offs, at = {}, {}, 0
            for p, w in enumerate(seq):
                occ.setdefault(w, []).append(p)
                offs.setdefault(w, []).append((at, at + len(w)))
                at += len(w) + 1
            toks = list(occ)
            off_col = "".join("".join(f"{s},{e};" for s, e in offs[w]) + "." for w in toks)
            pos_col = "".join("".join(f"{p};" for p in occ[w]) + "." for w in toks)
            f.write(f"t\t{' '.join(seq)}\t{' '.join(toks)}\t{off_col}\t{pos_col}\n")
    return vocab + list(fixed) + ["heavy", "lonely", "absent-term"]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6, 7, 8])
def test_random_corpora(tmp_path, seed):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    ld = os.path.join(tmp_path, "c.linedoc")
    terms = _corpus(ld, seed)
    d = os.path.join(tmp_path, "idx")
    os.makedirs(d)
    w.build_from_linedoc(ld, d, "WITH_POSITIONS")
    orc = OracleVacuum(d)
    rng = random.Random(100 + seed)
    items = []
    for _ in range(1000):
        n = rng.choice([1, 1, 2, 2, 2, 3, 4, 6])
        q = [rng.choice(terms) for _ in range(n)]
        items.append((q, rng.random() < 0.4, rng.choice([1, 2, 5, 10, 10, 33, 64])))
    for mode in sorted(DENSE_MODES):
        eng = _engine(d, mode)
        res = eng.SearchBatch([w.SearchQuery(q, n_results=k, is_phrase=ph) for q, ph, k in items])
        for (q, ph, k), r in zip(items, res):
            want, dfs = orc.search(q, k, phrase=ph)
            got = [(e.doc_id, e.doc_score) for e in r.entries]
            assert got == want, (mode, q, ph, k, got[:3], want[:3])
            if want:
                assert r.doc_freqs == dfs
        eng.close()
    orc.close()
