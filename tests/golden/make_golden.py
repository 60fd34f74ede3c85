#!/usr/bin/env python3
"""Regenerate tests/golden/results.json.gz: oracle results (doc ids, order and
exact f64 scores as float.hex) for fixed query sets over indexes written from
the reference's own fixture files.  The oracle is pinned by the reference's
known-answer tests (tests/test_oracle_kat.py); these vectors pin it (and the
GPU path, tests/test_gpu_parity.py) against regressions across rounds.

    python tests/golden/make_golden.py
"""
import gzip
import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
DATA = os.path.join(HERE, "data")


def query_sets(index_dirs):
    from oracle.oracle import OracleVacuum
    rng = random.Random(2026)
    sets = {}
    toks = open(os.path.join(DATA, "all-tokens.txt")).readline().split()
    o = OracleVacuum(index_dirs["wiki5"])
    freq = sorted(toks, key=lambda t: -o.df(t))[:60]
    sets["wiki5"] = ([[t] for t in rng.sample(toks, 1000)] +
                     [rng.sample(toks, 2) for _ in range(200)] +
                     [rng.sample(freq, 2) for _ in range(200)] +
                     [rng.sample(freq, 3) for _ in range(100)])
    vocab = sorted({t for line in open(os.path.join(DATA, "test_doc_tokenized")).read().splitlines()[1:]
                    for t in line.split("\t")[2].split()})
    sets["tok10k"] = ([[t] for t in rng.sample(vocab, 500)] +
                      [rng.sample(vocab[:400], 2) for _ in range(300)])
    terms = [f"t{i:07d}" for i in range(3000)]
    sets["synth20k"] = ([rng.sample(terms[:300], 2) for _ in range(200)] +
                        [[rng.choice(terms[:300]), rng.choice(terms[300:])] for _ in range(200)] +
                        [rng.sample(terms[:100], 3) for _ in range(100)])
    return sets


def build_indexes(root):
    import wiser_amd as w
    out = {}
    for name, src, fmt in [("wiki5", "line_doc_with_positions", "WITH_POSITIONS"),
                           ("tok10k", "test_doc_tokenized", "TOKEN_ONLY")]:
        out[name] = os.path.join(root, name)
        w.build_from_linedoc(os.path.join(DATA, src), out[name], fmt)
    out["synth20k"] = os.path.join(root, "synth20k")
    w.build_synthetic(out["synth20k"], n_docs=20000, vocab=20000, seed=0x5EED2026, threads=4)
    return out


def main():
    from oracle.oracle import OracleVacuum
    with tempfile.TemporaryDirectory() as root:
        dirs = build_indexes(root)
        sets = query_sets(dirs)
        golden = {}
        for name, qs in sets.items():
            o = OracleVacuum(dirs[name])
            rows = []
            for q in qs:
                r, dfs = o.search(q, 10)
                rows.append({"q": q, "k": 10, "df": dfs, "hits": [[d, s.hex()] for d, s in r]})
            golden[name] = rows
    with gzip.open(os.path.join(HERE, "results.json.gz"), "wt") as f:
        json.dump(golden, f, separators=(",", ":"))
    print({k: len(v) for k, v in golden.items()})


if __name__ == "__main__":
    main()
