#!/usr/bin/env python3
"""Write a linedoc of Zipf text (diagnostics and writer scale runs: exercises
bench.py's --linedoc path, configs[2] style, when no Wikipedia dump is at hand).

usage: make_linedoc.py OUT N_DOCS [TOKEN_ONLY|WITH_POSITIONS] [SEED]

WITH_POSITIONS rows are title | body | distinct tokens | offsets | positions,
the reference's linedoc columns (engine_loader.h:53-96): per token its
"s,e;" char spans (end inclusive) and "p;" word positions, '.'-terminated."""
import random
import sys

import numpy as np


def main():
    out, n_docs = sys.argv[1], int(sys.argv[2])
    fmt = sys.argv[3] if len(sys.argv) > 3 else "TOKEN_ONLY"
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    V = 20000 if fmt == "TOKEN_ONLY" else 200000
    vocab = [f"w{i}" for i in range(V)]
    if fmt == "TOKEN_ONLY":
        rng = random.Random(seed)
        weights = [1.0 / (i + 1) ** 1.07 for i in range(V)]
        with open(out, "w") as f:
            f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
            for d in range(n_docs):
                body = " ".join(rng.choices(vocab, weights, k=rng.randint(20, 300)))
                f.write(f"d{d}\t{body}\t{body}\n")
        return
    if fmt != "WITH_POSITIONS":
        raise SystemExit("format must be TOKEN_ONLY or WITH_POSITIONS")
    g = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, V + 1) ** 1.07
    cdf = np.cumsum(p / p.sum())
    wlen = np.array([len(w) for w in vocab])
    with open(out, "w", buffering=1 << 22) as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\toffsets\tpositions\n")
        for d in range(n_docs):
            n = int(g.integers(20, 300))
            seq = np.searchsorted(cdf, g.random(n))
            seq = np.minimum(seq, V - 1)
            starts = np.concatenate(([0], np.cumsum(wlen[seq] + 1)[:-1]))
            occ = {}
            for pos, (t, s) in enumerate(zip(seq.tolist(), starts.tolist())):
                occ.setdefault(t, []).append((pos, s))
            toks = list(occ)
            off_col = "".join("".join(f"{s},{s + wlen[t] - 1};" for _, s in occ[t]) + "." for t in toks)
            pos_col = "".join("".join(f"{q};" for q, _ in occ[t]) + "." for t in toks)
            body = " ".join(vocab[t] for t in seq.tolist())
            f.write(f"d{d}\t{body}\t{' '.join(vocab[t] for t in toks)}\t{off_col}\t{pos_col}\n")


if __name__ == "__main__":
    main()
