#!/usr/bin/env python3
"""Write a TOKEN_ONLY linedoc of Zipf text (diagnostics: exercises bench.py's
--linedoc path, configs[2] style, when no Wikipedia dump is at hand)."""
import random
import sys

out, n_docs = sys.argv[1], int(sys.argv[2])
rng = random.Random(1)
vocab = [f"w{i}" for i in range(20000)]
weights = [1.0 / (i + 1) ** 1.07 for i in range(len(vocab))]
with open(out, "w") as f:
    f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
    for d in range(n_docs):
        body = " ".join(rng.choices(vocab, weights, k=rng.randint(20, 300)))
        f.write(f"d{d}\t{body}\t{body}\n")
