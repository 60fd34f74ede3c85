"""SHA-256 of every file the linedoc writer produces for the writer cases
(tests/test_writer_stream.py), written to tests/golden/writer_sha256.json.

The hashes were taken from the whole-corpus in-memory writer (round 2) before
it was replaced by the streaming one: the test holds the streaming writer to
byte-identical output at every chunk size and thread count."""
import hashlib
import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
DATA = os.path.join(HERE, "data")
BLOOM = (0.0009, 5)


def positions_linedoc(path, n_docs, vocab, seed):
    """WITH_POSITIONS linedoc of Zipf word sequences (conftest's phrase fixture shape)."""
    rng = random.Random(seed)
    words = [f"w{i}" for i in range(vocab)]
    weights = [1.0 / (i + 1) for i in range(vocab)]
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\toffsets\tpositions\n")
        for _ in range(n_docs):
            seq = rng.choices(words, weights, k=rng.randint(1, 60))
            occ, offs, at = {}, {}, 0
            for p, w in enumerate(seq):
                occ.setdefault(w, []).append(p)
                offs.setdefault(w, []).append((at, at + len(w)))
                at += len(w) + 1
            toks = list(occ)
            off_col = "".join("".join(f"{s},{e};" for s, e in offs[w]) + "." for w in toks)
            pos_col = "".join("".join(f"{p};" for p in occ[w]) + "." for w in toks)
            f.write(f"t\t{' '.join(seq)}\t{' '.join(toks)}\t{off_col}\t{pos_col}\n")


def token_linedoc(path, n_docs, vocab, seed):
    rng = random.Random(seed)
    words = [f"w{i}" for i in range(vocab)]
    weights = [1.0 / (i + 1) ** 1.07 for i in range(vocab)]
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for d in range(n_docs):
            body = " ".join(rng.choices(words, weights, k=rng.randint(1, 300)))
            f.write(f"d{d}\t{body}\t{body}\n")


def cases(root):
    """name -> (linedoc, format, bloom)"""
    pos = os.path.join(root, "pos.linedoc")
    positions_linedoc(pos, 3000, 60, seed=11)
    tok = os.path.join(root, "tok.linedoc")
    token_linedoc(tok, 2000, 3000, seed=5)
    out = {
        "iter3": (os.path.join(DATA, "iter_test_3_docs"), "WITH_POSITIONS", None),
        "iter3_tf": (os.path.join(DATA, "iter_test_3_docs_tf"), "WITH_POSITIONS", None),
        "one_word": (os.path.join(DATA, "one_word_with_position"), "WITH_POSITIONS", None),
        "wiki5": (os.path.join(DATA, "line_doc_with_positions"), "WITH_POSITIONS", None),
        "wiki5_bloom": (os.path.join(DATA, "line_doc_with_positions"), "WITH_POSITIONS", BLOOM),
        "pre_suf_bloom": (os.path.join(DATA, "wiki_linedoc.toy.pre-suf-bloom"), "WITH_POSITIONS", BLOOM),
        "bi3_bloom": (os.path.join(DATA, "iter_test_3_docs_tf_bi-bloom"), "WITH_POSITIONS", BLOOM),
        "tok10k": (os.path.join(DATA, "test_doc_tokenized"), "TOKEN_ONLY", None),
        "pos3000": (pos, "WITH_POSITIONS", None),
        "pos3000_bloom": (pos, "WITH_POSITIONS", BLOOM),
        "tok2000": (tok, "TOKEN_ONLY", None),
        "tok2000_bloom": (tok, "TOKEN_ONLY", BLOOM),
    }
    return out


def digest(d):
    h = {}
    for name in sorted(os.listdir(d)):
        p = os.path.join(d, name)
        if os.path.isfile(p):
            h[name] = hashlib.sha256(open(p, "rb").read()).hexdigest()
    return h


def build_all(root, build):
    """build(linedoc, out_dir, fmt, bloom) for every case -> {case: {file: sha}}"""
    res = {}
    for name, (ld, fmt, bloom) in cases(root).items():
        d = os.path.join(root, name)
        os.makedirs(d, exist_ok=True)
        build(ld, d, fmt, bloom)
        res[name] = digest(d)
    return res


def main():
    import wiser_amd as w
    with tempfile.TemporaryDirectory() as root:
        res = build_all(root, lambda ld, d, fmt, bloom: w.build_from_linedoc(ld, d, fmt, bloom=bloom))
    with open(os.path.join(HERE, "writer_sha256.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(len(res), "cases")


if __name__ == "__main__":
    main()
