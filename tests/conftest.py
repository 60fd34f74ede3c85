import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "tests", "golden", "data")

# One HIP runtime per process, the same one bench.py uses: torch loads first,
# at collection time, and libwiser_hip.so (NEEDED libamdhip64.so.7 /
# librccl.so.1) then binds to the copies torch already mapped under those
# sonames.  (The other order maps a second libamdhip64 for torch, whose
# NEEDED name differs, and the two runtimes fight over the device.)
try:
    import torch  # noqa: F401,E402
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _torch_device_first():
    """torch's device state is initialised once, before any engine opens the
    device, whatever subset of tests runs (torch is imported above)."""
    try:
        import torch
        torch.cuda.is_available()
    except Exception:
        pass


@pytest.fixture(scope="session")
def built():
    """Make sure libwiser_hip.so and liboracle.so exist (hipcc cross-compiles on CPU)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", ROOT, "-j8", "all"])
    return True


def _build(tmp_root, name, linedoc, fmt):
    import wiser_amd as w
    d = os.path.join(tmp_root, name)
    os.makedirs(d, exist_ok=True)
    st = w.build_from_linedoc(os.path.join(DATA, linedoc) if not os.path.isabs(linedoc) else linedoc,
                              d, fmt)
    return d, st


@pytest.fixture(scope="session")
def indexes(built, tmp_path_factory):
    """Reference fixtures written as Vacuum indexes by the product writer."""
    root = str(tmp_path_factory.mktemp("idx"))
    three = os.path.join(root, "three.linedoc")
    with open(three, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for body in ["hello world", "hello wisconsin", "hello world big world"]:
            f.write(f"t\t{body}\t{body}\n")
    # tests_5.cc:16-52 shape: 5 docs, tf 3 for hello and world, lengths (5-i)*10
    order = os.path.join(root, "order.linedoc")
    with open(order, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(5):
            toks = ["hello"] * 3 + ["world"] * 3 + ["again"] * 3
            toks += [f"fill{j}" for j in range((5 - i) * 10 - len(toks))]
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    out = {}
    out["three"] = _build(root, "three", three, "TOKEN_ONLY") + (three, "TOKEN_ONLY")
    out["order"] = _build(root, "order", order, "TOKEN_ONLY") + (order, "TOKEN_ONLY")
    out["iter3"] = _build(root, "iter3", "iter_test_3_docs", "WITH_POSITIONS") + (
        os.path.join(DATA, "iter_test_3_docs"), "WITH_POSITIONS")
    out["one_word"] = _build(root, "one_word", "one_word_with_position", "WITH_POSITIONS") + (
        os.path.join(DATA, "one_word_with_position"), "WITH_POSITIONS")
    out["wiki5"] = _build(root, "wiki5", "line_doc_with_positions", "WITH_POSITIONS") + (
        os.path.join(DATA, "line_doc_with_positions"), "WITH_POSITIONS")
    out["tok10k"] = _build(root, "tok10k", "test_doc_tokenized", "TOKEN_ONLY") + (
        os.path.join(DATA, "test_doc_tokenized"), "TOKEN_ONLY")
    return out


@pytest.fixture(scope="session")
def synth_small(built, tmp_path_factory):
    """20k-doc synthetic Zipf index (same generator as the C2 bench index)."""
    import wiser_amd as w
    d = str(tmp_path_factory.mktemp("synth20k"))
    st = w.build_synthetic(d, n_docs=20000, vocab=20000, seed=0x5EED2026, threads=4)
    return d, st


def all_tokens():
    with open(os.path.join(DATA, "all-tokens.txt")) as f:
        return f.readline().split()


# ---- phrase fixtures (positions index with known token sequences) ----
def _write_positions_linedoc(path, n_docs, vocab, seed):
    """WITH_POSITIONS linedoc (title, body, tokens, offsets, positions) of random
    word sequences; returns the token sequence of every doc."""
    rng = random.Random(seed)
    words = [f"w{i}" for i in range(vocab)]
    weights = [1.0 / (i + 1) for i in range(vocab)]
    seqs = []
    with open(path, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\toffsets\tpositions\n")
        for _ in range(n_docs):
            seq = rng.choices(words, weights, k=rng.randint(1, 60))
            seqs.append(seq)
            body = " ".join(seq)
            occ, offs, at = {}, {}, 0
            for p, w in enumerate(seq):
                occ.setdefault(w, []).append(p)
                offs.setdefault(w, []).append((at, at + len(w)))
                at += len(w) + 1
            toks = list(occ)
            off_col = "".join("".join(f"{s},{e};" for s, e in offs[w]) + "." for w in toks)
            pos_col = "".join("".join(f"{p};" for p in occ[w]) + "." for w in toks)
            f.write(f"t\t{body}\t{' '.join(toks)}\t{off_col}\t{pos_col}\n")
    return seqs


@pytest.fixture(scope="module")
def positions_index(built, tmp_path_factory):
    """3000 docs over 60 Zipf words: lists of hundreds of postings with position
    boxes of many packs, so that bags straddle packs and skip intervals."""
    import wiser_amd as w
    root = str(tmp_path_factory.mktemp("phr"))
    path = os.path.join(root, "pos.linedoc")
    seqs = _write_positions_linedoc(path, 3000, 60, seed=11)
    d = os.path.join(root, "idx")
    os.makedirs(d)
    w.build_from_linedoc(path, d, "WITH_POSITIONS")
    return d, seqs


def has_phrase(seq, terms):
    n = len(terms)
    return any(seq[i:i + n] == terms for i in range(len(seq) - n + 1))


def phrase_cases(seqs, n, seed):
    rng = random.Random(seed)
    cases = []
    for _ in range(n):
        m = rng.choice([2, 2, 2, 3, 4])
        s = rng.choice(seqs)
        if len(s) >= m and rng.random() < 0.7:
            i = rng.randrange(len(s) - m + 1)
            cases.append(s[i:i + m])               # a phrase that occurs
        else:
            cases.append([f"w{rng.randrange(12)}" for _ in range(m)])   # head words, maybe repeated
    return cases


# ---- bloom-filter indexes (the same fixtures written with two-way phrase blooms) ----
BLOOM_RATIO, BLOOM_ENTRIES = 0.0009, 5   # BloomDumper defaults (bloom_filter.h:650-655)


def _build_bloom(src, d, fmt="WITH_POSITIONS", bloom=(BLOOM_RATIO, BLOOM_ENTRIES)):
    import wiser_amd as w
    os.makedirs(d, exist_ok=True)
    w.build_from_linedoc(src, d, fmt, bloom=bloom)
    return d


@pytest.fixture(scope="module")
def bloom_indexes(built, indexes, positions_index, tmp_path_factory):
    root = str(tmp_path_factory.mktemp("bloom"))
    out = {}
    out["bi3"] = (_build_bloom(os.path.join(DATA, "iter_test_3_docs_tf_bi-bloom"), f"{root}/bi3"),
                  _build_bloom(os.path.join(DATA, "iter_test_3_docs_tf_bi-bloom"), f"{root}/bi3_nb",
                         bloom=None))
    out["wiki5"] = (_build_bloom(indexes["wiki5"][2], f"{root}/wiki5"), indexes["wiki5"][0])
    pos_ld = os.path.join(os.path.dirname(positions_index[0]), "pos.linedoc")
    out["pos"] = (_build_bloom(pos_ld, f"{root}/pos"), positions_index[0])
    return out
