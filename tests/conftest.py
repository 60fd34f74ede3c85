import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "tests", "golden", "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


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
