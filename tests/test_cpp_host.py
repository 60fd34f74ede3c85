"""The C++ host class (include/wiser_hip_engine.hpp) above the C ABI: builds
on CPU; on the GPU its answers equal the oracle for a query log."""
import os
import random
import subprocess

import pytest

from conftest import ROOT, all_tokens

CLI = os.path.join(ROOT, "wiser_amd", "_lib", "engine_cli")


def test_cli_built(built):
    assert os.access(CLI, os.X_OK)


@pytest.mark.gpu
def test_cpp_host_matches_oracle(indexes, tmp_path):
    from oracle.oracle import OracleVacuum
    d = indexes["wiki5"][0]
    rng = random.Random(4)
    toks = all_tokens()
    qs = [[t] for t in rng.sample(toks, 100)] + [rng.sample(toks, 2) for _ in range(100)]
    log = tmp_path / "q.log"
    log.write_text("\n".join(" ".join(q) for q in qs) + "\n")
    out = subprocess.run([CLI, d, str(log), "10"], capture_output=True, text=True, check=True)
    lines = out.stdout.split("\n")
    assert lines[-1] == "" and len(lines) == len(qs) + 1, len(lines)   # one line per query, no truncation
    o = OracleVacuum(d)
    for q, line in zip(qs, lines):
        want, _ = o.search(q, 10)
        got = [(int(x.split(":")[0]), float.fromhex(x.split(":")[1])) for x in line.split()]
        assert got == want, q


@pytest.mark.gpu
def test_cpp_host_snippets_match_oracle(indexes, tmp_path):
    """VacuumHipEngine (C++ mirror) with return_snippets: the batched host
    snippet stage (wsr_snippets_batch) after the GPU top-k."""
    from oracle.oracle import OracleVacuum
    d = indexes["wiki5"][0]
    rng = random.Random(6)
    toks = all_tokens()
    qs = [[t] for t in rng.sample(toks, 60)] + [rng.sample(toks[:300], 2) for _ in range(60)]
    log = tmp_path / "q.log"
    log.write_text("\n".join(" ".join(q) for q in qs) + "\n")
    out = subprocess.run([CLI, d, str(log), "10", "snippets"], capture_output=True, text=True, check=True)
    lines = out.stdout.split("\n")
    assert lines[-1] == "" and len(lines) == 2 * len(qs) + 1, len(lines)   # two lines per query
    o = OracleVacuum(d)
    n = 0
    for i, q in enumerate(qs):
        want = o.search_snippets(q, 10)
        hits = [(int(x.split(":")[0]), float.fromhex(x.split(":")[1])) for x in lines[2 * i].split()]
        snips = [bytes.fromhex(x).decode() for x in lines[2 * i + 1].split(",")] if hits else []
        assert [(d_, s_, sn) for (d_, s_), sn in zip(hits, snips)] == want, q
        n += len(want)
    assert n > 100
