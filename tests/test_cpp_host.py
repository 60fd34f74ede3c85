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
    o = OracleVacuum(d)
    for q, line in zip(qs, lines):
        want, _ = o.search(q, 10)
        got = [(int(x.split(":")[0]), float.fromhex(x.split(":")[1])) for x in line.split()]
        assert got == want, q
