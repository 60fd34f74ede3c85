"""Committed golden vectors (tests/golden/results.json.gz, produced by
tests/golden/make_golden.py from the oracle over the reference's fixture
files): the oracle must reproduce them on CPU, the HIP engine on the GPU."""
import gzip
import json
import os

import pytest

from conftest import DATA, ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden", "results.json.gz")


@pytest.fixture(scope="module")
def golden_indexes(built, tmp_path_factory):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden
    root = str(tmp_path_factory.mktemp("golden"))
    return make_golden.build_indexes(root), json.load(gzip.open(GOLDEN, "rt"))


def _hits(r):
    return [[d, s.hex()] for d, s in r]


def test_oracle_reproduces_golden(golden_indexes):
    from oracle.oracle import OracleVacuum
    dirs, golden = golden_indexes
    for name, rows in golden.items():
        o = OracleVacuum(dirs[name])
        for row in rows:
            r, dfs = o.search(row["q"], row["k"])
            assert _hits(r) == row["hits"] and dfs == row["df"], (name, row["q"])


@pytest.mark.gpu
def test_engine_reproduces_golden(golden_indexes):
    import wiser_amd as w
    dirs, golden = golden_indexes
    for name, rows in golden.items():
        e = w.VacuumEngine(dirs[name])
        e.Load()
        res = e.SearchBatch([w.SearchQuery(row["q"], n_results=row["k"]) for row in rows])
        for row, r in zip(rows, res):
            got = [[x.doc_id, x.doc_score.hex()] for x in r.entries]
            assert got == row["hits"], (name, row["q"])
            assert (r.doc_freqs if row["hits"] else row["df"]) == row["df"]
        e.close()
