"""Offset-bucket probes on the GPU (tests/bucket_corpus.py): the lean kernel's
O1 through buckets -- inline offsets, the 8-byte window of a bucket of up to
nine, the walk past it -- further lists through buckets, and the general
kernel's first other list; every list dense (WSR_DENSE_DIV) or the default
threshold, whole image and doc-range shards (W = 2, 3 through the step's
region exchange); bit for bit against the oracle."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bucket_index(built, tmp_path_factory):
    from bucket_corpus import build_bucket_index
    return build_bucket_index(tmp_path_factory.mktemp("gbuckets"))


def _queries():
    us = [f"u{i}" for i in (0, 3, 7, 77, 400, 999)]
    qs = []
    for u in us:
        for o in ("g", "s", "z", "y"):
            qs += [[u, o], [o, u]]
        qs += [[u, "g", "s"], ["s", u, "g", "y"]]
    qs += [["g", "s"], ["s", "g"], ["g", "y"], ["z", "g"], ["g", "z", "s"], ["g"], ["s"], ["y", "g"]]
    return qs


@pytest.mark.parametrize("div", [0, 1 << 30])
@pytest.mark.parametrize("k", [10, 100])
def test_bucket_probes_equal_oracle(bucket_index, div, k, monkeypatch):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    if div:
        monkeypatch.setenv("WSR_DENSE_DIV", str(div))
    o = OracleVacuum(bucket_index)
    qs = _queries()
    eng = w.VacuumEngine(bucket_index, device=0, positions=False)
    eng.Load()
    res = eng.SearchBatch([w.SearchQuery(q, n_results=k) for q in qs])
    for q, r in zip(qs, res):
        assert [(x.doc_id, x.doc_score) for x in r.entries] == o.search(q, k)[0], q
    eng.close()
    o.close()


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_probes_shards(bucket_index, world, monkeypatch):
    from test_shard_gpu import _run_step_regions
    from oracle.oracle import OracleVacuum
    monkeypatch.setenv("WSR_DENSE_DIV", str(1 << 30))
    o = OracleVacuum(bucket_index)
    qs, got = _run_step_regions(bucket_index, _queries() * 2, 10, world, None)
    for q, g in zip(qs, got):
        assert g == o.search(q, 10)[0], q
    o.close()
