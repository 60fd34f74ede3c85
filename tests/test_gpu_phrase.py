"""GPU parity of phrase queries (SearchQuery::is_phrase) against the oracle.

The HIP path ranks a conjunctive survivor only when its position bags hold the
terms at consecutive positions (QueryProcessor::HandleTheFoundDoc,
query_processing.h:854-912; PhraseQueryProcessor2, :170-382).  Bit-exact: doc
ids, order (ties included) and f64 scores, over:
  * the reference's phrase fixtures (tests_15.cc:96-155, tests_18.cc:334-352);
  * a 3000-doc positions index with known token sequences (bags straddling
    packs and skip intervals), 2-4 term phrases that occur and ones that do
    not, repeated terms, k = 1, 10, 64;
  * the 20k-doc synthetic Zipf index (real token positions), head-term phrases;
  * every dense-list probe mode and doc-range shards.
"""
import os
import random

import pytest

from conftest import has_phrase, phrase_cases
from test_gpu_parity import DENSE_MODES, SCORE_RTOL, _engine

pytestmark = pytest.mark.gpu


def _check_phrase(eng, orc, queries, k, phrase=True):
    import wiser_amd as w
    res = eng.SearchBatch([w.SearchQuery(list(q), n_results=k, is_phrase=phrase) for q in queries])
    bad = []
    for q, r in zip(queries, res):
        want, dfs = orc.search(list(q), k, phrase=phrase)
        got = [(e.doc_id, e.doc_score) for e in r.entries]
        if got != want or (want and r.doc_freqs != dfs):
            bad.append((q, got[:3], want[:3]))
        for (gd, gs), (wd, ws) in zip(got, want):
            assert abs(gs - ws) <= SCORE_RTOL * max(1.0, abs(ws))
    assert not bad, f"{len(bad)}/{len(queries)} phrase queries differ, first: {bad[:3]}"
    return res


@pytest.fixture(scope="module", params=sorted(DENSE_MODES))
def mode(request):
    return request.param


def test_phrase_fixture_kat(indexes, mode):
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d = indexes["iter3"][0]
    eng = _engine(d, mode)
    r = eng.Search(w.SearchQuery(["a", "b"], n_results=10, is_phrase=True))
    assert sorted(e.doc_id for e in r.entries) == [1, 2]
    r = eng.Search(w.SearchQuery(["a", "b", "c"], n_results=10, is_phrase=True))
    assert [e.doc_id for e in r.entries] == [2]
    assert eng.Search(w.SearchQuery(["b", "a"], n_results=10, is_phrase=True)).Size() == 0
    orc = OracleVacuum(d)
    _check_phrase(eng, orc, [["a", "b"], ["b", "c"], ["a", "b", "c"], ["a", "c"], ["c", "b"],
                             ["a", "a"], ["a"], ["a", "b", "x"]], 10)
    eng.close()
    d = indexes["wiki5"][0]
    eng = _engine(d, mode)
    assert eng.Search(w.SearchQuery(["a", "b"], is_phrase=True)).Size() == 0
    assert eng.Search(w.SearchQuery(["anarchist", "movement"], is_phrase=True)).Size() == 1
    # every adjacent token pair and triple of the 5 long docs, and their reversals
    orc = OracleVacuum(d)
    qs = []
    with open(indexes["wiki5"][2]) as f:
        f.readline()
        for line in f:
            body = line.split("\t")[1].split()
            for i in range(0, len(body) - 2, 7):
                qs += [body[i:i + 2], body[i:i + 3], body[i:i + 2][::-1]]
    _check_phrase(eng, orc, qs, 10)
    eng.close()


def test_phrase_positions_index(positions_index, mode):
    from oracle.oracle import OracleVacuum
    d, seqs = positions_index
    eng = _engine(d, mode)
    orc = OracleVacuum(d)
    qs = phrase_cases(seqs, 600, seed=17)
    for k in (1, 10, 64):
        res = _check_phrase(eng, orc, qs, k)
    # the phrase filter is real: result sets are the brute-force phrase docs
    for q, r in zip(qs, res):
        docs = {i for i, s in enumerate(seqs) if has_phrase(s, q)}
        if len(docs) <= 64:
            assert {e.doc_id for e in r.entries} == docs
    # mixed batch: phrase and conjunctive queries side by side
    import wiser_amd as w
    mixed = [w.SearchQuery(q, n_results=10, is_phrase=(i % 2 == 0)) for i, q in enumerate(qs)]
    for q, r in zip(mixed, eng.SearchBatch(mixed)):
        want, _ = orc.search(q.terms, 10, phrase=q.is_phrase)
        assert [(e.doc_id, e.doc_score) for e in r.entries] == want
    eng.close()
    orc.close()


def test_phrase_synthetic_zipf(synth_small):
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    eng = _engine(d, "dense")
    orc = OracleVacuum(d)
    rng = random.Random(23)
    head = [f"t{i:07d}" for i in range(40)]
    qs = [rng.sample(head, 2) for _ in range(300)] + [rng.sample(head, 3) for _ in range(100)]
    qs += [[h, h] for h in head[:10]]
    res = _check_phrase(eng, orc, qs, 10)
    assert sum(r.Size() > 0 for r in res) > 100   # head phrases do occur
    eng.close()
    orc.close()


def test_phrase_doc_range_shards(positions_index):
    """Shard images keep the whole position box of a list; phrase results of a
    W-way doc-range split replayed in order equal the unsharded oracle."""
    from oracle.oracle import OracleVacuum
    from test_shard_gpu import _run_step_regions
    d, seqs = positions_index
    orc = OracleVacuum(d)
    qs = phrase_cases(seqs, 240, seed=29)
    for world in (2, 3, 8):
        qs2, got = _run_step_regions(d, qs, 10, world, slot=None, phrase=True)
        for q, g in zip(qs2, got):
            assert g == orc.search(q, 10, phrase=True)[0], (world, q)
    orc.close()


def test_phrase_needs_positions(indexes):
    import wiser_amd as w
    from wiser_amd._capi import WiserError
    e = w.VacuumEngine(indexes["iter3"][0], positions=False)
    e.Load()
    with pytest.raises(WiserError):
        e.Search(w.SearchQuery(["a", "b"], is_phrase=True))
    # a one-term phrase is an ordinary single-term query
    assert e.Search(w.SearchQuery(["a"], is_phrase=True)).Size() == 3
    e.close()


@pytest.mark.parametrize("name", ["bi3", "wiki5", "pos"])
def test_bloom_index_loads_and_matches(bloom_indexes, name):
    """An index written with two-way bloom filters (reference layout) loads; the
    GPU's exact position check gives the results of the reference's bloom-pruned
    path (oracle with bloom_enable_factor 1), for phrase and plain queries."""
    from conftest import all_tokens
    from oracle.oracle import OracleVacuum
    d, plain = bloom_indexes[name]
    eng = _engine(d, "dense")
    orc = OracleVacuum(d)
    assert orc.has_bloom()
    orc_plain = OracleVacuum(plain)
    rng = random.Random(len(name))
    if name == "pos":
        src = os.path.join(os.path.dirname(plain), "pos.linedoc")
        seqs = [l.rstrip("\n").split("\t")[1].split() for l in open(src).readlines()[1:]]
        qs = phrase_cases(seqs, 300, seed=43)
    else:
        words = ["a", "b", "c", "x"] if name == "bi3" else all_tokens()[:80]
        qs = [rng.sample(words, 2) for _ in range(150)] + [rng.sample(words, 3) for _ in range(50)]
    _check_phrase(eng, orc, qs, 10)
    _check_phrase(eng, orc, qs, 10, phrase=False)
    for q in qs[:100]:
        assert orc.search(q, 10, phrase=True) == orc_plain.search(q, 10, phrase=True)
    eng.close()


def _varint(b, i):
    v = sh = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << sh
        sh += 7
        if not c & 0x80:
            return v, i


def _blank_first_bloom_boxes(d, terms):
    """Mark every posting of the first bloom box of `terms` (both sections) as
    having no filter: the box's presence bitmap zeroed in place (the arrays stay
    but nothing points at them).  The reference's reader then answers "not
    present" for those postings (flash_iterators.h:1045-1050)."""
    import struct
    tip = open(os.path.join(d, "my.tip"), "rb").read()
    offs, at = {}, 0
    while at < len(tip):
        n = struct.unpack_from("<I", tip, at)[0]
        t = tip[at + 4:at + 4 + n].decode()
        v = struct.unpack_from("<q", tip, at + 4 + n)[0]
        offs[t] = v & ((1 << 48) - 1)
        at += 4 + n + 8
    vac = bytearray(open(os.path.join(d, "my.vacuum"), "rb").read())
    for t in terms:
        o = offs[t]
        assert vac[o] == 0xF4
        _, i = _varint(vac, o + 1)
        s0, i = _varint(vac, i)
        s1, _ = _varint(vac, i)
        for s in (s0, s1):
            p = o + s
            assert vac[p] == 0xA4
            _, p = _varint(vac, p + 1)
            first, _ = _varint(vac, p)
            b = o + first
            assert vac[b] == 0xF5
            n, q = _varint(vac, b + 1)
            vac[q:q + (n + 7) // 8] = bytes((n + 7) // 8)
    open(os.path.join(d, "my.vacuum"), "wb").write(bytes(vac))


@pytest.mark.parametrize("factor", [0, 1, 3])
def test_bloom_pruning_follows_reference(bloom_indexes, tmp_path, factor):
    """The GPU applies IsPossibleToPresent (query_processing.h:873-884) before
    the position check, with CreateSearchEngine's bloom_enable_factor: on an
    index whose head terms lose the filters of their first 128 postings, the
    reference prunes docs that do hold the phrase, and the GPU must prune
    exactly the same ones (which side is checked depends on the factor and on
    the lists' sizes; 0 = BLOOM_NEVER_USE)."""
    import shutil
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    src, plain = bloom_indexes["pos"]
    d = str(tmp_path / "tampered")
    shutil.copytree(src, d)
    heads = [f"w{i}" for i in range(8)]
    _blank_first_bloom_boxes(d, heads)
    ld = os.path.join(os.path.dirname(plain), "pos.linedoc")
    seqs = [l.rstrip("\n").split("\t")[1].split() for l in open(ld).readlines()[1:]]
    rng = random.Random(97)
    qs = phrase_cases(seqs, 200, seed=97)
    qs += [rng.sample(heads, 2) for _ in range(150)] + [rng.sample(heads, 3) for _ in range(50)]
    eng = w.VacuumEngine(d, bloom_factor=factor)
    eng.Load()
    orc = OracleVacuum(d, bloom_factor=factor)
    _check_phrase(eng, orc, qs, 10)
    _check_phrase(eng, orc, qs, 10, phrase=False)
    exact = OracleVacuum(d, bloom_factor=0)
    n_diff = sum(orc.search(q, 10, phrase=True) != exact.search(q, 10, phrase=True) for q in qs)
    if factor:
        assert n_diff > 0, "the tampered filters must change some results for this test to bite"
    else:
        assert n_diff == 0
    assert eng.image_info()["pos_bytes"] > 0
    eng.close()


def test_phrase_only_batch_stats_are_its_own(positions_index):
    """A batch of phrase queries alone launches neither the conjunctive lean
    kernel nor the general one (engine.cc batch_run); its statistics must not
    read those kernels' rows, which still hold the batch's previous run."""
    import wiser_amd as w
    from wiser_amd import _capi
    d, seqs = positions_index
    eng = _engine(d, "dense")
    qs = phrase_cases(seqs, 400, seed=5)
    ph = [q for q in qs if len(q) == 2]
    conj = [q for q in qs if len(q) >= 2]

    def upload(b, queries, phrase):
        arr = (_capi.Query * len(queries))()
        for i, q in enumerate(queries):
            arr[i] = eng.resolve(w.SearchQuery(q, n_results=10, is_phrase=phrase))[0]
        b.upload(arr)

    a = w.ResidentBatch(eng, len(conj), 10)
    upload(a, conj, False)
    a.run()
    a.fetch()
    assert a.stats().survivors > 0
    upload(a, ph, True)   # the same batch object: its conjunctive rows keep the last run's counts
    a.run()
    _, na = a.fetch()
    na = list(na)[:len(ph)]
    sa = a.stats()
    b = w.ResidentBatch(eng, len(conj), 10)
    upload(b, ph, True)
    b.run()
    _, nb = b.fetch()
    nb = list(nb)[:len(ph)]
    sb = b.stats()
    assert na == nb
    assert (sa.survivors, sa.driver_blocks, sa.algo_bytes) == (sb.survivors, sb.driver_blocks, sb.algo_bytes)
    a.close()
    b.close()
    eng.close()


def test_class_batches_resident(positions_index):
    """The engine's batch former (wsr_class_order) over a mixed log: class-pure
    resident batches, run back to back with several in flight, every result
    equal to the oracle's and scattered back to its query."""
    import wiser_amd as w
    from wiser_amd import _capi
    from oracle.oracle import OracleVacuum
    d, seqs = positions_index
    eng = w.VacuumEngine(d, positions=True)
    eng.Load()
    orc = OracleVacuum(d)
    rng = random.Random(31)
    qs = phrase_cases(seqs, 900, seed=37)
    items = [(q, rng.random() < 0.3) for q in qs]
    arr = (_capi.Query * len(items))(*[eng.resolve(w.SearchQuery(q, n_results=10, is_phrase=ph))[0]
                                       for q, ph in items])
    groups = w.class_batches(arr, 128)
    assert len({items[i][1] and len(items[i][0]) > 1 for i in groups[0]}) == 1
    bs = []
    for g in groups:
        b = w.ResidentBatch(eng, len(g), 10)
        b.upload((_capi.Query * len(g))(*[arr[i] for i in g]))
        bs.append(b)
    for _ in range(2):
        for b in bs:
            b.run()
    got = {}
    for g, b in zip(groups, bs):
        hits, nh = b.fetch()
        for j, i in enumerate(g):
            got[i] = [(hits[j * 10 + t].doc_id, hits[j * 10 + t].score) for t in range(nh[j])]
        b.close()
    for i, (q, ph) in enumerate(items):
        assert got[i] == orc.search(list(q), 10, phrase=ph)[0], (q, ph)
    eng.close()
    orc.close()
