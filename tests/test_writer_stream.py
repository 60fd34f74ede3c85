"""The streaming linedoc writer (writer.cc: run files per chunk of rows, k-way
merge by term, parallel encode) against the SHA-256 of the one-map writer it
replaced (tests/golden/writer_sha256.json, make_writer_sha.py): byte-identical
my.vacuum / my.tip / my.doc_length / doc store for every fixture case, bloom
filters on and off, at chunk sizes that cut the fixtures into many runs and at
1 and 4 threads; and malformed rows still fail with the first bad row."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_writer_sha as mws  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "writer_sha256.json")))


def _build_env(chunk, threads):
    import wiser_amd as w

    def build(ld, d, fmt, bloom):
        old = {k: os.environ.get(k) for k in ("WSR_WRITER_CHUNK_DOCS", "WSR_WRITER_THREADS")}
        os.environ["WSR_WRITER_CHUNK_DOCS"] = str(chunk)
        os.environ["WSR_WRITER_THREADS"] = str(threads)
        try:
            w.build_from_linedoc(ld, d, fmt, bloom=bloom)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        assert not os.path.exists(os.path.join(d, ".wsr_runs")), "run files left behind"
    return build


@pytest.mark.parametrize("chunk,threads", [(32768, 4), (1, 1), (7, 4), (500, 3)])
def test_byte_identical(built, tmp_path, chunk, threads):
    got = mws.build_all(str(tmp_path), _build_env(chunk, threads))
    assert set(got) == set(GOLDEN)
    for name in GOLDEN:
        assert got[name] == GOLDEN[name], name


def _linedoc(path, rows, header="FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\toffsets\tpositions"):
    with open(path, "w") as f:
        f.write(header + "\n")
        for r in rows:
            f.write(r + "\n")


@pytest.mark.parametrize("chunk", [1, 2, 100])
def test_first_bad_row(built, tmp_path, chunk):
    import wiser_amd as w
    from wiser_amd._capi import WiserError
    good = "t\ta b\ta b\t0,1;.2,3;.\t0;.1;."
    rows = [good, good, "t\ta a\ta a\t0,1;.2,3;.\t0;.1;.", good, "t\tshort", good]
    ld = str(tmp_path / "bad.linedoc")
    _linedoc(ld, rows)
    os.environ["WSR_WRITER_CHUNK_DOCS"] = str(chunk)
    try:
        with pytest.raises(WiserError, match="duplicate token 'a' in row 2"):
            w.build_from_linedoc(ld, str(tmp_path / "o1"), "WITH_POSITIONS")
        _linedoc(ld, rows[:2] + rows[3:])
        with pytest.raises(WiserError, match="row 3 has too few columns"):
            w.build_from_linedoc(ld, str(tmp_path / "o2"), "WITH_POSITIONS")
    finally:
        os.environ.pop("WSR_WRITER_CHUNK_DOCS", None)
    assert not os.path.exists(str(tmp_path / "o1" / ".wsr_runs"))


def test_log_generators_fail_on_unwritable_path(built, tmp_path):
    """a query-log generator whose output cannot be written fails
    the call instead of returning WSR_OK with no file."""
    import pytest
    import wiser_amd as w
    d = str(tmp_path / "idx")
    w.build_synthetic(d, n_docs=20000, vocab=20000, seed=3, threads=2)
    bad = str(tmp_path / "no_such_dir" / "q.log")
    for gen in (lambda p: w.gen_two_term_log(d, p, n_queries=10),
                lambda p: w.gen_mixed_log(d, p, n_queries=10),
                lambda p: w.gen_single_term_log(d, p, True, n_queries=10)):
        with pytest.raises(Exception):
            gen(bad)
        ok = str(tmp_path / "q.log")
        assert gen(ok) == 10
        assert len(open(ok).read().splitlines()) == 10
