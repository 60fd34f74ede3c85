"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so, the CPU
restatement of the reference query path (see oracle.h).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.dirname(HERE), "oracle/_build/liboracle.so"])


if not os.path.exists(LIB_PATH):
    build()

lib = C.CDLL(LIB_PATH)
_P = C.c_void_p
_I32P = C.POINTER(C.c_int32)
_F64P = C.POINTER(C.c_double)
for name, res, args in [
    ("orc_last_error", C.c_char_p, []),
    ("orc_num_bits", C.c_int, [C.c_uint32]),
    ("orc_char4_encode", C.c_uint8, [C.c_uint32]),
    ("orc_char4_decode", C.c_uint32, [C.c_uint8]),
    ("orc_varint_encode", C.c_int, [C.c_uint64, C.POINTER(C.c_uint8)]),
    ("orc_varint_decode", C.c_int, [C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)]),
    ("orc_pack128", C.c_int, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)]),
    ("orc_unpack128", C.c_int, [C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)]),
    ("orc_es_idf", C.c_double, [C.c_int, C.c_int]),
    ("orc_es_tfnorm", C.c_double, [C.c_int, C.c_int, C.c_double]),
    ("orc_tfnorm_lossy", C.c_double, [C.c_double, C.c_int, C.c_uint8]),
    ("orc_vacuum_open", _P, [C.c_char_p]),
    ("orc_vacuum_close", None, [_P]),
    ("orc_vacuum_term_count", C.c_int, [_P]),
    ("orc_vacuum_n_docs", C.c_int, [_P]),
    ("orc_vacuum_df", C.c_int, [_P, C.c_char_p]),
    ("orc_vacuum_list", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                  C.c_int]),
    ("orc_vacuum_search", C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int, C.c_int, _I32P, _F64P,
                                    _I32P]),
    ("orc_vacuum_search_phrase", C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int,
                                           _I32P, _F64P, _I32P]),
    ("orc_vacuum_positions", C.c_int, [_P, C.c_char_p, C.c_int, C.POINTER(C.c_uint32), C.c_int]),
    ("orc_phrase_lists", C.c_int, [C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_int), C.c_int,
                                   _I32P, C.c_int]),
    ("orc_vacuum_search_lines", C.c_int, [_P, C.c_char_p, C.c_int, C.c_int, _I32P, _F64P, _I32P,
                                          C.c_int]),
    ("orc_vacuum_bench_lines", C.c_int, [_P, C.c_char_p, C.c_int, C.c_int, C.c_double,
                                         C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    ("orc_qqmem_load", _P, [C.c_char_p, C.c_int64, C.c_char_p]),
    ("orc_qqmem_close", None, [_P]),
    ("orc_qqmem_term_count", C.c_int, [_P]),
    ("orc_qqmem_search", C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int, C.c_int, _I32P, _F64P,
                                   _I32P]),
    ("orc_ub_negative_char_index", C.c_int64, []),
    ("orc_qqmem_list", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int]),
    ("orc_qqmem_posting", C.c_int, [_P, C.c_char_p, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_int),
                                    C.POINTER(C.c_uint32), C.POINTER(C.c_int), C.c_int]),
    ("orc_posting_encode", C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_int,
                                     C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_uint8), C.c_int]),
    ("orc_pld_probe", C.c_int, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int, C.c_int,
                                C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_int),
                                _I32P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int, _I32P]),
    ("orc_vacuum_set_bloom_factor", None, [_P, C.c_int]),
    ("orc_vacuum_has_bloom", C.c_int, [_P]),
    ("orc_bloom_stats", None, [C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("orc_vacuum_bloom_check", C.c_int, [_P, C.c_char_p, C.c_int, C.c_int, C.c_char_p]),
    ("orc_vacuum_search_snippets", C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int,
                                             C.c_int, _I32P, _F64P, C.c_char_p, C.c_int64,
                                             C.POINTER(C.c_int64)]),
    ("orc_highlight", C.c_int, [_I32P, _I32P, C.c_int, C.c_int, C.c_char_p, C.c_char_p, C.c_int]),
    ("orc_docstore_get", C.c_int64, [_P, C.c_int, C.c_char_p, C.c_int64]),
    ("orc_vacuum_offsets", C.c_int, [_P, C.c_char_p, C.c_int, _I32P, C.c_int]),
    ("orc_vacuum_docid_ops", C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int64), C.c_int,
                                       C.POINTER(C.c_int64)]),
]:
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args


def _err():
    return lib.orc_last_error().decode(errors="replace")


def _search(fn, h, terms, k, *extra):
    arr = (C.c_char_p * max(len(terms), 1))(*[t.encode() for t in terms])
    kk = max(k, 1)
    docs = (C.c_int32 * kk)()
    scores = (C.c_double * kk)()
    freqs = (C.c_int32 * max(len(terms), 1))(*([-1] * max(len(terms), 1)))
    n = fn(h, arr, len(terms), k, *extra, docs, scores, freqs)
    if n < 0:
        raise RuntimeError(_err())
    dfs = [freqs[i] for i in range(len(terms))] if n > 0 or (len(terms) and freqs[0] >= 0) else []
    if any(d < 0 for d in dfs):
        dfs = []
    return [(docs[i], scores[i]) for i in range(n)], dfs


class OracleVacuum:
    """VacuumEngine restatement reading my.vacuum / my.tip / my.doc_length."""

    def __init__(self, index_dir: str, bloom_factor: int = 1):
        self.h = lib.orc_vacuum_open(index_dir.encode())
        if not self.h:
            raise RuntimeError(_err())
        lib.orc_vacuum_set_bloom_factor(self.h, bloom_factor)

    def has_bloom(self):
        return bool(lib.orc_vacuum_has_bloom(self.h))

    def bloom_check(self, term, posting, side, elem):
        """side 0 = prior (begin) filter, 1 = next (end) filter -> 1 / 0"""
        r = lib.orc_vacuum_bloom_check(self.h, term.encode(), posting, side, elem.encode())
        if r < -1:
            raise RuntimeError(_err())
        return r

    def close(self):
        if self.h:
            lib.orc_vacuum_close(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def term_count(self):
        return lib.orc_vacuum_term_count(self.h)

    def n_docs(self):
        return lib.orc_vacuum_n_docs(self.h)

    def df(self, term):
        return lib.orc_vacuum_df(self.h, term.encode())

    def postings(self, term):
        n = self.df(term)
        d = (C.c_uint32 * max(n, 1))()
        t = (C.c_uint32 * max(n, 1))()
        m = lib.orc_vacuum_list(self.h, term.encode(), d, t, n)
        if m < 0:
            raise RuntimeError(_err())
        return list(d[:m]), list(t[:m])

    def docid_ops(self, term, ops):
        """Drive the term's DocIdIterator: ops = [("advance",), ("skip_to", posting),
        ("skip_forward", doc)] -> [(PostingIndex, Value or None, IsEnd)] after each."""
        code = {"advance": 0, "skip_to": 1, "skip_forward": 2}
        flat = []
        for op in ops:
            flat += [code[op[0]], op[1] if len(op) > 1 else 0]
        arr = (C.c_int64 * max(len(flat), 1))(*flat)
        out = (C.c_int64 * max(3 * len(ops), 1))()
        if lib.orc_vacuum_docid_ops(self.h, term.encode(), arr, len(ops), out) < 0:
            raise RuntimeError(_err())
        return [(out[3 * i], None if out[3 * i + 1] < 0 else out[3 * i + 1], bool(out[3 * i + 2]))
                for i in range(len(ops))]

    def search(self, terms, k, phrase=False):
        """-> ([(doc, score)], doc_freqs); phrase = SearchQuery::is_phrase"""
        return _search(lib.orc_vacuum_search_phrase, self.h, terms, k, int(bool(phrase)))

    def search_snippets(self, terms, k, n_passages=3, phrase=False):
        """VacuumEngine::Search with return_snippets -> [(doc, score, snippet)]"""
        if k == 0:
            return []
        arr = (C.c_char_p * max(len(terms), 1))(*[t.encode() for t in terms])
        docs = (C.c_int32 * k)()
        scores = (C.c_double * k)()
        ends = (C.c_int64 * k)()
        cap = 1 << 22
        buf = C.create_string_buffer(cap)
        n = lib.orc_vacuum_search_snippets(self.h, arr, len(terms), k, int(bool(phrase)), n_passages,
                                           docs, scores, buf, cap, ends)
        if n < 0:
            raise RuntimeError(_err())
        raw = buf.raw
        out, at = [], 0
        for i in range(n):
            out.append((docs[i], scores[i], raw[at:ends[i]].decode("utf-8", errors="surrogateescape")))
            at = ends[i]
        return out

    def document(self, doc):
        """ChunkedDocStoreReader::Get"""
        cap = 1 << 24
        buf = C.create_string_buffer(cap)
        n = lib.orc_docstore_get(self.h, doc, buf, cap)
        if n < 0:
            raise RuntimeError(_err())
        return buf.raw[:n].decode("utf-8", errors="surrogateescape")

    def offsets(self, term, posting):
        """(start, end) offset pairs of one posting (OffsetPostingBagIterator)"""
        cap = 1 << 15
        out = (C.c_int32 * (2 * cap))()
        n = lib.orc_vacuum_offsets(self.h, term.encode(), posting, out, cap)
        if n < 0:
            raise RuntimeError(_err())
        return [(out[2 * i], out[2 * i + 1]) for i in range(min(n, cap))]

    def positions(self, term, posting):
        """positions of one posting (PositionPostingBagIterator)"""
        cap = 1 << 16
        out = (C.c_uint32 * cap)()
        n = lib.orc_vacuum_positions(self.h, term.encode(), posting, out, cap)
        if n < 0:
            raise RuntimeError(_err())
        return list(out[:min(n, cap)])

    def search_lines(self, lines, k, threads=1, phrases=None):
        """Many queries; returns list of [(doc, score)].  phrases[i] true: query
        i is a phrase query (written in double quotes, as the reference's log)."""
        def fmt(i, t):
            q = " ".join(t)
            return f'"{q}"' if phrases is not None and phrases[i] else q
        text = "\n".join(fmt(i, t) for i, t in enumerate(lines)).encode()
        nq = len(lines)
        docs = (C.c_int32 * (nq * k))()
        scores = (C.c_double * (nq * k))()
        nout = (C.c_int32 * nq)()
        lib.orc_vacuum_search_lines(self.h, text, k, threads, docs, scores, nout, nq)
        return [[(docs[q * k + i], scores[q * k + i]) for i in range(nout[q])] for q in range(nq)]


    def bench_lines(self, lines, k, threads, seconds, phrases=None):
        """(queries, seconds): `threads` persistent C++ workers over the log
        (cycled) for `seconds` (orc_vacuum_bench_lines)."""
        def fmt(i, t):
            q = " ".join(t)
            return f'"{q}"' if phrases is not None and phrases[i] else q
        text = "\n".join(fmt(i, t) for i, t in enumerate(lines)).encode()
        done, el = C.c_int64(), C.c_double()
        if lib.orc_vacuum_bench_lines(self.h, text, k, threads, seconds, C.byref(done), C.byref(el)) != 0:
            raise RuntimeError("orc_vacuum_bench_lines failed")
        return done.value, el.value


class OracleQqMem:
    """QqMemEngineDelta restatement built straight from a linedoc."""

    def __init__(self, linedoc: str, fmt: str, n_rows: int = -1):
        self.h = lib.orc_qqmem_load(linedoc.encode(), n_rows, fmt.encode())
        if not self.h:
            raise RuntimeError(_err())

    def close(self):
        if self.h:
            lib.orc_qqmem_close(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def term_count(self):
        return lib.orc_qqmem_term_count(self.h)

    def search(self, terms, k):
        return _search(lib.orc_qqmem_search, self.h, terms, k)

    def postings(self, term):
        """(docs, tfs) through PostingListDeltaIterator (varint postings)"""
        n = lib.orc_qqmem_list(self.h, term.encode(), None, None, 0)
        d = (C.c_uint32 * max(n, 1))()
        t = (C.c_uint32 * max(n, 1))()
        n = lib.orc_qqmem_list(self.h, term.encode(), d, t, n)
        return list(d[:n]), list(t[:n])

    def posting(self, term, i, cap=1 << 14):
        """(doc, [(start, end)], [positions]) of posting i"""
        o = (C.c_uint32 * cap)()
        p = (C.c_uint32 * cap)()
        no, np_ = C.c_int(), C.c_int()
        doc = lib.orc_qqmem_posting(self.h, term.encode(), i, o, C.byref(no), p, C.byref(np_), cap)
        if doc < 0:
            raise RuntimeError(_err())
        return doc, [(o[2 * j], o[2 * j + 1]) for j in range(no.value)], list(p[:np_.value])


def posting_encode(doc_delta, tf, offsets=(), positions=()):
    """StandardPosting::Encode (posting.h:130-151)"""
    flat = [v for pr in offsets for v in pr]
    o = (C.c_uint32 * max(1, len(flat)))(*flat)
    p = (C.c_uint32 * max(1, len(positions)))(*positions)
    out = (C.c_uint8 * 4096)()
    n = lib.orc_posting_encode(doc_delta, tf, o, len(offsets), p, len(positions), out, 4096)
    return bytes(out[:n])


def pld_probe(docs, tfs, span, targets):
    """PostingListDelta(span) over (doc, tf) postings -> (skip prev docs, skip
    offsets, HasSkip per posting, NextSpanDocId per posting, SkipForward hits)"""
    n = len(docs)
    d = (C.c_uint32 * n)(*docs)
    t = (C.c_uint32 * n)(*tfs)
    sp = (C.c_uint32 * (n + 1))()
    so = (C.c_uint64 * (n + 1))()
    ns = C.c_int()
    hs = (C.c_int32 * n)()
    sd = (C.c_uint32 * n)()
    tg = (C.c_uint32 * max(1, len(targets)))(*targets)
    fd = (C.c_int32 * max(1, len(targets)))()
    if lib.orc_pld_probe(d, t, n, span, sp, so, C.byref(ns), hs, sd, tg, len(targets), fd) < 0:
        raise RuntimeError(_err())
    return (list(sp[:ns.value]), list(so[:ns.value]), list(hs), list(sd), list(fd[:len(targets)]))


def pack128(values):
    v = (C.c_uint32 * 128)(*values)
    out = (C.c_uint8 * (2 + 512 + 8))()
    n = lib.orc_pack128(v, out)
    return bytes(out[:n])


def unpack128(data: bytes):
    buf = (C.c_uint8 * (len(data) + 16)).from_buffer_copy(data + b"\0" * 16)
    out = (C.c_uint32 * 128)()
    b = lib.orc_unpack128(buf, out)
    if b < 0:
        raise RuntimeError(_err())
    return list(out), b


def varint_encode(v):
    out = (C.c_uint8 * 10)()
    n = lib.orc_varint_encode(v, out)
    return bytes(out[:n])


def varint_decode(data: bytes):
    buf = (C.c_uint8 * (len(data) + 10)).from_buffer_copy(data + b"\0" * 10)
    v = C.c_uint64()
    n = lib.orc_varint_decode(buf, C.byref(v))
    return v.value, n


def phrase_lists(lists, cap=64):
    """PhraseQueryProcessor2 over plain position lists -> (n_matches, table)"""
    arrs = [(C.c_uint32 * max(len(l), 1))(*l) for l in lists]
    ptrs = (C.POINTER(C.c_uint32) * len(lists))(*[C.cast(a, C.POINTER(C.c_uint32)) for a in arrs])
    sizes = (C.c_int * len(lists))(*[len(l) for l in lists])
    table = (C.c_int32 * (len(lists) * cap))()
    m = lib.orc_phrase_lists(ptrs, sizes, len(lists), table, cap)
    return m, [[table[i * cap + j] for j in range(min(m, cap))] for i in range(len(lists))]


def highlight(offsets, n_passages, text):
    """SimpleHighlighter::highlightOffsetsEnums over explicit per-term (start, end) lists"""
    flat = [v for term in offsets for pr in term for v in pr]
    pairs = (C.c_int32 * max(1, len(flat)))(*flat)
    counts = (C.c_int32 * max(1, len(offsets)))(*[len(t) for t in offsets])
    cap = 1 << 20
    buf = C.create_string_buffer(cap)
    n = lib.orc_highlight(pairs, counts, len(offsets), n_passages, text.encode(), buf, cap)
    if n < 0:
        raise RuntimeError(_err())
    return buf.raw[:n].decode("utf-8", errors="surrogateescape")


def bloom_stats():
    """(bloom checks, docs pruned by a filter) over the process so far"""
    c, p = C.c_int64(), C.c_int64()
    lib.orc_bloom_stats(C.byref(c), C.byref(p))
    return c.value, p.value
