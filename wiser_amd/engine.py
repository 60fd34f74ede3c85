"""Python mirror of the reference operator surface for the Vacuum engine.

Same names, argument meaning and error behaviour as the reference's
``SearchEngineServiceNew`` implemented by ``VacuumEngine``
(src/qq_mem/src/engine_services.h:14-27, vacuum_engine.h:119-258) and its
``SearchQuery`` / ``SearchResult`` types (types.h:205-346); every call goes
through the C ABI of libwiser_hip.so into the HIP kernels.

    engine = CreateSearchEngine("vacuum:vacuum_dump:/path/to/index")
    engine.Load()
    result = engine.Search(SearchQuery(["hello", "world"], n_results=10))

Behaviour kept from the reference:
  * ``n_results == 0`` -> empty result (vacuum_engine.h:206-208);
  * any term missing from the dictionary -> empty result, ``doc_freqs`` left
    empty (vacuum_engine.h:210-215);
  * entries ordered as the reference heap pops them (SortHeap), f64 scores;
  * ``is_phrase`` with two or more terms ranks only docs holding the terms at
    consecutive positions (QueryProcessor, query_processing.h:854-912); the
    engine must be loaded with ``positions=True`` (the default).
Snippets (SearchQuery.return_snippets): a host stage after the GPU top-k, as
in the reference (vacuum_engine.h:243-253): offsets from the index, text from the
doc store (my.fdx / my.fdt), SimpleHighlighter -- wsr_snippet in the C ABI.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import _capi
from ._capi import check, lib


@dataclass
class SearchQuery:
    """types.h:205-256"""
    terms: List[str]
    n_results: int = 5
    return_snippets: bool = False
    n_snippet_passages: int = 3
    is_phrase: bool = False


@dataclass
class SearchResultEntry:
    """types.h:259-274 (snippet filled when the query asks for snippets)"""
    doc_id: int
    doc_score: float
    snippet: str = ""


@dataclass
class SearchResult:
    """types.h:297-346"""
    entries: List[SearchResultEntry] = field(default_factory=list)
    doc_freqs: List[int] = field(default_factory=list)

    def Size(self) -> int:
        return len(self.entries)

    def __getitem__(self, i):
        return self.entries[i]


def ParseUrl(url: str):
    """engine_factory.h:21-31: ``vacuum:<source_type>:<path>``."""
    parts = url.split(":", 2)
    if len(parts) != 3 or parts[0] != "vacuum":
        raise ValueError(f"not a vacuum url: {url}")
    return parts[1], parts[2]


def CreateSearchEngine(url: str, bloom_factor: int = 1, device: int = 0) -> "VacuumEngine":
    """engine_factory.h:33-50 (only ``vacuum:vacuum_dump:<dir>`` is served here)."""
    source, path = ParseUrl(url)
    if source != "vacuum_dump":
        raise ValueError(f"unsupported vacuum source type: {source}")
    return VacuumEngine(path, bloom_factor=bloom_factor, device=device)


class VacuumEngine:
    """SearchEngineServiceNew over the HIP engine (vacuum_engine.h:119-258)."""

    def __init__(self, engine_dir_path: str, bloom_factor: int = 1, device: int = 0,
                 doc_range: Optional[Sequence[int]] = None, threads: int = 0,
                 positions: bool = True):
        self.engine_dir_path = engine_dir_path
        self.positions = positions
        self.bloom_factor = bloom_factor
        self.device = device
        self.doc_range = doc_range
        self.threads = threads
        self.snippet_threads = 0     # host threads of the snippet stage (0 = all cores)
        self._h = None

    # ---- SearchEngineServiceNew -------------------------------------
    def Load(self) -> None:
        if self._h is not None:
            raise RuntimeError("Engine is already loaded.")  # vacuum_engine.h:145
        opts = _capi.OpenOpts()
        opts.device = self.device
        opts.doc_lo, opts.doc_hi = (self.doc_range if self.doc_range else (0, 0))
        opts.threads = self.threads
        opts.positions = 1 if self.positions else 0
        opts.bloom_factor = int(self.bloom_factor)
        h = C.c_void_p()
        check(lib.wsr_open(self.engine_dir_path.encode(), C.byref(opts), C.byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h is not None:
            lib.wsr_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def image_info(self) -> Dict[str, int]:
        """HBM bytes of this engine's image per buffer (wsr_image_info_get)."""
        i = _capi.ImageInfo()
        check(lib.wsr_image_info_get(self._h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in _capi.ImageInfo._fields_}

    def TermCount(self) -> int:
        n = C.c_int32()
        check(lib.wsr_term_count(self._h, C.byref(n)))
        return n.value

    def NumDocs(self) -> int:
        n = C.c_int32()
        check(lib.wsr_n_docs(self._h, C.byref(n)))
        return n.value

    def PostinglistSizes(self, terms: Sequence[str]) -> Dict[str, int]:
        out = {}
        for t in terms:
            lid, df = self.lookup(t)
            if lid >= 0:
                out[t] = df
        return out

    def Search(self, query: SearchQuery) -> SearchResult:
        return self.SearchBatch([query])[0]

    # ---- batched extension -----------------------------------------
    def lookup(self, term: str):
        lid, df = C.c_int32(), C.c_int32()
        check(lib.wsr_lookup(self._h, term.encode(), C.byref(lid), C.byref(df)))
        return lid.value, df.value

    def resolve(self, query: SearchQuery):
        """-> (wsr_query, doc_freqs or None) with the reference's empty-result rules.
        A query of more than MAX_TERMS terms carries the rest in more_ids (ctypes
        keeps the array alive with the Query and with every array it is copied into)."""
        if len(query.terms) > _capi.MAX_QUERY_TERMS:
            raise NotImplementedError(f"more than {_capi.MAX_QUERY_TERMS} terms per query")
        if query.n_results > _capi.MAX_K:
            raise NotImplementedError(f"n_results above {_capi.MAX_K}")
        q = _capi.Query()
        q.k = max(0, int(query.n_results))
        q.flags = _capi.QUERY_PHRASE if (query.is_phrase and len(query.terms) > 1) else 0
        ids, dfs = [], []
        for t in query.terms:
            lid, df = self.lookup(t)
            ids.append(lid)
            dfs.append(df)
        missing = any(i < 0 for i in ids) or not ids
        q.n_terms = 0 if (missing or q.k == 0) else len(ids)
        for i, lid in enumerate(ids[:_capi.MAX_TERMS]):
            q.list_ids[i] = lid
        if len(ids) > _capi.MAX_TERMS:
            more = (C.c_int32 * (len(ids) - _capi.MAX_TERMS))(*ids[_capi.MAX_TERMS:])
            q.more_ids = C.cast(more, C.POINTER(C.c_int32))
        freqs = None if (missing or q.k == 0) else dfs
        return q, freqs

    def SearchBatch(self, queries: Sequence[SearchQuery]) -> List[SearchResult]:
        if not queries:
            return []
        arr = (_capi.Query * len(queries))()
        freqs = []
        stride = 1
        for i, sq in enumerate(queries):
            q, f = self.resolve(sq)
            arr[i] = q
            freqs.append(f)
            stride = max(stride, q.k)
        hits = (_capi.Hit * (len(queries) * stride))()
        nh = (C.c_int32 * len(queries))()
        check(lib.wsr_search_batch(self._h, arr, len(queries), stride, hits, nh))
        out = []
        for i in range(len(queries)):
            r = SearchResult()
            if freqs[i] is not None:
                r.doc_freqs = list(freqs[i])
                for j in range(nh[i]):
                    h = hits[i * stride + j]
                    r.entries.append(SearchResultEntry(h.doc_id, h.score))
            out.append(r)
        # vacuum_engine.h:248-252: the snippet stage, all entries of the batch at
        # once on the host's threads (grouped by n_snippet_passages)
        groups: Dict[int, List[int]] = {}
        for i, sq in enumerate(queries):
            if sq.return_snippets and freqs[i] is not None and nh[i] > 0:
                groups.setdefault(int(sq.n_snippet_passages), []).append(i)
        for n_passages, idx in groups.items():
            sub_q = (_capi.Query * len(idx))(*[arr[i] for i in idx])
            sub_h = (_capi.Hit * (len(idx) * stride))()
            sub_n = (C.c_int32 * len(idx))(*[nh[i] for i in idx])
            for a, i in enumerate(idx):
                C.memmove(C.byref(sub_h, a * stride * C.sizeof(_capi.Hit)),
                          C.byref(hits, i * stride * C.sizeof(_capi.Hit)), stride * C.sizeof(_capi.Hit))
            snips = _capi.snippets_batch(self._h, sub_q, sub_h, sub_n, stride, n_passages,
                                         self.snippet_threads)
            for a, i in enumerate(idx):
                for e, sn in zip(out[i].entries, snips[a]):
                    e.snippet = sn
        return out

    def snippet(self, q, doc_id: int, n_passages: int) -> str:
        """VacuumEngine::GenerateSnippet for result entry doc_id of resolved query q."""
        # (a 1-term phrase query is a plain query in the reference's dispatch)
        return _capi.text_call(lib.wsr_snippet, self._h, C.byref(q), doc_id, n_passages)

    def GetDocument(self, doc_id: int) -> str:
        """The doc store's body text (ChunkedDocStoreReader::Get)."""
        return _capi.text_call(lib.wsr_doc_get, self._h, doc_id)

    def decode_block(self, list_id: int, block: int, which: int = 0):
        """Device decode of one block (test hook) -> list of values."""
        buf = (C.c_uint32 * 128)()
        cnt = C.c_int32()
        check(lib.wsr_debug_decode_block(self._h, list_id, block, which, buf, C.byref(cnt)))
        return list(buf[: cnt.value])


class DocsHost:
    """The snippet stage alone, without a device: the index dictionary and the doc
    store of a Vacuum dump (wsr_docs_*).  Same snippets as VacuumEngine's."""

    def __init__(self, engine_dir_path: str):
        h = C.c_void_p()
        check(lib.wsr_docs_open(engine_dir_path.encode(), C.byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h is not None:
            lib.wsr_docs_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def query(self, terms: Sequence[str], is_phrase: bool = False):
        q = _capi.Query()
        q.n_terms = len(terms)
        q.k = 1
        q.flags = _capi.QUERY_PHRASE if (is_phrase and len(terms) > 1) else 0
        for i, t in enumerate(terms):
            lid, df = C.c_int32(), C.c_int32()
            check(lib.wsr_docs_lookup(self._h, t.encode(), C.byref(lid), C.byref(df)))
            q.list_ids[i] = lid.value
        return q

    def snippet(self, terms: Sequence[str], doc_id: int, n_passages: int = 3,
                is_phrase: bool = False) -> str:
        q = self.query(terms, is_phrase)
        return _capi.text_call(lib.wsr_docs_snippet, self._h, C.byref(q), doc_id, n_passages)

    def GetDocument(self, doc_id: int) -> str:
        return _capi.text_call(lib.wsr_docs_get, self._h, doc_id)


class ResidentBatch:
    """A query batch kept in HBM (wsr_batch_*): upload once, run many times."""

    def __init__(self, engine: VacuumEngine, max_queries: int, hit_stride: int):
        self.engine = engine
        self.stride = hit_stride
        b = C.c_void_p()
        check(lib.wsr_batch_create(engine._h, max_queries, hit_stride, C.byref(b)))
        self._b = b
        self.nq = 0
        # page-locked result arrays, reused by every fetch
        ph, pn = C.c_void_p(), C.c_void_p()
        check(lib.wsr_pinned_alloc(C.sizeof(_capi.Hit) * max(max_queries, 1) * hit_stride, C.byref(ph)))
        check(lib.wsr_pinned_alloc(4 * max(max_queries, 1), C.byref(pn)))
        self._pin = (ph, pn)
        self._hits = C.cast(ph, C.POINTER(_capi.Hit * (max(max_queries, 1) * hit_stride))).contents
        self._nh = C.cast(pn, C.POINTER(C.c_int32 * max(max_queries, 1))).contents

    def upload(self, queries) -> None:
        """queries: ctypes array of _capi.Query."""
        check(lib.wsr_batch_upload(self.engine._h, self._b, queries, len(queries)))
        self.nq = len(queries)

    def run(self) -> None:
        check(lib.wsr_batch_run(self.engine._h, self._b))

    def fetch(self):
        """-> (hits, n_hits): views of the batch's page-locked arrays, valid until
        the next fetch"""
        check(lib.wsr_batch_fetch(self.engine._h, self._b, self._hits, self._nh))
        return self._hits, self._nh

    def ready(self) -> bool:
        """True once the batch's last run has finished on the device."""
        rc = lib.wsr_batch_ready(self.engine._h, self._b)
        if rc < 0:
            check(rc)
        return rc == 1

    def wait_ready(self) -> None:
        """Spin until the batch's last run has finished (a host-side throttle)."""
        while not self.ready():
            pass

    def stats(self) -> _capi.BatchStats:
        st = _capi.BatchStats()
        check(lib.wsr_batch_stats_get(self.engine._h, self._b, C.byref(st)))
        return st

    def close(self) -> None:
        if self._b is not None:
            lib.wsr_batch_destroy(self.engine._h, self._b)
            self._b = None
            for p in self._pin:
                lib.wsr_pinned_free(p)
            self._pin = ()


class Server:
    """Micro-batching front end (wsr_server_*): Search() may be called from many
    threads at once; concurrent calls are coalesced into GPU batches.  The
    analogue of the reference's gRPC workers sharing one engine
    (grpc_server_impl.h:260-263,382-389)."""

    def __init__(self, engine: VacuumEngine, max_batch: int = 4096, window_us: int = 200):
        self.engine = engine
        s = C.c_void_p()
        check(lib.wsr_server_open(engine._h, max_batch, window_us, C.byref(s)))
        self._s = s

    def Search(self, query: SearchQuery) -> SearchResult:
        q, freqs = self.engine.resolve(query)
        hits = (_capi.Hit * max(1, q.k))()
        n = C.c_int32()
        check(lib.wsr_server_search(self._s, C.byref(q), hits, C.byref(n)))
        r = SearchResult()
        if freqs is not None:
            r.doc_freqs = list(freqs)
            r.entries = [SearchResultEntry(hits[j].doc_id, hits[j].score) for j in range(n.value)]
        return r

    def bench(self, queries, n_clients: int = 16, depth: int = 256,
              seconds: float = 3.0) -> _capi.ServeStats:
        """closed-loop load: queries = ctypes array of _capi.Query"""
        st = _capi.ServeStats()
        check(lib.wsr_server_bench(self._s, queries, len(queries), n_clients, depth, seconds,
                                   C.byref(st)))
        return st

    def close(self) -> None:
        if self._s is not None:
            lib.wsr_server_close(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def image_size(index_dir: str, doc_range=None, positions: bool = False, bloom_factor: int = 0,
               threads: int = 0) -> Dict[str, int]:
    """HBM bytes per buffer of the image wsr_open would build for index_dir (or
    its doc range [lo, hi)), computed on the host without a device
    (wsr_image_size)."""
    lo, hi = doc_range or (0, 0)
    i = _capi.ImageInfo()
    check(lib.wsr_image_size(index_dir.encode(), lo, hi, 1 if positions else 0, bloom_factor, threads,
                             C.byref(i)))
    return {f: getattr(i, f) for f, _ in _capi.ImageInfo._fields_}


def sync(engine: VacuumEngine) -> None:
    check(lib.wsr_sync(engine._h))


# ---- index building (host only) -------------------------------------------
def build_from_linedoc(linedoc: str, out_dir: str, fmt: str = "WITH_POSITIONS",
                       n_rows: int = -1, bloom: Optional[Sequence] = None) -> _capi.BuildStats:
    """bloom = (ratio, expected_entries), e.g. (0.0009, 5): also write the
    two-way phrase bloom filters (flash_engine_dumper.h:412-525)."""
    st = _capi.BuildStats()
    if bloom:
        check(lib.wsr_build_from_linedoc_bloom(linedoc.encode(), n_rows, fmt.encode(),
                                               out_dir.encode(), float(bloom[0]), int(bloom[1]),
                                               C.byref(st)))
    else:
        check(lib.wsr_build_from_linedoc(linedoc.encode(), n_rows, fmt.encode(), out_dir.encode(),
                                         C.byref(st)))
    return st


def build_synthetic(out_dir: str, n_docs: int = 1_000_000, vocab: int = 500_000,
                    zipf_s: float = 1.07, seed: int = 0x5EED2026, with_positions: bool = True,
                    threads: int = 0) -> _capi.BuildStats:
    st = _capi.BuildStats()
    check(lib.wsr_build_synthetic(out_dir.encode(), n_docs, vocab, zipf_s, seed,
                                  1 if with_positions else 0, threads, C.byref(st)))
    return st


def build_wiki_standin(out_dir: str, n_docs: int = 5_500_000, term_scale: float = 1.0,
                       seed: int = 0x3C3C2026, threads: int = 0, topics: int = 0,
                       topics_per_term: int = 2, affinity: float = 0.6) -> _capi.BuildStats:
    """BASELINE configs[2] stand-in: df histogram of the reference's en-Wikipedia
    index (tools/gen_synthetic_log.py:8-16) x term_scale over n_docs docs.
    topics > 0: the topic-clustered variant (doc ids in `topics` contiguous
    ranges, every term under N/16 postings draws `affinity` of its docs from
    its topics_per_term home topics; the df histogram is unchanged)."""
    st = _capi.BuildStats()
    if topics > 0:
        check(lib.wsr_build_wiki_standin_topics(out_dir.encode(), n_docs, term_scale, seed, threads, topics,
                                                topics_per_term, affinity, C.byref(st)))
    else:
        check(lib.wsr_build_wiki_standin(out_dir.encode(), n_docs, term_scale, seed, threads,
                                         C.byref(st)))
    return st


def gen_two_term_log(index_dir: str, out_path: str, n_queries: int = 100_000, seed: int = 7) -> int:
    n = C.c_int64()
    check(lib.wsr_gen_two_term_log(index_dir.encode(), n_queries, seed, out_path.encode(),
                                   C.byref(n)))
    return n.value


def gen_mixed_log(index_dir: str, out_path: str, n_queries: int = 20_000, seed: int = 7) -> int:
    """1-5 term AND queries with the AOL term-count shares."""
    n = C.c_int64()
    check(lib.wsr_gen_mixed_log(index_dir.encode(), n_queries, seed, out_path.encode(),
                                C.byref(n)))
    return n.value


def gen_single_term_log(index_dir: str, out_path: str, high: bool, n_queries: int = 20_000, seed: int = 7) -> int:
    """Single-term queries of one df group (tools/gen_synthetic_log.py:171-189;
    run_exp.py:116-117's type_single.docfreq_high / _low)."""
    n = C.c_int64()
    check(lib.wsr_gen_single_term_log(index_dir.encode(), 1 if high else 0, n_queries, seed, out_path.encode(),
                                      C.byref(n)))
    return n.value


def gen_phrase_log(index_dir: str, out_path: str, n_queries: int = 10_000, seed: int = 7) -> int:
    """tools/gen_synthetic_log.py:254-265 over a synthetic index's phrase pool."""
    n = C.c_int64()
    check(lib.wsr_gen_phrase_log(index_dir.encode(), n_queries, seed, out_path.encode(),
                                 C.byref(n)))
    return n.value


def gen_realistic_log(index_dir: str, out_path: str, n_queries: int = 20_000, phrase_share: float = 0.1,
                      seed: int = 7) -> int:
    """One stream of the reference's mixed log (query_pool.h:363-375: quoted
    phrase lines among plain lines; run_exp.py's "type_realistic"): a share of
    two-term phrases from the index's phrase pool among 1-5-term AND queries
    (gen_mixed_log), interleaved in a seeded random order."""
    import os
    import random
    n_ph = int(round(n_queries * phrase_share))
    tmp_m, tmp_p = out_path + ".and.tmp", out_path + ".phr.tmp"
    gen_mixed_log(index_dir, tmp_m, n_queries=n_queries - n_ph, seed=seed)
    lines = open(tmp_m).read().splitlines()
    if n_ph:
        gen_phrase_log(index_dir, tmp_p, n_queries=n_ph, seed=seed + 1)
        lines += open(tmp_p).read().splitlines()
    for t in (tmp_m, tmp_p):
        if os.path.exists(t):
            os.remove(t)
    random.Random(seed).shuffle(lines)
    with open(out_path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return len(lines)


def class_order(queries) -> Tuple[List[int], int]:
    """wsr_class_order: a stable order of `queries` (a ctypes array of
    _capi.Query) with the conjunctive queries first and the phrase queries
    after them -> (order, n_conj).  Batches cut from it are class-pure."""
    n = len(queries)
    order = (C.c_int32 * max(n, 1))()
    nc = C.c_int32()
    check(lib.wsr_class_order(queries, n, order, C.byref(nc)))
    return list(order[:n]), nc.value


def class_batches(queries, batch: int) -> List[List[int]]:
    """The engine's batch former for a query stream: indices of `queries`
    (ctypes Query array) in batches of at most `batch`, each class cut
    separately (wsr_class_order), so no batch mixes phrase and conjunctive
    queries."""
    order, nc = class_order(queries)
    out = []
    for lo, hi in ((0, nc), (nc, len(order))):
        for s in range(lo, hi, batch):
            out.append(order[s:min(s + batch, hi)])
    return out


def read_query_log(path: str):
    """-> [(terms, is_phrase)]: one query per line, a phrase in double quotes"""
    out = []
    for line in open(path).read().splitlines():
        line = line.strip()
        if not line:
            continue
        ph = len(line) >= 2 and line[0] == '"' and line[-1] == '"'
        out.append(((line[1:-1] if ph else line).split(), ph))
    return out
