"""ctypes binding of include/wiser_hip.h (the engine's C ABI).

Loads the in-tree ``wiser_amd/_lib/libwiser_hip.so`` built by ``make`` (or
``__graft_entry__.build()``).  There is no fallback: if the library is missing
the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# WISER_HIP_LIB: an A/B build of the same sources (scripts only)
LIB_PATH = os.environ.get("WISER_HIP_LIB") or os.path.join(HERE, "_lib", "libwiser_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "wiser_hip.h")

MAX_TERMS = 16            # terms held in Query.list_ids (more: Query.more_ids)
MAX_QUERY_TERMS = 1024
MAX_PHRASE_TERMS = 8
MAX_K = 1024
SERVER_MAX_K = MAX_K

WSR_OK = 0
E_INVALID, E_IO, E_HIP, E_LIMIT, E_INTERNAL = -1, -2, -3, -4, -5
ERRORS = {-1: "WSR_E_INVALID", -2: "WSR_E_IO", -3: "WSR_E_HIP", -4: "WSR_E_LIMIT",
          -5: "WSR_E_INTERNAL"}


QUERY_PHRASE = 1


class OpenOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("doc_lo", C.c_uint32), ("doc_hi", C.c_uint32),
                ("threads", C.c_int32), ("positions", C.c_int32), ("bloom_factor", C.c_int32)]


class Query(C.Structure):
    _fields_ = [("n_terms", C.c_int32), ("k", C.c_int32), ("list_ids", C.c_int32 * MAX_TERMS),
                ("flags", C.c_int32), ("more_ids", C.POINTER(C.c_int32))]


class Hit(C.Structure):
    _fields_ = [("doc_id", C.c_int32), ("pad", C.c_int32), ("score", C.c_double)]


class BatchStats(C.Structure):
    _fields_ = [("work_items", C.c_uint64), ("survivors", C.c_uint64),
                ("driver_blocks", C.c_uint64), ("other_blocks", C.c_uint64),
                ("algo_bytes", C.c_uint64), ("plan_ms", C.c_double),
                ("segment_ms", C.c_double), ("replay_ms", C.c_double),
                ("events", C.c_uint64), ("max_query_events", C.c_uint64),
                ("lean_ms", C.c_double)]


class ImageInfo(C.Structure):
    _fields_ = [("total_bytes", C.c_uint64), ("blob_bytes", C.c_uint64), ("dense_bytes", C.c_uint64),
                ("tf8_bytes", C.c_uint64), ("plen_bytes", C.c_uint64), ("dir_bytes", C.c_uint64),
                ("pos_bytes", C.c_uint64), ("n_lists", C.c_uint32), ("dense_lists", C.c_uint32)]


class ServeStats(C.Structure):
    _fields_ = [("queries", C.c_uint64), ("seconds", C.c_double), ("qps", C.c_double),
                ("p50_ms", C.c_double), ("p99_ms", C.c_double), ("batches", C.c_uint64),
                ("mean_batch", C.c_double), ("queue_ms", C.c_double), ("gpu_ms", C.c_double),
                ("handoff_ms", C.c_double)]


class CommStats(C.Structure):
    _fields_ = [("groups", C.c_int64), ("steps", C.c_int64), ("replays_in_lean", C.c_int64),
                ("replays_on_stream", C.c_int64)]


class BuildStats(C.Structure):
    _fields_ = [("n_docs", C.c_int64), ("n_terms", C.c_int64), ("n_postings", C.c_int64),
                ("vacuum_bytes", C.c_int64), ("docs_char4_ge_0x80", C.c_int64),
                ("avg_length", C.c_double)]


class WiserError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build() "
                      "(the HIP engine has no CPU fallback)")

lib = C.CDLL(LIB_PATH)

_P = C.c_void_p
_sigs = {
    "wsr_last_error": (C.c_char_p, []),
    "wsr_version": (C.c_char_p, []),
    "wsr_runtime_info": (C.c_int, [C.c_char_p, C.c_int32]),
    "wsr_open": (C.c_int, [C.c_char_p, C.POINTER(OpenOpts), C.POINTER(_P)]),
    "wsr_close": (None, [_P]),
    "wsr_image_info_get": (C.c_int, [_P, C.POINTER(ImageInfo)]),
    "wsr_image_size": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_int32, C.c_int32, C.c_int32,
                                 C.POINTER(ImageInfo)]),
    "wsr_term_count": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "wsr_n_docs": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "wsr_lookup": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wsr_list_bytes": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_uint64)]),
    "wsr_search_batch": (C.c_int, [_P, C.POINTER(Query), C.c_int32, C.c_int32, C.POINTER(Hit),
                                   C.POINTER(C.c_int32)]),
    "wsr_check_query": (C.c_int, [_P, C.POINTER(Query)]),
    "wsr_resolve_text": (C.c_int, [_P, C.c_char_p, C.c_int64, C.c_int32, C.c_int32, C.POINTER(Query),
                                   C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int64]),
    "wsr_search_text": (C.c_int, [_P, C.c_char_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                  C.POINTER(Hit), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wsr_class_order": (C.c_int, [C.POINTER(Query), C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wsr_batch_create": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "wsr_batch_destroy": (None, [_P, _P]),
    "wsr_batch_upload": (C.c_int, [_P, _P, C.POINTER(Query), C.c_int32]),
    "wsr_batch_run": (C.c_int, [_P, _P]),
    "wsr_sync": (C.c_int, [_P]),
    "wsr_batch_fetch": (C.c_int, [_P, _P, C.POINTER(Hit), C.POINTER(C.c_int32)]),
    "wsr_batch_stats_get": (C.c_int, [_P, _P, C.POINTER(BatchStats)]),
    "wsr_batch_fetch_range": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.POINTER(Hit),
                                        C.POINTER(C.c_int32)]),
    "wsr_stream": (C.c_int, [_P, C.POINTER(_P)]),
    "wsr_batch_stream": (C.c_int, [_P, _P, C.POINTER(_P)]),
    "wsr_shard_fill": (C.c_int, [_P, _P, C.c_int32, C.POINTER(C.c_int64)]),
    "wsr_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "wsr_comm_open": (C.c_int, [C.POINTER(C.c_uint8), C.c_int32, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "wsr_comm_close": (None, [_P]),
    "wsr_loopback_create": (C.c_int, [C.c_int32, C.POINTER(_P)]),
    "wsr_loopback_destroy": (None, [_P]),
    "wsr_comm_open_loopback": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "wsr_comm_flush": (C.c_int, [_P]),
    "wsr_comm_stats_get": (C.c_int, [_P, C.POINTER(CommStats)]),
    "wsr_shard_step": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int64]),
    "wsr_shard_steps": (C.c_int, [_P, _P, C.c_int32, _P, C.c_int32, C.c_int64]),
    "wsr_shard_step_emit_async": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int64, _P]),
    "wsr_batch_stream_sync": (C.c_int, [_P, _P]),
    "wsr_batch_set_item_blocks": (C.c_int, [_P, _P, C.c_int32]),
    "wsr_shard_step_regions": (C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_uint64)]),
    "wsr_shard_step_emit": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int64, _P]),
    "wsr_shard_step_replay": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int64, _P]),
    "wsr_shard_step_replay_deferred": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int64, _P]),
    "wsr_debug_wg_stats": (C.c_int, [_P, _P, C.POINTER(C.c_uint32), C.c_int32,
                                     C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wsr_debug_fail_runs": (C.c_int, [C.c_int32]),
    "wsr_debug_decode_block": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32,
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]),
    "wsr_debug_dense_lookup": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_char_p,
                                         C.POINTER(C.c_uint32), C.c_int32, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32)]),
    "wsr_build_from_linedoc": (C.c_int, [C.c_char_p, C.c_int64, C.c_char_p, C.c_char_p,
                                         C.POINTER(BuildStats)]),
    "wsr_build_from_linedoc_bloom": (C.c_int, [C.c_char_p, C.c_int64, C.c_char_p, C.c_char_p,
                                               C.c_float, C.c_int32, C.POINTER(BuildStats)]),
    "wsr_build_synthetic": (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, C.c_double, C.c_uint64,
                                      C.c_int32, C.c_int32, C.POINTER(BuildStats)]),
    "wsr_build_wiki_standin": (C.c_int, [C.c_char_p, C.c_int64, C.c_double, C.c_uint64,
                                         C.c_int32, C.POINTER(BuildStats)]),
    "wsr_build_wiki_standin_topics": (C.c_int, [C.c_char_p, C.c_int64, C.c_double, C.c_uint64, C.c_int32,
                                                C.c_int32, C.c_int32, C.c_double, C.POINTER(BuildStats)]),
    "wsr_gen_two_term_log": (C.c_int, [C.c_char_p, C.c_int64, C.c_uint64, C.c_char_p,
                                       C.POINTER(C.c_int64)]),
    "wsr_batch_ready": (C.c_int, [_P, _P]),
    "wsr_pinned_alloc": (C.c_int, [C.c_uint64, C.POINTER(_P)]),
    "wsr_pinned_free": (None, [_P]),
    "wsr_batch_fetch_cols": (C.c_int, [_P, _P, C.POINTER(Hit), C.POINTER(C.c_int32), C.c_int32]),
    "wsr_server_open": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "wsr_server_close": (None, [_P]),
    "wsr_server_search": (C.c_int, [_P, C.POINTER(Query), C.POINTER(Hit), C.POINTER(C.c_int32)]),
    "wsr_server_bench": (C.c_int, [_P, C.POINTER(Query), C.c_int32, C.c_int32, C.c_int32,
                                   C.c_double, C.POINTER(ServeStats)]),
    "wsr_gen_mixed_log": (C.c_int, [C.c_char_p, C.c_int64, C.c_uint64, C.c_char_p,
                                    C.POINTER(C.c_int64)]),
    "wsr_gen_single_term_log": (C.c_int, [C.c_char_p, C.c_int32, C.c_int64, C.c_uint64, C.c_char_p,
                                          C.POINTER(C.c_int64)]),
    "wsr_gen_phrase_log": (C.c_int, [C.c_char_p, C.c_int64, C.c_uint64, C.c_char_p,
                                     C.POINTER(C.c_int64)]),
    "wsr_snippet": (C.c_int, [_P, C.POINTER(Query), C.c_int32, C.c_int32, C.c_char_p, C.c_int32,
                              C.POINTER(C.c_int32)]),
    "wsr_doc_get": (C.c_int, [_P, C.c_int32, C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
    "wsr_snippets_batch": (C.c_int, [_P, C.POINTER(Query), C.c_int32, C.POINTER(Hit),
                                     C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                     C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "wsr_docs_open": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "wsr_docs_close": (None, [_P]),
    "wsr_docs_lookup": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wsr_docs_snippet": (C.c_int, [_P, C.POINTER(Query), C.c_int32, C.c_int32, C.c_char_p, C.c_int32,
                                   C.POINTER(C.c_int32)]),
    "wsr_docs_get": (C.c_int, [_P, C.c_int32, C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
    "wsr_highlight": (C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                                C.c_char_p, C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
}
for _name, (_res, _args) in _sigs.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def check(rc):
    if rc != WSR_OK:
        raise WiserError(rc, lib.wsr_last_error().decode(errors="replace"))
    return rc


def text_call(fn, *args, cap: int = 4096) -> str:
    """Call a (..., char* out, int32 cap, int32* len) entry point, growing the
    buffer when the text is longer than it."""
    while True:
        buf = C.create_string_buffer(cap)
        n = C.c_int32()
        check(fn(*args, buf, cap, C.byref(n)))
        if n.value <= cap:
            return buf.raw[: n.value].decode("utf-8", errors="surrogateescape")
        cap = n.value


def snippets_batch(h, queries, hits, n_hits, stride: int, n_passages: int, threads: int = 0):
    """wsr_snippets_batch -> list (per query) of lists of snippet strings."""
    nq = len(n_hits)
    ends = (C.c_uint64 * max(1, nq * stride))()
    total = C.c_uint64()
    cap = 1 << 16
    while True:
        buf = C.create_string_buffer(cap)
        rc = lib.wsr_snippets_batch(h, queries, nq, hits, n_hits, stride, n_passages, threads, buf, cap,
                                    ends, C.byref(total))
        if rc == -4 and total.value > cap:   # WSR_E_LIMIT: grow to the reported size
            cap = total.value
            continue
        check(rc)
        break
    raw = buf.raw
    out, at = [], 0
    for i in range(nq):
        row = []
        for j in range(stride):
            e = ends[i * stride + j]
            if j < n_hits[i]:
                row.append(raw[at:e].decode("utf-8", errors="surrogateescape"))
            at = e
        out.append(row)
    return out


def highlight(offsets, n_passages: int, text: str) -> str:
    """SimpleHighlighter::highlightOffsetsEnums over explicit per-term (start, end) lists."""
    flat = [v for term in offsets for pr in term for v in pr]
    pairs = (C.c_int32 * max(1, len(flat)))(*flat)
    counts = (C.c_int32 * max(1, len(offsets)))(*[len(t) for t in offsets])
    return text_call(lib.wsr_highlight, pairs, counts, len(offsets), n_passages, text.encode())


def header_symbols(path: str = HEADER):
    """Function names declared in include/wiser_hip.h."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(wsr_\w+)\s*\(", text, re.M)))


def runtime_info() -> str:
    """hipRuntimeGetVersion and the loaded libamdhip64 / librccl paths."""
    buf = C.create_string_buffer(1024)
    check(lib.wsr_runtime_info(buf, 1024))
    return buf.value.decode()
