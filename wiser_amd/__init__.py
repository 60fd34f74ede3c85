"""wiser_amd: MI355X-native conjunctive-query + BM25 top-k engine for the
Vacuum (WiSER) index.  The compute path is libwiser_hip.so (hand-written HIP
for gfx950) behind the C ABI in include/wiser_hip.h; this package is the thin
Python mirror of the reference's SearchEngineServiceNew surface."""
from .engine import (CreateSearchEngine, DocsHost, ResidentBatch, SearchQuery, SearchResult,  # noqa: F401
                     class_batches, class_order,
                     SearchResultEntry, Server, VacuumEngine, build_from_linedoc, build_synthetic,
                     build_wiki_standin, gen_mixed_log, gen_phrase_log, gen_realistic_log,
                     gen_single_term_log, gen_two_term_log,
                     image_size, read_query_log, sync)

__all__ = ["CreateSearchEngine", "DocsHost", "VacuumEngine", "SearchQuery", "SearchResult",
           "SearchResultEntry", "ResidentBatch", "Server", "build_from_linedoc", "build_synthetic",
           "build_wiki_standin", "gen_mixed_log", "gen_phrase_log", "gen_realistic_log", "gen_single_term_log",
           "gen_two_term_log",
           "image_size", "read_query_log", "sync", "class_batches", "class_order"]
