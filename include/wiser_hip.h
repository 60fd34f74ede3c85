/*
 * wiser_hip.h -- C ABI of the MI355X conjunctive-query + BM25 top-k engine for
 * the Vacuum (WiSER) index.  Plain pointers and sizes only; no C++ or torch
 * types cross this boundary.  Every function returns 0 (WSR_OK) or a negative
 * WSR_E_* code and never aborts; wsr_last_error() gives a thread-local message.
 *
 * Reference interfaces replaced (paths under /root/reference/src/qq_mem/src):
 *   wsr_open / wsr_close ...... VacuumEngine::Load (vacuum_engine.h:144-180) and
 *                               CreateSearchEngine("vacuum:vacuum_dump:<dir>")
 *                               (engine_factory.h:21-50)
 *   wsr_term_count ............ SearchEngineServiceNew::TermCount (engine_services.h:20,
 *                               vacuum_engine.h:182-185)
 *   wsr_lookup ................ VacuumInvertedIndex::FindTermIndexResult +
 *                               VacuumPostingListIterator::Size
 *                               (vacuum_engine.h:75-99,187-199, flash_iterators.h:1030-1032)
 *   wsr_search_batch .......... VacuumEngine::Search (vacuum_engine.h:201-258) ->
 *                               qq_search::ProcessQueryDelta (query_processing.h:956-979),
 *                               n queries per call instead of one
 *   wsr_batch_* ............... the same, split into upload / enqueue / fetch so that a
 *                               serving loop (grpc_server_impl.h:382-389) or a bench
 *                               (engine_bench.cc:255-279) can keep query batches
 *                               resident in HBM and overlap them
 *   wsr_snippet / wsr_docs_* .. VacuumEngine::GenerateSnippet (vacuum_engine.h:286-296),
 *                               ChunkedDocStoreReader (doc_store.h:365-455),
 *                               SimpleHighlighter (highlighter.h:297-456); host stage
 *   wsr_build_* / wsr_gen_* ... index writer FlashEngineDumper::{LoadLocalDocuments,Dump}
 *                               (flash_engine_dumper.h:674-744) and the query generator
 *                               tools/gen_synthetic_log.py:191-214 (host only, no GPU)
 *
 * Threading: a handle may be used from several threads (the reference's
 * engine is shared read-only by its gRPC threads, grpc_server_impl.h:260-263):
 * its image is read-only after wsr_open, wsr_search_batch / wsr_search_text
 * may be called concurrently, and threads that each own a wsr_batch drive
 * them concurrently (a batch itself is used by one thread at a time).
 */
#ifndef WISER_HIP_H
#define WISER_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WSR_MAX_TERMS 16        /* terms held in wsr_query.list_ids (more: wsr_query.more_ids) */
#define WSR_MAX_QUERY_TERMS 1024 /* terms of a conjunctive query (AOL's longest query has 245) */
#define WSR_MAX_PHRASE_TERMS 8  /* terms of a phrase query (the reference's cap, query_processing.h:695) */
#define WSR_MAX_K 1024          /* n_results (k > 64 keeps the replay's heap in LDS) */
#define WSR_SERVER_MAX_K WSR_MAX_K  /* n_results through the micro-batcher (wsr_server_*) */

enum {
  WSR_OK = 0,
  WSR_E_INVALID = -1,   /* bad argument */
  WSR_E_IO = -2,        /* missing / malformed index files */
  WSR_E_HIP = -3,       /* HIP runtime error (no device, out of memory, ...) */
  WSR_E_LIMIT = -4,     /* n_terms > WSR_MAX_QUERY_TERMS (phrase: WSR_MAX_PHRASE_TERMS) or k > WSR_MAX_K */
  WSR_E_INTERNAL = -5
};

typedef struct wsr_handle wsr_handle;
typedef struct wsr_batch wsr_batch;

typedef struct wsr_open_opts {
  int32_t device;     /* HIP device ordinal */
  uint32_t doc_lo;    /* doc-id shard [doc_lo, doc_hi); doc_hi = 0 means all docs */
  uint32_t doc_hi;
  int32_t threads;    /* host threads for the load-time directory build (0 = all) */
  int32_t positions;  /* 1: also upload the position boxes (phrase queries) */
  int32_t bloom_factor; /* CreateSearchEngine's bloom_enable_factor (engine_factory.h:33-34,
                           reference default 1; 0 = BLOOM_NEVER_USE, types.h:54): with
                           positions and a bloom index, phrase candidates are pruned by
                           the two-way filters before the position check
                           (QueryProcessor::IsPossibleToPresent, query_processing.h:873-884).
                           Pruning only: results are the same at every factor. */
} wsr_open_opts;

/* A query with its terms already resolved by wsr_lookup (list id per term, in
 * query order; -1 = term not in the index => empty result, as the reference). */
typedef struct wsr_query {
  int32_t n_terms;
  int32_t k;          /* n_results; 0 => empty result */
  int32_t list_ids[WSR_MAX_TERMS];   /* terms 0 .. min(n_terms, 16) - 1 */
  int32_t flags;      /* WSR_QUERY_PHRASE: SearchQuery::is_phrase (types.h:205-256) --
                         a doc is ranked only if the terms occur at consecutive
                         positions (QueryProcessor::HandleTheFoundDoc,
                         query_processing.h:854-912); needs positions at wsr_open */
  const int32_t* more_ids;   /* n_terms > WSR_MAX_TERMS: list ids of terms 16 .. n_terms - 1
                                (caller's memory, read during the call that takes the
                                query; the reference's conjunctive processor has no
                                term cap, query_processing.h:710-728,810-852) */
} wsr_query;
#define WSR_QUERY_PHRASE 1

typedef struct wsr_hit {
  int32_t doc_id;
  int32_t pad;
  double score;       /* f64 BM25, bit-identical to the reference engine */
} wsr_hit;

/* ---- snippets (SearchQuery::return_snippets) ---------------------------
 * The snippet of result entry `doc_id` of query q: VacuumEngine::GenerateSnippet
 * (vacuum_engine.h:243-253,286-296) over ResultDocEntry::OffsetsForHighliting
 * (query_processing.h:446-492) and SimpleHighlighter::highlightOffsetsEnums
 * (highlighter.h:303-441).  A host stage after the GPU top-k, as in the
 * reference: the doc's offset (and, for a phrase, position) bags are read from
 * the mapped index, the text from the doc store (my.fdx / my.fdt,
 * ChunkedDocStoreReader, doc_store.h:365-455; WSR_E_INVALID if the index has
 * none).  Writes min(len, cap) bytes to out (no terminator) and the full
 * length to *len. */
int wsr_snippet(wsr_handle* h, const wsr_query* q, int32_t doc_id, int32_t n_passages,
                char* out, int32_t cap, int32_t* len);
/* The snippets of a batch's result entries, built by `threads` host threads
 * (0 = all cores): entry j of query i is hits[i * stride + j], j < n_hits[i]
 * (what wsr_search_batch / wsr_batch_fetch return).  The snippets are packed
 * into buf in entry order; ends[i * stride + j] = end offset of that entry's
 * snippet (entries past n_hits[i] are empty).  *total = bytes needed; if it
 * exceeds cap nothing is written and WSR_E_LIMIT is returned. */
int wsr_snippets_batch(wsr_handle* h, const wsr_query* q, int32_t nq, const wsr_hit* hits,
                       const int32_t* n_hits, int32_t stride, int32_t n_passages, int32_t threads,
                       char* buf, uint64_t cap, uint64_t* ends, uint64_t* total);
/* ChunkedDocStoreReader::Get: the doc's body text */
int wsr_doc_get(wsr_handle* h, int32_t doc_id, char* out, int32_t cap, int32_t* len);
/* The same host stage without a device: index dictionary + doc store only. */
typedef struct wsr_docs wsr_docs;
int wsr_docs_open(const char* dir, wsr_docs** out);
void wsr_docs_close(wsr_docs* d);
int wsr_docs_lookup(wsr_docs* d, const char* term, int32_t* list_id, int32_t* doc_freq);
int wsr_docs_snippet(wsr_docs* d, const wsr_query* q, int32_t doc_id, int32_t n_passages, char* out,
                     int32_t cap, int32_t* len);
int wsr_docs_get(wsr_docs* d, int32_t doc_id, char* out, int32_t cap, int32_t* len);
/* SimpleHighlighter::highlightOffsetsEnums over explicit offsets: term i has
 * counts[i] (start, end) pairs, consecutive in pairs[] (tests_2.cc:15-90). */
int wsr_highlight(const int32_t* pairs, const int32_t* counts, int32_t n_terms, int32_t n_passages,
                  const char* text, char* out, int32_t cap, int32_t* len);

/* Per-batch counters of the last run (for the roofline / profiles). */
typedef struct wsr_batch_stats {
  uint64_t work_items;       /* segments processed */
  uint64_t survivors;        /* docs in every list (scored) */
  uint64_t driver_blocks;    /* 128-posting blocks decoded from driver lists */
  uint64_t other_blocks;     /* blocks decoded from the other lists */
  uint64_t algo_bytes;       /* sum over queries of docid+tf span bytes of its lists (a phrase
                                query: + the lists' position boxes) + survivors * 1 B + k * 12 B
                                 */
  double plan_ms, segment_ms, replay_ms;  /* HIP-event times on the engine stream */
  uint64_t events;           /* segment heap-insertion events handed to the replay */
  uint64_t max_query_events; /* the largest per-query event count of the batch */
  double lean_ms;            /* lean_kernel alone (segment_ms spans it and the concurrent
                                general segment_kernel) */
} wsr_batch_stats;

/* HBM bytes of an engine's image, per buffer. */
typedef struct wsr_image_info {
  uint64_t total_bytes;
  uint64_t blob_bytes;    /* docid + tf spans, byte-exact from my.vacuum */
  uint64_t dense_bytes;   /* rank bitmaps of the dense lists */
  uint64_t tf8_bytes;     /* their 1-byte tfs */
  uint64_t plen_bytes;    /* per-posting doc-length codes */
  uint64_t dir_bytes;     /* list heads, block directory, decoded tails, doc lengths */
  uint64_t pos_bytes;     /* position boxes (positions = 1) */
  uint32_t n_lists, dense_lists;
} wsr_image_info;

const char* wsr_last_error(void);
const char* wsr_version(void);
/* the HIP runtime this process runs the engine on: hipRuntimeGetVersion and
 * the paths of the loaded libamdhip64 / librccl (one runtime per process) */
int wsr_runtime_info(char* buf, int32_t cap);

/* ---- engine ---------------------------------------------------------- */
int wsr_open(const char* vacuum_dir, const wsr_open_opts* opts, wsr_handle** out);
void wsr_close(wsr_handle* h);
int wsr_image_info_get(wsr_handle* h, wsr_image_info* out);
/* The same figures without a device (host only): the image wsr_open would
 * build for the doc range [doc_lo, doc_hi) (doc_hi 0 = all) of the index in
 * dir, with positions / blooms as wsr_open_opts and the same load-time knobs,
 * sized but never uploaded.  threads: host threads (0 = all). */
int wsr_image_size(const char* dir, uint32_t doc_lo, uint32_t doc_hi, int32_t positions, int32_t bloom_factor,
                   int32_t threads, wsr_image_info* out);
int wsr_term_count(wsr_handle* h, int32_t* out);
int wsr_n_docs(wsr_handle* h, int32_t* out);
/* list id (or -1) and document frequency (0 if absent) of one term */
int wsr_lookup(wsr_handle* h, const char* term, int32_t* list_id, int32_t* doc_freq);
/* bytes of docid+tf span held in HBM for a list (0 if absent from this shard) */
int wsr_list_bytes(wsr_handle* h, int32_t list_id, uint64_t* out);

/* The per-query checks wsr_batch_upload applies (term / k limits, flags, a
 * phrase query needs positions): WSR_OK or the code upload would return. */
int wsr_check_query(wsr_handle* h, const wsr_query* q);

/* Run nq queries synchronously.  hits: nq * hit_stride entries (hit_stride >=
 * every query's k); n_hits[q] = entries written for query q. */
int wsr_search_batch(wsr_handle* h, const wsr_query* q, int32_t nq, int32_t hit_stride,
                     wsr_hit* hits, int32_t* n_hits);

/* Queries as text, the reference's query-log format (QueryProducerByLog,
 * query_pool.h:319-378): one query per line, terms separated by spaces, a
 * line in double quotes is a phrase query.  Every term is resolved through the
 * term index (VacuumInvertedIndex::FindIteratorsSolid, vacuum_engine.h:89-99);
 * q[0..*nq) receives the queries (k results each).  The list ids of terms past
 * the first WSR_MAX_TERMS of a query go to the caller's more_store (more_cap
 * int32 entries; may be NULL when no query is that long) and the query's
 * more_ids points there, so the ids live as long as the caller's storage;
 * WSR_E_LIMIT when more_store is too small. */
int wsr_resolve_text(wsr_handle* h, const char* text, int64_t len, int32_t k, int32_t max_q,
                     wsr_query* q, int32_t* nq, int32_t* more_store, int64_t more_cap);
/* The whole Search chain from strings: wsr_resolve_text, then wsr_search_batch
 * (upload, run, results to the host). */
int wsr_search_text(wsr_handle* h, const char* text, int64_t len, int32_t k, int32_t hit_stride,
                    int32_t max_q, wsr_hit* hits, int32_t* n_hits, int32_t* nq);

/* The batch former for a stream of queries cut into batches.  The reference
 * scores every query on its own (grpc_server_impl.h:382-389, a query_pool.h
 * log mixes classes), so which queries share a batch is the engine's choice:
 * order[0..nq) receives a stable permutation of the queries that puts each
 * execution class together -- conjunctive queries (AND of any length, single
 * terms) first, then phrase queries of two or more terms -- and *n_conj the
 * size of the first class.  Batches cut from this order are class-pure: a
 * phrase query's position check then runs in batches of its own instead of
 * riding, a few hundred at a time, at the tail of every conjunctive batch
 * (DESIGN.md §4i).  Needs no handle. */
int wsr_class_order(const wsr_query* q, int32_t nq, int32_t* order, int32_t* n_conj);

/* ---- resident batches ------------------------------------------------ */
int wsr_batch_create(wsr_handle* h, int32_t max_queries, int32_t hit_stride, wsr_batch** out);
void wsr_batch_destroy(wsr_handle* h, wsr_batch* b);
/* copy queries to HBM (synchronous) and size the event workspace */
int wsr_batch_upload(wsr_handle* h, wsr_batch* b, const wsr_query* q, int32_t nq);
/* enqueue plan + segment + replay kernels on the batch's streams (asynchronous) */
int wsr_batch_run(wsr_handle* h, wsr_batch* b);
/* wait for the engine stream */
int wsr_sync(wsr_handle* h);
/* copy results to the host: the copies are queued behind the batch's kernels,
 * then one wait.  Fails with WSR_E_INTERNAL when the device raised an error
 * flag (hits / n_hits then hold no meaningful results). */
int wsr_batch_fetch(wsr_handle* h, wsr_batch* b, wsr_hit* hits, int32_t* n_hits);
int wsr_batch_stats_get(wsr_handle* h, wsr_batch* b, wsr_batch_stats* out);
/* as wsr_batch_fetch, but only the first `cols` (<= hit stride) entries of each
 * query: hits is nq x cols (a pitched copy; cols >= every query's k) */
int wsr_batch_fetch_cols(wsr_handle* h, wsr_batch* b, wsr_hit* hits, int32_t* n_hits, int32_t cols);
/* page-locked host memory for result arrays (their copies are then DMA'd) */
int wsr_pinned_alloc(uint64_t bytes, void** out);
void wsr_pinned_free(void* p);
/* 1 when the batch's last run has finished on the device, 0 while it runs */
int wsr_batch_ready(wsr_handle* h, wsr_batch* b);

/* ---- serving: micro-batcher over one handle --------------------------
 * The reference serves single queries from N gRPC worker threads sharing one
 * engine (grpc_server_impl.h:260-263,382-389).  wsr_server_search() may be
 * called from any number of threads; a dispatcher thread coalesces the calls
 * that arrive within window_us (or until max_batch are queued) into one GPU
 * batch; up to four batches are in flight, each on its own streams, and a
 * completer thread retires them in launch order and hands every caller its
 * result.  Each call blocks until its own result. */
typedef struct wsr_server wsr_server;
typedef struct wsr_serve_stats {
  uint64_t queries;      /* completed in the run */
  double seconds, qps;
  double p50_ms, p99_ms; /* per-query latency, submit -> result on the caller's thread */
  uint64_t batches;      /* GPU batches the dispatcher ran */
  double mean_batch;     /* queries per batch */
  /* where a query's latency goes (means over the run): */
  double queue_ms;       /* submit -> its batch launched (dispatcher) */
  double gpu_ms;         /* batch launched -> its end event seen by the completer */
  double handoff_ms;     /* end event seen -> the batch's last caller signalled */
} wsr_serve_stats;
/* Dispatch: a batch launches at once while fewer than `depth` batches are in
 * flight (WSR_SERVER_DEPTH, default 2: one running, one queued behind it on
 * the GPU, so batch size follows the load); with `depth` or more in flight it
 * launches when max_batch queries wait or the oldest has waited window_us, and
 * at most 4 batches are ever in flight. */
int wsr_server_open(wsr_handle* h, int32_t max_batch, int32_t window_us, wsr_server** out);
void wsr_server_close(wsr_server* s);
/* one query (k <= WSR_SERVER_MAX_K = WSR_MAX_K): hits receives n_hits <= k entries */
int wsr_server_search(wsr_server* s, const wsr_query* q, wsr_hit* hits, int32_t* n_hits);
/* closed-loop load (the reference client's threads, grpc_client_impl.h:557-620):
 * n_clients threads keep `depth` queries each in flight, drawn round-robin from
 * q[0..nq), for `seconds`; throughput and latency percentiles in *st */
int wsr_server_bench(wsr_server* s, const wsr_query* q, int32_t nq, int32_t n_clients,
                     int32_t depth, double seconds, wsr_serve_stats* st);

/* ---- doc-range shards (multi-GPU) ------------------------------------
 * A shard engine (wsr_open_opts.doc_lo/doc_hi) runs every query of a batch over
 * its doc range.  Queries are owned by contiguous slices of q_per_owner queries
 * (owner o = query / q_per_owner).  Per step, every shard's segment kernels
 * reduce each query's events to those of a heap run from empty over the shard
 * and append them to the owner's region of an exchange buffer; one all-to-all
 * moves the regions; the owner replays the events of all shards in shard (=
 * doc-id range) order.  Results are bit-identical to an unsharded run (see
 * DESIGN.md, "Why replaying events is exact").  A region = the {count, offset}
 * pairs of the owner's q_per_owner queries, padded to whole 16-byte events,
 * then a slot of `slot` events; a query whose events overflow the slot is
 * flagged (count -1 and an error flag that wsr_batch_fetch* reports). */
/* results of the batch's queries [q0, q0 + nq) (an owner's slice) */
int wsr_batch_fetch_range(wsr_handle* h, wsr_batch* b, int32_t q0, int32_t nq, wsr_hit* hits,
                          int32_t* n_hits);
/* the engine's HIP stream (a hipStream_t) for ordering the caller's work */
int wsr_stream(wsr_handle* h, void** stream);
/* the batch's own stream (a hipStream_t): its runs and its shard step's
 * emission are ordered on it */
int wsr_batch_stream(wsr_handle* h, wsr_batch* b, void** stream);
/* events appended per owner by the last shard step's emission (waits for the
 * batch), to size the slot */
int wsr_shard_fill(wsr_handle* h, wsr_batch* b, int32_t n_owners, int64_t* owner_totals);

/* ---- native RCCL exchange (one process per GPU; a C++ host needs no Python):
 * rank 0 makes the id, every rank opens the communicator with it (the id
 * travels by the caller's own rendezvous), then each step is one call: the
 * segments emit into per-owner regions ({count, offset} pairs + the event
 * slot) on the batch's stream, then, on the communicator's stream, one
 * ncclAllToAll of the regions over xGMI and the owner replay.  Nothing waits
 * on the host; wsr_batch_fetch* / wsr_batch_ready join the exchange.  Rank
 * r's owned queries are [r * q_per_owner, (r + 1) * q_per_owner) of a batch
 * of world * q_per_owner. */
#define WSR_COMM_ID_BYTES 128
typedef struct wsr_comm wsr_comm;
int wsr_comm_unique_id(uint8_t* id /* WSR_COMM_ID_BYTES */);
int wsr_comm_open(const uint8_t* id, int32_t world, int32_t rank, int32_t device, wsr_comm** out);
void wsr_comm_close(wsr_comm* c);
int wsr_shard_step(wsr_handle* h, wsr_batch* b, wsr_comm* c, int32_t q_per_owner, int64_t slot);
/* A step group: n batches of world * q_per_owner queries each, every one
 * emitted into its region of each owner's run of n regions (in one of the
 * communicator's exchange buffer sets), then ONE ncclAllToAll of the runs and
 * the n owner replays.  The same results as n wsr_shard_step calls, with one
 * collective's host cost instead of n.  The owner replays are deferred by
 * default (WSR_REPLAY_DEFER=0: not) into the lean kernels of the step group
 * two groups later; a fetch, wsr_batch_ready or the batch's next run enqueues
 * a still-pending one first.  A batch may be fetched, run or destroyed on
 * another thread than the one issuing steps (the communicator's lock orders
 * the deferred replays); close the communicator before the engine handles
 * whose batches it stepped. */
int wsr_shard_steps(wsr_handle* h, wsr_batch* const* b, int32_t n, wsr_comm* c, int32_t q_per_owner,
                    int64_t slot);
/* enqueue every deferred owner replay of the communicator (before timing the
 * whole job on a device synchronize, or closing) */
int wsr_comm_flush(wsr_comm* c);
/* What the communicator's step groups did so far: groups (collectives) and
 * steps (batches), and where each batch's owner replay ran -- in a later
 * group's lean kernel (deferred) or on the communicator's stream (not
 * deferred, wide queries, flushed by a fetch / flush / the batch's next step). */
typedef struct wsr_comm_stats {
  int64_t groups, steps, replays_in_lean, replays_on_stream;
} wsr_comm_stats;
int wsr_comm_stats_get(wsr_comm* c, wsr_comm_stats* out);
/* Loopback communicators (tests and one-GPU rehearsals, never a measurement):
 * the world ranks of a group live in ONE process, each with its own engine
 * (usually its doc-range shard image on the same device), and the step
 * groups' all-to-all is done by device copies between their exchange buffers
 * in place of ncclAllToAll -- the same regions, runs, slots and owner replays
 * as the RCCL path, so wsr_shard_steps at world > 1 runs exactly as it does
 * over xGMI except for the transport.  Every rank must submit the same step
 * groups in the same order (as with RCCL); a rank's collective completes on
 * its stream only once every rank has read its send buffer. */
typedef struct wsr_loopback wsr_loopback;
int wsr_loopback_create(int32_t world, wsr_loopback** out);
void wsr_loopback_destroy(wsr_loopback* l);   /* after closing its communicators */
int wsr_comm_open_loopback(wsr_loopback* l, int32_t rank, int32_t device, wsr_comm** out);
/* wsr_shard_step's two device halves with the transfer left to the caller (a
 * multi-rank rehearsal on one GPU, where RCCL refuses two ranks, or a host
 * exchange): the engine's own region buffers, in the exact layout the step's
 * ncclAllToAll moves -- world regions of *region_bytes (wsr_shard_step_regions);
 * region o = the {count, offset} pairs of owner o's q_per_owner queries,
 * padded to whole 16-byte events, then owner o's slot of `slot` events.
 * wsr_shard_step_emit runs the batch with fused emission and copies the send
 * regions to host_send (world * region_bytes); the caller delivers region o of
 * every rank g to rank o as its region g; wsr_shard_step_replay copies those
 * (host_recv, world * region_bytes) to the device and replays this rank's
 * owned queries on the batch's stream. */
int wsr_shard_step_regions(int32_t q_per_owner, int64_t slot, uint64_t* region_bytes);
int wsr_shard_step_emit(wsr_handle* h, wsr_batch* b, int32_t world, int32_t q_per_owner, int64_t slot,
                        void* host_send);
int wsr_shard_step_replay(wsr_handle* h, wsr_batch* b, int32_t rank, int32_t world, int32_t q_per_owner,
                          int64_t slot, const void* host_recv);
/* wsr_shard_step_replay deferred: the regions are copied to the device now and
 * the owner replay rides in the lean kernel of the next run of another batch
 * of the engine (a fetch, wsr_batch_ready, the batch's next run or its destroy
 * enqueues it on the batch's own stream first if no run has taken it). */
int wsr_shard_step_replay_deferred(wsr_handle* h, wsr_batch* b, int32_t rank, int32_t world, int32_t q_per_owner,
                                   int64_t slot, const void* host_recv);
/* wsr_shard_step_emit without the wait: the copy to host_send (page-locked,
 * wsr_pinned_alloc) is enqueued on the batch's stream; wsr_batch_stream_sync
 * waits for it, so a caller overlaps one batch's host exchange with the next
 * batch's kernels. */
int wsr_shard_step_emit_async(wsr_handle* h, wsr_batch* b, int32_t world, int32_t q_per_owner, int64_t slot,
                              void* host_send);
int wsr_batch_stream_sync(wsr_handle* h, wsr_batch* b);
/* Driver blocks per work item at most for this batch's runs (1..63, default
 * 63): shorter items cut a batch's latency (its longest item) at some cost in
 * throughput; the serving front end's batches use WSR_SERVER_ITEM_BLOCKS. */
int wsr_batch_set_item_blocks(wsr_handle* h, wsr_batch* b, int32_t blocks);

/* Decode one block of a list on the device (test hook for the decoder):
 * out[0..128) receives the block's values (doc ids when which == 0, tf when 1). */
int wsr_debug_decode_block(wsr_handle* h, int32_t list_id, int32_t block, int32_t which,
                           uint32_t* out, int32_t* count);

/* Raw per-workgroup counters of the last segment launch (diagnostics):
 * n_wg rows of `stride` u32 {survivors, driver blocks, other blocks, 0}.
 * out may be NULL to query. */
int wsr_debug_wg_stats(wsr_handle* h, wsr_batch* b, uint32_t* out, int32_t max_words,
                       int32_t* n_wg, int32_t* stride);

/* Fault injection (tests of the error paths): the next n batch runs -- plain
 * or the emission of a shard step -- fail with WSR_E_HIP before they enqueue
 * anything.  n = 0 clears it. */
int wsr_debug_fail_runs(int32_t n);

/* Host-only check of the dense-list image (no GPU): builds the image of
 * [doc_lo, doc_hi) (doc_hi 0 = all) with the given dense_div and looks each doc
 * up in the list's rank bitmap + tf bytes, exactly as the device probe does.
 * tf_out[i] = tf of docs[i] in the list, -1 when absent; *is_dense = 1 when
 * the list got a bitmap (otherwise tf_out is all -1). */
int wsr_debug_dense_lookup(const char* dir, uint32_t doc_lo, uint32_t doc_hi, uint32_t dense_div,
                           const char* term, const uint32_t* docs, int32_t n, int32_t* tf_out,
                           int32_t* is_dense);

/* ---- index building (host only; no GPU needed) ----------------------- */
typedef struct wsr_build_stats {
  int64_t n_docs, n_terms, n_postings, vacuum_bytes, docs_char4_ge_0x80;
  double avg_length;
} wsr_build_stats;

/* format: "TOKEN_ONLY" or "WITH_POSITIONS"; n_rows < 0 reads every row */
int wsr_build_from_linedoc(const char* linedoc, int64_t n_rows, const char* format,
                           const char* out_dir, wsr_build_stats* st);
/* the same, writing the two-way phrase bloom filters of every posting
 * (FlashEngineDumper::DumpPostingListWithBloom, flash_engine_dumper.h:412-525):
 * ratio / expected_entries as BloomDumper's (defaults 0.0009, 5) */
int wsr_build_from_linedoc_bloom(const char* linedoc, int64_t n_rows, const char* format,
                                 const char* out_dir, float ratio, int32_t expected_entries,
                                 wsr_build_stats* st);
int wsr_build_synthetic(const char* out_dir, int64_t n_docs, int64_t vocab, double zipf_s,
                        uint64_t seed, int32_t with_positions, int32_t threads,
                        wsr_build_stats* st);
/* BASELINE configs[2] stand-in: an index whose df histogram follows the
 * reference's en-Wikipedia one (tools/gen_synthetic_log.py:8-16) scaled by
 * term_scale, over n_docs docs (writer.h: WikiSpec); lists are streamed to
 * disk, so host memory does not grow with the corpus */
int wsr_build_wiki_standin(const char* out_dir, int64_t n_docs, double term_scale, uint64_t seed,
                           int32_t threads, wsr_build_stats* st);
/* the same df histogram with topic-clustered doc ids (writer.h WikiSpec::topics):
 * `topics` contiguous doc-id ranges, every term under N/16 postings draws
 * `affinity` of its docs from its `topics_per_term` home topics */
int wsr_build_wiki_standin_topics(const char* out_dir, int64_t n_docs, double term_scale, uint64_t seed,
                                  int32_t threads, int32_t topics, int32_t topics_per_term, double affinity,
                                  wsr_build_stats* st);
int wsr_gen_two_term_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                         const char* out_path, int64_t* n_written);
/* mixed 1-5 term AND log (AOL term-count shares; SURVEY 8d "C4") */
int wsr_gen_mixed_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                      const char* out_path, int64_t* n_written);
/* single-term log (tools/gen_synthetic_log.py:171-189, the run_exp.py:116-117
 * workloads type_single.docfreq_high / _low): terms drawn with replacement from
 * the df group, high != 0: df >= 10^4, else df < 10^4 */
int wsr_gen_single_term_log(const char* index_dir, int32_t high, int64_t n_queries, uint64_t seed,
                            const char* out_path, int64_t* n_written);
/* phrase log (tools/gen_synthetic_log.py:254-265) from a synthetic index's
 * phrase pool: one "t1 t2" per line, in double quotes */
int wsr_gen_phrase_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                       const char* out_path, int64_t* n_written);

#ifdef __cplusplus
}
#endif

#endif /* WISER_HIP_H */
