/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * (tailuzhecom/wiser, src/qq_mem/src) conjunctive-query + BM25 + top-k path,
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
 * the checker.  The product (wiser_amd, libwiser_hip.so) never links or calls
 * this library.
 *
 * Parity pinning: the reference C++ could not be built or run here (the
 * environment refused it), so this restatement is pinned
 * by the reference's own known-answer tests (tests/test_oracle_kat.py cites
 * each one) and by the Vacuum == QqMem differential test of tests_15.cc:158-210
 * re-run over the reference's own fixture files.
 */
#ifndef WISER_ORACLE_H
#define WISER_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_vacuum orc_vacuum;
typedef struct orc_qqmem orc_qqmem;

const char* orc_last_error(void);

/* ---- codecs (known-answer tests) ------------------------------------- */
int orc_num_bits(uint32_t v);
uint8_t orc_char4_encode(uint32_t v);
uint32_t orc_char4_decode(uint8_t c);
int orc_varint_encode(uint64_t v, uint8_t* out);               /* returns bytes */
int orc_varint_decode(const uint8_t* in, uint64_t* v);          /* returns bytes */
/* LittlePackedIntsWriter::Serialize: 2-byte header + 16*b bytes; returns size */
int orc_pack128(const uint32_t* values, uint8_t* out);
/* LittlePackedIntsReader::DecodeToCache over a serialised pack */
int orc_unpack128(const uint8_t* pack, uint32_t* out);
double orc_es_idf(int doc_count, int doc_freq);
double orc_es_tfnorm(int freq, int field_length, double avg);  /* calc_es_tfnorm */
double orc_tfnorm_lossy(double avg, int freq, uint8_t char4);   /* Bm25Similarity */

/* ---- Vacuum engine restatement --------------------------------------- */
orc_vacuum* orc_vacuum_open(const char* dir);
void orc_vacuum_close(orc_vacuum* h);
int orc_vacuum_term_count(orc_vacuum* h);
int orc_vacuum_n_docs(orc_vacuum* h);
/* posting list size (0 if absent) */
int orc_vacuum_df(orc_vacuum* h, const char* term);
/* iterate a whole list through DocIdIterator / TermFreqIterator */
int orc_vacuum_list(orc_vacuum* h, const char* term, uint32_t* docs, uint32_t* tfs, int cap);
/* doc-id iterator ops (0 Advance, 1 SkipTo posting, 2 SkipForward doc) ->
 * {PostingIndex, Value or -1, IsEnd} per op */
int orc_vacuum_docid_ops(orc_vacuum* h, const char* term, const int64_t* ops, int n, int64_t* out);
/* VacuumEngine::Search: returns n entries (<= k), fills docs/scores and doc_freqs
 * (doc_freqs filled only when every term exists, as the reference). */
int orc_vacuum_search(orc_vacuum* h, const char* const* terms, int n_terms, int k,
                      int32_t* docs, double* scores, int32_t* doc_freqs);
/* The same with SearchQuery::is_phrase (QueryProcessor's position check). */
int orc_vacuum_search_phrase(orc_vacuum* h, const char* const* terms, int n_terms, int k,
                             int is_phrase, int32_t* docs, double* scores, int32_t* doc_freqs);
/* bloom: QueryProcessor's bloom_enable_factor (1 by default, 0 = never use);
 * whether the index carries bloom filters; checks / prunes counted so far;
 * one posting's filter checked for an element (1 may be present, 0 not) */
void orc_vacuum_set_bloom_factor(orc_vacuum* h, int factor);
int orc_vacuum_has_bloom(orc_vacuum* h);
void orc_bloom_stats(int64_t* checks, int64_t* pruned);
int orc_vacuum_bloom_check(orc_vacuum* h, const char* term, int posting, int side, const char* elem);
/* positions of posting `posting` of a term (PositionPostingBagIterator); returns tf */
int orc_vacuum_positions(orc_vacuum* h, const char* term, int posting, uint32_t* out, int cap);
/* PhraseQueryProcessor2 over plain sorted position lists: NumOfMatches, and the
 * matched positions per list in table[list * cap + match] */
int orc_phrase_lists(const uint32_t* const* lists, const int* sizes, int n_lists, int32_t* table,
                     int cap);
/* SearchQuery::return_snippets: as orc_vacuum_search_phrase, plus each entry's
 * snippet (n_passages passages) concatenated into buf; snip_end[i] = end of
 * entry i's snippet.  Needs the doc store (my.fdx / my.fdt). */
int orc_vacuum_search_snippets(orc_vacuum* h, const char* const* terms, int n_terms, int k,
                               int is_phrase, int n_passages, int32_t* docs, double* scores,
                               char* buf, int64_t cap, int64_t* snip_end);
/* SimpleHighlighter over explicit offsets (pairs: sum(counts) start,end pairs) */
int orc_highlight(const int32_t* pairs, const int32_t* counts, int n_terms, int n_passages,
                  const char* doc, char* out, int cap);
/* ChunkedDocStoreReader::Get; returns the text length */
int64_t orc_docstore_get(orc_vacuum* h, int doc, char* out, int64_t cap);
/* offset pairs of one posting (OffsetPostingBagIterator); returns tf */
int orc_vacuum_offsets(orc_vacuum* h, const char* term, int posting, int32_t* out, int cap);
/* Many queries: queries are '\n'-separated lines of ' '-separated terms (a line
 * in double quotes is a phrase query).
 * Outputs are nq*k arrays plus n per query.  threads >= 1.  Returns nq. */
int orc_vacuum_search_lines(orc_vacuum* h, const char* text, int k, int threads,
                            int32_t* docs, double* scores, int32_t* n_out, int max_q);
/* CPU-baseline timing: `threads` persistent workers run the log's queries
 * (cycled) for `seconds`; no spawn, parse or result conversion inside the
 * interval.  Outputs the queries completed and the interval.  Returns 0. */
int orc_vacuum_bench_lines(orc_vacuum* h, const char* text, int k, int threads, double seconds,
                           int64_t* done_out, double* elapsed_out);

/* ---- QqMem (in-memory, varint postings) engine restatement ----------- */
orc_qqmem* orc_qqmem_load(const char* linedoc, int64_t n_rows, const char* format);
void orc_qqmem_close(orc_qqmem* h);
int orc_qqmem_term_count(orc_qqmem* h);
int orc_qqmem_search(orc_qqmem* h, const char* const* terms, int n_terms, int k,
                     int32_t* docs, double* scores, int32_t* doc_freqs);
/* the term's varint posting list through PostingListDeltaIterator; returns its size */
int orc_qqmem_list(orc_qqmem* h, const char* term, uint32_t* docs, uint32_t* tfs, int cap);
/* one posting's offset pairs (2 per pair) and positions; returns its doc id */
int orc_qqmem_posting(orc_qqmem* h, const char* term, int posting, uint32_t* offs, int* n_offs,
                      uint32_t* pos, int* n_pos, int cap);
/* StandardPosting::Encode (posting.h:130-151); returns the byte count */
int orc_posting_encode(uint32_t doc_delta, uint32_t tf, const uint32_t* offs, int n_pairs,
                       const uint32_t* pos, int n_pos, uint8_t* out, int cap);
/* PostingListDelta skip index and iterator walks (posting_list_delta.h:161-470) */
int orc_pld_probe(const uint32_t* docs, const uint32_t* tfs, int n, int span, uint32_t* skip_prev,
                  uint64_t* skip_off, int* n_skip, int32_t* has_skip, uint32_t* span_doc,
                  const uint32_t* targets, int n_targets, int32_t* found);

/* counters of reference-UB situations hit so far (negative cache index) */
int64_t orc_ub_negative_char_index(void);

#ifdef __cplusplus
}
#endif

#endif
