// Vacuum index writer (host, C++17): builds my.vacuum / my.tip / my.doc_length
// from a linedoc or from a seeded synthetic Zipf corpus.  Off the query hot
// path; it exists because the reference's own dumper cannot be built here
//  and the engine needs indexes in the reference layout.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace wiser {

struct SyntheticSpec {
  int64_t n_docs = 1000000;
  int64_t vocab = 500000;
  double zipf_s = 1.07;
  double len_mu = 5.0;
  double len_sigma = 0.8;
  int64_t len_max = 20000;
  uint64_t seed = 0x5EED2026ull;
  bool with_positions = true;  // write position + offset sections (reference layout)
  int threads = 0;             // 0 = hardware concurrency
};

// Two-way phrase bloom filters (bloom.h): off by default; the reference's
// BloomDumper defaults are ratio 0.0009, 5 expected entries (bloom_filter.h:650-655).
struct BloomSpec {
  bool on = false;
  float ratio = 0.0009f;
  int entries = 5;
};

struct BuildStats {
  int64_t n_docs = 0;
  int64_t n_terms = 0;
  int64_t n_postings = 0;
  int64_t vacuum_bytes = 0;
  int64_t docs_char4_ge_0x80 = 0;  // lengths >= 2^18: reference indexes its cache with a
                                   // negative signed char (UB, scoring.h:65-69)
  double avg_length = 0;
};

// format: "TOKEN_ONLY" or "WITH_POSITIONS" (engine_loader.h:53-96).
// Throws std::runtime_error on malformed input.
// bloom.on: every posting also gets its "begin" / "end" bloom filter over the
// terms before / after each occurrence of the term in the doc (from positions).
BuildStats build_from_linedoc(const std::string& linedoc, int64_t n_rows,
                              const std::string& format, const std::string& out_dir,
                              const BloomSpec& bloom = BloomSpec());

BuildStats build_synthetic(const SyntheticSpec& spec, const std::string& out_dir);

// English-Wikipedia-shaped stand-in (BASELINE configs[2], "C3"): no Wikipedia
// dump exists offline, so the posting lists are drawn straight from the df
// histogram the reference records for its en-Wikipedia index
// (tools/gen_synthetic_log.py:8-16: terms per df decade 4,996,891 / 520,675 /
// 94,721 / 22,139 / 5,717 / 1,434 / 38), times term_scale.  Per term: df from
// a power law inside its decade (density ~ df^-1.6, the decade-to-decade
// ratio of that histogram), df distinct uniform doc ids, tf = 1 + Exp(lambda)
// with lambda growing with the doc's verbosity (lognormal) and the term's
// df / N.  Doc length = sum of its tfs (every token is indexed), stored as
// Char4 with the reference's incremental mean.  Lists are generated per term
// from per-term seeds and written in term order, a few thousand at a time, so
// host memory stays bounded whatever the corpus size; position bags hold tf
// consecutive positions and the matching offset pairs (reference layout).
struct WikiSpec {
  int64_t n_docs = 5500000;
  double term_scale = 1.0;
  uint64_t seed = 0x3C3C2026ull;
  int threads = 0;
  // Topic-clustered variant (topics > 0; 0 = the uniform stand-in above): doc
  // ids are cut into `topics` contiguous ranges (a topic's articles sit
  // together, as a dump's ids follow creation order by portal / category), every
  // term below N/16 postings whose draws keep its home topics at most half full
  // gets topics_per_term home topics (from its id) and draws `affinity` of its
  // doc ids inside them, the rest uniformly; the df of every term, and so the
  // df histogram, is unchanged.  Terms with a common home topic then co-occur
  // far more often than independent draws.
  int topics = 0;
  int topics_per_term = 2;
  double affinity = 0.6;
};
BuildStats build_wiki_standin(const WikiSpec& spec, const std::string& out_dir);

// Two-term query log restating tools/gen_synthetic_log.py:191-214 over the
// df table of an index: group "low" = floor(log10 df) in 0..3, "high" = 4..6;
// each term picks a group uniformly then a term uniformly; t1 != t2; the pair
// is sorted; duplicates are dropped until n_queries distinct queries exist.
// Written one query per line (query_pool.h:319-378 format).
int64_t gen_two_term_log(const std::string& index_dir, int64_t n_queries, uint64_t seed,
                         const std::string& out_path);

// Mixed 1-5 term AND log (BASELINE configs[3], SURVEY 8d "C4"): terms per query
// by the AOL log's shares (36.8/25.2/17.3/10.0/5.3 %, renormalised), each term
// drawn as in gen_two_term_log, distinct and sorted, distinct queries.
int64_t gen_mixed_log(const std::string& index_dir, int64_t n_queries, uint64_t seed,
                      const std::string& out_path);

// Single-term query log restating tools/gen_synthetic_log.py:171-189
// (single_term_queries, the run_exp.py:116-117 workloads
// type_single.docfreq_high / _low): n terms drawn with replacement
// (rand_items_from_set, :47-58) from the whole df group, "high" (df >= 10^4)
// or "low" (df < 10^4).
int64_t gen_single_term_log(const std::string& index_dir, bool high, int64_t n_queries, uint64_t seed,
                            const std::string& out_path);

// Phrase query log restating tools/gen_synthetic_log.py:254-265: n phrases
// drawn without replacement from the index's phrase pool (phrases.txt, written
// by build_synthetic), one per line in double quotes.
int64_t gen_phrase_log(const std::string& index_dir, int64_t n_queries, uint64_t seed,
                       const std::string& out_path);

}  // namespace wiser
