// Snippets of result entries (SearchQuery::return_snippets), host side.
//
// The reference builds a snippet per top-k entry on the CPU after ranking
// (VacuumEngine::Search -> GenerateSnippet, vacuum_engine.h:243-253,286-296):
//   1. the (start, end) char offsets of every query term in the doc, read from
//      the term's offset box at the doc's posting (LazyBoundedOffsetPairIterator,
//      flash_iterators.h:711-769); for a phrase query only the offsets of the
//      matched occurrences (ResultDocEntry::FilterOffsetByPosition over the
//      PhraseQueryProcessor2 table, query_processing.h:446-492,170-382);
//   2. the doc text from the doc store (docstore.h);
//   3. SimpleHighlighter::highlightOffsetsEnums (highlighter.h:297-456):
//      sentences scored by a BM25-like passage score, the best n_passages kept,
//      printed in text order with <b>..<\b> around the matches.
// Here the GPU has already produced the top-k; this stage reads the k docs'
// posting blocks straight from the mapped index file.  Everything is
// recomputed per entry from the doc id, so no per-query iterator state is kept.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <unordered_map>
#include <string>
#include <utility>
#include <vector>

#include "docstore.h"
#include "index.h"

namespace wiser {

using OffsetPair = std::pair<int, int>;

// Decoded skip rows per list, shared by the threads of the snippet stage
// (the reference re-decodes a list's whole skip list for every iterator,
// flash_iterators.h:946-948; a snippet needs them for k docs per query).
class SkipRowCache {
 public:
  explicit SkipRowCache(const VacuumIndex& idx) : idx_(idx) {}
  // (entries are never dropped, so the reference stays valid; lookups take a
  // shared lock, a first decode an exclusive one)
  const std::vector<SkipRow>& get(int32_t list) const;

 private:
  const VacuumIndex& idx_;
  mutable std::shared_mutex mu_;
  mutable std::unordered_map<int32_t, std::unique_ptr<const std::vector<SkipRow>>> rows_;
};

// The snippet of doc `doc` for a query of n list ids (query order).  The doc
// must hold every term (it is a result entry); throws std::runtime_error otherwise.
std::string make_snippet(const VacuumIndex& idx, const SkipRowCache& rows, const DocStore& docs,
                         const int32_t* lists, int n, bool phrase, int32_t doc, int n_passages);

// SimpleHighlighter::highlightOffsetsEnums over explicit per-term offset lists
// (each non-empty).
std::string highlight_offsets(const std::vector<std::vector<OffsetPair>>& terms, int n_passages,
                              const std::string& text);

}  // namespace wiser
