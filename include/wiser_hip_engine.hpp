// wiser_hip_engine.hpp -- C++ host class above the C ABI (wiser_hip.h) that
// keeps the reference's operator surface:
//   SearchEngineServiceNew::{Load, Search, TermCount, PostinglistSizes}
//   (src/qq_mem/src/engine_services.h:14-27, vacuum_engine.h:119-258)
//   SearchQuery / SearchResultEntry / SearchResult (types.h:205-346)
// Header-only; link libwiser_hip.so.  Errors: the reference aborts (LOG(FATAL))
// on corrupt data; this class throws std::runtime_error instead, and keeps the
// reference's empty-result rules (n_results == 0, any missing term).
#ifndef WISER_HIP_ENGINE_HPP
#define WISER_HIP_ENGINE_HPP

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "wiser_hip.h"

namespace wiser_hip {

typedef std::vector<std::string> TermList;

struct SearchQuery {  // types.h:205-256
  SearchQuery() {}
  explicit SearchQuery(const TermList& t) : terms(t) {}
  SearchQuery(const TermList& t, bool snippets) : terms(t), return_snippets(snippets) {}
  TermList terms;
  int n_results = 5;
  bool return_snippets = false;  // entries get snippets (host stage, wsr_snippet)
  int n_snippet_passages = 3;
  bool is_phrase = false;        // >= 2 terms: consecutive positions required (WSR_QUERY_PHRASE)
};

struct SearchResultEntry {  // types.h:259-274
  std::string snippet;
  int doc_id = 0;
  double doc_score = 0;
};

struct SearchResult {  // types.h:297-346
  std::vector<SearchResultEntry> entries;
  std::vector<int> doc_freqs;
  std::size_t Size() const { return entries.size(); }
  const SearchResultEntry& operator[](int i) const { return entries[i]; }
};

inline void check(int rc) {
  if (rc != WSR_OK) throw std::runtime_error(std::string("wiser_hip: ") + wsr_last_error());
}

class VacuumHipEngine {
 public:
  // bloom_enable_factor: CreateSearchEngine's (engine_factory.h:33-34), default 1
  explicit VacuumHipEngine(const std::string& dir, int device = 0, int bloom_enable_factor = 1)
      : dir_(dir), device_(device), bloom_factor_(bloom_enable_factor) {}
  ~VacuumHipEngine() { wsr_close(h_); }
  VacuumHipEngine(const VacuumHipEngine&) = delete;
  VacuumHipEngine& operator=(const VacuumHipEngine&) = delete;

  void Load() {
    if (h_) throw std::runtime_error("Engine is already loaded.");
    wsr_open_opts o{device_, 0, 0, 0, 1, bloom_factor_};   // positions: phrase queries served
    check(wsr_open(dir_.c_str(), &o, &h_));
  }

  int TermCount() const {
    int32_t n = 0;
    check(wsr_term_count(h_, &n));
    return n;
  }

  std::map<std::string, int> PostinglistSizes(const TermList& terms) const {
    std::map<std::string, int> out;
    for (const auto& t : terms) {
      int32_t id, df;
      check(wsr_lookup(h_, t.c_str(), &id, &df));
      if (id >= 0) out[t] = df;
    }
    return out;
  }

  SearchResult Search(const SearchQuery& q) { return SearchBatch({q})[0]; }

  // VacuumEngine::GenerateSnippet (vacuum_engine.h:286-296) for a result entry
  std::string Snippet(const wsr_query& q, int doc_id, int n_passages) const {
    std::string s(4096, '\0');
    int32_t n = 0;
    check(wsr_snippet(h_, &q, doc_id, n_passages, &s[0], static_cast<int32_t>(s.size()), &n));
    if (n > static_cast<int32_t>(s.size())) {
      s.assign(n, '\0');
      check(wsr_snippet(h_, &q, doc_id, n_passages, &s[0], n, &n));
    }
    s.resize(n);
    return s;
  }

  std::vector<SearchResult> SearchBatch(const std::vector<SearchQuery>& qs) {
    std::vector<wsr_query> in(qs.size());
    std::vector<std::vector<int32_t>> more(qs.size());   // terms past WSR_MAX_TERMS
    std::vector<std::vector<int>> freqs(qs.size());
    std::vector<bool> empty(qs.size(), false);
    int stride = 1;
    for (size_t i = 0; i < qs.size(); ++i) {
      const SearchQuery& q = qs[i];
      if (q.terms.size() > WSR_MAX_QUERY_TERMS || q.n_results > WSR_MAX_K)
        throw std::runtime_error("query over the engine limits");
      wsr_query& w = in[i];
      w.more_ids = nullptr;
      w.k = q.n_results < 0 ? 0 : q.n_results;
      w.flags = (q.is_phrase && q.terms.size() > 1) ? WSR_QUERY_PHRASE : 0;
      bool missing = q.terms.empty();
      for (size_t t = 0; t < q.terms.size(); ++t) {
        int32_t id, df;
        check(wsr_lookup(h_, q.terms[t].c_str(), &id, &df));
        if (t < WSR_MAX_TERMS) w.list_ids[t] = id;
        else more[i].push_back(id);
        if (id < 0) missing = true;
        freqs[i].push_back(df);
      }
      if (!more[i].empty()) w.more_ids = more[i].data();
      empty[i] = missing || w.k == 0;
      w.n_terms = empty[i] ? 0 : static_cast<int32_t>(q.terms.size());
      if (w.k > stride) stride = w.k;
    }
    std::vector<wsr_hit> hits(qs.size() * stride);
    std::vector<int32_t> nh(qs.size());
    if (!qs.empty())
      check(wsr_search_batch(h_, in.data(), static_cast<int32_t>(qs.size()), stride, hits.data(),
                             nh.data()));
    std::vector<SearchResult> out(qs.size());
    for (size_t i = 0; i < qs.size(); ++i) {
      if (empty[i]) continue;  // vacuum_engine.h:206-215: nothing, doc_freqs unset
      out[i].doc_freqs = freqs[i];
      for (int j = 0; j < nh[i]; ++j) {
        SearchResultEntry e;
        e.doc_id = hits[i * stride + j].doc_id;
        e.doc_score = hits[i * stride + j].score;
        out[i].entries.push_back(e);
      }
    }
    // vacuum_engine.h:248-252: snippets of every entry, the batch at once on the
    // host's threads, one call per distinct n_snippet_passages
    std::map<int, std::vector<int32_t>> groups;   // n_passages -> n_hits masked to that group
    for (size_t i = 0; i < qs.size(); ++i) {
      if (!qs[i].return_snippets || empty[i] || nh[i] == 0) continue;
      auto& g = groups[qs[i].n_snippet_passages];
      if (g.empty()) g.assign(qs.size(), 0);
      g[i] = nh[i];
    }
    for (auto& kv : groups) {
      std::vector<uint64_t> ends(qs.size() * stride);
      uint64_t total = 0;
      std::string buf(1 << 16, '\0');
      int rc = wsr_snippets_batch(h_, in.data(), static_cast<int32_t>(qs.size()), hits.data(), kv.second.data(),
                                  stride, kv.first, 0, &buf[0], buf.size(), ends.data(), &total);
      if (rc == WSR_E_LIMIT && total > buf.size()) {
        buf.assign(total, '\0');
        rc = wsr_snippets_batch(h_, in.data(), static_cast<int32_t>(qs.size()), hits.data(), kv.second.data(),
                                stride, kv.first, 0, &buf[0], buf.size(), ends.data(), &total);
      }
      check(rc);
      uint64_t at = 0;
      for (size_t i = 0; i < qs.size(); ++i)
        for (int j = 0; j < stride; ++j) {
          const uint64_t e = ends[i * stride + j];
          if (j < kv.second[i]) out[i].entries[j].snippet.assign(buf, at, e - at);
          at = e;
        }
    }
    return out;
  }

 private:
  std::string dir_;
  int device_;
  int bloom_factor_ = 1;
  wsr_handle* h_ = nullptr;
};

}  // namespace wiser_hip

#endif
