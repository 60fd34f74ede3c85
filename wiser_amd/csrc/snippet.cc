// Snippets of result entries (see snippet.h).
#include "snippet.h"

#include <algorithm>
#include <cmath>
#include <memory>
#include <queue>
#include <stdexcept>

#include "format.h"

namespace wiser {
namespace {

// `take` entries of a position / offset box, starting `skip` entries after
// entry `idx` of the blob at file offset `blob`.  A box is a run of 128-value
// packs closed by one VInts blob (CozyBoxIterator, flash_iterators.h:280-412).
std::vector<uint32_t> box_entries(const uint8_t* file, uint64_t file_len, uint64_t blob, uint64_t idx,
                                  uint64_t skip, uint64_t take) {
  std::vector<uint32_t> out;
  out.reserve(take);
  const uint8_t* end = file + file_len;
  uint64_t at = idx + skip;   // entry index counted from the start of `blob`
  uint32_t vals[kPackSize];
  while (out.size() < take) {
    if (blob >= file_len) throw std::runtime_error("box runs past the index file");
    const uint8_t* p = file + blob;
    if (p[0] == kPackMagic) {
      const uint64_t bytes = 2 + 16ull * p[1];
      if (at >= kPackSize) { at -= kPackSize; blob += bytes; continue; }
      if (!host_decode_block(p, end, kPackSize, false, 0, vals)) throw std::runtime_error("bad box pack");
      for (uint64_t j = at; j < kPackSize && out.size() < take; ++j) out.push_back(vals[j]);
      at = 0;
      blob += bytes;
    } else if (p[0] == kVIntsMagic) {   // the box's last blob
      uint64_t nb = 0;
      const int l = get_varint(p + 1, end, &nb);
      if (!l) throw std::runtime_error("bad box VInts header");
      const uint8_t* q = p + 1 + l;
      const uint8_t* qe = q + nb;
      if (qe > end) throw std::runtime_error("box VInts runs past the index file");
      for (uint64_t j = 0; q < qe && out.size() < take; ++j) {
        uint64_t v = 0;
        const int m = get_varint(q, qe, &v);
        if (!m) throw std::runtime_error("bad box varint");
        q += m;
        if (j >= at) out.push_back(static_cast<uint32_t>(v));
      }
      if (out.size() < take) throw std::runtime_error("box shorter than its postings' tfs");
    } else {
      throw std::runtime_error("box blob format");
    }
  }
  return out;
}

// A doc's posting in one list: its skip row, slot in the row's block and the
// block's tfs (the bag of slot j starts after the tfs of slots 0..j-1).
struct Posting {
  SkipRow row;
  int slot = 0;
  int cnt = 0;
  uint32_t tf[kPackSize];
};

Posting locate(const VacuumIndex& idx, const SkipRowCache& cache, int32_t list, int32_t doc) {
  const std::vector<SkipRow>& rows = cache.get(list);
  const uint32_t df = idx.df(list);
  if (rows.empty()) throw std::runtime_error("empty posting list");
  // block r holds the docs in (prev_doc[r], prev_doc[r + 1]]; row 0 starts at 0
  const uint32_t d = static_cast<uint32_t>(doc);
  size_t r = std::partition_point(rows.begin() + 1, rows.end(),
                                  [&](const SkipRow& s) { return s.prev_doc < d; }) - rows.begin() - 1;
  Posting P;
  P.row = rows[r];
  P.cnt = static_cast<int>(std::min<uint64_t>(kPackSize, df - kPackSize * r));
  const uint8_t* end = idx.file() + idx.file_bytes();
  uint32_t ids[kPackSize];
  if (!host_decode_block(idx.file() + P.row.doc_off, end, P.cnt, true, P.row.prev_doc, ids) ||
      !host_decode_block(idx.file() + P.row.tf_off, end, P.cnt, false, 0, P.tf))
    throw std::runtime_error("bad posting block");
  const uint32_t* hit = std::lower_bound(ids, ids + P.cnt, d);
  if (hit == ids + P.cnt || *hit != d) throw std::runtime_error("doc is not in the posting list");
  P.slot = static_cast<int>(hit - ids);
  return P;
}

// The posting's bag, prefix-summed from 0: positions (pairs = false) or
// (start, end) offsets flattened (pairs = true, 2 x tf entries).
std::vector<uint32_t> bag(const VacuumIndex& idx, const Posting& P, bool pairs) {
  const uint64_t per = pairs ? 2 : 1;
  uint64_t skip = 0;
  for (int i = 0; i < P.slot; ++i) skip += P.tf[i] * per;
  std::vector<uint32_t> v = box_entries(idx.file(), idx.file_bytes(), pairs ? P.row.off_off : P.row.pos_off,
                                        pairs ? P.row.off_idx : P.row.pos_idx, skip, P.tf[P.slot] * per);
  uint32_t acc = 0;
  for (auto& x : v) { acc += x; x = acc; }
  return v;
}

std::vector<OffsetPair> as_pairs(const std::vector<uint32_t>& flat) {
  std::vector<OffsetPair> v(flat.size() / 2);
  for (size_t i = 0; i < v.size(); ++i)
    v[i] = OffsetPair(static_cast<int>(flat[2 * i]), static_cast<int>(flat[2 * i + 1]));
  return v;
}

// Term appearances (index of the occurrence in the term's position list) of
// every phrase match, per term: PhraseQueryProcessor2's table
// (ProcessTwoTerm :264-310, ProcessGeneral :312-336) over position arrays.
std::vector<std::vector<int>> phrase_table(const std::vector<std::vector<uint32_t>>& pos) {
  const int n = static_cast<int>(pos.size());
  std::vector<std::vector<int>> t(n);
  if (n == 2) {
    const auto& A = pos[0];
    const auto& B = pos[1];
    size_t ia = 0, ib = 0;             // next entry to take
    int pa = -100, pb = -200;          // last taken (pb shifted by one)
    bool done = false;
    auto take_a = [&]() { if (ia < A.size()) pa = static_cast<int>(A[ia++]); else done = true; };
    auto take_b = [&]() { if (ib < B.size()) pb = static_cast<int>(B[ib++]) - 1; else done = true; };
    while (!done) {
      if (pa < pb) {
        take_a();
      } else if (pa > pb) {
        take_b();
      } else {
        t[0].push_back(static_cast<int>(ia) - 1);
        t[1].push_back(static_cast<int>(ib) - 1);
        take_a();
        take_b();
      }
    }
    return t;
  }
  std::vector<size_t> at(n, 0);       // entries taken per term
  std::vector<int> last(n);
  for (int i = 0; i < n; ++i) {
    if (pos[i].empty()) return t;
    last[i] = static_cast<int>(pos[i][0]);
    at[i] = 1;
  }
  // advance every term to an adjusted position >= target; false when one runs out
  auto reach = [&](int target) {
    for (int i = 0; i < n; ++i) {
      while (at[i] < pos[i].size() && last[i] - i < target) last[i] = static_cast<int>(pos[i][at[i]++]);
      if (at[i] >= pos[i].size() && last[i] - i < target) return false;
    }
    return true;
  };
  for (;;) {
    int target = 0;
    for (int i = 0; i < n; ++i) target = std::max(target, last[i] - i);
    if (!reach(target)) break;
    bool all = true;
    for (int i = 0; i < n && all; ++i) all = last[i] - i == target;
    if (all) {
      for (int i = 0; i < n; ++i) t[i].push_back(static_cast<int>(at[i]) - 1);
      if (!reach(target + 1)) break;
    }
  }
  return t;
}

// ---------------------------------------------------------- highlighter ----
// float arithmetic as SimpleHighlighter (pivot 87, k1 1.2, b 0.75, :443-455)
constexpr float kPivot = 87, kK1 = 1.2f, kB = 0.75f;
float start_weight(int start) { return 1 + 1 / static_cast<float>(std::log(static_cast<float>(kPivot + start))); }
float freq_weight(int freq, int len) {
  const float norm = kK1 * ((1 - kB) + kB * (len / kPivot));
  return freq / (freq + norm);
}

struct Sentence {   // SentenceBreakIteratorNew::next(int offset) (:176-192)
  int start = -1, end = -1;
  bool around(const std::string& s, int offset) {
    const int last = static_cast<int>(s.size()) - 1;
    if (offset > last) return false;
    for (end = offset; end < last && s[end] != '.'; ++end) {}
    start = std::max(0, offset - 1);
    while (start > 0 && s[start] != '.') --start;
    if (start > 0) ++start;
    return true;
  }
};

struct Passage {
  int start = -1, end = -1;
  float score = 0;
  std::vector<OffsetPair> hits;
  void clear() { start = end = -1; score = 0; hits.clear(); }
  // Passage::to_string (:97-115): tags inserted from the last match backwards
  std::string render(const std::string& s) {
    std::string r = s.substr(start, end - start + 1) + "\n";
    std::sort(hits.begin(), hits.end(), [](const OffsetPair& a, const OffsetPair& b) { return a.first > b.first; });
    for (const auto& h : hits) {
      r.insert(h.second - start + 1, "<\\b>");
      r.insert(std::max(0, h.first - start), "<b>");
    }
    return r;
  }
};

struct Cursor {   // one term's offsets (Offset_Iterator, weight 1)
  const std::vector<OffsetPair>* v;
  size_t i;
  int start, end;
  void step() {
    if (++i < v->size()) { start = (*v)[i].first; end = (*v)[i].second; }
    else start = end = -1;
  }
};

}  // namespace

std::string highlight_offsets(const std::vector<std::vector<OffsetPair>>& terms, int n_passages,
                              const std::string& text) {
  if (terms.empty()) return "";
  const size_t cap = static_cast<size_t>(n_passages);
  auto by_start = [](const Cursor& a, const Cursor& b) { return a.start > b.start; };
  std::priority_queue<Cursor, std::vector<Cursor>, decltype(by_start)> cursors(by_start);
  for (const auto& t : terms) {
    if (t.empty()) throw std::runtime_error("highlight: a term without offsets");
    cursors.push(Cursor{&t, 0, t[0].first, t[0].second});
  }
  auto by_score = [](Passage* const& a, Passage* const& b) { return a->score > b->score; };
  std::priority_queue<Passage*, std::vector<Passage*>, decltype(by_score)> best(by_score);
  std::vector<std::unique_ptr<Passage>> owned;
  auto make = [&owned]() { owned.emplace_back(new Passage()); return owned.back().get(); };
  Sentence sent;
  float floor = -1;   // score of the weakest kept passage
  Passage* p = make();
  while (!cursors.empty()) {
    Cursor c = cursors.top();
    cursors.pop();
    if (c.start == -1) continue;
    if (c.end > p->end) {   // the match lies past the current sentence: close it
      if (p->start >= 0) {
        p->score = p->score * start_weight(p->start);
        if (best.size() == cap && p->score <= floor) {
          p->clear();
        } else {
          best.push(p);
          if (best.size() > cap) { p = best.top(); best.pop(); p->clear(); }
          else p = make();
          floor = best.top()->score;
        }
      }
      if (!sent.around(text, c.end)) break;
      p->start = sent.start;
      p->end = sent.end;
    }
    int freq = 0;   // this term's matches inside the sentence
    for (;;) {
      ++freq;
      p->hits.emplace_back(c.start, c.end);
      c.step();
      if (c.start == -1) break;
      if (c.end > p->end) { cursors.push(c); break; }
    }
    p->score = p->score + 1 * freq_weight(freq, p->end - p->start + 1);
  }
  p->score = p->score * start_weight(p->start);
  if (p->score > 0) {
    if (best.size() < cap) best.push(p);
    else if (p->score > floor) { best.pop(); best.push(p); }
  }
  std::vector<Passage*> keep;
  for (; !best.empty(); best.pop()) keep.push_back(best.top());
  std::sort(keep.begin(), keep.end(), [](Passage* const& a, Passage* const& b) { return a->start < b->start; });
  std::string out;
  for (Passage* k : keep) out += k->render(text);
  return out;
}

const std::vector<SkipRow>& SkipRowCache::get(int32_t list) const {
  {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto it = rows_.find(list);
    if (it != rows_.end()) return *it->second;
  }
  std::unique_ptr<const std::vector<SkipRow>> r(new std::vector<SkipRow>(idx_.rows(list)));
  std::unique_lock<std::shared_mutex> g(mu_);
  return *rows_.emplace(list, std::move(r)).first->second;   // (a racing decode is dropped)
}

std::string make_snippet(const VacuumIndex& idx, const SkipRowCache& rows, const DocStore& docs,
                         const int32_t* lists, int n, bool phrase, int32_t doc, int n_passages) {
  std::vector<Posting> ps;
  for (int i = 0; i < n; ++i) ps.push_back(locate(idx, rows, lists[i], doc));
  std::vector<std::vector<OffsetPair>> terms;
  if (phrase && n > 1) {
    // only the matched occurrences (FilterOffsetByPosition); the doc is a
    // result entry, so it holds the phrase
    std::vector<std::vector<uint32_t>> pos;
    for (const auto& p : ps) pos.push_back(bag(idx, p, false));
    const std::vector<std::vector<int>> t = phrase_table(pos);
    for (int i = 0; i < n && !t[i].empty(); ++i) {
      const std::vector<OffsetPair> all = as_pairs(bag(idx, ps[i], true));
      std::vector<OffsetPair> row;
      for (int a : t[i]) {
        if (a >= static_cast<int>(all.size())) throw std::runtime_error("offsets shorter than positions");
        row.push_back(all[a]);
      }
      terms.push_back(std::move(row));
    }
  } else {
    for (const auto& p : ps) terms.push_back(as_pairs(bag(idx, p, true)));
  }
  return highlight_offsets(terms, n_passages, docs.get(doc));
}

}  // namespace wiser
