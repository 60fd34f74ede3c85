// RegHeap (wiser_amd/csrc/regheap.h, compiled here for the host) against
// libstdc++'s own std::priority_queue with the reference's comparator
// (MinPointerHeap / EntryGreater, src/qq_mem/src/query_processing.h:510-524),
// RankDoc (:590-602) and SortHeap (:551-562): the doc ids, in order, must be
// identical, ties included.  Prints "ok <streams>" or the first mismatch.
#include <algorithm>
#include <cstdio>
#include <queue>
#include <random>
#include <vector>

#include "regheap.h"

struct Ent {
  double score;
  int32_t doc;
};
struct Greater {
  bool operator()(const Ent& a, const Ent& b) const { return a.score > b.score; }
};

static std::vector<Ent> reference(const std::vector<Ent>& ev, uint32_t k) {
  std::priority_queue<Ent, std::vector<Ent>, Greater> h;
  for (const Ent& e : ev) {
    if (h.size() < k) h.push(e);
    else if (e.score > h.top().score) { h.pop(); h.push(e); }
  }
  std::vector<Ent> out;
  while (!h.empty()) { out.push_back(h.top()); h.pop(); }
  std::reverse(out.begin(), out.end());
  return out;
}

static std::vector<Ent> regheap(const std::vector<Ent>& ev, uint32_t k) {
  wiser::RegHeap h;
  for (const Ent& e : ev) h.insert(k, e.score, e.doc);
  std::vector<Ent> out;
  while (h.n) { out.push_back({h.s[0], h.d[0]}); h.pop(); }
  std::reverse(out.begin(), out.end());
  return out;
}

int main() {
  std::mt19937_64 g(20261018);
  int streams = 0;
  for (uint32_t k = 1; k <= wiser::kRegHeapK; ++k) {
    for (int rep = 0; rep < 400; ++rep) {
      const int n = static_cast<int>(g() % 300);
      const int levels = 1 + static_cast<int>(g() % (rep % 3 == 0 ? 3 : 40));   // tie-heavy streams too
      std::vector<Ent> ev;
      for (int i = 0; i < n; ++i) {
        double s = 1.0 + static_cast<double>(g() % levels) * 0.25;
        if (rep % 5 == 1) s += i * 1e-3;   // rising: every event an insertion
        ev.push_back({s, i});
      }
      const auto a = reference(ev, k), b = regheap(ev, k);
      bool same = a.size() == b.size();
      for (size_t i = 0; same && i < a.size(); ++i) same = a[i].doc == b[i].doc && a[i].score == b[i].score;
      if (!same) {
        std::printf("mismatch k=%u rep=%d n=%d\n", k, rep, n);
        return 1;
      }
      ++streams;
    }
  }
  std::printf("ok %d\n", streams);
  return 0;
}
