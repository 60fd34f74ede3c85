#include "index.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <fcntl.h>
#include <fstream>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

#include "bloom.h"
#include "format.h"

namespace wiser {

VacuumIndex::~VacuumIndex() {
  if (map_) ::munmap(map_, map_len_);
}

namespace {
// FNV-1a, 64-bit
inline uint64_t term_hash(const char* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<uint8_t>(p[i])) * 0x100000001b3ull;
  return h ^ (h >> 29);
}
inline bool same(const std::string& t, const char* p, size_t n) {
  return t.size() == n && std::memcmp(t.data(), p, n) == 0;
}
}  // namespace

int32_t VacuumIndex::find(const std::string& term) const { return find(term.data(), term.size()); }

int32_t VacuumIndex::find(const char* p, size_t n) const {
  if (tslot_.empty()) return -1;
  const uint64_t h = term_hash(p, n);
  const uint32_t tag = static_cast<uint32_t>(h >> 32);
  for (uint64_t i = h & tmask_;; i = (i + 1) & tmask_) {
    const uint64_t e = tslot_[i];
    if (e == 0) return -1;
    if (static_cast<uint32_t>(e >> 32) == tag) {
      const int32_t id = static_cast<int32_t>(static_cast<uint32_t>(e)) - 1;
      if (same(terms_[id], p, n)) return id;
    }
  }
}

void VacuumIndex::find_many(const char* const* p, const uint32_t* n, size_t cnt, int32_t* out) const {
  if (tslot_.empty()) {
    for (size_t i = 0; i < cnt; ++i) out[i] = -1;
    return;
  }
  constexpr size_t G = 32;
  uint64_t h[G];
  int32_t cand[G];
  for (size_t g0 = 0; g0 < cnt; g0 += G) {
    const size_t m = std::min(G, cnt - g0);
    for (size_t i = 0; i < m; ++i) {   // hashes; prefetch the home slots
      h[i] = term_hash(p[g0 + i], n[g0 + i]);
      __builtin_prefetch(&tslot_[h[i] & tmask_]);
    }
    for (size_t i = 0; i < m; ++i) {   // first tag match; prefetch its string
      const uint32_t tag = static_cast<uint32_t>(h[i] >> 32);
      cand[i] = -1;
      for (uint64_t s = h[i] & tmask_;; s = (s + 1) & tmask_) {
        const uint64_t e = tslot_[s];
        if (e == 0) break;
        if (static_cast<uint32_t>(e >> 32) == tag) {
          cand[i] = static_cast<int32_t>(static_cast<uint32_t>(e)) - 1;
          __builtin_prefetch(&terms_[cand[i]]);
          break;
        }
      }
    }
    for (size_t i = 0; i < m; ++i) {   // confirm (a tag collision falls back to the full probe)
      const int32_t c = cand[i];
      out[g0 + i] = (c >= 0 && same(terms_[c], p[g0 + i], n[g0 + i])) ? c
                    : (c < 0 ? -1 : find(p[g0 + i], n[g0 + i]));
    }
  }
}

int32_t VacuumIndex::insert_term(const char* p, size_t n, int32_t id) {
  const uint64_t h = term_hash(p, n);
  const uint32_t tag = static_cast<uint32_t>(h >> 32);
  for (uint64_t i = h & tmask_;; i = (i + 1) & tmask_) {
    const uint64_t e = tslot_[i];
    if (e == 0) {
      tslot_[i] = (static_cast<uint64_t>(tag) << 32) | static_cast<uint32_t>(id + 1);
      return id;
    }
    if (static_cast<uint32_t>(e >> 32) == tag) {
      const int32_t old = static_cast<int32_t>(static_cast<uint32_t>(e)) - 1;
      if (same(terms_[old], p, n)) return old;
    }
  }
}

void VacuumIndex::open(const std::string& dir) {
  // --- my.doc_length (doc_length_store.h:163-190)
  {
    std::ifstream f(dir + "/my.doc_length", std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + dir + "/my.doc_length");
    int32_t count = 0;
    f.read(reinterpret_cast<char*>(&count), 4);
    f.read(reinterpret_cast<char*>(&avg_), 8);
    if (!f || count < 0) throw std::runtime_error("truncated my.doc_length");
    std::string rec(static_cast<size_t>(count) * 5, '\0');
    f.read(&rec[0], rec.size());
    if (!f) throw std::runtime_error("truncated my.doc_length records");
    for (int32_t i = 0; i < count; ++i) {
      int32_t id;
      std::memcpy(&id, &rec[5 * i], 4);
      if (id < 0) throw std::runtime_error("negative doc id in my.doc_length");
      if (static_cast<size_t>(id) >= c4_.size()) c4_.resize(static_cast<size_t>(id) + 1, 0);
      c4_[id] = static_cast<uint8_t>(rec[5 * i + 4]);
    }
    n_docs_ = count;
  }
  // Bm25Similarity::BuildCache (scoring.h:85-90): k1 * (1 - b + b * len / avg)
  {
    const double k1 = 1.2, b = 0.75;
    for (int i = 0; i < 256; ++i) {
      const uint32_t fl = char4_to_length(static_cast<uint8_t>(i));
      cache_[i] = k1 * (1 - b + b * fl / avg_);
    }
  }
  // --- my.vacuum
  {
    int fd = ::open((dir + "/my.vacuum").c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + dir + "/my.vacuum");
    struct stat sb;
    if (::fstat(fd, &sb) != 0) { ::close(fd); throw std::runtime_error("stat my.vacuum"); }
    map_len_ = static_cast<uint64_t>(sb.st_size);
    void* p = map_len_ ? ::mmap(nullptr, map_len_, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
    ::close(fd);
    if (map_len_ && p == MAP_FAILED) throw std::runtime_error("mmap my.vacuum failed");
    map_ = static_cast<uint8_t*>(p);
    if (map_len_ < 1 || map_[0] != kVacuumMagic)
      throw std::runtime_error("my.vacuum: wrong first byte (expected 0x88)");
    // Bloom fields: has_bloom_begin, bytes, entries, f32 ratio; same for end.
    const uint8_t* q = map_ + 1;
    const uint8_t* e = map_ + std::min<uint64_t>(map_len_, kVacuumHeaderBytes);
    uint64_t has_bloom[2] = {0, 0}, bytes[2] = {0, 0}, entries[2] = {0, 0};
    float ratio[2] = {0, 0};
    for (int s = 0; s < 2; ++s) {
      int l = get_varint(q, e, &has_bloom[s]); q += l;
      l = get_varint(q, e, &bytes[s]); q += l;
      l = get_varint(q, e, &entries[s]); q += l;
      if (q + 4 <= e) std::memcpy(&ratio[s], q, 4);
      q += 4;
      if (q > e) throw std::runtime_error("my.vacuum: truncated header");
    }
    // Bloom filters (has_bloom) only add sections between the tf and the
    // position boxes of each list; every box is located through the skip
    // rows, so the image is built the same way.  Phrase images can carry
    // them (build_image(..., blooms)) to prune before the position check.
    has_bloom_ = has_bloom[1] != 0;
    bloom_bytes_ = static_cast<uint32_t>(bytes[1]);
    bloom_entries_ = static_cast<uint32_t>(entries[1]);
    bloom_ratio_ = ratio[1];
  }
  // --- my.tip (term_index.h:147-159)
  {
    std::ifstream f(dir + "/my.tip", std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + dir + "/my.tip");
    f.seekg(0, std::ios::end);
    std::string all(static_cast<size_t>(f.tellg()), '\0');
    f.seekg(0);
    f.read(&all[0], all.size());
    if (!f) throw std::runtime_error("cannot read " + dir + "/my.tip");
    // entry positions first (sequential), then every list header checked in
    // parallel (millions of terms: one page of my.vacuum touched per list)
    struct Ent { size_t at; uint32_t len; uint64_t off, df; };
    std::vector<Ent> ents;
    for (size_t at = 0; at < all.size();) {
      if (at + 4 > all.size()) throw std::runtime_error("truncated my.tip");
      uint32_t len;
      std::memcpy(&len, &all[at], 4);
      if (at + 4 + len + 8 > all.size()) throw std::runtime_error("truncated my.tip entry");
      int64_t v;
      std::memcpy(&v, &all[at + 4 + len], 8);
      ents.push_back(Ent{at + 4, len, tip_offset(v), 0});
      at += 4 + len + 8;
    }
    {
      const size_t n = ents.size();
      const int nt = static_cast<int>(std::max<size_t>(1, std::min<size_t>(16, n / 65536)));
      std::atomic<size_t> bad{~size_t{0}};
      auto work = [&](int t) {
        for (size_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
          Ent& e = ents[i];
          uint64_t df = 0;
          if (e.off + 2 > map_len_ || map_[e.off] != kPostingListMagic ||
              !get_varint(map_ + e.off + 1, map_ + map_len_, &df) || df == 0) {
            size_t cur = bad.load();
            while (i < cur && !bad.compare_exchange_weak(cur, i)) {}
            return;
          }
          e.df = df;
        }
      };
      std::vector<std::thread> ts;
      for (int t = 1; t < nt; ++t) ts.emplace_back(work, t);
      work(0);
      for (auto& t : ts) t.join();
      if (bad.load() != ~size_t{0})
        throw std::runtime_error("posting list of '" + all.substr(ents[bad].at, ents[bad].len) +
                                 "' has a wrong magic byte or a bad doc freq");
    }
    uint64_t cap = 16;
    while (cap < 2 * ents.size()) cap <<= 1;
    tslot_.assign(cap, 0);
    tmask_ = cap - 1;
    terms_.reserve(ents.size());
    off_.reserve(ents.size());
    df_.reserve(ents.size());
    for (const Ent& e : ents) {
      const uint64_t off = e.off, df = e.df;
      const int32_t next = static_cast<int32_t>(terms_.size());
      // (the candidate string must be in terms_ for the table's compare)
      terms_.emplace_back(all, e.at, e.len);
      const int32_t id = insert_term(terms_.back().data(), terms_.back().size(), next);
      if (id != next) { // later entries win, as htrie_map assignment does
        terms_.pop_back();
        off_[id] = off;
        df_[id] = static_cast<uint32_t>(df);
        continue;
      }
      off_.push_back(off);
      df_.push_back(static_cast<uint32_t>(df));
    }
  }
  // calc_es_idf (scoring.h:21-25) with N = doc_lengths.Size() (vacuum_engine.h:240)
  idf_.resize(df_.size());
  for (size_t i = 0; i < df_.size(); ++i) {
    const int N = n_docs_, d = static_cast<int>(df_[i]);
    idf_[i] = std::log(1 + (N - d + 0.5) / (d + 0.5));
  }
}

std::vector<SkipRow> VacuumIndex::rows(int32_t id) const {
  std::vector<SkipRow> out;
  rows_into(id, &out);
  return out;
}

void VacuumIndex::rows_into(int32_t id, std::vector<SkipRow>* dst) const {
  const uint8_t* end = map_ + map_len_;
  const uint8_t* p = map_ + off_[id];
  uint64_t v;
  int l = get_varint(p + 1, end, &v);
  if (!l) throw std::runtime_error("bad df varint");
  p += 1 + l + 8;  // magic | df | 8 reserved bytes (bloom section pointers)
  if (p >= end || p[0] != kSkipListMagic) throw std::runtime_error("bad skip list magic");
  uint64_t n = 0;
  l = get_varint(p + 1, end, &n);
  p += 1 + l;
  if (n > map_len_) throw std::runtime_error("bad skip list length");
  std::vector<SkipRow>& out = *dst;
  out.resize(n);
  // fields: d prev_doc, d docid off, d tf off, d pos off, pos idx, d off off, off idx
  uint64_t pd = 0, pdo = 0, pto = 0, ppo = 0, poo = 0;
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t f[7];
    for (int k = 0; k < 7; ++k) {
      l = get_varint(p, end, &f[k]);
      if (!l) throw std::runtime_error("truncated skip list");
      p += l;
    }
    pd = static_cast<uint32_t>(pd + f[0]);
    pdo += f[1]; pto += f[2]; ppo += f[3]; poo += f[5];
    out[r] = SkipRow{static_cast<uint32_t>(pd), pdo, pto, ppo, static_cast<uint32_t>(f[4]), poo,
                     static_cast<uint32_t>(f[6])};
  }
}

bool host_decode_block(const uint8_t* p, const uint8_t* end, int cnt, bool delta,
                       uint32_t prev, uint32_t* out) {
  if (p >= end) return false;
  if (p[0] == kPackMagic) {
    if (cnt != kPackSize || p + 2 > end) return false;
    const int b = p[1];
    if (b < 1 || b > 32 || p + 2 + 16 * b > end) return false;
    const uint8_t* d = p + 2;
    const uint64_t mask = b == 32 ? 0xFFFFFFFFull : ((1ull << b) - 1);
    for (int j = 0; j < kPackSize; ++j) {
      const uint64_t bit = static_cast<uint64_t>(j) * b;
      uint64_t w = 0;
      const uint64_t at = bit >> 3, avail = 16u * b - at;  // bytes of the pack from `at`
      std::memcpy(&w, d + at, avail < 8 ? avail : 8);     // little-endian bit order
      out[j] = static_cast<uint32_t>((w >> (bit & 7)) & mask);
    }
  } else if (p[0] == kVIntsMagic) {
    uint64_t nb = 0;
    int l = get_varint(p + 1, end, &nb);
    if (!l) return false;
    const uint8_t* q = p + 1 + l;
    const uint8_t* qe = q + nb;
    if (qe > end) return false;
    for (int j = 0; j < cnt; ++j) {
      uint64_t v;
      int m = get_varint(q, qe, &v);
      if (!m) return false;
      q += m;
      out[j] = static_cast<uint32_t>(v);
    }
  } else {
    return false;
  }
  if (delta) {
    uint32_t acc = prev;
    for (int j = 0; j < cnt; ++j) { acc += out[j]; out[j] = acc; }
  }
  return true;
}

namespace {
// Runs fn(id) for every list id on `threads` threads; the first exception wins.
template <class F>
void for_each_list(int32_t L, int threads, F&& fn) {
  std::atomic<int32_t> next{0};
  std::atomic<bool> failed{false};
  std::string err;
  std::mutex err_mu;
  auto work = [&](int worker) {
    try {
      // small lists dominate the count: take them 256 at a time
      for (int32_t s; (s = next.fetch_add(256)) < L && !failed;)
        for (int32_t id = s; id < std::min(L, s + 256) && !failed; ++id) fn(id, worker);
    } catch (const std::exception& ex) {
      std::lock_guard<std::mutex> g(err_mu);
      if (!failed.exchange(true)) err = ex.what();
    }
  };
  std::vector<std::thread> ts;
  for (int i = 1; i < threads; ++i) ts.emplace_back(work, i);
  work(0);
  for (auto& t : ts) t.join();
  if (failed) throw std::runtime_error(err);
}
}  // namespace

// Three passes over the lists, none of which allocates per list: (1) size the
// list's part of every image array, (2) prefix sums in list-id order, (3) fill
// the arrays in place.  (Millions of one-block lists -- the en-Wikipedia shape
// -- made per-list vectors and their serial concatenation the load's cost.)
HostImage build_image(const VacuumIndex& idx, uint32_t doc_lo, uint32_t doc_hi, int threads,
                      uint32_t dense_div, bool positions, uint64_t dense_budget, bool blooms,
                      uint64_t hbm_free) {
  const int32_t L = idx.n_lists();
  const uint8_t* file = idx.file();
  const uint8_t* fend = file + idx.file_bytes();
  // doc ids a bitmap covers: the image's range clipped to the doc-length records
  const uint64_t span_end = std::min<uint64_t>(doc_hi, static_cast<uint64_t>(std::max(idx.n_docs(), 0)));
  const uint32_t span = span_end > doc_lo ? static_cast<uint32_t>(span_end - doc_lo) : 0u;
  const uint64_t n_ent = (static_cast<uint64_t>(span) + kDenseDocs - 1) / kDenseDocs;   // entries per bitmap
  const std::vector<uint8_t>& c4 = idx.char4_lengths();
  const double* norm = idx.bm25_cache();   // Bm25Similarity cache_ (scoring.h:85-90)
  struct Info {            // pass 1: the list's share of the image
    uint32_t r0 = 0, r1 = 0;   // image rows [r0, r1); r0 >= r1: no docs in the image
    uint32_t fcnt = 0;         // postings of the list's final row
    uint32_t tail_cnt = 0;     // postings of the image's last row
    uint64_t bytes = 0;        // docid span + tf span
    uint8_t dense = 0, vtail = 0;
    uint8_t shift = 0;         // dense: bucket shift (0: a bitmap)
  };
  std::vector<Info> info(L);
  struct Scratch {   // per worker thread, reused from list to list
    std::vector<SkipRow> rows;
    std::vector<uint32_t> last, docs, tfs;
  };
  if (threads < 1) threads = 1;
  std::vector<Scratch> scratch(threads);
  // rows and last doc of every row (prev of the next row; the final row decoded)
  auto load_rows = [&](int32_t id, Scratch& s, uint32_t* fcnt) {
    idx.rows_into(id, &s.rows);
    const uint32_t df = idx.df(id);
    const uint64_t nrows = s.rows.size();
    if (nrows == 0 || nrows != (df + kPackSize - 1) / kPackSize)
      throw std::runtime_error("skip rows do not match df for '" + idx.term(id) + "'");
    s.last.resize(nrows);
    for (uint64_t r = 0; r + 1 < nrows; ++r) s.last[r] = s.rows[r + 1].prev_doc;
    *fcnt = static_cast<uint32_t>(df - kPackSize * (nrows - 1));
    uint32_t tmp[kPackSize];
    if (!host_decode_block(file + s.rows[nrows - 1].doc_off, fend, static_cast<int>(*fcnt), true,
                           s.rows[nrows - 1].prev_doc, tmp))
      throw std::runtime_error("cannot decode the last block of '" + idx.term(id) + "'");
    s.last[nrows - 1] = tmp[*fcnt - 1];
  };
  auto row_cnt = [](const Info& in, uint64_t r, uint64_t nrows) {
    return r + 1 == nrows ? static_cast<int>(in.fcnt) : kPackSize;
  };

  const bool timing = std::getenv("WSR_LOAD_TIMING") != nullptr;
  auto t_mark = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[wsr load] %s %.3f s\n", what, std::chrono::duration<double>(now - t_mark).count());
    t_mark = now;
  };
  // ---- pass 1
  for_each_list(L, threads, [&](int32_t id, int worker) {
    Scratch& s = scratch[worker];
    Info& in = info[id];
    load_rows(id, s, &in.fcnt);
    const uint64_t nrows = s.rows.size();
    // blocks whose docs can fall into [doc_lo, doc_hi): docs of block r lie in
    // (prev_doc, last] (block 0: [first, last]).
    uint64_t r0 = nrows, r1 = 0;
    for (uint64_t r = 0; r < nrows; ++r) {
      const bool below_hi = (r == 0) || (static_cast<uint64_t>(s.rows[r].prev_doc) + 1 < doc_hi);
      if (below_hi && s.last[r] >= doc_lo) { r0 = std::min(r0, r); r1 = r + 1; }
    }
    if (r0 >= r1) { in.r0 = in.r1 = 0; return; }
    in.r0 = static_cast<uint32_t>(r0);
    in.r1 = static_cast<uint32_t>(r1);
    const uint64_t d0 = s.rows[r0].doc_off;
    const uint64_t d1 = s.rows[r1 - 1].doc_off + blob_bytes(file + s.rows[r1 - 1].doc_off, fend);
    const uint64_t t0 = s.rows[r0].tf_off;
    const uint64_t t1 = s.rows[r1 - 1].tf_off + blob_bytes(file + s.rows[r1 - 1].tf_off, fend);
    if (d1 <= d0 || t1 <= t0 || d1 > idx.file_bytes() || t1 > idx.file_bytes() ||
        d1 - d0 + (t1 - t0) >= (1ull << 32))
      throw std::runtime_error("bad blob span for '" + idx.term(id) + "'");
    in.bytes = (d1 - d0) + (t1 - t0);
    in.tail_cnt = (r1 == nrows) ? in.fcnt : kPackSize;
    in.vtail = r1 == nrows && file[s.rows[nrows - 1].doc_off] == kVIntsMagic;
    const uint64_t n_img = (r1 - r0 - 1) * kPackSize + in.tail_cnt;
    if (dense_div && span && n_img * dense_div >= span) {
      // a doc inside [doc_lo, doc_hi) but past the doc-length records cannot be
      // represented in a bitmap: such a list stays on the block path
      bool ok = true;
      const uint64_t lim = static_cast<uint64_t>(doc_lo) + span;
      for (uint64_t r = r0; r < r1 && ok; ++r) {
        if (s.last[r] < lim) continue;
        if (r > 0 && static_cast<uint64_t>(s.rows[r].prev_doc) + 1 >= doc_hi) continue;
        uint32_t docs[kPackSize];
        const int cnt = row_cnt(in, r, nrows);
        if (!host_decode_block(file + s.rows[r].doc_off, fend, cnt, true, s.rows[r].prev_doc, docs))
          throw std::runtime_error("cannot decode a block for the dense image");
        for (int i = 0; i < cnt; ++i)
          if (docs[i] >= lim && docs[i] < doc_hi) ok = false;
      }
      in.dense = ok;
      // the probe structure follows the density inside the range (a shard's
      // edge blocks also hold postings outside it)
      // (block r's docs lie in (prev_doc, last]; only edge blocks are decoded)
      uint64_t n_in = 0;
      for (uint64_t r = r0; r < r1 && ok; ++r) {
        const int cnt = row_cnt(in, r, nrows);
        const bool inside = (r == 0 ? doc_lo == 0 : s.rows[r].prev_doc + 1ull >= doc_lo) && s.last[r] < lim;
        if (inside) {
          n_in += static_cast<uint64_t>(cnt);
        } else {
          uint32_t docs[kPackSize];
          if (!host_decode_block(file + s.rows[r].doc_off, fend, cnt, true, s.rows[r].prev_doc, docs))
            throw std::runtime_error("cannot decode a block for the dense image");
          for (int i = 0; i < cnt; ++i) n_in += docs[i] >= doc_lo && docs[i] < lim;
        }
      }
      in.shift = static_cast<uint8_t>(bucket_shift(n_in, span));
      if (in.shift) {   // crowded buckets (postings clustered in the range): a bitmap
        const uint32_t c = in.shift;
        uint64_t crowded = 0, run = 0, cur = ~0ull;
        for (uint64_t r = r0; r < r1; ++r) {
          uint32_t docs[kPackSize];
          const int cnt = row_cnt(in, r, nrows);
          if (!host_decode_block(file + s.rows[r].doc_off, fend, cnt, true, s.rows[r].prev_doc, docs))
            throw std::runtime_error("cannot decode a block for the dense image");
          for (int i = 0; i < cnt; ++i) {
            if (docs[i] < doc_lo || docs[i] >= lim) continue;
            const uint64_t bk = (docs[i] - doc_lo) >> c;
            if (bk != cur) { cur = bk; run = 0; }
            if (++run == kBucketWindow + 1) ++crowded;
          }
        }
        if (crowded * kBucketCrowdedDiv > bucket_count(span, c)) in.shift = 0;
      }
    }
  });

  lap("pass 1 (sizes)");
  if (hbm_free) {
    // the rest of the image: blob, directory, plen and bmax (156 B per block),
    // decoded tails, blooms (positions are not sized yet: the 10 % margin)
    uint64_t other = static_cast<uint64_t>(std::max(idx.n_docs(), 0));
    for (int32_t id = 0; id < L; ++id) {
      const Info& in = info[id];
      if (in.r1 <= in.r0) continue;
      const uint64_t nbl = in.r1 - in.r0;
      other += in.bytes + nbl * (sizeof(BlockDev) + 12 + kPackSize) + (in.vtail ? 8ull * in.tail_cnt : 0);
      if (blooms && positions) other += nbl * kPackSize * 32;
    }
    const uint64_t cap = hbm_free / 10 * 9;
    const uint64_t room = cap > other ? cap - other : 0;
    if (!dense_budget || dense_budget > room) dense_budget = room ? room : 1;
  }
  // bitmap budget: when the dense lists' bitmaps + 1-byte tfs would exceed it,
  // the longest lists keep theirs (they are the ones probed most)
  if (dense_budget) {
    std::vector<std::pair<uint64_t, int32_t>> cand;   // (postings in the image, list)
    for (int32_t id = 0; id < L; ++id)
      if (info[id].dense)
        cand.emplace_back((info[id].r1 - info[id].r0 - 1) * uint64_t{kPackSize} + info[id].tail_cnt, id);
    std::sort(cand.begin(), cand.end(), [](const auto& a, const auto& b) {
      return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    uint64_t used = 0;
    for (const auto& c : cand) {
      const uint32_t sh = info[c.second].shift;
      const uint64_t bytes = (sh ? 4 * bucket_words(c.first, span, sh) : n_ent * kDenseEntBytes) + c.first;
      if (used + bytes > dense_budget) info[c.second].dense = 0;
      else used += bytes;
    }
  }
  // ---- pass 2: offsets in list-id order
  HostImage img;
  img.doc_lo = doc_lo;
  img.doc_hi = doc_hi;
  img.dense_span = span;
  img.lists.resize(L);
  img.list_bytes.resize(L);
  img.has_positions = positions;
  uint64_t at = 0, nb = 0, ne = 0, ntf8 = 0, ntail = 0, nbk = 0;
  for (int32_t id = 0; id < L; ++id) {
    const Info& in = info[id];
    ListDev& ld = img.lists[id];
    const uint32_t nbl = in.r1 > in.r0 ? in.r1 - in.r0 : 0u;
    ld.base = at;
    ld.blk0 = static_cast<uint32_t>(nb);
    ld.nblk = nbl;
    ld.df = idx.df(id);
    ld.tail_cnt = nbl ? in.tail_cnt : 0u;
    ld.idf = idx.idf(id);
    ld.bm = kNoDense;
    ld.tf8 = 0;
    ld.tail = kNoTail;
    ld.last = 0;
    ld.tfmax = 0;
    if (!nbl) { img.list_bytes[id] = 0; continue; }
    if (in.vtail) { ld.tail = ntail; ntail += 2ull * in.tail_cnt; }
    if (in.dense) {
      const uint64_t n_img = (nbl - 1) * static_cast<uint64_t>(kPackSize) + in.tail_cnt;
      if (in.shift) {   // offset buckets (nbk: in words, entries are 8-byte aligned)
        ld.bm = (static_cast<uint64_t>(in.shift) << kProbeShiftBit) | (nbk / 2);
        nbk += bucket_words(n_img, span, in.shift);
        ++img.bucket_lists;
      } else {
        ld.bm = ne;
        ne += n_ent;
      }
      ld.tf8 = ntf8;
      ntf8 += n_img;
      ++img.dense_lists;
    }
    img.list_bytes[id] = in.bytes;
    img.docid_tf_bytes += in.bytes;
    at += (in.bytes + 15) & ~15ull;
    nb += nbl;
  }
  if (nb >= (1ull << 32)) throw std::runtime_error("more than 2^32 blocks in one image");
  // (every byte of these is written by pass 3, in parallel)
  img.blob.resize(at + 64);   // tail pad: lanes read whole dwords past a blob end
  std::memset(&img.blob[at], 0, 64);
  img.blocks.resize(nb);
  img.blk_last.resize(nb);
  img.blk_meta.resize(nb);
  img.plen.resize(nb * kPackSize);
  img.bmax.resize(nb);
  img.tails.resize(ntail);
  img.dense.resize(ne);
  img.dense_rank.resize(kRankWords * ne);
  img.tf8.resize(ntf8);
  img.bkt.resize(nbk + 4);   // (+16 B: the last list's 8-byte offset windows)
  for (uint64_t i = nbk; i < nbk + 4; ++i) img.bkt[i] = 0;

  lap("pass 2 (offsets, allocation)");
  // ---- pass 3: fill in place
  struct PosPart {   // positions (phrase engines only): the list's box, packs, bag starts
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> pk, tail;
  };
  std::vector<PosPart> pos_parts(positions ? L : 0);
  if (positions) {
    img.pos_start.assign(2 * nb * kPackSize, 0);
  }
  // phrase bloom filters: shape from the header's "end" fields; one 16-byte
  // slot per filter, so bit arrays of more than 16 bytes stay on the host
  const BloomShape bshape(static_cast<int>(idx.bloom_entries()), idx.bloom_ratio());
  const uint32_t bbytes = idx.bloom_bytes();
  const bool with_blm = blooms && positions && idx.has_bloom() && bbytes >= 1 && bbytes <= 16 &&
                        bshape.bits > 0 && static_cast<uint32_t>(bshape.bits) <= 8 * bbytes && bshape.hashes > 0;
  if (with_blm) {
    img.has_blooms = true;
    img.blm_bits = static_cast<uint32_t>(bshape.bits);
    img.blm_hashes = static_cast<uint32_t>(bshape.hashes);
    img.blm.resize(nb * kPackSize * 32);
    img.blm_hash.assign(2 * static_cast<size_t>(L), 0);
  }
  for_each_list(L, threads, [&](int32_t id, int worker) {
    const Info& in = info[id];
    if (with_blm) {   // bloom_check's two hashes of the term (the element looked up)
      const std::string& t = idx.term(id);
      const uint32_t a = murmurhash2(t.data(), static_cast<int>(t.size()), 0x9747b28c);
      img.blm_hash[2 * id] = a;
      img.blm_hash[2 * id + 1] = murmurhash2(t.data(), static_cast<int>(t.size()), a);
    }
    if (in.r1 <= in.r0) return;
    Scratch& s = scratch[worker];
    uint32_t fcnt;
    load_rows(id, s, &fcnt);
    const uint64_t nrows = s.rows.size();
    const uint64_t r0 = in.r0, r1 = in.r1;
    const ListDev& ld = img.lists[id];
    const uint64_t d0 = s.rows[r0].doc_off;
    const uint64_t d1 = s.rows[r1 - 1].doc_off + blob_bytes(file + s.rows[r1 - 1].doc_off, fend);
    const uint64_t t0 = s.rows[r0].tf_off;
    const uint64_t t1 = s.rows[r1 - 1].tf_off + blob_bytes(file + s.rows[r1 - 1].tf_off, fend);
    std::memcpy(&img.blob[ld.base], file + d0, d1 - d0);
    std::memcpy(&img.blob[ld.base + (d1 - d0)], file + t0, t1 - t0);
    const uint64_t gap = ((in.bytes + 15) & ~15ull) - in.bytes;   // alignment padding
    if (gap) std::memset(&img.blob[ld.base + in.bytes], 0, gap);
    const uint64_t n_img = (r1 - r0 - 1) * kPackSize + in.tail_cnt;
    if (in.dense) { s.docs.resize(n_img); s.tfs.resize(n_img); }
    uint32_t tfmax = 0;   // (ListDev::tfmax: exact where the tfs are decoded, else pack maxima)
    for (uint64_t r = r0; r < r1; ++r) {
      const uint64_t j = ld.blk0 + (r - r0);
      img.blocks[j] = BlockDev{s.rows[r].prev_doc, s.last[r], static_cast<uint32_t>(s.rows[r].doc_off - d0),
                               static_cast<uint32_t>((d1 - d0) + s.rows[r].tf_off - t0)};
      img.blk_last[j] = s.last[r];
      if (r == r1 - 1) img.lists[id].last = s.last[r];   // (this worker's own list)
      const uint8_t* pd = file + s.rows[r].doc_off;
      const uint8_t* pf = file + s.rows[r].tf_off;
      const uint32_t bd = pd[0] == kPackMagic ? pd[1] : 0u;
      const uint32_t bf = pf[0] == kPackMagic ? pf[1] : 0u;
      if ((pd[0] != kPackMagic && pd[0] != kVIntsMagic) || (pf[0] != kPackMagic && pf[0] != kVIntsMagic) ||
          bd > 32 || bf > 32 || (pd[0] == kPackMagic && bd == 0) || (pf[0] == kPackMagic && bf == 0))
        throw std::runtime_error("bad blob header in '" + idx.term(id) + "'");
      img.blk_meta[j] = bd | (bf << 8);
      // doc-length codes in posting order: a block's 128 codes are one
      // contiguous line for the kernels instead of a gather over the doc ids
      // (docs past the length records get code 0, as in the kernels)
      const int cnt = row_cnt(in, r, nrows);
      uint32_t docs[kPackSize], tfs[kPackSize];
      if (!host_decode_block(pd, fend, cnt, true, s.rows[r].prev_doc, docs))
        throw std::runtime_error("cannot decode a block of '" + idx.term(id) + "'");
      uint8_t* o = &img.plen[j * kPackSize];
      for (int i = 0; i < cnt; ++i) o[i] = docs[i] < c4.size() ? c4[docs[i]] : 0;
      for (int i = cnt; i < kPackSize; ++i) o[i] = 0;
      const bool last_vints = in.vtail && r + 1 == nrows;
      if (!host_decode_block(pf, fend, cnt, false, 0, tfs))
        throw std::runtime_error("cannot decode the tfs of '" + idx.term(id) + "'");
      // the block's largest TfNormLossy, by the kernels' operations in their
      // order (f64), then rounded up to f32 so that idf times it never falls
      // below a score of the block
      double bm = 0.0;
      for (int i = 0; i < cnt; ++i) {
        tfmax = std::max(tfmax, tfs[i]);
        const double f = static_cast<double>(static_cast<int32_t>(tfs[i]));
        const double t = (f * (1.2 + 1)) / (f + norm[o[i]]);
        bm = t > bm ? t : bm;
      }
      float bmf = static_cast<float>(bm);
      if (static_cast<double>(bmf) < bm) bmf = std::nextafter(bmf, std::numeric_limits<float>::infinity());
      img.bmax[j] = bmf;
      if (last_vints) {   // the list's VInts tail, decoded once (the kernels read it as words)
        std::memcpy(&img.tails[ld.tail], docs, cnt * sizeof(uint32_t));
        std::memcpy(&img.tails[ld.tail + cnt], tfs, cnt * sizeof(uint32_t));
      }
      if (in.dense) {
        std::memcpy(&s.docs[(r - r0) * kPackSize], docs, cnt * sizeof(uint32_t));
        std::memcpy(&s.tfs[(r - r0) * kPackSize], tfs, cnt * sizeof(uint32_t));
      }
    }
    img.lists[id].tfmax = tfmax;   // (this worker's own list)
    if (in.dense && in.shift) {
      // offset buckets: per 2^c docs the rank and count of its postings and the
      // offsets of its first four; then every posting's offset
      const uint32_t c = in.shift, w = 1u << c;
      const uint64_t nbkt = bucket_count(span, c);
      uint32_t* ent = &img.bkt[2 * (ld.bm & kProbeBaseMask)];
      uint8_t* offs = reinterpret_cast<uint8_t*>(ent + 2 * nbkt);
      uint64_t i = 0;
      for (uint64_t e = 0; e < nbkt; ++e) {
        const uint64_t start = doc_lo + (e << c);
        while (i < n_img && s.docs[i] < start) ++i;
        uint64_t j = i;
        uint32_t in4 = 0xFFFFFFFFu;
        while (j < n_img && s.docs[j] < start + w) {
          const uint32_t o = static_cast<uint32_t>(s.docs[j] - start);
          offs[j] = static_cast<uint8_t>(o);
          if (j - i < kBucketInline) in4 = (in4 & ~(0xFFu << (8 * (j - i)))) | (o << (8 * (j - i)));
          ++j;
        }
        ent[2 * e] = static_cast<uint32_t>(i << 9 | (j - i));   // (j - i <= 2^c <= 256)
        ent[2 * e + 1] = in4;
      }
      for (uint64_t j = n_img; j < (n_img + 7) / 8 * 8; ++j) offs[j] = 0;
      uint8_t* t8 = &img.tf8[ld.tf8];
      for (uint64_t j = 0; j < n_img; ++j) t8[j] = static_cast<uint8_t>(s.tfs[j] < kTf8Escape ? s.tfs[j] : kTf8Escape);
    } else if (in.dense) {
      // rank bitmap: per kDenseDocs docs the doc mask and the rank record (the
      // postings before them, the tfs of the word's first four postings; 255:
      // none, or escaped)
      DenseEnt* de = &img.dense[ld.bm];
      uint64_t i = 0;
      for (uint64_t e = 0; e < n_ent; ++e) {
        const uint64_t start = doc_lo + e * kDenseDocs;
        while (i < n_img && s.docs[i] < start) ++i;
        DenseEnt ent{};
        img.dense_rank[kRankWords * (ld.bm + e)] = static_cast<uint32_t>(i);
        uint32_t t4 = 0xFFFFFFFFu;
        for (uint64_t j = i, n = 0; n < 4 && j < n_img && s.docs[j] < start + kDenseDocs; ++j, ++n) {
          const uint32_t t = s.tfs[j] < kTf8Escape ? s.tfs[j] : kTf8Escape;
          t4 = (t4 & ~(0xFFu << (8 * n))) | (t << (8 * n));
        }
        img.dense_rank[kRankWords * (ld.bm + e) + 1] = t4;
        for (uint64_t j = i; j < n_img && s.docs[j] < start + kDenseDocs; ++j)
          ent.w |= 1u << static_cast<uint32_t>(s.docs[j] - start);
        de[e] = ent;
      }
      uint8_t* t8 = &img.tf8[ld.tf8];
      for (uint64_t j = 0; j < n_img; ++j) t8[j] = static_cast<uint8_t>(s.tfs[j] < kTf8Escape ? s.tfs[j] : kTf8Escape);
    }
    if (positions) {
      // The list's position cozy box (flash_engine_dumper.h:78-104): the bag of
      // posting p holds tf(p) entries starting at entry sum(tf before p).  Walked
      // from row 0's blob; every skip row's (blob, in-blob index) must agree with
      // the walk (PositionPostingBagIterator::GoToSkipPostingBag, flash_iterators.h:504-513).
      PosPart& pt = pos_parts[id];
      const std::string& term = idx.term(id);
      std::vector<uint64_t> cum(nrows * kPackSize + 1, 0);
      uint64_t n = 0;
      for (uint64_t r = 0; r < nrows; ++r) {
        const int cnt = row_cnt(in, r, nrows);
        uint32_t tfs[kPackSize];
        if (!host_decode_block(file + s.rows[r].tf_off, fend, cnt, false, 0, tfs))
          throw std::runtime_error("cannot decode the tfs of '" + term + "'");
        for (int i = 0; i < cnt; ++i) { cum[n + 1] = cum[n] + tfs[i]; ++n; }
      }
      const uint64_t total = cum[n];
      if (total >= (1ull << 32)) throw std::runtime_error("position box of '" + term + "' over 2^32 entries");
      const uint64_t p0 = s.rows[0].pos_off;
      const uint64_t npk = total / kPackSize, rem = total % kPackSize;
      std::vector<uint64_t> blob_at(npk + (rem ? 1 : 0));
      std::vector<uint32_t> width(npk);
      uint64_t pa = p0;
      for (uint64_t k = 0; k < npk; ++k) {
        const uint8_t* b = file + pa;
        if (b + 2 > fend || b[0] != kPackMagic || b[1] < 1 || b[1] > 32)
          throw std::runtime_error("bad position pack in '" + term + "'");
        blob_at[k] = pa;
        width[k] = b[1];
        pa += 2 + 16ull * b[1];
      }
      if (rem) {
        blob_at[npk] = pa;
        pt.tail.resize(rem);
        if (file[pa] != kVIntsMagic ||
            !host_decode_block(file + pa, fend, static_cast<int>(rem), false, 0, pt.tail.data()))
          throw std::runtime_error("bad position VInts blob in '" + term + "'");
        pa += blob_bytes(file + pa, fend);
      }
      if (pa > idx.file_bytes() || pa - p0 >= (1ull << 32))
        throw std::runtime_error("position box of '" + term + "' out of range");
      for (uint64_t r = 0; r < nrows; ++r) {
        const uint64_t e = cum[r * kPackSize];
        if (s.rows[r].pos_off != blob_at[e / kPackSize] || s.rows[r].pos_idx != e % kPackSize)
          throw std::runtime_error("skip row position pointer disagrees with the box of '" + term + "'");
      }
      // The image keeps the slice of the box its blocks' bags lie in: packs
      // [k0, k1) and the VInts remainder when the slice reaches it, entries
      // renumbered from pack k0 (a doc-range shard holds a fraction of each
      // box; the whole image keeps all of it)
      const uint64_t e_lo = cum[r0 * kPackSize], e_hi = cum[std::min<uint64_t>(n, r1 * kPackSize)];
      const uint64_t k0 = std::min<uint64_t>(e_lo / kPackSize, npk);
      const uint64_t k1 = std::min<uint64_t>((e_hi + kPackSize - 1) / kPackSize, npk);
      const bool with_tail = rem && e_hi > npk * kPackSize;
      const uint64_t b_lo = k0 < blob_at.size() ? blob_at[k0] : pa;
      const uint64_t b_hi = k1 < blob_at.size() ? blob_at[k1] : pa;
      for (uint64_t k = k0; k < k1; ++k) {
        pt.pk.push_back(static_cast<uint32_t>(blob_at[k] - b_lo));
        pt.pk.push_back(width[k]);
      }
      if (!with_tail) pt.tail.clear();
      pt.bytes.assign(file + b_lo, file + std::max(b_lo, b_hi));
      const uint64_t e0 = k0 * kPackSize;
      const uint64_t n_pk = k1 - k0;   // the slice's packs (pt.pk pairs)
      for (uint64_t r = r0; r < r1; ++r)
        for (uint64_t i = 0; i < kPackSize && r * kPackSize + i < n; ++i) {
          const uint64_t slot = (ld.blk0 + r - r0) * kPackSize + i;
          const uint64_t er = cum[r * kPackSize + i] - e0;
          img.pos_start[2 * slot] = static_cast<uint32_t>(er);
          const uint64_t kk = er / kPackSize;
          if (kk < n_pk && pt.pk[2 * kk] < (1u << 26))
            img.pos_start[2 * slot + 1] = (pt.pk[2 * kk] << 6) | pt.pk[2 * kk + 1];
        }
    }
    if (with_blm) {
      // The list's two bloom sections (flash_engine_dumper.h:620-646): the 8
      // reserved header bytes hold their offsets from the list start (prior,
      // next); a section = 0xA4 | n boxes | delta offsets of the boxes, a box
      // = 0xF5 | n | MSB-first presence bitmap | the present bit arrays
      // (BloomSkipList / BloomBoxIterator, flash_containers.h:560-687).  Box b
      // holds postings [128 b, 128 b + n): its arrays go to the image slots of
      // skip row b, whose blocks this image holds when r0 <= b < r1.
      const std::string& term = idx.term(id);
      const uint8_t* pl = file + idx.list_offset(id);
      uint64_t v, so[2];
      const uint8_t* q = pl + 1;
      int l = get_varint(q, fend, &v);
      q += l;
      for (int side = 0; side < 2; ++side) {
        l = get_varint(q, fend, &so[side]);
        if (!l) throw std::runtime_error("bad bloom section pointer in '" + term + "'");
        q += l;
      }
      uint8_t* dst = &img.blm[ld.blk0 * kPackSize * 32];
      std::memset(dst, 0, (r1 - r0) * kPackSize * 32);
      for (int side = 0; side < 2; ++side) {
        const uint8_t* p = pl + so[side];
        uint64_t nbox = 0;
        if (p >= fend || p[0] != kBloomSkipListMagic || !(l = get_varint(p + 1, fend, &nbox)) || nbox != nrows)
          throw std::runtime_error("bad bloom skip list in '" + term + "'");
        p += 1 + l;
        uint64_t boff = 0;
        for (uint64_t b = 0; b < r1; ++b) {
          uint64_t d;
          if (!(l = get_varint(p, fend, &d))) throw std::runtime_error("truncated bloom skip list in '" + term + "'");
          p += l;
          boff += d;
          if (b < r0) continue;
          const uint8_t* bx = pl + boff;
          uint64_t n = 0;
          if (bx >= fend || bx[0] != kBloomBoxMagic || !(l = get_varint(bx + 1, fend, &n)) || n > kPackSize)
            throw std::runtime_error("bad bloom box in '" + term + "'");
          const uint8_t* bm = bx + 1 + l;
          const uint8_t* items = bm + (n + 7) / 8;
          if (items > fend) throw std::runtime_error("bloom box bitmap of '" + term + "' out of range");
          uint64_t phys = 0;
          for (uint64_t i = 0; i < n; ++i) {
            if (!(bm[i / 8] & (0x80u >> (i % 8)))) continue;
            const uint8_t* a = items + phys * bbytes;
            if (a + bbytes > fend) throw std::runtime_error("bloom box of '" + term + "' out of range");
            std::memcpy(dst + ((b - r0) * kPackSize + i) * 32 + side * 16, a, bbytes);
            ++phys;
          }
        }
      }
    }
  });

  lap("pass 3 (fill)");
  if (positions) {
    uint64_t pb = 0;
    for (auto& p : pos_parts) pb += (p.bytes.size() + 15) & ~15ull;
    img.pos_blob.resize(pb + 64, 0);   // tail pad: lanes read whole dwords
    img.pos_lists.resize(L, PosDev{0, 0, 0, 0});
    img.pos_list_bytes.assign(L, 0);
    uint64_t pat = 0;
    for (int32_t id = 0; id < L; ++id) {
      PosPart& p = pos_parts[id];
      PosDev& pd = img.pos_lists[id];
      pd.base = pat;
      pd.pk0 = static_cast<uint32_t>(img.pos_pk.size() / 2);
      pd.npk = static_cast<uint32_t>(p.pk.size() / 2);
      pd.tail = img.pos_tail.size();
      img.pos_list_bytes[id] = p.bytes.size();
      if (!p.bytes.empty()) std::memcpy(&img.pos_blob[pat], p.bytes.data(), p.bytes.size());
      pat += (p.bytes.size() + 15) & ~15ull;
      img.pos_pk.insert(img.pos_pk.end(), p.pk.begin(), p.pk.end());
      img.pos_tail.insert(img.pos_tail.end(), p.tail.begin(), p.tail.end());
      PosPart().bytes.swap(p.bytes);
    }
  }
  return img;
}

int64_t dense_lookup_host(const HostImage& img, const ListDev& L, uint32_t doc) {
  if (L.bm == kNoDense || doc < img.doc_lo || doc >= img.doc_hi) return -1;
  const uint32_t rel = doc - img.doc_lo;
  if (rel >= img.dense_span) return -1;
  uint32_t idx = 0;
  if (const uint32_t c = probe_shift(L.bm)) {   // offset buckets: scan the bucket's offsets
    const uint64_t base = L.bm & kProbeBaseMask;
    const uint32_t* ent = &img.bkt[2 * (base + (rel >> c))];
    const uint8_t* offs = reinterpret_cast<const uint8_t*>(&img.bkt[2 * (base + bucket_count(img.dense_span, c))]);
    const uint32_t rank = ent[0] >> 9, cnt = ent[0] & 511u, o = rel & ((1u << c) - 1u);
    bool hit = false;
    for (uint32_t j = 0; j < cnt && !hit; ++j) {
      const uint32_t b = j < kBucketInline ? (ent[1] >> (8 * j)) & 255u : offs[rank + j];
      if (b == o) { hit = true; idx = rank + j; }
    }
    if (!hit) return -1;
  } else {
    const DenseEnt& e = img.dense[L.bm + rel / kDenseDocs];
    const uint32_t sh = rel % kDenseDocs;
    if (!dense_ent_bit(e, sh)) return -1;
    idx = dense_ent_rank(e, img.dense_rank[kRankWords * (L.bm + rel / kDenseDocs)], sh);
  }
  const uint8_t t = img.tf8[L.tf8 + idx];
  if (t != kTf8Escape) return t;
  const uint32_t j = idx / kPackSize;
  const BlockDev& bd = img.blocks[L.blk0 + j];
  const uint32_t cnt = j + 1 == L.nblk ? L.tail_cnt : kPackSize;
  uint32_t out[kPackSize];
  const uint8_t* p = img.blob.data() + L.base + bd.tf_rel;
  if (!host_decode_block(p, img.blob.data() + img.blob.size(), static_cast<int>(cnt), false, 0, out))
    return -1;
  return out[idx % kPackSize];
}

}  // namespace wiser
