#include "index.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <fcntl.h>
#include <fstream>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

#include "format.h"

namespace wiser {

VacuumIndex::~VacuumIndex() {
  if (map_) ::munmap(map_, map_len_);
}

int32_t VacuumIndex::find(const std::string& term) const {
  auto it = lookup_.find(term);
  return it == lookup_.end() ? -1 : it->second;
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
    uint64_t has_bloom[2] = {0, 0};
    for (int s = 0; s < 2; ++s) {
      uint64_t v;
      int l = get_varint(q, e, &has_bloom[s]); q += l;
      l = get_varint(q, e, &v); q += l;
      l = get_varint(q, e, &v); q += l;
      q += 4;
      if (q > e) throw std::runtime_error("my.vacuum: truncated header");
    }
    // Bloom filters (has_bloom) only add sections between the tf and the
    // position boxes of each list; every box is located through the skip
    // rows, so the image is built the same way.  The position check of
    // phrase queries is exact, so the filters (pruning only) are not uploaded.
    has_bloom_ = has_bloom[1] != 0;
  }
  // --- my.tip (term_index.h:147-159)
  {
    std::ifstream f(dir + "/my.tip", std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + dir + "/my.tip");
    std::string all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    size_t at = 0;
    while (at < all.size()) {
      if (at + 4 > all.size()) throw std::runtime_error("truncated my.tip");
      uint32_t len;
      std::memcpy(&len, &all[at], 4);
      at += 4;
      if (at + len + 8 > all.size()) throw std::runtime_error("truncated my.tip entry");
      std::string term = all.substr(at, len);
      at += len;
      int64_t v;
      std::memcpy(&v, &all[at], 8);
      at += 8;
      const uint64_t off = tip_offset(v);
      if (off + 2 > map_len_ || map_[off] != kPostingListMagic)
        throw std::runtime_error("posting list of '" + term + "' has a wrong magic byte");
      uint64_t df = 0;
      if (!get_varint(map_ + off + 1, map_ + map_len_, &df) || df == 0)
        throw std::runtime_error("posting list of '" + term + "' has a bad doc freq");
      auto ins = lookup_.emplace(term, static_cast<int32_t>(terms_.size()));
      if (!ins.second) { // later entries win, as htrie_map assignment does
        const int32_t id = ins.first->second;
        off_[id] = off;
        df_[id] = static_cast<uint32_t>(df);
        continue;
      }
      terms_.push_back(term);
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
  std::vector<SkipRow> out(n);
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
  return out;
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

HostImage build_image(const VacuumIndex& idx, uint32_t doc_lo, uint32_t doc_hi, int threads,
                      uint32_t dense_div, bool positions) {
  const int32_t L = idx.n_lists();
  const uint8_t* file = idx.file();
  const uint8_t* fend = file + idx.file_bytes();
  // doc ids a bitmap covers: the image's range clipped to the doc-length records
  const uint64_t span_end = std::min<uint64_t>(doc_hi, static_cast<uint64_t>(std::max(idx.n_docs(), 0)));
  const uint32_t span = span_end > doc_lo ? static_cast<uint32_t>(span_end - doc_lo) : 0u;
  const uint64_t n_ent = (static_cast<uint64_t>(span) + kDenseDocs - 1) / kDenseDocs;
  struct Part {
    std::vector<BlockDev> blocks;  // doc_rel / tf_rel relative to the list's span
    std::vector<uint32_t> meta;
    std::vector<uint8_t> bytes;    // docid span followed by tf span
    uint32_t tail_cnt = 0;
    std::vector<DenseEnt> dense;   // rank bitmap (dense lists only)
    std::vector<uint8_t> tf8;
    std::vector<uint8_t> plen;     // doc-length code of every posting, 128 per block
    std::vector<uint32_t> tail;    // VInts last block decoded: doc ids, then tfs
    // positions: the whole box, its pack directory, VInts remainder, bag starts
    std::vector<uint8_t> pos_bytes;
    std::vector<uint32_t> pos_pk;
    std::vector<uint32_t> pos_tail;
    std::vector<uint32_t> pos_start;
  };
  const std::vector<uint8_t>& c4 = idx.char4_lengths();
  std::vector<Part> parts(L);
  // decode the image's postings of one list and lay down its bitmap + tf bytes
  auto build_dense = [&](Part& pt, const std::vector<SkipRow>& rows, uint64_t r0, uint64_t r1,
                         uint64_t n_img) {
    std::vector<uint32_t> docs(n_img), tfs(n_img);
    for (uint64_t r = r0; r < r1; ++r) {
      const int cnt = r + 1 == r1 ? static_cast<int>(pt.tail_cnt) : kPackSize;
      const uint64_t at = (r - r0) * kPackSize;
      if (!host_decode_block(file + rows[r].doc_off, fend, cnt, true, rows[r].prev_doc, &docs[at]) ||
          !host_decode_block(file + rows[r].tf_off, fend, cnt, false, 0, &tfs[at]))
        throw std::runtime_error("cannot decode a block for the dense image");
    }
    // a doc inside [doc_lo, doc_hi) but past the doc-length records cannot be
    // represented: keep the list on the block path
    for (uint64_t i = 0; i < n_img; ++i)
      if (docs[i] >= doc_lo && docs[i] < doc_hi && docs[i] - doc_lo >= span) return;
    pt.dense.assign(n_ent, DenseEnt{0, 0});
    uint64_t i = 0;
    for (uint64_t e = 0; e < n_ent; ++e) {
      const uint64_t start = doc_lo + e * kDenseDocs;
      while (i < n_img && docs[i] < start) ++i;
      pt.dense[e].rank = static_cast<uint32_t>(i);
      for (uint64_t j = i; j < n_img && docs[j] < start + kDenseDocs; ++j) {
        const uint32_t bit = static_cast<uint32_t>(docs[j] - start);
        pt.dense[e].w |= 1u << bit;
      }
    }
    pt.tf8.resize(n_img);
    for (uint64_t j = 0; j < n_img; ++j) pt.tf8[j] = static_cast<uint8_t>(tfs[j] < kTf8Escape ? tfs[j] : kTf8Escape);
  };
  // The list's position cozy box (flash_engine_dumper.h:78-104): the bag of
  // posting p holds tf(p) entries starting at entry sum(tf before p).  Walked
  // from row 0's blob; every skip row's (blob, in-blob index) must agree with
  // the walk (PositionPostingBagIterator::GoToSkipPostingBag, flash_iterators.h:504-513).
  auto build_positions = [&](Part& pt, const std::vector<SkipRow>& rows, uint64_t r0, uint64_t r1,
                             int fcnt, const std::string& term) {
    const uint64_t nrows = rows.size();
    std::vector<uint64_t> cum(nrows * kPackSize + 1, 0);
    uint64_t n = 0;
    for (uint64_t r = 0; r < nrows; ++r) {
      const int cnt = r + 1 == nrows ? fcnt : kPackSize;
      uint32_t tfs[kPackSize];
      if (!host_decode_block(file + rows[r].tf_off, fend, cnt, false, 0, tfs))
        throw std::runtime_error("cannot decode the tfs of '" + term + "'");
      for (int i = 0; i < cnt; ++i) { cum[n + 1] = cum[n] + tfs[i]; ++n; }
    }
    const uint64_t total = cum[n];
    if (total >= (1ull << 32)) throw std::runtime_error("position box of '" + term + "' over 2^32 entries");
    const uint64_t p0 = rows[0].pos_off;
    const uint64_t npk = total / kPackSize, rem = total % kPackSize;
    std::vector<uint64_t> blob_at(npk + (rem ? 1 : 0));
    uint64_t at = p0;
    for (uint64_t k = 0; k < npk; ++k) {
      const uint8_t* b = file + at;
      if (b + 2 > fend || b[0] != kPackMagic || b[1] < 1 || b[1] > 32)
        throw std::runtime_error("bad position pack in '" + term + "'");
      blob_at[k] = at;
      pt.pos_pk.push_back(static_cast<uint32_t>(at - p0));
      pt.pos_pk.push_back(b[1]);
      at += 2 + 16ull * b[1];
    }
    if (rem) {
      blob_at[npk] = at;
      pt.pos_tail.resize(rem);
      if (file[at] != kVIntsMagic ||
          !host_decode_block(file + at, fend, static_cast<int>(rem), false, 0, pt.pos_tail.data()))
        throw std::runtime_error("bad position VInts blob in '" + term + "'");
      at += blob_bytes(file + at, fend);
    }
    if (at > idx.file_bytes() || at - p0 >= (1ull << 32))
      throw std::runtime_error("position box of '" + term + "' out of range");
    for (uint64_t r = 0; r < nrows; ++r) {
      const uint64_t e = cum[r * kPackSize];
      if (rows[r].pos_off != blob_at[e / kPackSize] || rows[r].pos_idx != e % kPackSize)
        throw std::runtime_error("skip row position pointer disagrees with the box of '" + term + "'");
    }
    pt.pos_bytes.assign(file + p0, file + at);
    pt.pos_start.assign((r1 - r0) * kPackSize, 0);
    for (uint64_t r = r0; r < r1; ++r)
      for (uint64_t i = 0; i < kPackSize && r * kPackSize + i < n; ++i)
        pt.pos_start[(r - r0) * kPackSize + i] = static_cast<uint32_t>(cum[r * kPackSize + i]);
  };
  std::atomic<int32_t> next{0};
  std::atomic<bool> failed{false};
  std::string err;
  auto work = [&] {
    try {
      for (int32_t id; (id = next++) < L && !failed;) {
        const std::vector<SkipRow> rows = idx.rows(id);
        const uint32_t df = idx.df(id);
        const uint64_t nrows = rows.size();
        if (nrows != (df + kPackSize - 1) / kPackSize)
          throw std::runtime_error("skip rows do not match df for '" + idx.term(id) + "'");
        // last doc of each block: prev of the next row; decode the final block.
        std::vector<uint32_t> last(nrows);
        for (uint64_t r = 0; r + 1 < nrows; ++r) last[r] = rows[r + 1].prev_doc;
        const int fcnt = static_cast<int>(df - kPackSize * (nrows - 1));
        {
          uint32_t tmp[kPackSize];
          if (!host_decode_block(file + rows[nrows - 1].doc_off, fend, fcnt, true,
                                 rows[nrows - 1].prev_doc, tmp))
            throw std::runtime_error("cannot decode the last block of '" + idx.term(id) + "'");
          last[nrows - 1] = tmp[fcnt - 1];
        }
        // blocks whose docs can fall into [doc_lo, doc_hi): docs of block r lie in
        // (prev_doc, last] (block 0: [first, last]).
        uint64_t r0 = nrows, r1 = 0;
        for (uint64_t r = 0; r < nrows; ++r) {
          const bool below_hi = (r == 0) || (static_cast<uint64_t>(rows[r].prev_doc) + 1 < doc_hi);
          if (below_hi && last[r] >= doc_lo) { r0 = std::min(r0, r); r1 = r + 1; }
        }
        Part& pt = parts[id];
        if (r0 >= r1) continue;  // list has no docs in this shard
        const uint64_t d0 = rows[r0].doc_off;
        const uint64_t d1 = rows[r1 - 1].doc_off + blob_bytes(file + rows[r1 - 1].doc_off, fend);
        const uint64_t t0 = rows[r0].tf_off;
        const uint64_t t1 = rows[r1 - 1].tf_off + blob_bytes(file + rows[r1 - 1].tf_off, fend);
        if (d1 <= d0 || t1 <= t0 || d1 > idx.file_bytes() || t1 > idx.file_bytes())
          throw std::runtime_error("bad blob span for '" + idx.term(id) + "'");
        pt.bytes.assign(file + d0, file + d1);
        pt.bytes.insert(pt.bytes.end(), file + t0, file + t1);
        for (uint64_t r = r0; r < r1; ++r) {
          pt.blocks.push_back(BlockDev{rows[r].prev_doc, last[r],
                                       static_cast<uint32_t>(rows[r].doc_off - d0),
                                       static_cast<uint32_t>((d1 - d0) + rows[r].tf_off - t0)});
          const uint8_t* pd = file + rows[r].doc_off;
          const uint8_t* pf = file + rows[r].tf_off;
          const uint32_t bd = pd[0] == kPackMagic ? pd[1] : 0u;
          const uint32_t bf = pf[0] == kPackMagic ? pf[1] : 0u;
          if ((pd[0] != kPackMagic && pd[0] != kVIntsMagic) || (pf[0] != kPackMagic && pf[0] != kVIntsMagic) ||
              bd > 32 || bf > 32 || (pd[0] == kPackMagic && bd == 0) || (pf[0] == kPackMagic && bf == 0))
            throw std::runtime_error("bad blob header in '" + idx.term(id) + "'");
          pt.meta.push_back(bd | (bf << 8));
        }
        pt.tail_cnt = (r1 == nrows) ? static_cast<uint32_t>(fcnt) : kPackSize;
        // doc-length codes in posting order: a block's 128 codes are one
        // contiguous line for the kernels instead of a gather over the doc ids
        // (docs past the length records get code 0, as in the kernels)
        pt.plen.assign((r1 - r0) * kPackSize, 0);
        for (uint64_t r = r0; r < r1; ++r) {
          const int cnt = r + 1 == nrows ? fcnt : kPackSize;
          uint32_t docs[kPackSize];
          if (!host_decode_block(file + rows[r].doc_off, fend, cnt, true, rows[r].prev_doc, docs))
            throw std::runtime_error("cannot decode a block of '" + idx.term(id) + "'");
          uint8_t* o = &pt.plen[(r - r0) * kPackSize];
          for (int i = 0; i < cnt; ++i) o[i] = docs[i] < c4.size() ? c4[docs[i]] : 0;
          if (r + 1 == nrows && (pt.meta.back() & 0xFF) == 0) {
            // the list's VInts tail, decoded once (the kernels read it as words)
            uint32_t tfs[kPackSize];
            if (!host_decode_block(file + rows[r].tf_off, fend, cnt, false, 0, tfs))
              throw std::runtime_error("cannot decode the tf tail of '" + idx.term(id) + "'");
            pt.tail.assign(docs, docs + cnt);
            pt.tail.insert(pt.tail.end(), tfs, tfs + cnt);
          }
        }
        const uint64_t n_img = (r1 - r0 - 1) * kPackSize + pt.tail_cnt;
        if (dense_div && span && n_img * dense_div >= span) build_dense(pt, rows, r0, r1, n_img);
        if (positions) build_positions(pt, rows, r0, r1, fcnt, idx.term(id));
      }
    } catch (const std::exception& ex) {
      if (!failed.exchange(true)) err = ex.what();
    }
  };
  if (threads < 1) threads = 1;
  std::vector<std::thread> ts;
  for (int i = 0; i < threads; ++i) ts.emplace_back(work);
  for (auto& t : ts) t.join();
  if (failed) throw std::runtime_error(err);

  HostImage img;
  img.doc_lo = doc_lo;
  img.doc_hi = doc_hi;
  img.dense_span = span;
  img.lists.resize(L);
  img.list_bytes.resize(L);
  uint64_t total = 0, nb = 0;
  for (auto& p : parts) { total += (p.bytes.size() + 15) & ~15ull; nb += p.blocks.size(); }
  img.blob.resize(total + 64, 0);  // tail pad: lanes read whole dwords past a blob end
  img.blocks.reserve(nb);
  img.blk_last.reserve(nb);
  img.blk_meta.reserve(nb);
  img.plen.reserve(nb * kPackSize);
  img.has_positions = positions;
  if (positions) {
    uint64_t pb = 0;
    for (auto& p : parts) pb += (p.pos_bytes.size() + 15) & ~15ull;
    img.pos_blob.resize(pb + 64, 0);   // tail pad: lanes read whole dwords
    img.pos_lists.resize(L, PosDev{0, 0, 0, 0});
    img.pos_start.reserve(nb * kPackSize);
    uint64_t pat = 0;
    for (int32_t id = 0; id < L; ++id) {
      Part& p = parts[id];
      PosDev& pd = img.pos_lists[id];
      pd.base = pat;
      pd.pk0 = static_cast<uint32_t>(img.pos_pk.size() / 2);
      pd.npk = static_cast<uint32_t>(p.pos_pk.size() / 2);
      pd.tail = img.pos_tail.size();
      if (!p.pos_bytes.empty()) std::memcpy(&img.pos_blob[pat], p.pos_bytes.data(), p.pos_bytes.size());
      pat += (p.pos_bytes.size() + 15) & ~15ull;
      img.pos_pk.insert(img.pos_pk.end(), p.pos_pk.begin(), p.pos_pk.end());
      img.pos_tail.insert(img.pos_tail.end(), p.pos_tail.begin(), p.pos_tail.end());
      img.pos_start.insert(img.pos_start.end(), p.pos_start.begin(), p.pos_start.end());
      std::vector<uint8_t>().swap(p.pos_bytes);
      std::vector<uint32_t>().swap(p.pos_pk);
      std::vector<uint32_t>().swap(p.pos_tail);
      std::vector<uint32_t>().swap(p.pos_start);
    }
  }
  uint64_t at = 0;
  for (int32_t id = 0; id < L; ++id) {
    Part& p = parts[id];
    ListDev& ld = img.lists[id];
    ld.base = at;
    ld.blk0 = static_cast<uint32_t>(img.blocks.size());
    ld.nblk = static_cast<uint32_t>(p.blocks.size());
    ld.df = idx.df(id);
    ld.tail_cnt = p.tail_cnt;
    ld.idf = idx.idf(id);
    ld.bm = kNoDense;
    ld.tf8 = 0;
    ld.tail = kNoTail;
    ld.pad = 0;
    if (!p.tail.empty()) {
      ld.tail = img.tails.size();
      img.tails.insert(img.tails.end(), p.tail.begin(), p.tail.end());
      std::vector<uint32_t>().swap(p.tail);
    }
    if (!p.dense.empty()) {
      ld.bm = img.dense.size();
      ld.tf8 = img.tf8.size();
      img.dense.insert(img.dense.end(), p.dense.begin(), p.dense.end());
      img.tf8.insert(img.tf8.end(), p.tf8.begin(), p.tf8.end());
      ++img.dense_lists;
      std::vector<DenseEnt>().swap(p.dense);
      std::vector<uint8_t>().swap(p.tf8);
    }
    if (!p.bytes.empty()) std::memcpy(&img.blob[at], p.bytes.data(), p.bytes.size());
    img.docid_tf_bytes += p.bytes.size();
    img.list_bytes[id] = p.bytes.size();
    at += (p.bytes.size() + 15) & ~15ull;
    for (auto& b : p.blocks) { img.blocks.push_back(b); img.blk_last.push_back(b.last); }
    img.blk_meta.insert(img.blk_meta.end(), p.meta.begin(), p.meta.end());
    img.plen.insert(img.plen.end(), p.plen.begin(), p.plen.end());
    std::vector<uint8_t>().swap(p.bytes);
    std::vector<uint8_t>().swap(p.plen);
  }
  return img;
}

int64_t dense_lookup_host(const HostImage& img, const ListDev& L, uint32_t doc) {
  if (L.bm == kNoDense || doc < img.doc_lo || doc >= img.doc_hi) return -1;
  const uint32_t rel = doc - img.doc_lo;
  if (rel >= img.dense_span) return -1;
  const DenseEnt& e = img.dense[L.bm + rel / kDenseDocs];
  const uint32_t sh = rel % kDenseDocs;
  if (!((e.w >> sh) & 1u)) return -1;
  const uint32_t idx = e.rank + static_cast<uint32_t>(__builtin_popcount(e.w & ((1u << sh) - 1u)));
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
