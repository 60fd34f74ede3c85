// TEST INFRASTRUCTURE ONLY -- see oracle.h.  A single-threaded-per-query CPU
// restatement of the reference's query path, written from its behaviour; each
// piece cites the reference file:line it restates (paths relative to
// /root/reference/src/qq_mem/src).  Deliberately iterator-shaped like the
// reference (linear skip-row walk, whole-pack unpack, per-posting heap test)
// so that it doubles as the CPU baseline timed by bench.py.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fcntl.h>
#include <fstream>
#include <iterator>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <queue>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;
std::atomic<int64_t> g_ub_neg{0};

constexpr int kPack = 128;                 // PACK_ITEM_CNT, packed_value.h:13
constexpr uint8_t kSkipMagic = 0xA3;       // types.h:44
constexpr uint8_t kPostingMagic = 0xF4;    // types.h:46
constexpr uint8_t kPackMagic = 0xD6;       // types.h:47
constexpr uint8_t kVIntsMagic = 0x9B;      // types.h:48
constexpr uint8_t kVacuumMagic = 0x88;     // types.h:50

// utils.h:249-266 varint_decode_64bit
int varint_decode(const uint8_t* b, uint64_t* v) {
  uint64_t r = b[0] & 0x7f;
  int i = 1;
  if (b[0] < 0x80) { *v = b[0]; return 1; }
  while (b[i - 1] & 0x80) { r += static_cast<uint64_t>(b[i] & 0x7f) << (7 * i); ++i; }
  *v = r;
  return i;
}

// utils.cc:257-270 varint_encode
int varint_encode(uint64_t v, uint8_t* out) {
  int i = 0;
  while (i == 0 || v > 0) { out[i++] = static_cast<uint8_t>((v & 0x7f) | 0x80); v >>= 7; }
  out[i - 1] &= 0x7f;
  return i;
}

// utils.h:286-294
int num_bits(uint32_t v) { int n = 0; while (v) { v >>= 1; ++n; } return n; }

// utils.h:301-313 UintToChar4 (returns the char's bit pattern)
uint8_t char4_encode(uint32_t val) {
  if (val < 0x08) return static_cast<uint8_t>(val & 0xff);
  int shift = num_bits(val) - 4;
  uint32_t enc = (val >> shift) & 0x07;
  enc |= static_cast<uint32_t>(shift + 1) << 3;
  return static_cast<uint8_t>(enc);
}

// utils.h:315-329 Char4ToUint
uint32_t char4_decode(uint8_t c) {
  uint32_t bits = c & 0x07;
  int shift = ((c & 0xff) >> 3) - 1;
  if (shift == -1) return bits;
  return (bits | 0x08) << shift;
}

// LittleIntPacker turbounpack32 (turbobitpacking32.c:3863-3868, layout from
// scripts/turbopacking32.py:83-112): value j at bits [j*b, j*b+b) of the
// little-endian stream of 64-bit words.
void turbo_unpack(const uint8_t* in, int b, uint32_t* out) {
  for (int j = 0; j < kPack; ++j) {
    uint64_t v = 0;
    for (int k = 0; k < b; ++k) {
      uint64_t bit = static_cast<uint64_t>(j) * b + k;
      v |= static_cast<uint64_t>((in[bit >> 3] >> (bit & 7)) & 1) << k;
    }
    out[j] = static_cast<uint32_t>(v);
  }
}

// turbopack32 restated the same way (packed_value.h:87-128 caller)
void turbo_pack(const uint32_t* in, int b, uint8_t* out) {
  std::memset(out, 0, 16 * b);
  for (int j = 0; j < kPack; ++j)
    for (int k = 0; k < b; ++k)
      if ((in[j] >> k) & 1) {
        uint64_t bit = static_cast<uint64_t>(j) * b + k;
        out[bit >> 3] |= static_cast<uint8_t>(1u << (bit & 7));
      }
}

// scoring.h:21-25
double es_idf(int doc_count, int doc_freq) {
  return std::log(1 + (doc_count - doc_freq + 0.5) / (doc_freq + 0.5));
}

// Bm25Similarity (scoring.h:43-97)
struct Bm25 {
  static constexpr double k1 = 1.2, b = 0.75;
  double avg = 1;
  double cache[256];
  void reset(double a) {
    avg = a;
    for (int i = 0; i < 256; ++i) {
      uint32_t fl = char4_decode(static_cast<uint8_t>(i & 0xff));
      cache[i] = k1 * (1 - b + b * fl / avg);
    }
  }
  double tfnorm_lossy(int freq, uint8_t c) const {
    // cache_[field_length] with a signed char index: negative for c >= 0x80 (UB in
    // the reference).  Counted, and read as the unsigned byte like the GPU path.
    if (static_cast<signed char>(c) < 0) ++g_ub_neg;
    return (freq * (k1 + 1)) / (freq + cache[c]);
  }
};

// --------------------------------------------------------------- codecs --
// LittlePackedIntsReader (packed_value.h:184-235)
struct PackReader {
  const uint8_t* buf = nullptr;
  int bits = 0;
  uint32_t cache[kPack];
  void reset(const uint8_t* p) {
    buf = p;
    if (p[0] != kPackMagic) throw std::runtime_error("pack magic");
    bits = p[1];
  }
  void decode() { turbo_unpack(buf + 2, bits, cache); }
};

// VIntsIterator (packed_value.h:400-460) over VarintIteratorEndBound (compression.h:131-196)
struct VIntsIter {
  const uint8_t* data = nullptr;
  int cur = 0, end = 0, next_index = 0;
  void reset(const uint8_t* p) {
    if (p[0] != kVIntsMagic) throw std::runtime_error("vints magic");
    uint64_t nb;
    int l = varint_decode(p + 1, &nb);
    data = p + 1 + l;
    cur = 0;
    end = static_cast<int>(nb);
    next_index = 0;
  }
  bool is_end() const { return cur >= end; }
  uint64_t peek() const { uint64_t v; varint_decode(data + cur, &v); return v; }
  uint64_t pop() { uint64_t v; cur += varint_decode(data + cur, &v); ++next_index; return v; }
  int index() const { return next_index; }
  void skip_to(int i) { while (index() < i) pop(); }
};

// SkipList::Load (flash_containers.h:354-391): docid / tf / position / offset
// columns (the offset columns feed snippets, vacuum_engine.h:248-252).
struct SkipEntry {
  uint32_t prev_doc;
  uint64_t doc_off, tf_off, pos_off;
  uint32_t pos_idx;
  uint64_t off_off;
  uint32_t off_idx;
};
std::vector<SkipEntry> load_skip_list(const uint8_t* buf) {
  if (buf[0] != kSkipMagic) throw std::runtime_error("skip list magic");
  uint64_t n;
  int l = varint_decode(buf + 1, &n);
  const uint8_t* p = buf + 1 + l;
  std::vector<SkipEntry> rows;
  rows.reserve(n);
  uint32_t pd = 0;
  uint64_t pdo = 0, pto = 0, ppo = 0, poo = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t f[7];
    for (int k = 0; k < 7; ++k) p += varint_decode(p, &f[k]);
    uint32_t prev = static_cast<uint32_t>(f[0] + pd);
    uint64_t dof = f[1] + pdo, tof = f[2] + pto, pof = f[3] + ppo, oof = f[5] + poo;
    rows.push_back(SkipEntry{prev, dof, tof, pof, static_cast<uint32_t>(f[4]), oof,
                             static_cast<uint32_t>(f[6])});
    pd = prev; pdo = dof; pto = tof; ppo = pof; poo = oof;
  }
  return rows;
}

// DocIdIterator (flash_iterators.h:121-262) with DeltaEncodedPackedIntsIterator /
// DeltaEncodedVIntsIterator (packed_value.h:320-369,463-507).
class DocIdIter {
 public:
  void reset(const uint8_t* file, const std::vector<SkipEntry>* sl, int n) {
    file_ = file; sl_ = sl; n_ = n; fmt_ = 0; cur_ = 0;
    skip_to(0);
  }
  int posting_index() const { return cur_; }
  bool is_end() const { return cur_ == n_; }
  uint32_t value() const {
    if (fmt_ == 1) return static_cast<uint32_t>(pack_prev_ + pack_.cache[pack_idx_]);
    return static_cast<uint32_t>(vprev_ + vints_.peek());
  }
  void advance() { skip_to(cur_ + 1); }
  void skip_to(int posting) {
    const int blob = posting / kPack, off = posting % kPack;
    if (fmt_ == 0 || cur_blob() != blob) {
      if (posting >= n_) { cur_ = n_; return; }
      setup(blob);
    }
    if (fmt_ == 2) { while (vints_.index() < off) vprev_ += vints_.pop(); }
    else { while (pack_idx_ < off) { pack_prev_ = value(); ++pack_idx_; } }
    cur_ = posting;
  }
  // flash_iterators.h:181-199: linear walk over skip rows, then in-blob scan
  void skip_forward(uint32_t val) {
    int blob_to_go = cur_blob();
    const int last = (n_ - 1) / kPack;
    while (blob_to_go + 1 <= last && (*sl_)[blob_to_go + 1].prev_doc < val) ++blob_to_go;
    const int base = blob_to_go * kPack;
    if (blob_to_go != cur_blob()) skip_to(base);
    if (fmt_ == 2) {
      while (!vints_.is_end() && vprev_ + vints_.peek() < val) vprev_ += vints_.pop();
      cur_ = base + vints_.index();
    } else {
      while (pack_idx_ != kPack && value() < val) { pack_prev_ = value(); ++pack_idx_; }
      cur_ = base + pack_idx_;
    }
  }

 private:
  int cur_blob() const { return cur_ / kPack; }
  void setup(int blob) {
    const SkipEntry& e = (*sl_)[blob];
    const uint8_t* p = file_ + e.doc_off;
    if (p[0] == kPackMagic) {
      fmt_ = 1; pack_.reset(p); pack_.decode(); pack_idx_ = 0; pack_prev_ = e.prev_doc;
    } else if (p[0] == kVIntsMagic) {
      fmt_ = 2; vints_.reset(p); vprev_ = e.prev_doc;
    } else {
      throw std::runtime_error("docid blob format");
    }
  }
  const uint8_t* file_ = nullptr;
  const std::vector<SkipEntry>* sl_ = nullptr;
  int n_ = 0, cur_ = 0, fmt_ = 0;  // fmt: 0 none, 1 pack, 2 vints
  PackReader pack_;
  int pack_idx_ = 0;
  long pack_prev_ = 0;
  VIntsIter vints_;
  long vprev_ = 0;
};

// TermFreqIterator (flash_iterators.h:43-118)
class TfIter {
 public:
  void reset(const uint8_t* file, const std::vector<SkipEntry>* sl) { file_ = file; sl_ = sl; fmt_ = 0; cur_ = 0; }
  uint32_t at(int posting) {
    const int blob = posting / kPack, off = posting % kPack;
    if (fmt_ == 0 || cur_ / kPack != blob) {
      const uint8_t* p = file_ + (*sl_)[blob].tf_off;
      if (p[0] == kPackMagic) { fmt_ = 1; pack_.reset(p); pack_.decode(); }
      else { fmt_ = 2; vints_.reset(p); }
    }
    cur_ = posting;
    if (fmt_ == 1) return pack_.cache[off];
    vints_.skip_to(off);
    return static_cast<uint32_t>(vints_.peek());
  }

 private:
  const uint8_t* file_ = nullptr;
  const std::vector<SkipEntry>* sl_ = nullptr;
  int fmt_ = 0, cur_ = 0;
  PackReader pack_;
  VIntsIter vints_;
};

// ---------------------------------------------------------------- bloom --
std::atomic<int64_t> g_bloom_checks{0}, g_bloom_pruned{0};

// MurmurHash2 (libbloom/murmur2/MurmurHash2.c:15-64), little-endian reads
uint32_t murmur2(const void* key, int len, uint32_t seed) {
  const uint32_t m = 0x5bd1e995;
  uint32_t h = seed ^ static_cast<uint32_t>(len);
  const uint8_t* d = static_cast<const uint8_t*>(key);
  for (; len >= 4; d += 4, len -= 4) {
    uint32_t k = static_cast<uint32_t>(d[0]) | static_cast<uint32_t>(d[1]) << 8 |
                 static_cast<uint32_t>(d[2]) << 16 | static_cast<uint32_t>(d[3]) << 24;
    k *= m; k ^= k >> 24; k *= m;
    h *= m; h ^= k;
  }
  if (len == 3) h ^= static_cast<uint32_t>(d[2]) << 16;
  if (len >= 2) h ^= static_cast<uint32_t>(d[1]) << 8;
  if (len >= 1) { h ^= d[0]; h *= m; }
  h ^= h >> 13; h *= m; h ^= h >> 15;
  return h;
}

// bloom_set (libbloom/bloom.c:84-115) + bloom_check (:48-75): 1 = may be present
struct BloomParams {
  int bits = 0, hashes = 0;
  void set(int entries, double error) {
    const double bpe = -(std::log(error) / 0.480453013918201);
    bits = static_cast<int>(static_cast<double>(entries) * bpe);
    hashes = static_cast<int>(std::ceil(0.693147180559945 * bpe));
  }
  int check(const uint8_t* bf, const std::string& s) const {
    const uint32_t a = murmur2(s.data(), static_cast<int>(s.size()), 0x9747b28c);
    const uint32_t b = murmur2(s.data(), static_cast<int>(s.size()), a);
    int hits = 0;
    for (uint32_t i = 0; i < static_cast<uint32_t>(hashes); ++i) {
      const uint32_t x = (a + i * b) % static_cast<uint32_t>(bits);
      if (bf[x >> 3] & (1u << (x % 8))) ++hits;
    }
    return hits == hashes ? 1 : 0;
  }
};

// VacuumHeader (flash_iterators.h:826-889): the "end" fields are the ones used
// by both readers
struct VacHeader {
  bool has_bloom = false;
  uint32_t bit_array_bytes = 0, expected_entries = 0;
  float ratio = 0;
  void load(const uint8_t* p) {
    ++p;
    uint64_t v[3];
    for (int s = 0; s < 2; ++s) {
      for (int i = 0; i < 3; ++i) p += varint_decode(p, &v[i]);
      float r;
      std::memcpy(&r, p, 4);
      p += 4;
      if (s == 1) {
        has_bloom = v[0] != 0;
        bit_array_bytes = static_cast<uint32_t>(v[1]);
        expected_entries = static_cast<uint32_t>(v[2]);
        ratio = r;
      }
    }
  }
};

// BloomFilterColumnReader (flash_iterators.h:776-823) over BloomSkipList and
// BloomBoxIterator (flash_containers.h:560-687): the bit array of a posting,
// nullptr when its box bitmap marks it absent
class BloomColumn {
 public:
  void reset(const uint8_t* pl, uint64_t section_off, uint32_t item_bytes) {
    pl_ = pl; sec_ = pl + section_off; item_bytes_ = item_bytes; loaded_ = false; box_ = -1;
  }
  const uint8_t* bit_array(int posting) {
    if (!loaded_) {   // LoadSkipList: 0xA4 | n | delta offsets from the list start
      if (sec_[0] != 0xA4) throw std::runtime_error("bloom skip list magic");
      uint64_t n, prev = 0;
      const uint8_t* p = sec_ + 1;
      p += varint_decode(p, &n);
      boxes_.clear();
      for (uint64_t i = 0; i < n; ++i) { uint64_t d; p += varint_decode(p, &d); prev += d; boxes_.push_back(prev); }
      loaded_ = true;
    }
    const int box = posting / kPack;
    if (box != box_) {   // BloomBoxIterator::Fill
      const uint8_t* b = pl_ + boxes_.at(box);
      if (b[0] != 0xF5) throw std::runtime_error("bloom box magic");
      uint64_t n;
      const uint8_t* p = b + 1;
      p += varint_decode(p, &n);
      int phys = 0;
      for (uint64_t i = 0; i < n; ++i) {
        const bool has = p[i / 8] & (0x80u >> (i % 8));   // DecodeBitmapByte, MSB first
        map_[i] = has ? phys++ : -1;
      }
      items_ = p + (n + 7) / 8;
      n_ = static_cast<int>(n);
      box_ = box;
    }
    const int i = posting % kPack;
    if (i >= n_ || map_[i] < 0) return nullptr;
    return items_ + static_cast<uint64_t>(map_[i]) * item_bytes_;
  }

 private:
  const uint8_t* pl_ = nullptr;
  const uint8_t* sec_ = nullptr;
  uint32_t item_bytes_ = 0;
  bool loaded_ = false;
  std::vector<uint64_t> boxes_;
  int box_ = -1, n_ = 0;
  int map_[kPack];
  const uint8_t* items_ = nullptr;
};

// CozyBoxIterator (flash_iterators.h:280-412): a run of packs then one VInts
// blob; it does not know where the box ends (the caller counts entries).
class CozyIter {
 public:
  void reset(const uint8_t* file) { file_ = file; type_ = 0; blob_off_ = 0; idx_ = 0; }
  int type() const { return type_; }
  // GoToCozyEntry (:294-305)
  void go(uint64_t blob_off, int in_blob) {
    if (type_ == 0 || blob_off_ != blob_off) setup(blob_off);
    if (type_ == 2) vints_.skip_to(in_blob);
    idx_ = in_blob;
  }
  uint32_t value() const {  // :339-348
    return type_ == 1 ? pack_.cache[idx_] : static_cast<uint32_t>(vints_.peek());
  }
  void advance() {  // :309-315
    go(blob_off_, idx_ + 1);
    if (at_blob_end()) go(blob_off_ + blob_bytes(), 0);
  }
  void advance_by(int n) {  // AdvanceBy (:319-337)
    while (n > 0) {
      if (type_ == 1) {
        const int remain = kPack - idx_;
        if (n < remain) { idx_ += n; n = 0; }
        else { go(blob_off_ + blob_bytes(), 0); n -= remain; }
      } else {
        advance();
        --n;
      }
    }
  }

 private:
  bool at_blob_end() const { return type_ == 1 ? idx_ >= kPack : vints_.is_end(); }
  // PackedIntsIterator / VIntsIterator::SerializationSize (packed_value.h:426-428
  // assumes a 1-byte length varint; a VInts blob is always a box's last)
  uint64_t blob_bytes() const { return type_ == 1 ? 2 + 16ull * pack_.bits : 2 + vints_.end; }
  void setup(uint64_t blob_off) {  // SetupBlob (:390-403)
    const uint8_t* p = file_ + blob_off;
    if (p[0] == kPackMagic) { type_ = 1; pack_.reset(p); pack_.decode(); }
    else if (p[0] == kVIntsMagic) { type_ = 2; vints_.reset(p); }
    else throw std::runtime_error("cozy box blob format");
    blob_off_ = blob_off;
    idx_ = 0;
  }
  const uint8_t* file_ = nullptr;
  int type_ = 0;  // 0 none, 1 pack, 2 vints
  uint64_t blob_off_ = 0;
  int idx_ = 0;
  PackReader pack_;
  VIntsIter vints_;
};

// PositionPostingBagIterator (flash_iterators.h:458-634): the positions of one
// posting ("bag", tf entries, delta coded from 0 inside the bag).  Bags are
// found from the skip row of their 128-posting interval plus the tfs before.
// offsets = true: OffsetPostingBagIterator (:667-704) -- 2 x tf entries per bag
// (start, end pairs), the skip rows' offset columns -- popped as
// LazyBoundedOffsetPairIterator::SinglePop (:748-760), whose running value also
// starts from 0 at the bag.
class PosBagIter {
 public:
  void reset(const uint8_t* file, const std::vector<SkipEntry>* sl, bool offsets = false) {
    cozy_.reset(file); sl_ = sl; tf_.reset(file, sl); cur_bag_ = 0; mult_ = offsets ? 2 : 1;
  }
  void skip_to(int bag) {  // SkipTo (:570-591)
    if (cozy_.type() == 0 || bag / kPack > cur_bag_ / kPack) {
      jump(bag);
    } else {
      cozy_.advance_by(entries_between(cur_bag_, bag) - n_adv_);
    }
    cur_bag_ = bag;
    prev_ = 0;
    tf_cur_ = static_cast<int>(tf_.at(bag)) * mult_;
    n_popped_ = 0;
    n_adv_ = 0;
  }
  uint32_t pop() {  // PopInBag (:593-604)
    const uint32_t pos = prev_ + cozy_.value();
    prev_ = pos;
    ++n_popped_;
    if (n_popped_ < tf_cur_) { cozy_.advance(); ++n_adv_; }
    return pos;
  }
  bool is_end() const { return n_popped_ >= tf_cur_; }  // IsEndInBag (:606-608)

 private:
  int entries_between(int a, int b) {  // NumCozyEntriesBetween (:619-628)
    int n = 0;
    for (int i = a; i < b; ++i) n += static_cast<int>(tf_.at(i)) * mult_;
    return n;
  }
  void jump(int bag) {  // JumpToPostingBag / FindSkipInterval / GoToSkipPostingBag (:504-536)
    int i = cur_bag_ / kPack;
    while (i + 1 < static_cast<int>(sl_->size()) && (i + 1) * kPack <= bag) ++i;
    const SkipEntry& e = (*sl_)[i];
    if (mult_ == 2) cozy_.go(e.off_off, static_cast<int>(e.off_idx));
    else cozy_.go(e.pos_off, static_cast<int>(e.pos_idx));
    cur_bag_ = i * kPack;
    cozy_.advance_by(entries_between(i * kPack, bag));
  }
  CozyIter cozy_;
  const std::vector<SkipEntry>* sl_ = nullptr;
  TfIter tf_;
  int cur_bag_ = 0, n_popped_ = 0, n_adv_ = 0, tf_cur_ = 0, mult_ = 1;
  uint32_t prev_ = 0;
};

// PhraseQueryProcessor2 (query_processing.h:170-382) over pop-iterators
// (IsEnd / Pop); returns NumOfMatches and, when `table` is given, the matched
// positions per term (PositionInfoTable2 rows).
template <class PosIt>
int phrase_process(std::vector<PosIt*>& its, std::vector<std::vector<int>>* table,
                   std::vector<std::vector<int>>* apr = nullptr) {
  const int n = static_cast<int>(its.size());
  int matches = 0;
  // AppendPositionCol / pos_table_.Append: PositionInfo{pos, term_appearance}
  auto append = [&](int row, int pos, int ap) {
    if (table) (*table)[row].push_back(pos);
    if (apr) (*apr)[row].push_back(ap);
  };
  if (table) table->assign(n, {});
  if (apr) apr->assign(n, {});
  if (n == 2) {  // ProcessTwoTerm (:264-310)
    PosIt* it0 = its[0];
    PosIt* it1 = its[1];
    int pos0 = -100, pos1 = -200;
    int apr0 = -1, apr1 = -1;
    bool tried_pop_end = false;
    while (!tried_pop_end) {
      if (pos0 < pos1) {
        if (!it0->is_end()) { pos0 = static_cast<int>(it0->pop()); ++apr0; }
        else tried_pop_end = true;
      } else if (pos0 > pos1) {
        if (!it1->is_end()) { pos1 = static_cast<int>(it1->pop()) - 1; ++apr1; }
        else tried_pop_end = true;
      } else {
        append(0, pos0, apr0);
        append(1, pos1 + 1, apr1);
        ++matches;
        if (!it0->is_end()) { pos0 = static_cast<int>(it0->pop()); ++apr0; }
        else tried_pop_end = true;
        if (!it1->is_end()) { pos1 = static_cast<int>(it1->pop()) - 1; ++apr1; }
        else tried_pop_end = true;
      }
    }
    return matches;
  }
  // ProcessGeneral (:312-336) with InitializeLastPopped / FindMaxAdjustedLastPopped /
  // MovePoppedBeyond / IsPoppedMatch (:180-252); positions are int (Position)
  std::vector<int> last(n), ap(n, 0);
  for (int i = 0; i < n; ++i) {
    if (its[i]->is_end()) return 0;
    last[i] = static_cast<int>(its[i]->pop());
    ap[i] = 0;
  }
  auto move_beyond = [&](int mx) {
    for (int i = 0; i < n; ++i) {
      while (!its[i]->is_end() && last[i] - i < mx) { last[i] = static_cast<int>(its[i]->pop()); ++ap[i]; }
      if (its[i]->is_end() && last[i] - i < mx) return false;
    }
    return true;
  };
  for (;;) {
    int mx = 0;
    for (int i = 0; i < n; ++i) mx = std::max(mx, last[i] - i);
    if (!move_beyond(mx)) break;
    bool match = true;
    for (int i = 0; i < n; ++i) match = match && last[i] - i == mx;
    if (match) {
      for (int i = 0; i < n; ++i) append(i, last[i], ap[i]);
      ++matches;
      if (!move_beyond(mx + 1)) break;
    }
  }
  return matches;
}

// VacuumPostingListIterator (flash_iterators.h:893-1079).  Bloom filters are
// not read: with an index written without them the reference's HasTerm answers
// BLM_MAY_PRESENT (:1039-1058) and every found doc goes to the position check.
class VacuumIter {
 public:
  VacuumIter(const uint8_t* file, uint64_t off, const VacHeader* hdr = nullptr,
             const std::string* term = nullptr)
      : hdr_(hdr), term_(term) {
    const uint8_t* buf = file + off;
    if (buf[0] != kPostingMagic) throw std::runtime_error("posting list magic");
    uint64_t df;
    int l = varint_decode(buf + 1, &df);
    n_ = static_cast<int>(df);
    if (hdr_ && hdr_->has_bloom) {   // the 8 reserved bytes: section offsets (:923-944)
      uint64_t b0, b1;
      const uint8_t* p = buf + 1 + l;
      p += varint_decode(p, &b0);
      varint_decode(p, &b1);
      blm_ = std::make_shared<std::vector<BloomColumn>>(2);
      (*blm_)[0].reset(buf, b0, hdr_->bit_array_bytes);
      (*blm_)[1].reset(buf, b1, hdr_->bit_array_bytes);
      bparams_.set(static_cast<int>(hdr_->expected_entries), static_cast<double>(hdr_->ratio));
    }
    skip_ = std::make_shared<std::vector<SkipEntry>>(load_skip_list(buf + 1 + l + 8));
    file_ = file;
    doc_.reset(file, skip_.get(), n_);
    tf_.reset(file, skip_.get());
    pos_ = std::make_shared<PosBagIter>();
    pos_->reset(file, skip_.get());
  }
  int size() const { return n_; }
  bool is_end() const { return doc_.is_end(); }
  int doc_id() const { return static_cast<int>(doc_.value()); }
  int term_freq() { return static_cast<int>(tf_.at(doc_.posting_index())); }
  void advance() { doc_.advance(); }
  void skip_forward(uint32_t d) { doc_.skip_forward(d); }
  void skip_to(int posting) { doc_.skip_to(posting); }   // DocIdIterator::SkipTo (flash_iterators.h:170-179)
  // AssignPositionBegin (:1002-1005)
  PosBagIter* position_begin() { pos_->skip_to(doc_.posting_index()); return pos_.get(); }
  int posting_index() const { return doc_.posting_index(); }
  // OffsetPairsBegin (:1007-1012) -> LazyBoundedOffsetPairIterator drained by
  // ResultDocEntry::ExpandOffsets (query_processing.h:454-466): the (start, end)
  // pairs of posting `posting`
  std::vector<std::pair<int, int>> offset_pairs(int posting) const {
    PosBagIter it;
    it.reset(file_, skip_.get(), true);
    it.skip_to(posting);
    std::vector<std::pair<int, int>> v;
    while (!it.is_end()) {
      const int a = static_cast<int>(it.pop());
      const int b = static_cast<int>(it.pop());
      v.emplace_back(a, b);
    }
    return v;
  }
  const std::string& term() const { return *term_; }
  // HasPriorTerm / HasNextTerm / HasTerm (:994-1000,1039-1058): 0 = not present,
  // 1 = may be present (always, without bloom filters)
  int has_prior_term(const std::string& t) { return has_term(0, t); }
  int has_next_term(const std::string& t) { return has_term(1, t); }

 private:
  int has_term(int side, const std::string& t) {
    if (!blm_) return 1;
    ++g_bloom_checks;
    const uint8_t* bf = (*blm_)[side].bit_array(doc_.posting_index());
    const int r = bf ? bparams_.check(bf, t) : 0;
    if (!r) ++g_bloom_pruned;
    return r;
  }
  const VacHeader* hdr_ = nullptr;
  const std::string* term_ = nullptr;
  std::shared_ptr<std::vector<BloomColumn>> blm_;
  BloomParams bparams_;
  int n_ = 0;
  const uint8_t* file_ = nullptr;
  std::shared_ptr<std::vector<SkipEntry>> skip_;
  DocIdIter doc_;
  TfIter tf_;
  std::shared_ptr<PosBagIter> pos_;
};

// ----------------------------------------------- qq_mem varint postings ----
// StandardPosting::Encode (posting.h:130-151): content_size | doc_id_delta | TF |
// off_size | offsets (start, end), each a delta to the previous value, from an
// imaginary 0 (:85-99) | positions, deltas from an imaginary 0 (:101-113);
// content_size counts everything after itself, off_size the offset bytes.
void vb_append(std::string* s, uint64_t v) {
  uint8_t b[10];
  const int n = varint_encode(v, b);
  s->append(reinterpret_cast<const char*>(b), n);
}

std::string standard_posting_encode(uint32_t doc_delta, uint32_t tf,
                                    const std::vector<std::pair<uint32_t, uint32_t>>& offs,
                                    const std::vector<uint32_t>& pos) {
  std::string info, off, pbuf, out;
  vb_append(&info, doc_delta);
  vb_append(&info, tf);
  uint32_t last = 0;
  for (auto& pr : offs) {
    vb_append(&off, pr.first - last);
    last = pr.first;
    vb_append(&off, pr.second - last);
    last = pr.second;
  }
  std::string off_sized;
  vb_append(&off_sized, off.size());   // VarintBuffer::Prepend(Size())
  off_sized += off;
  last = 0;
  for (uint32_t p : pos) { vb_append(&pbuf, p - last); last = p; }
  vb_append(&out, info.size() + off_sized.size() + pbuf.size());
  out += info;
  out += off_sized;
  out += pbuf;
  return out;
}

// PostingListDelta (posting_list_delta.h:397-470): postings appended as
// StandardPosting bytes with doc-id deltas (posting[-1] = posting[0], so the
// first delta is 0); every skip_span postings a skip entry (doc id of the
// posting before, byte offset of the span's first posting).
struct PostingListDelta {
  int span = 100;   // :399
  std::string data;
  std::vector<std::pair<uint32_t, uint64_t>> skip;   // (prev_doc_id, start_offset)
  int n = 0;
  uint32_t last = 0;
  void add(uint32_t doc, uint32_t tf, const std::vector<std::pair<uint32_t, uint32_t>>& offs,
           const std::vector<uint32_t>& pos) {
    if (n == 0) last = doc;
    else if (doc <= last) throw std::runtime_error("doc ids must increase in a posting list");
    if (n % span == 0) skip.emplace_back(last, data.size());
    data += standard_posting_encode(doc - last, tf, offs, pos);
    last = doc;
    ++n;
  }
};

// PostingListDeltaIterator (posting_list_delta.h:161-394): DecodeToCache reads
// content size, doc delta, tf, offset size; Advance moves to the next posting;
// SkipForward walks postings, jumping a whole span when the next span's first
// doc (its skip entry's prev_doc_id) is still below the target.
class DeltaIter {
 public:
  explicit DeltaIter(const PostingListDelta* pl) : pl_(pl), addr_(0), idx_(0), prev_(pl->skip[0].first) {
    decode();
  }
  int size() const { return pl_->n; }
  bool is_end() const { return idx_ == pl_->n; }
  int doc_id() const { return static_cast<int>(doc_); }
  int term_freq() const { return static_cast<int>(tf_); }
  int posting_index() const { return idx_; }
  void advance() {
    addr_ = next_;
    ++idx_;
    prev_ = doc_;
    decode();
  }
  bool has_skip() const { return idx_ % pl_->span == 0 && idx_ + pl_->span < pl_->n; }
  uint32_t next_span_doc_id() const { return pl_->skip[idx_ / pl_->span + 1].first; }
  void skip_to_next_span() {
    const int s = idx_ / pl_->span + 1;
    addr_ = pl_->skip[s].second;
    idx_ = s * pl_->span;
    prev_ = pl_->skip[s].first;
    decode();
  }
  void skip_forward(uint32_t v) {
    while (idx_ < pl_->n && doc_ < v) {
      if (has_skip() && next_span_doc_id() < v) skip_to_next_span();
      else advance();
    }
  }
  // the current posting's offset pairs and positions (CompressedPairIterator /
  // CompressedPositionIterator, posting_list_delta.h:281-296)
  std::vector<std::pair<uint32_t, uint32_t>> offsets() const {
    std::vector<std::pair<uint32_t, uint32_t>> out;
    uint64_t at = off_start_, last = 0;
    while (at < pos_start_) {
      uint64_t a, b;
      at += varint_decode(raw() + at, &a);
      at += varint_decode(raw() + at, &b);
      const uint32_t s = static_cast<uint32_t>(last + a);
      const uint32_t e = static_cast<uint32_t>(s + b);
      out.emplace_back(s, e);
      last = e;
    }
    return out;
  }
  std::vector<uint32_t> positions() const {
    std::vector<uint32_t> out;
    uint64_t at = pos_start_, last = 0;
    while (at < next_) {
      uint64_t d;
      at += varint_decode(raw() + at, &d);
      last += d;
      out.push_back(static_cast<uint32_t>(last));
    }
    return out;
  }
  PosBagIter* position_begin() { throw std::runtime_error("phrase queries need a Vacuum index"); }
  const std::string& term() const { throw std::runtime_error("phrase queries need a Vacuum index"); }
  int has_prior_term(const std::string&) { return 1; }
  int has_next_term(const std::string&) { return 1; }

 private:
  const uint8_t* raw() const { return reinterpret_cast<const uint8_t*>(pl_->data.data()); }
  void decode() {   // DecodeToCache (:299-318); nothing to read past the last posting
    if (idx_ >= pl_->n) return;
    uint64_t content, delta, tf, osz;
    uint64_t at = addr_;
    at += varint_decode(raw() + at, &content);
    next_ = at + content;
    at += varint_decode(raw() + at, &delta);
    doc_ = static_cast<uint32_t>(prev_ + delta);
    at += varint_decode(raw() + at, &tf);
    tf_ = static_cast<uint32_t>(tf);
    at += varint_decode(raw() + at, &osz);
    off_start_ = at;
    pos_start_ = at + osz;
  }
  const PostingListDelta* pl_;
  uint64_t addr_;
  int idx_;
  uint32_t prev_;
  uint32_t doc_ = 0, tf_ = 0;
  uint64_t next_ = 0, off_start_ = 0, pos_start_ = 0;
};

// ----------------------------------------------------------- the heap ----
// std::priority_queue<unique_ptr<ResultDocEntry>, vector, EntryGreater>
// (query_processing.h:510-524) with libstdc++'s __push_heap / __adjust_heap /
// __pop_heap restated; comp(a, b) = a.score > b.score.
// With snippets on, an entry also keeps what ResultDocEntry keeps for them
// (query_processing.h:386-445): each list's posting index at the doc (its
// LazyBoundedOffsetPairIterator), the phrase match table's term appearances
// (PositionInfoTable2, RankDocForPhrase) and is_phrase.
struct Entry {
  int doc;
  double score;
  std::vector<int> post;
  std::vector<std::vector<int>> apr;
  bool phrase = false;
};
class MinHeap {
 public:
  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  const Entry& top() const { return v_[0]; }
  void push(const Entry& e) {
    v_.push_back(e);
    push_hole(static_cast<long>(v_.size()) - 1, 0, e);
  }
  void pop() {
    if (v_.size() > 1) {
      const long len = static_cast<long>(v_.size()) - 1;
      Entry value = v_[len];
      v_[len] = v_[0];
      adjust(0, len, value);
    }
    v_.pop_back();
  }

 private:
  static bool comp(const Entry& a, const Entry& b) { return a.score > b.score; }
  void push_hole(long hole, long top, Entry value) {
    long parent = (hole - 1) / 2;
    while (hole > top && comp(v_[parent], value)) {
      v_[hole] = v_[parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    v_[hole] = value;
  }
  void adjust(long hole, long len, Entry value) {
    const long top = hole;
    long child = hole;
    while (child < (len - 1) / 2) {
      child = 2 * (child + 1);
      if (comp(v_[child], v_[child - 1])) --child;
      v_[hole] = v_[child];
      hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
      child = 2 * (child + 1);
      v_[hole] = v_[child - 1];
      hole = child - 1;
    }
    push_hole(hole, top, value);
  }
  std::vector<Entry> v_;
};

// ProcessorBase / NonPhraseProcessorBase / *QueryProcessor (query_processing.h:527-950)
template <class It>
class Processor {
 public:
  Processor(const Bm25& sim, std::vector<It>* its, const std::vector<uint8_t>& lens, int n_docs, int k,
            bool phrase = false, int bloom_factor = 1)
      : sim_(sim), its_(*its), lens_(lens), k_(k), phrase_(phrase), bloom_factor_(bloom_factor) {
    for (auto& it : its_) idf_.push_back(es_idf(n_docs, it.size()));   // :544-547
  }
  // qq_search::ProcessQueryDelta dispatch (:966-978): one term ->
  // SingleTermQueryProcessor; two terms, not a phrase -> TwoTermNonPhrase; else
  // QueryProcessor (ProcessTwoTerm / ProcessMultipleTerms, same intersection
  // loops, HandleTheFoundDoc :886-895 on every doc found)
  std::vector<Entry> run() {
    if (its_.size() == 1) single();
    else if (its_.size() == 2) two();
    else multi();
    return sort_heap();
  }
  int64_t phrase_checks() const { return n_phrase_checks_; }
  void capture(bool on) { capture_ = on; }

 private:
  // CalcDocScoreLossy (scoring.h:124-145), terms in query order
  double score(int doc) {
    double s = 0;
    const uint8_t c = static_cast<size_t>(doc) < lens_.size() ? lens_[doc] : 0;
    for (size_t i = 0; i < its_.size(); ++i) {
      const int tf = its_[i].term_freq();
      double tfn = sim_.tfnorm_lossy(tf, c);
      double t = idf_[i] * tfn;
      s += t;
    }
    return s;
  }
  // RankDoc (query_processing.h:588-603) / RankDocForPhrase (:897-912) and
  // InsertToHeap (:605-616, :914-925)
  void rank(int doc, std::vector<std::vector<int>>* apr = nullptr) {
    const double s = score(doc);
    if (heap_.size() < static_cast<size_t>(k_)) insert(doc, s, apr);
    else if (s > heap_.top().score) { heap_.pop(); insert(doc, s, apr); }
  }
  void insert(int doc, double s, std::vector<std::vector<int>>* apr) {
    Entry e{doc, s};
    if (capture_) {
      for (auto& it : its_) e.post.push_back(it.posting_index());
      if (apr) { e.apr = *apr; e.phrase = true; }
    }
    heap_.push(e);
  }
  // HandleTheFoundDoc (:886-895): a phrase query ranks the doc only when the
  // positions hold the phrase (FindPhrase :854-867; RankDocForPhrase scores and
  // inserts exactly as RankDoc, :897-912)
  // IsPossibleToPresent (:873-884) with CheckBloomWithEnableFactor (:796-807) and
  // CheckBloomFallBack (:784-794); BLOOM_NEVER_USE = 0 (types.h:54)
  bool possible() {
    if (bloom_factor_ == 0) return true;
    if (its_.size() != 2) {
      for (size_t i = 0; i + 1 < its_.size(); ++i)
        if (its_[i].has_next_term(its_[i + 1].term()) == 0) return false;
      return true;
    }
    const size_t s1 = static_cast<size_t>(its_[0].size()), s2 = static_cast<size_t>(its_[1].size());
    const size_t f = static_cast<size_t>(bloom_factor_);
    if (f * s1 <= s2) return its_[0].has_next_term(its_[1].term()) != 0;
    if (f * s2 < s1) return its_[1].has_prior_term(its_[0].term()) != 0;
    return true;
  }
  void found(int doc) {
    if (phrase_ && its_.size() > 1) {
      ++n_phrase_checks_;
      if (!possible()) return;   // FindPhrase returns 0 matches
      std::vector<PosBagIter*> ps;
      for (auto& it : its_) ps.push_back(it.position_begin());
      std::vector<std::vector<int>> apr;
      if (phrase_process(ps, nullptr, capture_ ? &apr : nullptr) > 0) rank(doc, capture_ ? &apr : nullptr);
    } else {
      rank(doc);
    }
  }
  void single() {  // :632-641
    auto& it = its_[0];
    while (!it.is_end()) { rank(it.doc_id()); it.advance(); }
  }
  void two() {  // TwoTermNonPhraseQueryProcessor::Process :656-677
    auto& a = its_[0];
    auto& b = its_[1];
    while (!a.is_end() && !b.is_end()) {
      const int d0 = a.doc_id(), d1 = b.doc_id();
      if (d0 > d1) b.skip_forward(d0);
      else if (d0 < d1) a.skip_forward(d1);
      else { found(d0); a.advance(); b.advance(); }
    }
  }
  void multi() {  // ProcessMultipleTerms / FindMax / FindMatch :710-728,810-852
    for (;;) {
      int mx = -1;
      bool fin = false;
      for (auto& it : its_) {
        if (it.is_end()) { fin = true; break; }
        if (it.doc_id() > mx) mx = it.doc_id();
      }
      if (fin) break;
      for (size_t i = 0; i < its_.size(); ++i) {
        auto& it = its_[i];
        it.skip_forward(static_cast<uint32_t>(mx));
        if (it.is_end()) { fin = true; break; }
        if (it.doc_id() != mx) break;
        if (i == its_.size() - 1) {
          found(mx);
          for (auto& x : its_) x.advance();
        }
      }
      if (fin) break;
    }
  }
  std::vector<Entry> sort_heap() {  // :551-562
    std::vector<Entry> r;
    int kk = k_;
    while (!heap_.empty() && kk != 0) { r.push_back(heap_.top()); heap_.pop(); --kk; }
    std::reverse(r.begin(), r.end());
    return r;
  }
  const Bm25& sim_;
  std::vector<It>& its_;
  const std::vector<uint8_t>& lens_;
  int k_;
  bool phrase_;
  int bloom_factor_;
  int64_t n_phrase_checks_ = 0;
  bool capture_ = false;
  std::vector<double> idf_;
  MinHeap heap_;
};

// ----------------------------------------------------------- snippets ----
// LZ4 is the reference's own third-party codec for the doc store
// (doc_store.h:15,26-128); the system liblz4 1.9.3 is linked.
extern "C" int LZ4_decompress_safe(const char* src, char* dst, int compressed_size, int dst_capacity);

// ChunkedDocStoreReader (doc_store.h:365-455) with DecompressText /
// DecodeHeader (:50-128): my.fdx = varint n_doc_ids | varint buffer size |
// n x int64 (offset << 1 | aligned); my.fdt chunks = 0x33 | varint n_chunks |
// varint chunk sizes | LZ4 blocks.
class DocStoreReader {
 public:
  ~DocStoreReader() { if (fdt_) munmap(fdt_, fdt_len_); }
  void load(const std::string& dir) {
    std::ifstream f(dir + "/my.fdx", std::ios::binary);
    if (!f) throw std::runtime_error("cannot open my.fdx");
    std::string raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const uint8_t* a = reinterpret_cast<const uint8_t*>(raw.data());
    uint64_t n, bs;
    size_t at = varint_decode(a, &n);
    at += varint_decode(a + at, &bs);
    n_ = static_cast<int>(n);
    buf_size_ = static_cast<int>(bs);
    for (int i = 0; i < n_; ++i) {
      int64_t v;
      std::memcpy(&v, a + at, 8);
      at += 8;
      offsets_.push_back(v);
    }
    int fd = ::open((dir + "/my.fdt").c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open my.fdt");
    struct stat sb;
    fstat(fd, &sb);
    fdt_len_ = sb.st_size;
    if (fdt_len_) {
      void* p = mmap(nullptr, fdt_len_, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) { ::close(fd); throw std::runtime_error("mmap my.fdt"); }
      fdt_ = static_cast<uint8_t*>(p);
    }
    ::close(fd);
  }
  std::string get(int id) const {  // Get (:426-443)
    if (id < 0 || id >= n_) throw std::runtime_error("doc id outside the doc store");
    int64_t start = offsets_[id];
    if (start & 1) { start >>= 1; start = start + 4096 - start % 4096; }
    else start >>= 1;
    const uint8_t* c = fdt_ + start;
    if (c[0] != 0x33) throw std::runtime_error("Compressed doc has the wrong magic number");
    VIntsHeaderless hdr{c + 1};
    const uint64_t nch = hdr.pop();
    std::vector<uint64_t> sizes;
    for (uint64_t i = 0; i < nch; ++i) sizes.push_back(hdr.pop());
    const char* chunk = reinterpret_cast<const char*>(c + 1 + hdr.off);
    std::vector<char> buf(buf_size_);
    std::string text;
    for (uint64_t i = 0; i < nch; ++i) {
      const int got = LZ4_decompress_safe(chunk, buf.data(), static_cast<int>(sizes[i]), buf_size_);
      if (got < 0) throw std::runtime_error("Failed to decompresse.");
      chunk += sizes[i];
      text.append(buf.data(), got);
    }
    return text;
  }

 private:
  struct VIntsHeaderless {   // VarintIteratorUnbounded
    const uint8_t* p;
    size_t off = 0;
    uint64_t pop() { uint64_t v; off += varint_decode(p + off, &v); return v; }
  };
  int n_ = 0, buf_size_ = 0;
  std::vector<int64_t> offsets_;
  uint8_t* fdt_ = nullptr;
  size_t fdt_len_ = 0;
};

// SimpleHighlighter::highlightOffsetsEnums (highlighter.h:297-456) with
// SentenceBreakIteratorNew (:118-197), Passage (:79-116), Offset_Iterator
// (:46-73).  float arithmetic as the reference (pivot 87, k1 1.2, b 0.75).
using OffPair = std::pair<int, int>;
struct HlOffsetIt {
  const std::vector<OffPair>* offs;
  size_t i = 0;
  int start, end, weight = 1;
  explicit HlOffsetIt(const std::vector<OffPair>* o) : offs(o) {
    start = (*o)[0].first;   // (the reference dereferences begin() unchecked)
    end = (*o)[0].second;
  }
  void next() {
    ++i;
    if (i == offs->size()) { start = end = -1; return; }
    start = (*offs)[i].first;
    end = (*offs)[i].second;
  }
};
struct HlPassage {
  int start = -1, end = -1;
  float score = 0;
  std::vector<OffPair> matches;
  void reset() { start = end = -1; score = 0; matches.clear(); }
  std::string to_string(const std::string& doc) {   // :97-115
    std::string res = doc.substr(start, end - start + 1) + "\n";
    std::sort(matches.begin(), matches.end(),
              [](const OffPair& a, const OffPair& b) { return a.first > b.first; });
    for (auto& m : matches) {
      res.insert(m.second - start + 1, "<\\b>");
      res.insert(std::max(0, m.first - start), "<b>");
    }
    return res;
  }
};
struct HlSentences {   // SentenceBreakIteratorNew::next(int offset) (:176-192)
  const std::string* text;
  int start = -1, end = -1, last;
  explicit HlSentences(const std::string& t) : text(&t), last(static_cast<int>(t.size()) - 1) {}
  int next(int offset) {
    if (offset > last) return 0;
    for (end = offset; end < last; ++end)
      if ((*text)[end] == '.') break;
    for (start = std::max(0, offset - 1); start > 0; --start) {
      if ((*text)[start] == '.') { ++start; break; }
    }
    return 1;
  }
};
float hl_passage_norm(int start) {
  const float pivot = 87;
  return 1 + 1 / static_cast<float>(std::log(static_cast<float>(pivot + start)));
}
float hl_tf_norm(int freq, int len) {
  const float pivot = 87, k1 = 1.2f, b = 0.75f;
  const float norm = k1 * ((1 - b) + b * (len / pivot));
  return freq / (freq + norm);
}
std::string highlight(const std::vector<std::vector<OffPair>>& table, int max_passages,
                      const std::string& doc) {
  if (table.empty()) return "";
  HlSentences sent(doc);
  auto cmp_off = [](const HlOffsetIt& a, const HlOffsetIt& b) { return a.start > b.start; };
  std::priority_queue<HlOffsetIt, std::vector<HlOffsetIt>, decltype(cmp_off)> offq(cmp_off);
  for (auto& row : table) offq.push(HlOffsetIt(&row));
  auto cmp_pass = [](HlPassage* const& a, HlPassage* const& b) { return a->score > b->score; };
  std::priority_queue<HlPassage*, std::vector<HlPassage*>, decltype(cmp_pass)> pq(cmp_pass);
  std::vector<std::unique_ptr<HlPassage>> pool;
  auto fresh = [&]() { pool.emplace_back(new HlPassage()); return pool.back().get(); };
  float min_score = -1;
  HlPassage* cur = fresh();
  while (!offq.empty()) {
    HlOffsetIt it = offq.top();
    offq.pop();
    int s = it.start;
    if (s == -1) continue;
    int e = it.end;
    if (e > cur->end) {
      if (cur->start >= 0) {
        cur->score = cur->score * hl_passage_norm(cur->start);
        if (pq.size() == static_cast<size_t>(max_passages) && cur->score <= min_score) {
          cur->reset();
        } else {
          pq.push(cur);
          if (pq.size() > static_cast<size_t>(max_passages)) {
            cur = pq.top();
            pq.pop();
            cur->reset();
          } else {
            cur = fresh();
          }
          min_score = pq.top()->score;
        }
      }
      if (sent.next(e) <= 0) break;
      cur->start = sent.start;
      cur->end = sent.end;
    }
    int tf = 0;
    for (;;) {
      ++tf;
      cur->matches.emplace_back(s, e);
      it.next();
      if (it.start == -1) break;
      s = it.start;
      e = it.end;
      if (e > cur->end) { offq.push(it); break; }
    }
    cur->score = cur->score + it.weight * hl_tf_norm(tf, cur->end - cur->start + 1);
  }
  cur->score = cur->score * hl_passage_norm(cur->start);
  if (cur->score > 0) {
    if (pq.size() < static_cast<size_t>(max_passages)) {
      pq.push(cur);
    } else if (cur->score > min_score) {
      pq.pop();
      pq.push(cur);
    }
  }
  std::vector<HlPassage*> out;
  while (!pq.empty()) { out.push_back(pq.top()); pq.pop(); }
  std::sort(out.begin(), out.end(), [](HlPassage* const& a, HlPassage* const& b) { return a->start < b->start; });
  std::string res;
  for (auto* p : out) res += p->to_string(doc);
  return res;
}

// ResultDocEntry::OffsetsForHighliting (query_processing.h:446-492) then
// VacuumEngine::GenerateSnippet (vacuum_engine.h:286-296)
std::string entry_snippet(const std::vector<VacuumIter>& its, const Entry& e, const DocStoreReader& ds,
                          int n_passages) {
  std::vector<std::vector<OffPair>> table;
  if (e.phrase) {   // FilterOffsetByPosition: the pair of each matched appearance
    for (size_t r = 0; r < e.apr.size() && !e.apr[r].empty(); ++r) {
      const auto pairs = its[r].offset_pairs(e.post[r]);
      std::vector<OffPair> row;
      int cur = -1;
      OffPair pr{0, 0};
      for (int ap : e.apr[r]) {
        while (cur < ap) {
          if (cur + 1 >= static_cast<int>(pairs.size()))
            throw std::runtime_error("offset_iter does not suppose to reach the end.");
          pr = pairs[cur + 1];
          ++cur;
        }
        row.push_back(pr);
      }
      table.push_back(row);
    }
  } else {          // ExpandOffsets
    for (size_t i = 0; i < its.size(); ++i) table.push_back(its[i].offset_pairs(e.post[i]));
  }
  return highlight(table, n_passages, ds.get(e.doc));
}

int emit(const std::vector<Entry>& r, int32_t* docs, double* scores) {
  for (size_t i = 0; i < r.size(); ++i) { docs[i] = r[i].doc; scores[i] = r[i].score; }
  return static_cast<int>(r.size());
}

std::vector<std::string> explode(const std::string& s, char c) {  // utils.cc:29-42
  std::vector<std::string> v;
  std::string cur;
  for (char ch : s) {
    if (ch != c) cur += ch;
    else if (!cur.empty()) { v.push_back(cur); cur.clear(); }
  }
  if (!cur.empty()) v.push_back(cur);
  return v;
}

std::vector<std::string> explode_strict(const std::string& s, char c) {  // utils.cc:52-67
  std::vector<std::string> v;
  std::string cur;
  for (char ch : s) {
    if (ch != c) cur += ch;
    else { v.push_back(cur); cur.clear(); }
  }
  v.push_back(cur);
  return v;
}

}  // namespace

// ------------------------------------------------------------ handles ----
struct orc_vacuum {
  uint8_t* map = nullptr;
  size_t len = 0;
  VacHeader hdr;
  int bloom_factor = 1;   // CreateSearchEngine's bloom_enable_factor default (engine_factory.h:33-34)
  std::unordered_map<std::string, uint64_t> tip;  // term -> posting list offset
  std::vector<uint8_t> lens;                      // DocLengthCharStore
  int n_docs = 0;
  Bm25 sim;
  std::string dir;
  std::unique_ptr<DocStoreReader> docs;   // loaded on first use (snippets)
  const DocStoreReader& doc_store() {
    if (!docs) { docs.reset(new DocStoreReader()); docs->load(dir); }
    return *docs;
  }
};

struct orc_qqmem {
  std::map<std::string, PostingListDelta> index;   // varint postings (posting_list_delta.h)
  std::vector<uint8_t> lens;
  double avg = 0;
  int n_docs = 0;
  Bm25 sim;
};

extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }
int orc_num_bits(uint32_t v) { return num_bits(v); }
uint8_t orc_char4_encode(uint32_t v) { return char4_encode(v); }
uint32_t orc_char4_decode(uint8_t c) { return char4_decode(c); }
int orc_varint_encode(uint64_t v, uint8_t* out) { return varint_encode(v, out); }
int orc_varint_decode(const uint8_t* in, uint64_t* v) { return varint_decode(in, v); }
int64_t orc_ub_negative_char_index(void) { return g_ub_neg.load(); }

int orc_pack128(const uint32_t* values, uint8_t* out) {  // packed_value.h:93-116
  int b = 0;
  for (int i = 0; i < kPack; ++i) { int n = num_bits(values[i]); n = n == 0 ? 1 : n; b = std::max(b, n); }
  out[0] = kPackMagic;
  out[1] = static_cast<uint8_t>(b);
  turbo_pack(values, b, out + 2);
  return 2 + (b * kPack + 7) / 8;
}

int orc_unpack128(const uint8_t* pack, uint32_t* out) {
  try {
    PackReader r;
    r.reset(pack);
    r.decode();
    std::memcpy(out, r.cache, sizeof r.cache);
    return r.bits;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

double orc_es_idf(int n, int df) { return es_idf(n, df); }

double orc_es_tfnorm(int freq, int field_length, double avg) {  // scoring.h:28-40
  const double k1 = 1.2, b = 0.75;
  return (freq * (k1 + 1)) / (freq + k1 * (1 - b + ((b * field_length) / avg)));
}

double orc_tfnorm_lossy(double avg, int freq, uint8_t c) {
  Bm25 s;
  s.reset(avg);
  return s.tfnorm_lossy(freq, c);
}

// VacuumEngine::Load (vacuum_engine.h:144-180) minus doc store / mlock / profiler
orc_vacuum* orc_vacuum_open(const char* dir) {
  std::unique_ptr<orc_vacuum> h(new orc_vacuum());
  try {
    const std::string d(dir);
    h->dir = d;
    {  // DocLengthCharStore::Deserialize (doc_length_store.h:163-190)
      std::ifstream f(d + "/my.doc_length", std::ios::binary);
      if (!f) throw std::runtime_error("cannot open my.doc_length");
      int32_t count;
      double avg;
      f.read(reinterpret_cast<char*>(&count), 4);
      f.read(reinterpret_cast<char*>(&avg), 8);
      for (int32_t i = 0; i < count; ++i) {
        int32_t id;
        char c;
        f.read(reinterpret_cast<char*>(&id), 4);
        f.read(&c, 1);
        if (!f) throw std::runtime_error("truncated my.doc_length");
        if (static_cast<size_t>(id) >= h->lens.size()) h->lens.resize(id + 1, 0);
        h->lens[id] = static_cast<uint8_t>(c);
      }
      h->n_docs = count;
      h->sim.reset(avg);  // similarity_.Reset(doc_lengths_.GetAvgLength())
    }
    {  // TermTrieIndex::Load (term_index.h:106-159)
      std::ifstream f(d + "/my.tip", std::ios::binary);
      if (!f) throw std::runtime_error("cannot open my.tip");
      for (;;) {
        uint32_t n;
        if (!f.read(reinterpret_cast<char*>(&n), 4)) break;
        std::string t(n, '\0');
        int64_t v;
        f.read(&t[0], n);
        f.read(reinterpret_cast<char*>(&v), 8);
        // DecodePrefetchZoneAndOffset (flash_containers.h:14-19)
        h->tip[t] = static_cast<uint64_t>(v) & ((~0ull << 16) >> 16);
      }
    }
    {  // MapPostingLists + VacuumHeader::Load (flash_iterators.h:826-873)
      int fd = ::open((d + "/my.vacuum").c_str(), O_RDONLY);
      if (fd < 0) throw std::runtime_error("cannot open my.vacuum");
      struct stat sb;
      fstat(fd, &sb);
      h->len = sb.st_size;
      void* p = mmap(nullptr, h->len, PROT_READ, MAP_PRIVATE, fd, 0);
      ::close(fd);
      if (p == MAP_FAILED) throw std::runtime_error("mmap");
      h->map = static_cast<uint8_t*>(p);
      if (h->map[0] != kVacuumMagic) throw std::runtime_error("Vacuum's first byte is wrong");
      h->hdr.load(h->map);
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
  return h.release();
}

void orc_vacuum_close(orc_vacuum* h) {
  if (!h) return;
  if (h->map) munmap(h->map, h->len);
  delete h;
}

int orc_vacuum_term_count(orc_vacuum* h) { return static_cast<int>(h->tip.size()); }
void orc_vacuum_set_bloom_factor(orc_vacuum* h, int f) { h->bloom_factor = f; }
int orc_vacuum_has_bloom(orc_vacuum* h) { return h->hdr.has_bloom ? 1 : 0; }
void orc_bloom_stats(int64_t* checks, int64_t* pruned) {
  *checks = g_bloom_checks.load();
  *pruned = g_bloom_pruned.load();
}
// the bloom bit array of one posting (0 = prior / begin, 1 = next / end) checked
// for `elem`: 1 may be present, 0 not present (also: no filter), -1 no bloom
int orc_vacuum_bloom_check(orc_vacuum* h, const char* term, int posting, int side, const char* elem) {
  auto f = h->tip.find(term);
  if (f == h->tip.end() || !h->hdr.has_bloom) return -1;
  try {
    VacuumIter it(h->map, f->second, &h->hdr, &f->first);
    for (int i = 0; i < posting; ++i) it.advance();
    return side ? it.has_next_term(elem) : it.has_prior_term(elem);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -2;
  }
}
int orc_vacuum_n_docs(orc_vacuum* h) { return h->n_docs; }

int orc_vacuum_df(orc_vacuum* h, const char* term) {
  auto it = h->tip.find(term);
  if (it == h->tip.end()) return 0;
  return VacuumIter(h->map, it->second).size();
}

int orc_vacuum_list(orc_vacuum* h, const char* term, uint32_t* docs, uint32_t* tfs, int cap) {
  auto f = h->tip.find(term);
  if (f == h->tip.end()) return 0;
  try {
    VacuumIter it(h->map, f->second);
    int n = 0;
    while (!it.is_end()) {
      if (n < cap) { docs[n] = it.doc_id(); tfs[n] = it.term_freq(); }
      ++n;
      it.advance();
    }
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// The doc-id iterator of a term's list driven op by op (tests_11.cc:218-424,
// tests_12.cc:33-270): ops[2i] = 0 Advance, 1 SkipTo(posting arg), 2
// SkipForward(doc arg); after each op out[3i..3i+2] = {PostingIndex, Value (-1
// at the end), IsEnd}.  Returns n, or -1 (unknown term / error).
int orc_vacuum_docid_ops(orc_vacuum* h, const char* term, const int64_t* ops, int n, int64_t* out) {
  auto f = h->tip.find(term);
  if (f == h->tip.end()) { g_err = "unknown term"; return -1; }
  try {
    VacuumIter it(h->map, f->second);
    for (int i = 0; i < n; ++i) {
      const int64_t op = ops[2 * i], arg = ops[2 * i + 1];
      if (op == 0) it.advance();
      else if (op == 1) it.skip_to(static_cast<int>(arg));
      else it.skip_forward(static_cast<uint32_t>(arg));
      out[3 * i] = it.posting_index();
      out[3 * i + 1] = it.is_end() ? -1 : it.doc_id();
      out[3 * i + 2] = it.is_end() ? 1 : 0;
    }
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// VacuumEngine::Search (vacuum_engine.h:201-258), no snippets
int orc_vacuum_search_phrase(orc_vacuum* h, const char* const* terms, int n_terms, int k,
                             int is_phrase, int32_t* docs, double* scores, int32_t* doc_freqs) {
  if (k == 0) return 0;
  try {
    std::vector<VacuumIter> its;
    for (int i = 0; i < n_terms; ++i) {  // FindIteratorsSolid (vacuum_engine.h:89-99)
      auto f = h->tip.find(terms[i]);
      if (f != h->tip.end()) its.emplace_back(h->map, f->second, &h->hdr, &f->first);
    }
    if (its.empty() || static_cast<int>(its.size()) < n_terms) return 0;
    if (doc_freqs) for (size_t i = 0; i < its.size(); ++i) doc_freqs[i] = its[i].size();
    Processor<VacuumIter> p(h->sim, &its, h->lens, h->n_docs, k, is_phrase != 0, h->bloom_factor);
    return emit(p.run(), docs, scores);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// VacuumEngine::Search with SearchQuery::return_snippets (vacuum_engine.h:243-253)
int orc_vacuum_search_snippets(orc_vacuum* h, const char* const* terms, int n_terms, int k,
                               int is_phrase, int n_passages, int32_t* docs, double* scores,
                               char* buf, int64_t cap, int64_t* snip_end) {
  if (k == 0) return 0;
  try {
    std::vector<VacuumIter> its;
    for (int i = 0; i < n_terms; ++i) {
      auto f = h->tip.find(terms[i]);
      if (f != h->tip.end()) its.emplace_back(h->map, f->second, &h->hdr, &f->first);
    }
    if (its.empty() || static_cast<int>(its.size()) < n_terms) return 0;
    Processor<VacuumIter> p(h->sim, &its, h->lens, h->n_docs, k, is_phrase != 0, h->bloom_factor);
    p.capture(true);
    const std::vector<Entry> r = p.run();
    const DocStoreReader& ds = h->doc_store();
    int64_t at = 0;
    for (size_t i = 0; i < r.size(); ++i) {
      docs[i] = r[i].doc;
      scores[i] = r[i].score;
      const std::string sn = entry_snippet(its, r[i], ds, n_passages);
      if (at + static_cast<int64_t>(sn.size()) > cap) throw std::runtime_error("snippet buffer too small");
      std::memcpy(buf + at, sn.data(), sn.size());
      at += static_cast<int64_t>(sn.size());
      snip_end[i] = at;
    }
    return static_cast<int>(r.size());
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// SimpleHighlighter::highlightOffsetsEnums on explicit offset pairs (tests_2.cc:15-90):
// pairs holds sum(counts) (start, end) pairs, term by term.  Returns the length.
int orc_highlight(const int32_t* pairs, const int32_t* counts, int n_terms, int n_passages,
                  const char* doc, char* out, int cap) {
  try {
    std::vector<std::vector<OffPair>> table(n_terms);
    for (int t = 0; t < n_terms; ++t) {
      for (int j = 0; j < counts[t]; ++j) table[t].emplace_back(pairs[0], pairs[1]), pairs += 2;
    }
    const std::string s = highlight(table, n_passages, doc);
    if (static_cast<int>(s.size()) > cap) throw std::runtime_error("highlight buffer too small");
    std::memcpy(out, s.data(), s.size());
    return static_cast<int>(s.size());
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// ChunkedDocStoreReader::Get (doc_store.h:426-443).  Returns the length.
int64_t orc_docstore_get(orc_vacuum* h, int doc, char* out, int64_t cap) {
  try {
    const std::string s = h->doc_store().get(doc);
    if (static_cast<int64_t>(s.size()) > cap) throw std::runtime_error("doc buffer too small");
    std::memcpy(out, s.data(), s.size());
    return static_cast<int64_t>(s.size());
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// The (start, end) offset pairs of posting `posting` of a term (OffsetPostingBagIterator).
int orc_vacuum_offsets(orc_vacuum* h, const char* term, int posting, int32_t* out, int cap) {
  auto f = h->tip.find(term);
  if (f == h->tip.end()) return 0;
  try {
    VacuumIter it(h->map, f->second);
    if (posting < 0 || posting >= it.size()) return 0;
    const auto v = it.offset_pairs(posting);
    for (size_t i = 0; i < v.size() && static_cast<int>(i) < cap; ++i) {
      out[2 * i] = v[i].first;
      out[2 * i + 1] = v[i].second;
    }
    return static_cast<int>(v.size());
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int orc_vacuum_search(orc_vacuum* h, const char* const* terms, int n_terms, int k, int32_t* docs,
                      double* scores, int32_t* doc_freqs) {
  return orc_vacuum_search_phrase(h, terms, n_terms, k, 0, docs, scores, doc_freqs);
}

// The positions of one posting through PositionPostingBagIterator (test hook).
int orc_vacuum_positions(orc_vacuum* h, const char* term, int posting, uint32_t* out, int cap) {
  auto f = h->tip.find(term);
  if (f == h->tip.end()) return 0;
  try {
    VacuumIter it(h->map, f->second);
    if (posting < 0 || posting >= it.size()) return 0;
    it.skip_forward(0);
    for (int i = 0; i < posting; ++i) it.advance();
    PosBagIter* p = it.position_begin();
    int n = 0;
    while (!p->is_end()) {
      const uint32_t v = p->pop();
      if (n < cap) out[n] = v;
      ++n;
    }
    return n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// PhraseQueryProcessor2 over plain position lists (tests_5.cc:447-581 shape):
// returns NumOfMatches; table (n_lists x cap) receives the matched positions.
int orc_phrase_lists(const uint32_t* const* lists, const int* sizes, int n_lists, int32_t* table,
                     int cap) {
  struct ListIt {
    const uint32_t* v; int n; int i;
    bool is_end() const { return i >= n; }
    uint32_t pop() { return v[i++]; }
  };
  std::vector<ListIt> its(n_lists);
  std::vector<ListIt*> ps;
  for (int i = 0; i < n_lists; ++i) { its[i] = ListIt{lists[i], sizes[i], 0}; ps.push_back(&its[i]); }
  std::vector<std::vector<int>> t;
  const int m = phrase_process(ps, &t);
  if (table)
    for (int i = 0; i < n_lists; ++i)
      for (int j = 0; j < m && j < cap; ++j) table[i * cap + j] = t[i][j];
  return m;
}

int orc_vacuum_search_lines(orc_vacuum* h, const char* text, int k, int threads, int32_t* docs,
                            double* scores, int32_t* n_out, int max_q) {
  std::vector<std::string> lines = explode(text, '\n');
  const int nq = std::min<int>(static_cast<int>(lines.size()), max_q);
  std::atomic<int> next{0};
  auto work = [&] {
    for (int q; (q = next++) < nq;) {
      // a line in double quotes is a phrase query (gen_synthetic_log.py:262)
      std::string line = lines[q];
      const bool phrase = line.size() >= 2 && line.front() == '"' && line.back() == '"';
      if (phrase) line = line.substr(1, line.size() - 2);
      std::vector<std::string> t = explode(line, ' ');
      std::vector<const char*> tp;
      for (auto& s : t) tp.push_back(s.c_str());
      n_out[q] = orc_vacuum_search_phrase(h, tp.data(), static_cast<int>(tp.size()), k, phrase,
                                          docs + static_cast<int64_t>(q) * k,
                                          scores + static_cast<int64_t>(q) * k, nullptr);
    }
  };
  if (threads <= 1) work();
  else {
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
  }
  return nq;
}

// CPU baseline timing (bench.py cpu_baseline): `threads` workers share the
// read-only index, as the reference's gRPC threads share one engine
// (grpc_server_impl.h:260-263).  The log is parsed once, the workers are
// started and parked before the clock starts, each query's results go to the
// worker's own preallocated arrays, and the workers take queries from one
// shared counter (the log cycled) until the main thread stops them after
// `seconds`.  Nothing is spawned, parsed or converted inside the interval.
int orc_vacuum_bench_lines(orc_vacuum* h, const char* text, int k, int threads, double seconds,
                           int64_t* done_out, double* elapsed_out) {
  struct Q { std::vector<std::string> terms; std::vector<const char*> ptr; bool phrase; };
  std::vector<Q> qs;
  for (auto& raw : explode(text, '\n')) {
    std::string line = raw;
    const bool phrase = line.size() >= 2 && line.front() == '"' && line.back() == '"';
    if (phrase) line = line.substr(1, line.size() - 2);
    Q q;
    q.terms = explode(line, ' ');
    q.terms.erase(std::remove(q.terms.begin(), q.terms.end(), std::string()), q.terms.end());
    if (q.terms.empty()) continue;
    for (auto& s : q.terms) q.ptr.push_back(s.c_str());
    q.phrase = phrase;
    qs.push_back(std::move(q));
  }
  if (qs.empty() || threads < 1 || k < 1) return -1;
  std::atomic<int64_t> next{0};
  std::atomic<int> ready{0};
  std::atomic<bool> go{false}, stop{false};
  std::vector<int64_t> done(threads, 0);
  auto work = [&](int t) {
    std::vector<int32_t> docs(k);
    std::vector<double> scores(k);
    ready.fetch_add(1);
    while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
    int64_t n = 0;
    while (!stop.load(std::memory_order_relaxed)) {
      const Q& q = qs[static_cast<size_t>(next.fetch_add(1, std::memory_order_relaxed) %
                                          static_cast<int64_t>(qs.size()))];
      orc_vacuum_search_phrase(h, q.ptr.data(), static_cast<int>(q.ptr.size()), k, q.phrase,
                               docs.data(), scores.data(), nullptr);
      ++n;
    }
    done[t] = n;
  };
  std::vector<std::thread> ts;
  for (int i = 0; i < threads; ++i) ts.emplace_back(work, i);
  while (ready.load() < threads) std::this_thread::yield();
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop.store(true);
  for (auto& t : ts) t.join();
  const auto t1 = std::chrono::steady_clock::now();
  int64_t total = 0;
  for (int64_t n : done) total += n;
  *done_out = total;
  *elapsed_out = std::chrono::duration<double>(t1 - t0).count();
  return 0;
}

// QqMemEngineDelta::LoadLocalDocuments / AddDocument (qq_mem_engine.h:271-305):
// TOKEN_ONLY: tokens = body = column 2, tf = token count (utils.cc:167-180),
// length = count_terms(body); WITH_POSITIONS: tokens column 2, tf = offset pairs
// of the term (column 3), length = count_terms(column 1) (types.cc:38-40).
orc_qqmem* orc_qqmem_load(const char* linedoc, int64_t n_rows, const char* format) {
  std::unique_ptr<orc_qqmem> h(new orc_qqmem());
  try {
    const std::string fmt(format);
    const bool tok_only = fmt == "TOKEN_ONLY";
    if (!tok_only && fmt != "WITH_POSITIONS") throw std::runtime_error("format");
    std::ifstream in(linedoc);
    if (!in) throw std::runtime_error("cannot open linedoc");
    std::string line;
    std::getline(in, line);  // LineDoc header (utils.h:54-67)
    int doc = 0;
    int cnt = 0;
    while ((n_rows < 0 || doc < n_rows) && std::getline(in, line)) {
      auto items = explode_strict(line, '\t');
      int length;
      if (tok_only) {
        // AddDocumentNaive (qq_mem_engine.h:217-239): tf = count_tokens, the
        // offsets of extract_offset_pairs (utils.cc:184-217: [start, end]
        // inclusive of each occurrence in the token text), no positions
        const std::string& text = items[2];
        std::map<std::string, std::vector<std::pair<uint32_t, uint32_t>>> occ;
        size_t i = 0;
        while (i < text.size()) {
          if (text[i] == ' ') { ++i; continue; }
          size_t j = i;
          while (j < text.size() && text[j] != ' ') ++j;
          occ[text.substr(i, j - i)].emplace_back(static_cast<uint32_t>(i), static_cast<uint32_t>(j - 1));
          i = j;
        }
        int ntok = 0;
        for (auto& kv : occ) {
          h->index[kv.first].add(doc, static_cast<uint32_t>(kv.second.size()), kv.second, {});
          ntok += static_cast<int>(kv.second.size());
        }
        length = ntok;
      } else {
        // AddDocumentWithPositions (qq_mem_engine.h:194-215): tf = the term's
        // offset pairs (utils::parse_offsets, utils.cc:105-141), positions column 4
        auto toks = explode(items[2], ' ');
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> offs;
        std::vector<std::vector<uint32_t>> poss;
        {
          std::string grp;
          for (char ch : items[3]) {
            if (ch != '.') { grp += ch; continue; }
            if (grp.empty()) continue;
            std::vector<std::pair<uint32_t, uint32_t>> term;
            std::string buf;
            for (char c2 : grp) {
              if (c2 != ';') buf += c2;
              else if (!buf.empty()) {
                const size_t c = buf.find(',');
                term.emplace_back(std::stoul(buf.substr(0, c)), std::stoul(buf.substr(c + 1)));
                buf.clear();
              }
            }
            offs.push_back(term);
            grp.clear();
          }
        }
        for (auto& g : explode(items[4], '.')) {
          std::vector<uint32_t> pv;
          for (auto& x : explode(g, ';')) pv.push_back(static_cast<uint32_t>(std::stoul(x)));
          poss.push_back(pv);
        }
        for (size_t i = 0; i < toks.size(); ++i)
          h->index[toks[i]].add(doc, static_cast<uint32_t>(offs.at(i).size()), offs.at(i),
                                i < poss.size() ? poss[i] : std::vector<uint32_t>{});
        length = static_cast<int>(explode(items[1], ' ').size());
      }
      // DocLengthCharStore::AddLength (doc_length_store.h:104-112)
      h->avg = h->avg + (length - h->avg) / (cnt + 1);
      if (static_cast<size_t>(doc) >= h->lens.size()) h->lens.resize(doc + 1, 0);
      h->lens[doc] = char4_encode(static_cast<uint32_t>(length));
      ++cnt;
      ++doc;
    }
    h->n_docs = cnt;
    h->sim.reset(h->avg);
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
  return h.release();
}

void orc_qqmem_close(orc_qqmem* h) { delete h; }
int orc_qqmem_term_count(orc_qqmem* h) { return static_cast<int>(h->index.size()); }

// QqMemEngineDelta::Search (qq_mem_engine.h:335-368)
int orc_qqmem_search(orc_qqmem* h, const char* const* terms, int n_terms, int k, int32_t* docs,
                     double* scores, int32_t* doc_freqs) {
  if (k == 0) return 0;
  std::vector<DeltaIter> its;
  for (int i = 0; i < n_terms; ++i) {
    auto f = h->index.find(terms[i]);
    if (f != h->index.end()) its.emplace_back(&f->second);
  }
  if (its.empty() || static_cast<int>(its.size()) < n_terms) return 0;
  if (doc_freqs) for (size_t i = 0; i < its.size(); ++i) doc_freqs[i] = its[i].size();
  Processor<DeltaIter> p(h->sim, &its, h->lens, h->n_docs, k);
  return emit(p.run(), docs, scores);
}

// A whole varint posting list through PostingListDeltaIterator: docs, tfs and
// (optionally) the i-th posting's offset pairs / positions; returns the size.
int orc_qqmem_list(orc_qqmem* h, const char* term, uint32_t* docs, uint32_t* tfs, int cap) {
  auto f = h->index.find(term);
  if (f == h->index.end()) return 0;
  DeltaIter it(&f->second);
  int n = 0;
  for (; !it.is_end(); it.advance(), ++n)
    if (n < cap) { docs[n] = static_cast<uint32_t>(it.doc_id()); tfs[n] = static_cast<uint32_t>(it.term_freq()); }
  return n;
}

int orc_qqmem_posting(orc_qqmem* h, const char* term, int posting, uint32_t* offs, int* n_offs,
                      uint32_t* pos, int* n_pos, int cap) {
  auto f = h->index.find(term);
  if (f == h->index.end() || posting < 0 || posting >= f->second.n) { g_err = "no such posting"; return -1; }
  DeltaIter it(&f->second);
  for (int i = 0; i < posting; ++i) it.advance();
  auto o = it.offsets();
  auto p = it.positions();
  *n_offs = static_cast<int>(o.size());
  *n_pos = static_cast<int>(p.size());
  for (int i = 0; i < static_cast<int>(o.size()) && 2 * i + 1 < cap; ++i) { offs[2 * i] = o[i].first; offs[2 * i + 1] = o[i].second; }
  for (int i = 0; i < static_cast<int>(p.size()) && i < cap; ++i) pos[i] = p[i];
  return it.doc_id();
}

// StandardPosting::Encode of one posting (tests_4.cc:114-146)
int orc_posting_encode(uint32_t doc_delta, uint32_t tf, const uint32_t* offs, int n_pairs,
                       const uint32_t* pos, int n_pos, uint8_t* out, int cap) {
  std::vector<std::pair<uint32_t, uint32_t>> o;
  for (int i = 0; i < n_pairs; ++i) o.emplace_back(offs[2 * i], offs[2 * i + 1]);
  const std::string b = standard_posting_encode(doc_delta, tf, o, std::vector<uint32_t>(pos, pos + n_pos));
  if (static_cast<int>(b.size()) > cap) return -1;
  std::memcpy(out, b.data(), b.size());
  return static_cast<int>(b.size());
}

// PostingListDelta with skip span `span` over (doc, tf) postings without
// offsets (tests_4.cc:240-330): the skip entries and, per posting, HasSkip /
// NextSpanDocId, and SkipForward / SkipToNextSpan walks.
int orc_pld_probe(const uint32_t* docs, const uint32_t* tfs, int n, int span, uint32_t* skip_prev,
                  uint64_t* skip_off, int* n_skip, int32_t* has_skip, uint32_t* span_doc,
                  const uint32_t* targets, int n_targets, int32_t* found) {
  try {
    PostingListDelta pl;
    pl.span = span;
    for (int i = 0; i < n; ++i) pl.add(docs[i], tfs[i], {}, {});
    *n_skip = static_cast<int>(pl.skip.size());
    for (size_t i = 0; i < pl.skip.size(); ++i) { skip_prev[i] = pl.skip[i].first; skip_off[i] = pl.skip[i].second; }
    DeltaIter it(&pl);
    for (int i = 0; i < n; ++i, it.advance()) {
      has_skip[i] = it.has_skip() ? 1 : 0;
      span_doc[i] = it.has_skip() ? it.next_span_doc_id() : 0;
    }
    DeltaIter st(&pl);   // SkipForward over increasing targets
    for (int i = 0; i < n_targets; ++i) {
      st.skip_forward(targets[i]);
      found[i] = st.is_end() ? -1 : st.doc_id();
    }
    return pl.n;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"
