// Host-side Vacuum index loader and HBM image builder.
//
// VacuumIndex::open() is the equivalent of VacuumEngine::Load()
// (vacuum_engine.h:144-180) minus the doc store: it reads my.doc_length
// (doc_length_store.h:163-190), the term dictionary my.tip (term_index.h:106-159)
// and memory-maps my.vacuum (VacuumHeader::Load, flash_iterators.h:826-873).
//
// build_image() decodes every list's skip list ONCE (the reference re-decodes
// it on every query, flash_iterators.h:946-948) into a struct-of-arrays block
// directory and copies the [docid | tf] byte span of every list -- the
// reference's "prefetch zone" minus the header -- unchanged into one blob that
// is uploaded to HBM.  A doc-id range [lo, hi) restricts the image to the
// blocks that can hold docs of that range (multi-GPU doc-range shards).
#pragma once

#include <cstdint>
#include <string>
#include <memory>
#include <unordered_map>
#include <utility>
#include <vector>

#include "engine_types.h"

namespace wiser {

struct SkipRow {
  uint32_t prev_doc;
  uint64_t doc_off;  // absolute file offsets of the docid / tf blobs of this row
  uint64_t tf_off;
  uint64_t pos_off;  // position blob holding the row's first bag, and the bag's
  uint32_t pos_idx;  // entry index inside that blob (flash_containers.h:312-350)
  uint64_t off_off;  // the same for the offset box (snippets)
  uint32_t off_idx;
};

class VacuumIndex {
 public:
  VacuumIndex() = default;
  ~VacuumIndex();
  VacuumIndex(const VacuumIndex&) = delete;
  VacuumIndex& operator=(const VacuumIndex&) = delete;

  void open(const std::string& dir);  // throws std::runtime_error

  int32_t n_lists() const { return static_cast<int32_t>(terms_.size()); }
  int32_t find(const std::string& term) const;  // -1 when absent
  int32_t find(const char* p, size_t n) const;
  // n terms at once (the batch path): hashes first, then the table slots and
  // the candidate strings prefetched a group at a time, so the lookups' cache
  // misses overlap instead of running one after another
  void find_many(const char* const* p, const uint32_t* n, size_t cnt, int32_t* out) const;
  const std::string& term(int32_t id) const { return terms_[id]; }
  uint32_t df(int32_t id) const { return df_[id]; }
  uint64_t list_offset(int32_t id) const { return off_[id]; }
  double idf(int32_t id) const { return idf_[id]; }

  // N = number of doc-length records (DocLengthCharStore::Size()).
  int32_t n_docs() const { return n_docs_; }
  double avg_length() const { return avg_; }
  const std::vector<uint8_t>& char4_lengths() const { return c4_; }
  const double* bm25_cache() const { return cache_; }

  // Skip rows of one list (decoded on demand).
  std::vector<SkipRow> rows(int32_t id) const;
  void rows_into(int32_t id, std::vector<SkipRow>* out) const;   // reuses out's storage
  const uint8_t* file() const { return map_; }
  bool has_bloom() const { return has_bloom_; }
  // the filters' shape: VacuumHeader's "end" fields, the ones both bloom
  // readers use (flash_iterators.h:826-889)
  uint32_t bloom_bytes() const { return bloom_bytes_; }
  uint32_t bloom_entries() const { return bloom_entries_; }
  float bloom_ratio() const { return bloom_ratio_; }
  uint64_t file_bytes() const { return map_len_; }

 private:
  std::vector<std::string> terms_;
  // term -> id: open addressing, linear probing, one 8-byte slot per entry
  // (high half: the hash's high 32 bits, low half: id + 1; 0 = empty), at most
  // half full.  (A std::unordered_map lookup costs two dependent cache misses;
  // this one, one for the slot and one for the string compare.)
  std::vector<uint64_t> tslot_;
  uint64_t tmask_ = 0;
  int32_t insert_term(const char* p, size_t n, int32_t id);   // existing id, or id when new
  std::vector<uint64_t> off_;
  std::vector<uint32_t> df_;
  std::vector<double> idf_;
  std::vector<uint8_t> c4_;
  int32_t n_docs_ = 0;
  double avg_ = 0;
  double cache_[256] = {0};
  uint8_t* map_ = nullptr;
  uint64_t map_len_ = 0;
  bool has_bloom_ = false;
  uint32_t bloom_bytes_ = 0, bloom_entries_ = 0;
  float bloom_ratio_ = 0;
};

// Allocator whose resize() leaves trivial elements uninitialised: the image's
// large arrays are written in full by the parallel fill pass, so a serial
// zeroing first would only fault the pages in twice.
template <class T>
struct uninit_alloc : std::allocator<T> {
  template <class U>
  struct rebind { using other = uninit_alloc<U>; };
  uninit_alloc() = default;
  template <class U>
  uninit_alloc(const uninit_alloc<U>&) {}
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    if constexpr (sizeof...(A) == 0) ::new (static_cast<void*>(p)) U;
    else ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using big_vector = std::vector<T, uninit_alloc<T>>;

struct HostImage {
  big_vector<uint8_t> blob;
  std::vector<ListDev> lists;   // indexed by list id
  big_vector<BlockDev> blocks;
  big_vector<uint32_t> blk_last;
  big_vector<uint32_t> blk_meta;    // docid pack bits | tf pack bits << 8 (0 = VInts)
  std::vector<uint64_t> list_bytes;  // docid+tf span bytes per list in the image
  uint32_t doc_lo = 0, doc_hi = 0;
  uint64_t docid_tf_bytes = 0;  // sum of all lists' docid+tf spans in the image
  big_vector<DenseEnt> dense;   // rank bitmaps of the dense lists
  big_vector<uint32_t> dense_rank;   // the rank record of each DenseEnt (kRankWords u32), same index
  big_vector<uint8_t> tf8;      // 1-byte tfs of the dense lists (kTf8Escape = look up the blob)
  big_vector<uint32_t> bkt;     // offset buckets of the sparser dense lists (engine_types.h): per
                                // list its BucketEnts (2 words each), then its offset bytes
  uint32_t dense_span = 0;      // doc ids covered by a bitmap: [doc_lo, doc_lo + dense_span)
  uint32_t dense_lists = 0;     // lists with a probe structure (bitmap or buckets)
  uint32_t bucket_lists = 0;    //   of them with buckets
  big_vector<uint32_t> tails;   // decoded VInts last blocks (ListDev::tail)
  big_vector<uint8_t> plen;     // doc-length code (Char4) of every posting: block j of the
                                // image at [j * 128, j * 128 + 128), 0 past the length records
  big_vector<float> bmax;       // per block: the largest TfNormLossy (tf * 2.2) / (tf + cache_[c4])
                                // of its postings (scoring.h:65-69), f32 rounded up: idf times it
                                // bounds every score of the block (single-term block skipping)
  // positions (build_image(..., positions = true)): see PosDev
  bool has_positions = false;
  std::vector<uint8_t> pos_blob;
  std::vector<PosDev> pos_lists;            // indexed by list id
  std::vector<uint32_t> pos_pk;             // per full pack: byte offset, bit width (pairs)
  std::vector<uint32_t> pos_tail;
  // per posting slot (as plen), two words: the bag's start entry, and the pack
  // it starts in: (byte offset of the pack from the box base << 6) | its bit
  // width, 0 when the bag starts in the VInts remainder or the offset needs
  // more than 26 bits (the kernel then reads pos_pk).  One 8-byte load, one
  // line, instead of the start and then a dependent pos_pk load.
  std::vector<uint32_t> pos_start;
  std::vector<uint64_t> pos_list_bytes;     // bytes of each list's position box (algorithmic bytes)
  // two-way phrase bloom filters (build_image(..., blooms = true), positions
  // images of bloom indexes whose bit arrays fit 16 bytes): per posting slot
  // (as plen) 32 bytes, its "prior" (begin) then its "next" (end) bit array,
  // zero when the box bitmap marks the posting absent (an all-zero array
  // answers "not present", as a missing one does); per list the two
  // MurmurHash2 values of its term (bloom_check's a and b, libbloom/bloom.c:48-75)
  bool has_blooms = false;
  uint32_t blm_bits = 0, blm_hashes = 0;
  big_vector<uint8_t> blm;
  std::vector<uint32_t> blm_hash;           // (a, b) per list id
};

// Decode one block (pack or VInts) at p into out[0..cnt); delta-coded blocks
// are seeded with prev.  Returns false on a malformed blob.
bool host_decode_block(const uint8_t* p, const uint8_t* end, int cnt, bool delta,
                       uint32_t prev, uint32_t* out);

// dense_div > 0: lists with at least span / dense_div postings in the image get
// a rank bitmap + 1-byte tf array (0 disables them); dense_budget > 0 caps the
// bytes of all bitmaps + tf arrays (the longest lists keep theirs).  hbm_free >
// 0 (the device's free bytes): the budget is also clamped to 90 % of it minus
// the rest of the image, so that an image never fails to fit for its bitmaps.
HostImage build_image(const VacuumIndex& idx, uint32_t doc_lo, uint32_t doc_hi, int threads,
                      uint32_t dense_div = 0, bool positions = false, uint64_t dense_budget = 0,
                      bool blooms = false, uint64_t hbm_free = 0);

// Host restatement of the device's dense probe (bitmap or buckets): tf of doc
// in list L of the image, -1 when absent or when L has no probe structure.
int64_t dense_lookup_host(const HostImage& img, const ListDev& L, uint32_t doc);

}  // namespace wiser
