// Plain structs shared by the host planner and the HIP kernels.  All of them
// live in HBM; sizes are fixed so the host and device agree byte for byte.
#pragma once

#include <cstdint>

namespace wiser {

constexpr int kMaxTerms = 16;        // terms held inline in a QueryIn (and the plan's one-round loads)
constexpr int kMaxQueryTerms = 1024; // terms per conjunctive query (past kMaxTerms: QueryIn::ext)
constexpr int kMaxPhraseTerms = 8;   // terms per phrase query (the reference's cap, query_processing.h:695)
constexpr int kMaxK = 64;            // n_results of the wave top-k: running top-k and heap in one wave's lanes
constexpr int kMaxKWide = 1024;      // n_results per query; k > kMaxK: every survivor is an event and the
                                     // replay keeps the heap in LDS (wide_replay_kernel)

// One posting list in the HBM image.
struct ListDev {
  uint64_t base;      // byte offset of the list's docid span in the blob
  uint32_t blk0;      // first entry in the block directory
  uint32_t nblk;      // blocks of this list in the image
  uint32_t df;        // GLOBAL document frequency (drives idf and planning)
  uint32_t tail_cnt;  // postings in the image's last block (128 unless a VInts tail)
  double idf;         // calc_es_idf(N, df) computed on the host with libm log
  uint64_t bm;        // first DenseEnt of the list's doc bitmap, kNoDense when it has none
  uint64_t tf8;       // byte offset of the list's 1-byte tf array (posting order)
  uint64_t tail;      // its last block decoded (tail_cnt doc ids, then tail_cnt tfs) in the
                      // image's tails array when that block is a VInts blob, else kNoTail
  uint32_t last;      // last doc id of its last block in the image (= blk_last of that block)
  uint32_t tfmax;     // an upper bound of its tfs in the image: exact for dense lists (their tfs
                      // are decoded at load), else the largest pack width's maximum (~0u: unknown)
};
static_assert(sizeof(ListDev) == 64, "ListDev layout");
constexpr uint64_t kNoTail = ~0ull;

constexpr uint64_t kNoDense = ~0ull;
constexpr uint8_t kTf8Escape = 255;   // tf >= 255: read the tf blob instead

// A list's probe structure (ListDev::bm, QueryDesc::o_bm): bits 0-55 its
// first entry, bits 56-63 the bucket shift c (0: a rank bitmap of DenseEnt).
//
// Offset buckets (c = 3..8) are for lists of density below 1/kBucketDensity
// in the image's doc range, where a bitmap costs a 128-byte line per 1,024
// docs probed whatever the list holds: a driver a few hundred docs apart
// fetches nearly every mask line of the range, ~8x the list's compressed
// bytes at 1 % density (scripts/traffic_model.py).  The range is cut into
// buckets of 2^c docs, c chosen so that a bucket holds 1-2 postings on
// average (below 2.5 % density that is >= 64 docs: an entry line covers at
// least as many docs as a mask line); per bucket
// one 8-byte BucketEnt {rank << 9 | count, the in-bucket
// offsets (doc - bucket start) of its first four postings, one byte each}, and
// after the list's entries (at byte 8 * n_buckets of its region) the in-bucket
// offset of every posting, one byte each, for buckets of more than four.  A
// probe reads one entry (a line covers 16 buckets: 4,096 docs at c = 8) and
// compares four bytes at once; a hit's posting index is rank + its position,
// and its tf comes from tf8 as for a bitmap.  A probe past the fourth posting
// of a larger bucket reads the next offset bytes (one 8-byte window: counts up
// to 9 cost no further wait); past the ninth it walks them.  A list whose
// postings crowd (more than 1/1024 of its buckets over kBucketWindow, as a
// topic-clustered term's do) keeps a bitmap: every wave would walk.
constexpr uint32_t kProbeShiftBit = 56;
constexpr uint64_t kProbeBaseMask = (1ull << kProbeShiftBit) - 1;
constexpr uint32_t kBucketDensity = 40;     // buckets below 2.5 % density, bitmaps above
constexpr uint32_t kBucketMinShift = 3, kBucketMaxShift = 8;
constexpr uint32_t kBucketInline = 4;       // offsets held in the entry
constexpr uint32_t kBucketWindow = 9;       // counts served without a walk
constexpr uint32_t kBucketCrowdedDiv = 1024;   // more crowded buckets than 1/this: a bitmap
inline uint32_t probe_shift(uint64_t bm) { return static_cast<uint32_t>(bm >> kProbeShiftBit); }
inline uint64_t bucket_count(uint32_t span, uint32_t c) { return (static_cast<uint64_t>(span) + (1u << c) - 1) >> c; }
// bucket shift for n postings over span docs (0: a bitmap): 1-2 postings per bucket
inline uint32_t bucket_shift(uint64_t n, uint32_t span) {
  // (ranks travel in 23 bits; a shard image's edge blocks add < 256 postings)
  if (!span || n * kBucketDensity >= span || n >= (1u << 23) - 1024) return 0;
  uint32_t c = kBucketMinShift;
  while (c < kBucketMaxShift && (n << (c + 1)) <= 2ull * span) ++c;   // doubled, the mean stays <= 2
  return c;
}
// words (u32) of a bucket list's region: entries, then one offset byte per posting
inline uint64_t bucket_words(uint64_t n, uint32_t span, uint32_t c) {
  return 2 * bucket_count(span, c) + (n + 7) / 8 * 2;
}

// Dense lists (df >= span / dense_div) also carry a rank bitmap of their doc
// ids over the image's doc range, so that a probe costs one load + a popcount
// instead of decoding the list's blocks.  The masks and the rank records are
// two arrays at the same index: DenseEnt = the 32-doc mask word (bit
// (d - doc_lo) % 32 of doc d), HostImage::dense_rank = per entry an 8-byte
// rank record {postings of the list (in the image's blocks) before the
// entry's first doc, the 1-byte tfs of the word's first four postings (255:
// more, or tf >= 255: read tf8)}; posting index = rank + popcount of the lower
// bits, block = index / 128.  The lean kernel's probe of the most selective
// other list reads the mask word alone (a 128-byte line covers 1,024 docs) and
// only a hit reads its rank record, whose tf bytes give the hit's tf in the
// same line.  At the en-Wikipedia shape a high-df driver's postings are ~180
// docs apart, so with the ranks beside the masks (8 bytes per 32 docs, 512
// docs per line) nearly every probe fetched a line of its own from HBM, and
// those line fetches bound the lean kernel (profiles/r03_probe_sweep.jsonl:
// ~12 CU-cycles per HBM line; r03_probe_forms.txt).  Other users (further
// lists, the general kernel) load both words at once: one probe = two
// independent loads.
constexpr uint32_t kDenseDocs = 32;   // doc ids per DenseEnt
struct DenseEnt {
  uint32_t w;        // bit (d - doc_lo) % 32 of doc d; its rank record: HostImage::dense_rank, same index
};
static_assert(sizeof(DenseEnt) == 4, "DenseEnt layout");
constexpr uint32_t kRankWords = 2;                          // u32 per rank record
constexpr uint64_t kDenseEntBytes = 4 + 4 * kRankWords;     // mask + rank record

// Host form of an entry's bit test and rank (the kernels have their own).
inline bool dense_ent_bit(const DenseEnt& e, uint32_t sh) { return (e.w >> sh) & 1u; }
inline uint32_t dense_ent_rank(const DenseEnt& e, uint32_t rank, uint32_t sh) {   // postings before bit sh
  return rank + static_cast<uint32_t>(__builtin_popcount(e.w & ((1u << sh) - 1u)));
}

// One 128-posting block (= one skip-list row, flash_containers.h:312-350).
struct BlockDev {
  uint32_t prev;      // previous_doc_id: delta seed, doc id of posting 128*i - 1
  uint32_t last;      // doc id of the block's last posting
  uint32_t doc_rel;   // docid blob offset relative to ListDev::base
  uint32_t tf_rel;    // tf blob offset relative to ListDev::base
};
static_assert(sizeof(BlockDev) == 16, "BlockDev layout");

struct QueryIn {
  int32_t n_terms;          // 0 => empty result
  int32_t k;                // n_results (0 => empty result)
  int32_t list[kMaxTerms];  // list ids in query order; -1 => term missing => empty
  int32_t flags;            // kQueryPhrase: SearchQuery::is_phrase (types.h:205-256)
  uint32_t ext;             // n_terms > kMaxTerms: all n_terms list ids are at
                            // reinterpret_cast<const int32_t*>(batch's QueryIn array) + ext
};
static_assert(sizeof(QueryIn) == 80, "QueryIn layout");
constexpr int32_t kQueryPhrase = 1;

// Positions of one posting list in the image (phrase queries).  The list's
// position cozy box (flash_engine_dumper.h:78-104: full packs of 128 entries,
// then one VInts blob) is copied byte-identical to pos_blob at `base`; pack i
// starts at base + pos_pk[pk0 + i].x and has bit width pos_pk[pk0 + i].y; the
// VInts remainder is decoded at load (pos_tail[tail ..]).  Entry e of the box
// is in pack e / 128 when e < 128 * npk.  The bag of posting p (tf entries,
// delta coded from 0, flash_iterators.h:593-604) starts at entry
// pos_start[image slot of p] (slots as plen: 128 per image block).
struct PosDev {
  uint64_t base;
  uint64_t tail;
  uint32_t pk0;
  uint32_t npk;
};
static_assert(sizeof(PosDev) == 24, "PosDev layout");

// Written by the plan kernel for every query of a batch.
struct QueryPlan {
  uint32_t item_base;   // first work item of this query
  uint32_t n_items;     // segments (0 for empty queries)
  uint32_t seg_blocks;  // driver blocks per segment
  uint32_t driver;      // query slot of the shortest list (bits 0-7) | item cost bucket << 8
  uint64_t ev_base;     // first event slot (capacity = driver blocks * 128)
};
static_assert(sizeof(QueryPlan) == 24, "QueryPlan layout");

// Per-query work description of a lean query (every other list probed by
// bitmap, or a single term), written by the plan kernels so that a lean item's
// setup is one load of this record.
struct QueryDesc {
  uint64_t a_base;      // driver: blob base of its [docid | tf] span
  uint64_t a_tail;      //   decoded VInts last block (ListDev::tail)
  uint64_t o_bm;        // O1 (the other list with the fewest blocks): first bitmap entry
  uint64_t o_tf8;       //   offset of its 1-byte tfs
  uint64_t ev_base;     // = QueryPlan::ev_base
  uint64_t rsv0, rsv1;
  double a_idf, o_idf;
  uint32_t a_blk0, a_nblk, a_tail_cnt;
  uint32_t min_last;    // smallest last doc id over the other lists
  uint32_t item_base, n_items, seg;
  uint32_t slots;       // driver slot | O1 slot << 16 (kNoSlot: single term)
  uint32_t o_list;      // O1's list id
  uint32_t k;           // n_results (> kMaxK: wide, every survivor is an event)
  // score bound of a driver posting before the other lists are probed (f32,
  // the lean kernel's pre-probe pruning): b_id * tf / (tf + norm) is its own
  // term (b_id = 2.2 * idf), b_iom / (b_m + norm) bounds all the other terms
  // (b_m = their largest tfmax, b_iom = sum of 2.2 * idf over them, times b_m)
  float b_id, b_iom, b_m;
  uint32_t nt;          // n_terms
};
static_assert(sizeof(QueryDesc) == 128, "QueryDesc layout");
constexpr uint32_t kNoSlot = 0xFFFFu;

// A heap-insertion event: a survivor that a top-k heap run from empty over its
// segment inserts (query_processing.h:595-602).
struct Event {
  double score;
  int32_t doc;
  int32_t pad;
};
static_assert(sizeof(Event) == 16, "Event layout");

struct HitDev {
  int32_t doc;
  int32_t pad;
  double score;
};
static_assert(sizeof(HitDev) == 16, "HitDev layout");

}  // namespace wiser
