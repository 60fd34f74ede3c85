// Launch interface of kernels.hip (host side).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine_types.h"

namespace wiser {

// Kernel view of one HBM index image (a whole index or one doc-range shard).
struct IndexArgs {
  const uint8_t* blob;      // [docid | tf] spans of every list, byte-exact from my.vacuum
  const ListDev* lists;
  const BlockDev* blocks;
  const uint32_t* blk_last; // dense copy of BlockDev::last for the block searches
  const uint32_t* blk_meta; // docid pack bits | tf pack bits << 8 (0 = VInts blob)
  const uint8_t* c4;        // 1-byte lossy doc length per doc id
  const double* cache;      // Bm25Similarity cache_[256]
  uint32_t n_c4;
  uint32_t n_lists;
  uint32_t doc_lo, doc_hi;  // doc-id range of this image (shard)
  double avg;               // average doc length stored in my.doc_length
  const DenseEnt* dense;    // rank bitmaps of the dense lists (ListDev::bm)
  const uint32_t* dense_rk; // their rank records (same index, kRankWords u32 each)
  const uint2* bkt;         // offset buckets of the sparser dense lists (ListDev::bm with a shift)
  const uint8_t* tf8;       // their 1-byte tfs (ListDev::tf8)
  uint32_t dense_span;      // bitmaps cover doc ids [doc_lo, doc_lo + dense_span)
  float dense_ratio;        // probe list B by bitmap when nblk(B) >= dense_ratio * nblk(driver)
  uint32_t seg_cap;         // driver blocks per work item at most (kSegCost; the batch's own, see
                            // wsr_batch_set_item_blocks: a latency-bound caller takes shorter items)
  const uint8_t* plen;      // doc-length code of each posting, 128 per block (HostImage::plen)
  const float* bmax;        // per block: its largest TfNormLossy, f32 rounded up (HostImage::bmax)
  const uint32_t* tails;    // decoded VInts last blocks (ListDev::tail)
  // positions (phrase queries; null unless the engine was opened with them)
  const uint8_t* pos_blob;  // every list's position cozy box, byte-exact from my.vacuum
  const PosDev* pos_lists;  // indexed by list id
  const uint2* pos_pk;      // per full pack: byte offset from PosDev::base, bit width
  const uint32_t* pos_tail; // decoded VInts remainders
  const uint2* pos_start;   // per posting (128 slots per image block): the bag's start entry,
                            // the pack it starts in (offset << 6 | width; 0: read pos_pk)
  // phrase bloom filters (null / 0 unless a bloom index was opened with
  // positions and bloom_factor > 0): per posting slot two 16-byte bit arrays
  // (prior, next), per list its term's two hashes; bloom_factor as
  // CheckBloomWithEnableFactor's (query_processing.h:796-807)
  const uint4* blm;
  const uint2* blm_hash;
  uint32_t blm_bits, blm_hashes, bloom_factor;
};

// counters[] (zeroed before every batch): 0 total items, 2 event capacity used,
// 4 error flags, 6 end of the lean items, 8 end of the conjunctive lean items
// (items [0, lean conj) run in lean_kernel's conjunctive instance, [lean
// conj, lean) -- the lean phrase queries' -- in its phrase instance, the rest
// in segment_kernel); each work queue has one head per XCD-sized shard, each
// on its own 64-byte line (kCtrHead0 + 16*s lean conjunctive, kCtrPHead0 +
// 16*s lean phrase, kCtrGHead0 + 16*s general), so the dequeues of the
// persistent workers do not serialise on a single line.
enum { kCtrItems = 0, kCtrEvCap = 2, kCtrError = 4, kCtrLean = 6, kCtrLeanConj = 8, kCtrHead0 = 16,
       kQueueShards = 8,
       kCtrPHead0 = kCtrHead0 + 16 * kQueueShards,
       kCtrGHead0 = kCtrPHead0 + 16 * kQueueShards,
       kNumCounters = kCtrGHead0 + 16 * kQueueShards };
// QueryPlan::driver = driver slot | cost bucket << kPlanBucketShift | kPlanLean
// (| kPlanPhrase: a lean phrase query, the phrase instance's items)
constexpr uint32_t kPlanSlotMask = 0x7FFu;   // (kMaxQueryTerms <= 2048)
constexpr int kPlanBucketShift = 12;
constexpr uint32_t kPlanLean = 1u << 16;
constexpr uint32_t kPlanPhrase = 1u << 17;
static_assert(kMaxQueryTerms <= static_cast<int>(kPlanSlotMask) + 1, "driver slot field");
constexpr int kLeanWaves = 4;   // independent waves per lean_kernel workgroup
// per-workgroup statistics written by the segment kernels (no atomics):
// stats[wg * kStatStride + {0 survivors, 1 driver blocks, 2 other blocks}]
constexpr int kStatStride = 4;
enum { kErrLimit = 1, kErrCapacity = 2, kErrExchange = 4, kErrClass = 8 };
constexpr int kMaxOwners = 1024;   // doc-range shards (ranks) of one exchange

// Target block decodes per work item, for every class (lean, general,
// phrase); bounds seg_blocks (< 64).  Phrase items have been this long since
// round 3 (5 blocks before, while every conjunctive survivor ran the position
// check; now only the running top-k's candidates do, and longer items prune
// more: C5 leg 3.50 -> 4.95 M q/s at 63 blocks, 16: 4.27, 32: 4.56 M,
// profiles/r03_phrase_item_ab.txt).
constexpr int kSegCost = 63;
static_assert(kSegCost < 64, "a segment's driver directory is one entry per lane");
// A single-term item spans up to this many items' worth of blocks, which
// single_segment runs window by window: most of its blocks are skipped by
// their block bounds, so a short item would be mostly fixed cost.
constexpr int kSingleWindows = 8;
// Driver blocks per item of a phrase query at most: a batch's phrase items
// are its tail when they are few (the realistic mix in log order: 15.4 -> 16.5
// M q/s at 32 against 63, C5 unchanged; 16: 16.0 / 8.5 M, round 5).  Since the
// batch former puts phrases in batches of their own (round 6), 48: C5 15.3 ->
// 16.1 M, the class-ordered mix 27.6 -> 27.2 M (63: 16.1 / 27.2 M;
// profiles/r06/phrase_cap_ab/).
constexpr uint32_t kPhraseSegCap = 48;
// item cost classes for the longest-first queue order (QueryPlan::driver >> kPlanBucketShift);
// kItemFixedCost = an item's setup (dequeue, directory loads), in block decodes
// item cost buckets: log2(cost) < 3, 3, 4, >= 5, and (the heaviest) the items
// of a query of at least kHeavyQueryItems items
constexpr int kCostBuckets = 5;
// A query of this many items or more is queued before every other item of
// its class: its replay, the batch's longest chain of heap insertions, then
// starts while the lighter items still run, instead of ending the batch.
constexpr uint32_t kHeavyQueryItems = 4;
constexpr float kItemFixedCost = 4.0f;

// Replay fused into the segment kernel: the workgroup that completes a
// query's last item replays it (q_done: per-query completed items, zeroed by
// the plan kernel).  q_done == nullptr: no fusion (separate replay launch, or
// doc-range shard mode where events are exchanged first).
//
// Fused shard emission (wsr_shard_step, x_send != nullptr): the worker that
// completes a query's last item reduces the query's events to those of a heap
// run from empty over this shard (EventFilter; every survivor for k > kMaxK),
// appends them to the owner's slot of the send buffer at an offset taken from
// the owner's fill counter, and records {count, offset} for the query
// (count -1 and kErrExchange when the slot is full).  No reduce, scan or pack
// launch is left between the segment kernels and the exchange.
// A deferred owner replay (wsr_shard_steps): after their own items, the waves
// of a lean kernel replay owned queries of an earlier step group's exchange --
// owner_replay_meta_kernel's work without its launch (nq 0: none).  Only
// batches without wide queries are deferred.
struct OwnerJob {
  const QueryIn* qs;      // the replayed batch's queries; owned ones from q0
  const int32_t* meta;    // {count, offset} of owned query i from shard g at meta + g * meta_stride + 2 * i
  const Event* recv;      // shard g's events at recv + g * stride + offset
  HitDev* hits;
  int32_t* n_hits;
  uint32_t* counters;     // the replayed batch's (error flags)
  uint64_t meta_stride, stride;
  int32_t q0, nq, n_shards, hit_stride;
};

struct FusedReplay {
  uint32_t* q_done;
  HitDev* hits;
  int hit_stride;
  int32_t* n_hits;
  Event* x_send;        // owner o's slot at x_send + o * x_stride (x_slot events)
  int32_t* x_meta;      // {count, offset in the owner's slot} of query i of owner o at
                        //   x_meta + o * x_meta_stride + 2 * i
  uint32_t* x_fill;     // per owner: events appended (zeroed before the batch)
  uint32_t* x_err;      // error flags word
  uint64_t x_slot;      // slot capacity (events)
  uint64_t x_stride;    // events between owners' slots
  uint64_t x_meta_stride;   // int32 between owners' meta blocks
  int32_t x_qpr;        // queries per owner
  OwnerJob oj;          // (lean kernel only)
  __device__ int32_t* meta_of(uint32_t q) const {
    const uint32_t o = q / static_cast<uint32_t>(x_qpr);
    return x_meta + o * x_meta_stride + 2ull * (q - o * static_cast<uint32_t>(x_qpr));
  }
};

// Plan pass 1 -> pass 2: per plan workgroup (kPlanThreads queries), its items
// per item key (class, cost bucket) and its event capacity.
constexpr int kPlanThreads = 256;
struct PlanPart {
  uint32_t items[3 * kCostBuckets];
  uint64_t cap;
};

// phrase scratch words per general workgroup / lean wave (null when the batch
// has no phrase query)
constexpr int kPhraseScratch = kMaxPhraseTerms * 256;

// plan queries (2 launches); part: per plan workgroup of kPlanThreads queries
hipError_t launch_plan(const IndexArgs& ix, const QueryIn* q, int nq, QueryPlan* plan,
                       uint32_t* counters, uint64_t ev_capacity, uint32_t item_capacity,
                       int lean_grid, int lean_grid_ph, int seg_grid, const FusedReplay& fr, uint32_t* item_q,
                       uint64_t* pub, QueryDesc* desc, PlanPart* part, hipStream_t st);
hipError_t launch_segments(const IndexArgs& ix, const QueryIn* q, const QueryPlan* plan, int nq,
                           uint32_t* counters, Event* events, uint32_t* ev_cnt, uint32_t* stats,
                           int grid, const FusedReplay& fr, const uint32_t* item_q,
                           uint64_t* pub, uint32_t* ph, hipStream_t st);

// lean_grid workgroups of kLeanWaves waves; stats of wave w at stats[w * kStatStride];
// phrase: the lean phrase queries' items (the phrase instance; their lean
// ones have two terms), else the conjunctive lean items;
// two: every query of those items has two terms and k <= kMaxK;
// one (conjunctive only): every query of those items has one term
hipError_t launch_lean(const IndexArgs& ix, const QueryIn* q, const QueryPlan* plan, int nq,
                       uint32_t* counters, Event* events, uint32_t* ev_cnt, uint32_t* stats,
                       int lean_wgs, const FusedReplay& fr, const uint32_t* item_q,
                       uint64_t* pub, const QueryDesc* desc, bool phrase, bool two, bool one,
                       hipStream_t st);
int lean_kernel_occupancy(bool phrase);   // workgroups per CU
// queries with k > kMaxK (their segments emitted every survivor): heap in LDS
hipError_t launch_wide_replay(const QueryIn* q, const QueryPlan* plan, int nq, const Event* events,
                              const uint32_t* ev_cnt, HitDev* hits, int hit_stride, int32_t* n_hits,
                              hipStream_t st);
hipError_t launch_decode_probe(const uint8_t* p, uint32_t bits, uint32_t cnt, bool delta,
                               uint32_t seed, uint32_t* out, hipStream_t st);
// owner side of the fused exchange: meta[(g * nq + i) * 2] = {count, offset}
// sent by shard g for owned query i, its events at recv + g * slot + offset
// (meta of shard g at meta + g * meta_stride, its events at recv + g * stride)
hipError_t launch_owner_replay_meta(const QueryIn* q, int q0, int nq, int n_shards, const int32_t* meta,
                                    uint64_t meta_stride, uint64_t stride, const Event* recv, HitDev* hits,
                                    int hit_stride, int32_t* n_hits, uint32_t* counters, bool any_wide,
                                    hipStream_t st);
// resident 64-thread segment workgroups per CU
int segment_kernel_occupancy();

}  // namespace wiser
