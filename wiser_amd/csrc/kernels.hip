// HIP kernels for the conjunctive (AND) BM25 top-k path on gfx950 (MI355X).
//
// Replaces, in the reference (/root/reference/src/qq_mem/src):
//   posting-list decode ........ LittlePackedIntsReader / turbounpack32,
//                                DeltaEncoded{PackedInts,VInts}Iterator
//                                (packed_value.h:184-235,320-369,400-507)
//   intersect / skip iterator .. DocIdIterator::SkipForward, TwoTermNonPhrase-
//                                QueryProcessor::Process, QueryProcessor::FindMatch
//                                (flash_iterators.h:141-227, query_processing.h:656-677,810-852)
//   Bm25Similarity scorer ...... CalcDocScoreLossy / TfNormLossy (scoring.h:65-69,124-145)
//   top-k heap ................. MinPointerHeap / RankDoc / SortHeap
//                                (query_processing.h:510-524,551-562,588-616)
//
// Launches per query batch:
//   plan_*_kernel   per query pick the shortest list as driver and cut its
//                   blocks into segments of similar cost (one thread per query),
//                   then exclusive-scan segment counts and event capacities.
//   lean_kernel     persistent, independent waves: items whose other lists all
//                   carry a rank bitmap (the common case) -- a software pipeline
//                   over the driver's blocks, one bitmap probe per posting.
//   segment_kernel  persistent, one wave per workgroup, beside lean_kernel on a
//                   second stream: the general items.  Per driver block (128
//                   postings): wave-decode doc ids (2 per lane; bit-unpack or
//                   ballot-parallel varint), gallop each other list's block
//                   directory per lane, decode the touched blocks into LDS once,
//                   lower_bound in LDS, score survivors in fp64 in query-term
//                   order, and keep a running top-k (one f64 per lane) to emit
//                   the survivors a heap started empty at the segment start
//                   would insert ("events", in doc-id order).
//   The worker that finishes a query's last item replays its events, in doc-id
//   order, through a restatement of libstdc++'s push_heap / pop_heap with the
//   reference comparator, then SortHeap (wide_replay_kernel for k > 64).
//
// Exactness of the event filter: survivor i is inserted by a heap run from
// empty over a sequence iff fewer than k earlier survivors have a score >= s_i.
// A segment's events are therefore a superset of the global run's insertions
// inside that segment, and replaying only events reproduces every heap state
// (and so the tie order) of the reference bit for bit.
//
// Compiled with -ffp-contract=off: the reference build has no FMA
// (CMakeLists.txt:6,12), so tf*(k1+1), tf+cache, the division and the
// left-to-right sum are each rounded once, exactly as on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels.h"

namespace wiser {

constexpr uint32_t kNoBlock = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t l = threadIdx.x & 63;
  return l ? (~0ull >> (64 - l)) : 0ull;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), lane);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), lane);
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}

// DPP lane shuffles (no LDS crossbar, no per-width address registers).
// Lanes whose source is outside the row / wave read 0.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, ROWMASK, 0xF, false));
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143, kWaveShr1 = 0x138;

// inclusive sum inside aligned groups of W lanes (W = 2..64).  A row_shr lane
// whose source lies outside its 16-lane row keeps the 0 it was given, so for
// W >= 16 no lane test is needed and each step folds into one v_add_u32_dpp;
// groups narrower than a row must not take sums across their own boundary.
template <int W>
__device__ __forceinline__ uint32_t group_incl_scan(uint32_t x) {
  const uint32_t r = threadIdx.x & ((W < 16 ? W : 16) - 1);
  constexpr bool kRow = W >= 16;
  uint32_t y;
  y = dpp<kRowShr1>(x); if (kRow || r >= 1) x += y;
  if (W > 2) { y = dpp<kRowShr2>(x); if (kRow || r >= 2) x += y; }
  if (W > 4) { y = dpp<kRowShr4>(x); if (kRow || r >= 4) x += y; }
  if (W > 8) { y = dpp<kRowShr8>(x); x += y; }
  if (W > 16) { y = dpp<kRowBcast15, 0xA>(x); x += y; }
  if (W > 32) { y = dpp<kRowBcast31, 0xC>(x); x += y; }
  return x;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) { return group_incl_scan<64>(x); }

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// A wave-uniform value kept in a vector register: for values only ever used as
// VALU operands, so that they do not compete for the scalar registers of a
// loop that already needs more than the 106 it can have.
template <class T>
__device__ __forceinline__ T in_vgpr(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// max over the lanes below this one (0 for lane 0)
__device__ __forceinline__ uint32_t wave_excl_max(uint32_t x) {
  // (out-of-row lanes read 0, the identity of an unsigned max)
  x = dpp<kWaveShr1>(x);
  uint32_t y;
  y = dpp<kRowShr1>(x); x = umax(x, y);
  y = dpp<kRowShr2>(x); x = umax(x, y);
  y = dpp<kRowShr4>(x); x = umax(x, y);
  y = dpp<kRowShr8>(x); x = umax(x, y);
  y = dpp<kRowBcast15, 0xA>(x); x = umax(x, y);
  y = dpp<kRowBcast31, 0xC>(x); x = umax(x, y);
  return x;
}

// value of lane l-1 (lane 0 reads 0)
__device__ __forceinline__ double wave_shr1_f64(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = dpp<kWaveShr1>(static_cast<uint32_t>(u));
  const uint32_t hi = dpp<kWaveShr1>(static_cast<uint32_t>(u >> 32));
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}

// Value j of a 128-value pack whose data bytes start at d (bit width b):
// bits [j*b, j*b+b) of an LSB-first little-endian stream.  Reads the two
// aligned dwords that cover the value (the blob is padded at its end).
// (Addresses are formed from the global blob pointer with __builtin_align_down,
// not through integer casts, so the loads stay global_load and never become flat.)
__device__ __forceinline__ uint32_t pack_value(const uint8_t* d, uint32_t b, uint32_t j) {
  const uint32_t bit = j * b;
  const uint8_t* a = d + (bit >> 3);
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a) & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(__builtin_align_down(a, 4));
  const uint32_t sh = (mis << 3) + (bit & 7);
  const uint64_t v = (static_cast<uint64_t>(w[1]) << 32) | w[0];
  const uint32_t mask = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
  return static_cast<uint32_t>(v >> sh) & mask;
}

// (__builtin_align_down keeps the pointer's provenance, so the load stays
// global and a uniform byte is never fetched by a scalar load whose base is
// misaligned with the alignment folded into its immediate offset.)
__device__ __forceinline__ uint32_t load_byte(const uint8_t* p) {
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t w = *reinterpret_cast<const uint32_t*>(__builtin_align_down(p, 4));
  return (w >> (mis << 3)) & 0xFFu;
}

// Wave-cooperative decode of one block (pack of 128 or VInts tail of cnt) into
// out[0..cnt); delta blocks are prefix-summed from `seed` (doc ids), raw blocks
// are term frequencies.  `bits` is the pack width from the block directory
// (0 = VInts blob), so no dependent header load precedes the data loads.
// Ends with the wave's LDS writes visible to every lane.
// kWave: the caller's waves run independently (lean kernel): LDS ordering
// inside one wave needs only a compiler barrier, never a workgroup barrier.
template <bool kWave = false>
__device__ __forceinline__ void block_sync() {
  if (kWave) __builtin_amdgcn_wave_barrier();
  else __syncthreads();
}

template <bool kWave = false>
__device__ void decode_block(const uint8_t* p, uint32_t bits, uint32_t cnt, bool delta,
                             uint32_t seed, uint32_t* out) {
  const uint32_t l = threadIdx.x & 63;
  uint32_t x0, x1;
  if (bits) {
    x0 = pack_value(p + 2, bits, 2 * l);
    x1 = pack_value(p + 2, bits, 2 * l + 1);
  } else {
    // 0x9B | varint nbytes | LEB128 values.  Terminator bytes (MSB clear) are
    // found with a ballot per 64-byte chunk; a terminator's rank is its value
    // index, the previous terminator + 1 is its first byte.
    uint32_t nb = 0, hl = 0;
    {
      uint32_t sh = 0, byte;
      do {
        byte = uni(load_byte(p + 1 + hl));
        nb |= (byte & 0x7Fu) << sh;
        sh += 7;
        ++hl;
      } while ((byte & 0x80u) && hl < 5);
    }
    const uint8_t* q = p + 1 + hl;
    uint32_t before = 0;
    int32_t prev_term = -1;
    for (uint32_t c = 0; c < nb; c += 64) {
      const uint32_t i = c + l;
      const uint32_t byte = i < nb ? load_byte(q + i) : 0x80u;
      const bool term = i < nb && !(byte & 0x80u);
      const uint64_t m = __ballot(term);
      if (term) {
        const uint64_t below = m & lanemask_lt();
        const int32_t start = below ? static_cast<int32_t>(c + 63 - __clzll(below)) + 1 : prev_term + 1;
        uint32_t v = 0;
        for (int32_t j = start, s = 0; j <= static_cast<int32_t>(i); ++j, s += 7)
          v |= (load_byte(q + j) & 0x7Fu) << s;
        const uint32_t rank = before + __popcll(below);
        if (rank < 128) out[rank] = v;
      }
      before += __popcll(m);
      if (m) prev_term = static_cast<int32_t>(c + 63 - __clzll(m));
    }
    block_sync<kWave>();
    x0 = 2 * l < cnt ? out[2 * l] : 0;
    x1 = 2 * l + 1 < cnt ? out[2 * l + 1] : 0;
    block_sync<kWave>();
  }
  if (delta) {
    const uint32_t s = x0 + x1;
    const uint32_t inc = wave_incl_scan(s);
    x0 = seed + (inc - s) + x0;
    x1 = x0 + x1;
  }
  out[2 * l] = x0;
  out[2 * l + 1] = x1;
  block_sync<kWave>();
}

// lower_bound over sorted LDS values s[0..n)
__device__ __forceinline__ uint32_t lds_lower_bound(const uint32_t* s, uint32_t n, uint32_t x) {
  uint32_t lo = 0;
  while (n > 0) {
    const uint32_t h = n >> 1;
    if (s[lo + h] < x) { lo += h + 1; n -= h + 1; } else { n = h; }
  }
  return lo;
}

// First block j in [cur, nblk) of a list with last[j] >= x (nblk if none):
// the block DocIdIterator::GetBlobIndexToGo walks to (flash_iterators.h:218-227).
// Doc ids of a list are spread over the id space, so one interpolation probe
// between the cursor block and the list's last block lands next to the answer;
// galloping from the probe and a short bisection finish it.  This keeps the
// chain of dependent directory loads short for the far jumps of skewed pairs.
__device__ __forceinline__ uint32_t find_block(const uint32_t* last, uint32_t cur, uint32_t nblk,
                                               uint32_t x) {
  if (cur >= nblk) return nblk;
  const uint32_t a = last[cur];
  const uint32_t z = last[nblk - 1];
  if (a >= x) return cur;
  if (z < x) return nblk;
  uint32_t lo = cur + 1, hi = nblk - 1;  // last[lo-1] < x <= last[hi]
  if (lo < hi) {
    const float f = static_cast<float>(x - a) * __frcp_rn(static_cast<float>(z - a) + 1.0f);
    uint32_t g = lo + static_cast<uint32_t>(static_cast<float>(hi - lo) * f);
    g = g < lo ? lo : (g > hi ? hi : g);
    if (last[g] >= x) {
      hi = g;
      for (uint32_t s = 1; hi >= lo + s; s <<= 1) {
        const uint32_t p = hi - s;
        if (last[p] < x) { lo = p + 1; break; }
        hi = p;
      }
    } else {
      lo = g + 1;
      for (uint32_t s = 1; lo + s - 1 < hi; s <<= 1) {
        const uint32_t p = lo + s - 1;
        if (last[p] >= x) { hi = p; break; }
        lo = p + 1;
      }
    }
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (last[mid] < x) lo = mid + 1; else hi = mid;
    }
  }
  return lo;
}

// ---------------------------------------------------------- dense lists --
// Other list B is probed through its rank bitmap when it has one and is at
// least dense_ratio times as long as the driver (then a block decode per
// probe would mostly decode postings nobody asks for).  A bitmap probe round
// adds nothing to an item's plan cost: a lean item is kSegCost driver blocks
// (with the pre-probe bound and the floor refresh, longer items prune more and
// carry less fixed work per block: main leg 26.6 -> 28.0 M q/s against
// 42-block items, profiles/r02_sy_item_size_ab.txt).
__device__ __forceinline__ bool use_dense(const IndexArgs& ix, bool has_bm, uint32_t nblk_b,
                                          uint32_t nblk_driver) {
  return has_bm && static_cast<float>(nblk_b) >= ix.dense_ratio * static_cast<float>(nblk_driver);
}

// A bitmap entry as loaded for a probe: x = rank, y = mask word (two
// independent loads, one from each array).
using DenseVal = uint2;
__device__ __forceinline__ bool dense_bit(const DenseVal v, uint32_t sh) { return (v.y >> sh) & 1u; }
__device__ __forceinline__ uint32_t dense_rank(const DenseVal v, uint32_t sh) {
  return v.x + __popc(v.y & ((1u << sh) - 1u));
}
// entry e of the bitmap that starts at entry bm (ListDev::bm)
__device__ __forceinline__ DenseVal dense_at(const IndexArgs& ix, uint64_t bm, uint32_t e) {
  return make_uint2(ix.dense_rk[kRankWords * (bm + e)], ix.dense[bm + e].w);
}

// Bit of doc a in a prefetched bitmap entry; on a hit *idx = posting index.
__device__ __forceinline__ bool dense_hit(const IndexArgs& ix, uint32_t a, const DenseVal v,
                                          uint32_t* idx) {
  const uint32_t rel = a - ix.doc_lo;
  if (rel >= ix.dense_span) return false;
  const uint32_t sh = rel % kDenseDocs;
  if (!dense_bit(v, sh)) return false;
  *idx = dense_rank(v, sh);
  return true;
}

// tf of posting `idx` of B read from the tf blob (tf >= 255): pack value, or
// a per-lane walk of the VInts tail (0x9B | varint nbytes | LEB128 values).
__device__ __forceinline__ uint32_t dense_tf_slow(const IndexArgs& ix, const ListDev& B, uint32_t idx) {
  const uint32_t j = idx >> 7, pos = idx & 127;
  const BlockDev bb = ix.blocks[B.blk0 + j];
  const uint32_t tbits = ix.blk_meta[B.blk0 + j] >> 8;
  const uint8_t* p = ix.blob + B.base + bb.tf_rel;
  if (tbits) return pack_value(p + 2, tbits, pos);
  const uint8_t* q = p + 1;
  for (int i = 0; i < 5 && (*q++ & 0x80); ++i) {}   // nbytes
  for (uint32_t v = 0; v < pos; ++v)
    for (int i = 0; i < 5 && (*q++ & 0x80); ++i) {}
  uint32_t val = 0;
  for (int i = 0; i < 5; ++i) {
    const uint8_t c = *q++;
    val |= static_cast<uint32_t>(c & 0x7F) << (7 * i);
    if (!(c & 0x80)) break;
  }
  return val;
}

// ---- offset buckets (engine_types.h): an entry v = {rank << 9 | count,
// the first four in-bucket offsets}.  bucket_pos: the position (0..3) of
// offset o among the first four, kBucketMiss, or kBucketScan when o lies past
// the fourth of a bucket of more (offsets ascend): the offset bytes decide.
// Four bytes at once: t has a zero byte where v.y's byte equals o; the lowest
// byte the borrow test flags is always a true zero (a false flag needs a zero
// below it), and padding bytes past the count are ruled out by position.
constexpr uint32_t kBucketMiss = 4, kBucketScan = 5;
__device__ __forceinline__ uint32_t bucket_pos(const uint2 v, uint32_t o) {
  const uint32_t cnt = v.x & 511u;
  const uint32_t t = v.y ^ (o * 0x01010101u);
  const uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;
  const uint32_t pos = z ? (static_cast<uint32_t>(__builtin_ctz(z)) >> 3) : 4u;
  if (pos < min(cnt, kBucketInline)) return pos;
  return (cnt > kBucketInline && o > (v.y >> 24)) ? kBucketScan : kBucketMiss;
}
// the offset bytes of a bucket list (after its entries)
__device__ __forceinline__ const uint8_t* bucket_offsets(const IndexArgs& ix, uint64_t bm) {
  const uint32_t c = static_cast<uint32_t>(bm >> kProbeShiftBit);
  return reinterpret_cast<const uint8_t*>(ix.bkt + (bm & kProbeBaseMask) +
                                          ((static_cast<uint64_t>(ix.dense_span) + (1u << c) - 1) >> c));
}
// postings j0.. of a bucket of cnt starting at posting `rank`: is one at offset o?
__device__ __forceinline__ bool bucket_scan(const uint8_t* offs, uint32_t rank, uint32_t cnt, uint32_t o,
                                            uint32_t* idx, uint32_t j0 = kBucketInline) {
  for (uint32_t j = j0; j < cnt; ++j) {
    const uint32_t b = load_byte(offs + rank + j);
    if (b >= o) {
      *idx = rank + j;
      return b == o;
    }
  }
  return false;
}

// The window of a bucket's next eight offset bytes (postings 4..) as two
// aligned words w0, w1 from offs + rank + 4: is o among its first
// min(cnt - 4, available) bytes?  (its position, < 8; kWindowMiss; or, past
// a window that holds fewer than the remaining count with o beyond its last
// byte, kWindowScan: walk from `*next`.)
constexpr uint32_t kWindowMiss = 8, kWindowScan = 9;
__device__ __forceinline__ uint32_t bucket_window(uint32_t w0, uint32_t w1, uint32_t mis, uint32_t cnt, uint32_t o,
                                                  uint32_t* next) {
  const uint32_t avail = 8u - mis;
  const uint64_t w = ((static_cast<uint64_t>(w1) << 32) | w0) >> (mis << 3);
  const uint64_t t = w ^ (o * 0x0101010101010101ull);
  const uint64_t z = (t - 0x0101010101010101ull) & ~t & 0x8080808080808080ull;
  const uint32_t pos = z ? static_cast<uint32_t>(__builtin_ctzll(z)) >> 3 : 8u;
  if (pos < min(cnt - kBucketInline, avail)) return pos;
  *next = kBucketInline + avail;
  return (cnt - kBucketInline > avail && o > ((w >> ((avail - 1) << 3)) & 0xFFu)) ? kWindowScan : kWindowMiss;
}

// A list's probe entry for doc offset rel (in: rel inside the range, else a
// dummy read): its bitmap entry {rank, mask} or its bucket entry.  The shift
// comes from the list record, so the branch is uniform.
__device__ __forceinline__ DenseVal probe_at(const IndexArgs& ix, uint64_t bm, uint32_t rel, bool in) {
  const uint32_t c = static_cast<uint32_t>(bm >> kProbeShiftBit);
  if (c) return ix.bkt[(bm & kProbeBaseMask) + (in ? rel >> c : 0u)];
  return dense_at(ix, bm, in ? rel / kDenseDocs : 0u);
}
// Doc a in a prefetched probe entry; on a hit *idx = posting index.
__device__ __forceinline__ bool probe_hit(const IndexArgs& ix, uint64_t bm, uint32_t a, const DenseVal v,
                                          uint32_t* idx) {
  const uint32_t c = static_cast<uint32_t>(bm >> kProbeShiftBit);
  if (!c) return dense_hit(ix, a, v, idx);
  const uint32_t rel = a - ix.doc_lo;
  if (rel >= ix.dense_span) return false;
  const uint32_t o = rel & ((1u << c) - 1u);
  const uint32_t pos = bucket_pos(v, o);
  const uint32_t rank = v.x >> 9;
  if (pos < kBucketInline) {
    *idx = rank + pos;
    return true;
  }
  if (pos != kBucketScan) return false;
  // the next eight offset bytes at once, a walk past them
  const uint8_t* offs = bucket_offsets(ix, bm);
  const uint8_t* p = offs + rank + kBucketInline;
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(__builtin_align_down(p, 4));
  uint32_t next = 0;
  const uint32_t wpos = bucket_window(wp[0], wp[1], static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 3u,
                                      v.x & 511u, o, &next);
  if (wpos < 8u) {
    *idx = rank + kBucketInline + wpos;
    return true;
  }
  return wpos == kWindowScan && bucket_scan(offs, rank, v.x & 511u, o, idx, next);
}

// Is doc a in B?  One 8-byte load (dense_load, issued early) and, on a hit,
// the posting's rank gives its tf (dense_resolve).
__device__ __forceinline__ DenseVal dense_load(const IndexArgs& ix, const ListDev& B, uint32_t a,
                                               bool act) {
  const uint32_t rel = a - ix.doc_lo;
  return probe_at(ix, B.bm, rel, act && rel < ix.dense_span);
}

__device__ __forceinline__ bool dense_resolve(const IndexArgs& ix, const ListDev& B, uint32_t a,
                                              const DenseVal v, uint32_t* tf, uint32_t* pidx = nullptr) {
  uint32_t idx;
  if (!probe_hit(ix, B.bm, a, v, &idx)) return false;
  if (pidx) *pidx = idx;
  uint32_t t = ix.tf8[B.tf8 + idx];
  if (t == kTf8Escape) t = dense_tf_slow(ix, B, idx);
  *tf = t;
  return true;
}

// A query's list ids in query order: inline up to kMaxTerms, else in the
// batch's term table after the QueryIn array (QueryIn::ext, int32 units from qs).
__device__ __forceinline__ const int32_t* qlist_of(const QueryIn* qs, int qi) {
  const QueryIn* q = qs + qi;
  return q->n_terms <= kMaxTerms ? q->list : reinterpret_cast<const int32_t*>(qs) + q->ext;
}

// ----------------------------------------------------------------- plan --
// Item order: class-major (conjunctive lean items first, then the lean phrase
// queries', then general ones), then cost bucket-major, heaviest bucket first
// (query order inside a bucket, a query's items consecutive), so the
// persistent workers take the long items first and the short ones fill the
// tail (longest-first list scheduling).  The first bucket holds the items of
// queries of kHeavyQueryItems items or more, whose replays are the longest.
constexpr int kPlanKeys = 3 * kCostBuckets;   // classes: lean conjunctive, lean phrase, general
__device__ __forceinline__ uint32_t plan_key(uint32_t drv) {
  const uint32_t bucket = (drv >> kPlanBucketShift) & 0xFu;
  const uint32_t cls = (drv & kPlanLean) ? ((drv & kPlanPhrase) ? 1u : 0u) : 2u;
  return cls * kCostBuckets + (kCostBuckets - 1 - bucket);
}

// block-wide sums over the 256 threads of a plan workgroup (4 waves)
template <class T>
__device__ __forceinline__ T wave_incl_scan_any(T x) {
  const uint32_t l = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(x, d, 64);
    if (l >= static_cast<uint32_t>(d)) x += y;
  }
  return x;
}
// Exclusive prefixes over the workgroup's threads of N u32 values and one
// u64, and their workgroup totals, with one pair of barriers for all of them
// (the plan kernels' per-key item counts and event capacity).
template <int N>
struct ScanLds {
  uint32_t w[N][kPlanThreads / 64];
  uint64_t w64[kPlanThreads / 64];
};
template <int N>
__device__ __forceinline__ void block_excl_scan_n(const uint32_t (&x)[N], uint64_t y, uint32_t (&ex)[N],
                                                  uint32_t (&tot)[N], uint64_t& ey, uint64_t& toty,
                                                  ScanLds<N>& S) {
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  uint32_t inc[N];
#pragma unroll
  for (int k = 0; k < N; ++k) inc[k] = wave_incl_scan(x[k]);
  const uint64_t incy = wave_incl_scan_any(y);
  __syncthreads();
  if (l == 63) {
#pragma unroll
    for (int k = 0; k < N; ++k) S.w[k][w] = inc[k];
    S.w64[w] = incy;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    uint32_t below = 0, t = 0;
#pragma unroll
    for (uint32_t i = 0; i < kPlanThreads / 64; ++i) {
      below += i < w ? S.w[k][i] : 0u;
      t += S.w[k][i];
    }
    ex[k] = below + inc[k] - x[k];
    tot[k] = t;
  }
  uint64_t below = 0, t = 0;
#pragma unroll
  for (uint32_t i = 0; i < kPlanThreads / 64; ++i) {
    below += i < w ? S.w64[i] : 0ull;
    t += S.w64[i];
  }
  ey = below + incy - y;
  toty = t;
}

// Pass 1, one thread per query: driver (shortest list here), segment length
// (driver blocks per work item, so that items cost about kSegCost block
// decodes), item count and cost bucket; then the workgroup's item totals per
// key and its event capacity go to part[blockIdx.x] for pass 2.
__global__ __launch_bounds__(kPlanThreads) void plan_query_kernel(IndexArgs ix, const QueryIn* __restrict__ qs,
                                                         int nq, QueryPlan* __restrict__ plan,
                                                         uint32_t* __restrict__ counters, FusedReplay fr,
                                                         QueryDesc* __restrict__ desc,
                                                         PlanPart* __restrict__ part) {
  __shared__ ScanLds<kPlanKeys> S;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  QueryPlan p{0, 0, 1, 0, 0};
  if (i < nq) {
    const QueryIn q = qs[i];
    const int32_t* ql = qlist_of(qs, i);
    const int nt = q.n_terms;
    bool ok = nt > 0 && q.k > 0;
    if (nt > kMaxQueryTerms || q.k > kMaxKWide || (nt > kMaxPhraseTerms && (q.flags & kQueryPhrase))) {
      ok = false;
      atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrLimit));
    }
    // Driver (fewest blocks here), cost, class, O1 (the most selective other
    // list) and the smallest last doc of the others.  Up to kMaxTerms terms:
    // one round of loads, every term's block count, bitmap and last doc in
    // registers (each load's predicate depends on the query record only, so
    // all of them are in flight together); longer queries: plain loops.
    uint32_t d = 0, nd = 0xFFFFFFFFu, o1 = kNoSlot, min_last = 0xFFFFFFFFu;
    float cost = 1.0f;
    bool lean = true;
    if (nt <= kMaxTerms) {
      uint32_t nb[kMaxTerms], last[kMaxTerms];
      bool dn[kMaxTerms];
#pragma unroll
      for (int s = 0; s < kMaxTerms; ++s) {
        nb[s] = 0xFFFFFFFFu;
        last[s] = 0xFFFFFFFFu;
        dn[s] = false;
        const int32_t id = q.list[s];
        const bool in = s < nt;
        if (in && (id < 0 || static_cast<uint32_t>(id) >= ix.n_lists)) ok = false;
        if (in && id >= 0 && static_cast<uint32_t>(id) < ix.n_lists) {
          const ListDev& L = ix.lists[id];
          nb[s] = L.nblk;
          dn[s] = L.bm != kNoDense;
          last[s] = L.last;
        }
      }
#pragma unroll
      for (int s = 0; s < kMaxTerms; ++s)
        if (s < nt && nb[s] == 0) ok = false;  // no docs of this list in this shard: empty AND
      nd = nb[0];
#pragma unroll
      for (int s = 1; s < kMaxTerms; ++s) if (nb[s] < nd) { d = s; nd = nb[s]; }
      uint32_t o_nb = 0xFFFFFFFFu;
#pragma unroll
      for (int s = 0; s < kMaxTerms; ++s) {
        if (s >= nt || s == static_cast<int>(d)) continue;
        const bool dense = use_dense(ix, dn[s], nb[s], nd);
        cost += dense ? 0.0f : fminf(static_cast<float>(nb[s]) / nd, 64.0f);
        if (!dense) lean = false;
        min_last = last[s] < min_last ? last[s] : min_last;
        if (nb[s] < o_nb) { o1 = s; o_nb = nb[s]; }
      }
    } else if (ok) {
      for (int s = 0; s < nt; ++s) {
        const int32_t id = ql[s];
        if (id < 0 || static_cast<uint32_t>(id) >= ix.n_lists) { ok = false; break; }
        const uint32_t n = ix.lists[id].nblk;
        if (n == 0) ok = false;
        if (n < nd) { d = s; nd = n; }
      }
      uint32_t o_nb = 0xFFFFFFFFu;
      for (int s = 0; ok && s < nt; ++s) {
        if (s == static_cast<int>(d)) continue;
        const ListDev& L = ix.lists[ql[s]];
        const bool dense = use_dense(ix, L.bm != kNoDense, L.nblk, nd);
        cost += dense ? 0.0f : fminf(static_cast<float>(L.nblk) / nd, 64.0f);
        if (!dense) lean = false;
        min_last = L.last < min_last ? L.last : min_last;
        if (L.nblk < o_nb) { o1 = s; o_nb = L.nblk; }
      }
    }
    // a phrase query of more than two terms runs in the general class (the
    // lean kernel checks positions of two-term phrases only, in registers)
    if (nt > 2 && (q.flags & kQueryPhrase)) lean = false;
    if (ok) {
      uint32_t seg = static_cast<uint32_t>(kSegCost / cost);
      seg = seg > ix.seg_cap ? ix.seg_cap : seg;
      if (nt == 1) seg *= kSingleWindows;   // (single_segment: windows of 64 blocks)
      if (nt > 1 && (q.flags & kQueryPhrase)) seg = seg > kPhraseSegCap ? kPhraseSegCap : seg;
      seg = seg < 1 ? 1 : (seg > nd ? nd : seg);
      // cost class of one item (log2 of its block decodes, plus a fixed part
      // for the per-item setup): the queue hands out heavy items first
      const float item_cost = static_cast<float>(seg) * cost + kItemFixedCost;
      const uint32_t ic = static_cast<uint32_t>(item_cost);
      const uint32_t lg = 31u - __clz(ic > 4u ? ic : 4u);    // >= 2
      const uint32_t n_items = (nd + seg - 1) / seg;
      const uint32_t bucket = n_items >= kHeavyQueryItems ? static_cast<uint32_t>(kCostBuckets - 1)
                                                          : min(lg - 2u, static_cast<uint32_t>(kCostBuckets - 2));
      // (a lean phrase query has two terms: the one-term "phrase" is a plain term)
      const bool lean_ph = lean && nt > 1 && (q.flags & kQueryPhrase);
      p.driver = d | (bucket << kPlanBucketShift) | (lean ? kPlanLean : 0u) | (lean_ph ? kPlanPhrase : 0u);
      p.seg_blocks = seg;
      p.n_items = n_items;
      if (lean) {
        // the lean kernel's record (bases are added by plan_fill_kernel)
        // (the driver's and O1's records: a second round of loads, side by side)
        const ListDev A = ix.lists[ql[d]];
        QueryDesc D;
        D.a_base = A.base;
        D.a_tail = A.tail;
        D.a_idf = A.idf;
        D.a_blk0 = A.blk0;
        D.a_nblk = A.nblk;
        D.a_tail_cnt = A.tail_cnt;
        D.o_bm = 0; D.o_tf8 = 0; D.o_idf = 0.0; D.o_list = 0;
        if (o1 != kNoSlot) {
          const ListDev O = ix.lists[ql[o1]];
          D.o_bm = O.bm; D.o_tf8 = O.tf8; D.o_idf = O.idf;
          D.o_list = static_cast<uint32_t>(ql[o1]);
        }
        D.min_last = min_last;
        D.ev_base = 0;
        D.item_base = 0;
        D.n_items = p.n_items;
        D.seg = seg;
        D.slots = d | (o1 << 16);
        D.k = static_cast<uint32_t>(q.k);
        // pre-probe score bound: the other terms' BM25 parts are at most
        // sum(2.2 idf) * M / (M + norm) with M their largest tf bound
        double io = 0.0;
        uint32_t mm = 0;
        for (int s = 0; s < nt; ++s) {
          if (s == static_cast<int>(d)) continue;
          const ListDev& L = ix.lists[ql[s]];
          io += 2.2 * L.idf;
          mm = L.tfmax > mm ? L.tfmax : mm;
        }
        const float mf = o1 != kNoSlot ? static_cast<float>(mm) : 1.0f;
        D.b_id = static_cast<float>(2.2 * A.idf);
        D.b_m = mf;
        D.b_iom = static_cast<float>(io * static_cast<double>(mf));
        D.nt = static_cast<uint32_t>(nt);
        desc[i] = D;
      }
    }
    plan[i] = p;
    if (fr.q_done) {
      fr.q_done[i] = 0;
      if (p.n_items == 0) fr.n_hits[i] = 0;   // no item will replay an empty query
      if (p.n_items == 0 && fr.x_meta) {      // ... nor emit it: no events for its owner
        int32_t* m = fr.meta_of(static_cast<uint32_t>(i));
        m[0] = 0;
        m[1] = 0;
      }
    }
  }
  // the workgroup's items per key and event capacity (pass 2 scans them)
  const uint32_t key = plan_key(p.driver);
  uint32_t v[kPlanKeys], ex[kPlanKeys], tot[kPlanKeys];
#pragma unroll
  for (int k = 0; k < kPlanKeys; ++k) v[k] = key == static_cast<uint32_t>(k) ? p.n_items : 0u;
  uint64_t cex, ctot;
  block_excl_scan_n<kPlanKeys>(v, static_cast<uint64_t>(p.n_items) * p.seg_blocks * 128, ex, tot, cex, ctot, S);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < kPlanKeys; ++k) part[blockIdx.x].items[k] = tot[k];
    part[blockIdx.x].cap = ctot;
  }
}

// Pass 2, the same workgroups: every workgroup sums the partials of all
// workgroups (their totals give the key bases, those of the lower workgroups
// its own offsets), scans its queries per key, and writes each query's item and
// event bases, its lean record's bases, and its items' item -> query map and
// zeroed score floors (one thread per query, a few stores each; at most the
// query's driver blocks / segment length).
__global__ __launch_bounds__(kPlanThreads) void plan_fill_kernel(int nq, QueryPlan* __restrict__ plan,
                                                        const PlanPart* __restrict__ part, int n_part,
                                                        uint32_t* __restrict__ counters,
                                                        uint64_t ev_capacity, uint32_t item_capacity,
                                                        uint32_t lean_grid, uint32_t lean_grid_ph,
                                                        uint32_t seg_grid,
                                                        uint32_t* __restrict__ item_q,
                                                        uint64_t* __restrict__ pub,
                                                        QueryDesc* __restrict__ desc) {
  __shared__ ScanLds<kPlanKeys> S;
  __shared__ uint32_t s_key_all[kPlanKeys], s_key_below[kPlanKeys];
  __shared__ uint64_t s_cap_all, s_cap_below;
  const uint32_t t = threadIdx.x;
  // partial sums of all workgroups / of the lower ones: the first wave strides
  // over the partials and reduces across its lanes (no barrier until the end)
  if (t < 64) {
    uint32_t all[kPlanKeys], below[kPlanKeys];
#pragma unroll
    for (int k = 0; k < kPlanKeys; ++k) all[k] = below[k] = 0;
    uint64_t call = 0, cbelow = 0;
    for (int g = static_cast<int>(t); g < n_part; g += 64) {
      const PlanPart P = part[g];
      const bool lo = g < static_cast<int>(blockIdx.x);
#pragma unroll
      for (int k = 0; k < kPlanKeys; ++k) { all[k] += P.items[k]; below[k] += lo ? P.items[k] : 0u; }
      call += P.cap;
      cbelow += lo ? P.cap : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kPlanKeys; ++k) {
      all[k] = __builtin_amdgcn_readlane(wave_incl_scan(all[k]), 63);
      below[k] = __builtin_amdgcn_readlane(wave_incl_scan(below[k]), 63);
    }
    call = wave_incl_scan_any(call);
    cbelow = wave_incl_scan_any(cbelow);
    if (t == 63) {
#pragma unroll
      for (int k = 0; k < kPlanKeys; ++k) { s_key_all[k] = all[k]; s_key_below[k] = below[k]; }
      s_cap_all = call;
      s_cap_below = cbelow;
    }
  }
  __syncthreads();
  uint32_t key_base[kPlanKeys];
  uint32_t run = 0, n_lean = 0, n_conj = 0;
#pragma unroll
  for (int k = 0; k < kPlanKeys; ++k) {
    key_base[k] = run + s_key_below[k];
    run += s_key_all[k];
    if (k == kCostBuckets - 1) n_conj = run;
    if (k == 2 * kCostBuckets - 1) n_lean = run;
  }
  const uint32_t total_items = run;
  const bool fits = s_cap_all <= ev_capacity && total_items <= item_capacity;
  // this workgroup's queries: offsets inside their key and event bases
  const int i = blockIdx.x * blockDim.x + t;
  QueryPlan p{0, 0, 1, 0, 0};
  if (i < nq) p = plan[i];
  const uint32_t key = plan_key(p.driver);
  uint32_t v[kPlanKeys], ex[kPlanKeys], tot[kPlanKeys];
#pragma unroll
  for (int k = 0; k < kPlanKeys; ++k) v[k] = key == static_cast<uint32_t>(k) ? p.n_items : 0u;
  const uint64_t cap = static_cast<uint64_t>(p.n_items) * p.seg_blocks * 128;
  uint64_t cex, ctot;
  block_excl_scan_n<kPlanKeys>(v, cap, ex, tot, cex, ctot, S);
  uint32_t base = 0;
#pragma unroll
  for (int k = 0; k < kPlanKeys; ++k)
    if (key == static_cast<uint32_t>(k)) base = key_base[k] + ex[k];
  const uint64_t cb = s_cap_below + cex;
  if (i < nq) {
    plan[i].item_base = base;
    plan[i].ev_base = cb;
    // (skipped when the plan does not fit the workspace: never written past it)
    if (fits && (p.driver & kPlanLean)) {
      desc[i].item_base = base;
      desc[i].ev_base = cb;
    }
  }
  // The workgroup's items (item -> query, zeroed floor), spread over all its
  // threads: item j of the workgroup's run belongs to the last query whose
  // first item is at or before j (a binary search over the scan in LDS), so a
  // query of hundreds of items is not stored by its own thread alone.
  __shared__ ScanLds<1> S1;
  __shared__ uint32_t s_off[kPlanThreads + 1], s_base[kPlanThreads];
  const uint32_t mine[1] = {(i < nq && fits) ? p.n_items : 0u};
  uint32_t off[1], n_run[1];
  uint64_t u_ex, u_tot;
  block_excl_scan_n<1>(mine, 0ull, off, n_run, u_ex, u_tot, S1);
  s_off[t] = off[0];
  s_base[t] = base;
  if (t == 0) s_off[kPlanThreads] = n_run[0];
  __syncthreads();
  for (uint32_t j = t; j < n_run[0]; j += kPlanThreads) {
    uint32_t lo = 0, hi = kPlanThreads;   // s_off[lo] <= j < s_off[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_off[mid] <= j) lo = mid;
      else hi = mid;
    }
    const uint32_t slot = s_base[lo] + (j - s_off[lo]);
    item_q[slot] = blockIdx.x * blockDim.x + lo;
    if (pub) pub[slot] = 0;
  }
  if (blockIdx.x == 0) {
    if (t == 0) {
      if (!fits) atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrCapacity));
      // a class whose kernel the host did not launch (grid 0: its restatement
      // of the class rule found no such query) must hold no item: loud if it does
      if ((lean_grid == 0 && n_conj > 0) || (lean_grid_ph == 0 && n_lean > n_conj) ||
          (seg_grid == 0 && total_items > n_lean))
        atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrClass));
      counters[kCtrItems] = fits ? total_items : 0u;  // never write past the workspace
      counters[kCtrLean] = fits ? n_lean : 0u;
      counters[kCtrLeanConj] = fits ? n_conj : 0u;
      counters[kCtrEvCap] = static_cast<uint32_t>(s_cap_all > 0xFFFFFFFFull ? 0xFFFFFFFFull : s_cap_all);
    }
    // Work queues: shard s serves relative items s, s+8, s+16, ...; worker w
    // starts on relative item w without a dequeue, so shard s's head starts past
    // those first items (lean: one worker per wave; general: per workgroup).
    if (t < kQueueShards) {
      counters[kCtrHead0 + 16 * t] = (lean_grid + kQueueShards - 1 - t) / kQueueShards;
      counters[kCtrPHead0 + 16 * t] = (lean_grid_ph + kQueueShards - 1 - t) / kQueueShards;
      counters[kCtrGHead0 + 16 * t] = (seg_grid + kQueueShards - 1 - t) / kQueueShards;
    }
  }
}

// -------------------------------------------------------------- segment --
constexpr uint32_t kWin = 64;  // directory window: one entry per lane

struct WaveLds {
  uint32_t mb[8][128];   // doc ids of up to 8 other-list blocks decoded side by side
  uint32_t dtd[128];     // the driver's VInts tail block: doc ids
  uint32_t dtt[128];     //   and tfs
  Event evs[64];         // events buffered for one coalesced store
  double norm[256];      // Bm25Similarity cache_ (host table, scoring.h:85-90)
  uint32_t cur[kMaxTerms];  // per other slot (the first kMaxTerms): cursor into its block directory
  uint4 dblk[64];        // the driver's directory entries of the current segment
  uint32_t dmeta[64];
  uint32_t tf[128];      // cooperative decode of a VInts tf tail
  uint32_t dl[128];      // distinct other-list blocks probed by the driver block
  BlockDev wblk[kWin];   // directory window of the current other list: entries cur..cur+63
  uint32_t wlast[kWin];
  uint32_t wmeta[kWin];
};

// tf of posting `pos` of a block: packs are raw (not delta coded), so a lane
// reads its value directly; VInts tails are decoded by the whole wave.
__device__ __forceinline__ uint32_t pack_tf(const uint8_t* p, uint32_t bits, uint32_t pos) {
  return pack_value(p + 2, bits, pos);
}

// Directory entry j of list B: from the LDS window when it covers j.
// (Address-space-typed pointers keep the compiler from merging the two loads
// into one flat load of a selected pointer.)
#define WSR_LDS __attribute__((address_space(3)))
#define WSR_GLB __attribute__((address_space(1)))
__device__ __forceinline__ void dir_entry(const IndexArgs& ix, const ListDev& B, const WaveLds& S,
                                          uint32_t c, uint32_t wn, uint32_t j, BlockDev* bd,
                                          uint32_t* meta) {
  if (j - c < wn) {
    const WSR_LDS BlockDev* wb = (const WSR_LDS BlockDev*)(S.wblk);
    const WSR_LDS uint32_t* wm = (const WSR_LDS uint32_t*)(S.wmeta);
    const WSR_LDS BlockDev& e = wb[j - c];
    bd->prev = e.prev; bd->last = e.last; bd->doc_rel = e.doc_rel; bd->tf_rel = e.tf_rel;
    *meta = wm[j - c];
  } else {
    const WSR_GLB BlockDev* gb = (const WSR_GLB BlockDev*)(ix.blocks);
    const WSR_GLB uint32_t* gm = (const WSR_GLB uint32_t*)(ix.blk_meta);
    const WSR_GLB BlockDev& e = gb[B.blk0 + j];
    bd->prev = e.prev; bd->last = e.last; bd->doc_rel = e.doc_rel; bd->tf_rel = e.tf_rel;
    *meta = gm[B.blk0 + j];
  }
}

// G packed blocks side by side: group g (64/G lanes) unpacks block dl[base+g],
// 2G values per lane, prefix-sums them from the block's previous doc id and
// writes them to mb[g].  Skewed pairs probe many blocks with few docs each;
// decoding them together turns G dependent rounds into one.
template <int G>
__device__ __forceinline__ void grouped_decode(const IndexArgs& ix, const ListDev& B, WaveLds& S,
                                               uint32_t c, uint32_t wn, uint32_t base, uint32_t n) {
  constexpr int W = 64 / G, V = 2 * G;
  const uint32_t l = threadIdx.x & 63;
  const uint32_t g = l / W, li = l % W;
  const bool act = base + g < n;
  const uint32_t jj = act ? S.dl[base + g] : S.dl[base];
  BlockDev bb;
  uint32_t bm;
  dir_entry(ix, B, S, c, wn, jj, &bb, &bm);
  const uint32_t bits = bm & 0xFF;
  const uint8_t* p = ix.blob + B.base + bb.doc_rel;
  uint32_t* out = &S.mb[0][0];   // [t][lane]: conflict-free rows of 64 dwords
  uint32_t sum = 0;
#pragma unroll 2
  for (int t = 0; t < V; ++t) {
    const uint32_t x = pack_value(p + 2, bits, li * V + t);
    out[t * 64 + l] = x;   // raw deltas first: keeps them out of registers
    sum += x;
  }
  const uint32_t inc = group_incl_scan<W>(sum);
  uint32_t run = bb.prev + (inc - sum);
#pragma unroll 4
  for (int t = 0; t < V; ++t) { run += out[t * 64 + l]; out[t * 64 + l] = run; }
}

// lower_bound over the 128 doc ids of group g of a grouped decode
template <int G>
__device__ __forceinline__ uint32_t grouped_lower_bound(const WaveLds& S, uint32_t g, uint32_t x) {
  constexpr int W = 64 / G, V = 2 * G;
  const uint32_t* m = &S.mb[0][0];
  uint32_t lo = 0, n = 128;
  while (n > 0) {
    const uint32_t h = n >> 1, i = lo + h;
    if (m[(i % V) * 64 + g * W + i / V] < x) { lo = i + 1; n -= h + 1; } else { n = h; }
  }
  return lo;
}

template <int G>
__device__ __forceinline__ uint32_t grouped_at(const WaveLds& S, uint32_t g, uint32_t i) {
  constexpr int W = 64 / G, V = 2 * G;
  return (&S.mb[0][0])[(i % V) * 64 + g * W + i / V];
}

// Bm25Similarity: cache_[c] = k1 * (1 - b + b * Char4ToUint(c) / avg) (scoring.h:85-90),
// evaluated with the same operations in the same order as the host table.
__device__ __forceinline__ double length_norm(uint32_t c4, double avg) {
  const uint32_t mant = c4 & 0x07;
  const int sh = static_cast<int>(c4 >> 3) - 1;
  const uint32_t fl = sh < 0 ? mant : ((mant | 0x08u) << sh);
  const double k1 = 1.2, b = 0.75;
  return k1 * (1 - b + b * fl / avg);
}

__device__ __forceinline__ double bm25_term(double idf, uint32_t tf, double norm) {
  // TfNormLossy (scoring.h:65-69) times idf (scoring.h:136-140)
  const double f = static_cast<double>(static_cast<int32_t>(tf));
  const double k1p1 = 1.2 + 1;
  const double tfn = (f * k1p1) / (f + norm);
  return idf * tfn;
}

// global-address-space views (loads through them are global_load, not flat_load)
typedef __attribute__((address_space(1))) const uint64_t GlobalU64;
typedef __attribute__((address_space(1))) const uint32_t GlobalU32;

// --------------------------------------------------------------- replay --
// Events handed from one workgroup to another inside the segment kernel
// (fused replay) travel with agent-scope relaxed atomics, which gfx950 issues
// as sc1 (coherent across the XCDs' L2s) loads and stores; the hand-off itself
// is a per-query counter.  No buffer_wbl2 / buffer_inv of whole L2s needed.
__device__ __forceinline__ void store_event_coherent(Event* dst, const Event& e) {
  uint64_t* w = reinterpret_cast<uint64_t*>(dst);
  __hip_atomic_store(w, static_cast<uint64_t>(__double_as_longlong(e.score)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 1, static_cast<uint64_t>(static_cast<uint32_t>(e.doc)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kCoherent>
__device__ __forceinline__ void load_event(const Event* src, double* sc, int32_t* dc) {
  if (kCoherent) {
    // global (not flat) loads: a flat load also counts in lgkmcnt, so every
    // LDS or scalar wait would wait for it too; the doc alone (no load into
    // the pad's register, which the compiler reuses and then must wait for)
    const GlobalU64* w = (const GlobalU64*)src;
    *sc = __longlong_as_double(static_cast<long long>(
        __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    *dc = static_cast<int32_t>(__hip_atomic_load((const GlobalU32*)w + 2, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT));
  } else {
    *sc = src->score;
    *dc = src->doc;
  }
}

template <bool kCoherent>
__device__ __forceinline__ uint32_t load_count(const uint32_t* p) {
  if (kCoherent)
    return __hip_atomic_load((const GlobalU32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

__device__ __forceinline__ double shfl_f64(double v, uint32_t src) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __shfl(static_cast<uint32_t>(u), static_cast<int>(src), 64);
  const uint32_t hi = __shfl(static_cast<uint32_t>(u >> 32), static_cast<int>(src), 64);
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}

// libstdc++ std::priority_queue<unique_ptr<ResultDocEntry>, vector, EntryGreater>
// (query_processing.h:510-524): push = push_back + __push_heap, pop = __pop_heap
// (+ __adjust_heap) + pop_back, with comp(a, b) = a.score > b.score.
// The heap lives in the wave's registers, lane i = heap[i] (k <= 64), and each
// library operation runs as a few wave-wide steps instead of a scalar walk
// (the same array after every operation; tests/test_heap_parallel.py checks the
// model of this against the serial restatement):
//  * a sift up (__push_heap) of value v from `hole`: along the hole's ancestors
//    the scores never decrease going down, so the ancestors with score > v are
//    the deepest part of the chain; each of them moves one level down and v
//    lands at the shallowest (at the hole when there is none);
//  * __adjust_heap from the root: the path of "second children" (the right
//    child unless it is > the left) is a short uniform walk; the path shifts up
//    one level, then the old last entry sifts up from the path's end.
struct WaveHeap {
  double hs = 0.0;
  int32_t hd = 0;
  uint32_t n = 0;

  __device__ __forceinline__ double at(uint32_t i) const { return readlane_f64(hs, static_cast<int>(i)); }
  __device__ __forceinline__ int32_t doc(uint32_t i) const {
    return static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(hd), static_cast<int>(i)));
  }
  // __push_heap(first, hole, 0, value); anc = the hole's ancestors (bit mask)
  __device__ __forceinline__ void sift_up(uint32_t hole, uint64_t anc, double vs, int32_t vd) {
    const uint32_t l = threadIdx.x & 63;
    const bool on = (anc >> l) & 1ull;
    const uint64_t down = __ballot(on && hs > vs);   // ancestors that move one level down
    if (down == 0) {
      if (l == hole) { hs = vs; hd = vd; }
      return;
    }
    const uint32_t par = l ? (l - 1) >> 1 : 0u;
    const double ps = shfl_f64(hs, par);
    const int32_t pd = __shfl(hd, static_cast<int>(par), 64);
    if ((on || l == hole) && l != 0 && ((down >> par) & 1ull)) { hs = ps; hd = pd; }
    if (l == static_cast<uint32_t>(__builtin_ctzll(down))) { hs = vs; hd = vd; }
  }
  __device__ __forceinline__ void push(double vs, int32_t vd) {
    const uint32_t h = n++;
    uint64_t anc = 0;
    for (uint32_t x = h; x > 0;) {
      x = (x - 1) >> 1;
      anc |= 1ull << x;
    }
    sift_up(h, anc, vs, vd);
  }
  __device__ __forceinline__ void pop() {
    if (n > 1) {
      const uint32_t len = n - 1;
      const double vs = at(len);
      const int32_t vd = doc(len);
      // __adjust_heap(first, 0, len, value)
      const uint32_t l = threadIdx.x & 63;
      const double vl = shfl_f64(hs, min(2 * l + 1, 63u));
      const double vr = shfl_f64(hs, min(2 * l + 2, 63u));
      const uint32_t nxt = vr > vl ? 2 * l + 1 : 2 * l + 2;
      uint32_t h = 0, src = l;
      uint64_t path = 1;
      while (h < (len - 1) / 2) {
        const uint32_t c = __builtin_amdgcn_readlane(nxt, static_cast<int>(h));
        if (l == h) src = c;
        h = c;
        path |= 1ull << h;
      }
      if ((len & 1) == 0 && h == (len - 2) / 2) {
        const uint32_t c = 2 * h + 1;
        if (l == h) src = c;
        h = c;
        path |= 1ull << h;
      }
      const double ss = shfl_f64(hs, src);
      const int32_t sd = __shfl(hd, static_cast<int>(src), 64);
      hs = ss;
      hd = sd;
      sift_up(h, path & ~(1ull << h), vs, vd);
    }
    --n;
  }
};

// Running filter over a query's event stream, in doc-id order: an event is
// one the reference heap inserts iff fewer than k earlier events have a score
// >= its score (the top-k multiset of any prefix is carried by its events).
// `emit(score, doc)` is called, wave-uniformly, for exactly those events.
struct EventFilter {
  double pt = 0.0;    // running top-k of events, lane t = rank t
  uint32_t pt_n = 0;
  uint32_t k = 0;
  // one chunk of up to 64 events, lane i = event i of the chunk
  template <class Emit>
  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&& emit) {
    const uint32_t l = threadIdx.x & 63;
    const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
    uint64_t cm = __ballot(valid && (pt_n < k || sc > kth));
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      const double sv = readlane_f64(sc, fl);
      const int32_t dv = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(dc), fl));
      const uint32_t pos = __popcll(__ballot(l < pt_n && pt >= sv));
      if (pos < k) {
        emit(sv, dv);
        const double up = wave_shr1_f64(pt);
        if (l > pos) pt = up;
        else if (l == pos) pt = sv;
        pt_n = pt_n + 1 > k ? k : pt_n + 1;
      }
    }
  }
};

// The events of `nseg` segments (doc-id order), consumed as one stream in
// chunks of 64: the segment counts are loaded 64 at a time and scanned, lane r
// holding segment r's count and offset; a chunk finds each lane's segment by
// walking the few segments that overlap it (readlane, no memory), and the next
// chunk's loads are issued before the current chunk is filtered.  (Round 1
// searched an LDS copy of the offsets per lane; inside the out-of-line replay
// those were flat accesses whose waits also waited for the in-flight event
// loads, so every search step cost a full memory round trip.)
// count_of(r) and base_of(r) give segment r's event count and first event.
template <bool kCoherent = false, class Filter, class CountOf, class BaseOf, class Emit>
__device__ __forceinline__ void consume_stream(Filter& F, uint32_t nseg, CountOf count_of,
                                               BaseOf base_of, Emit&& emit) {
  const uint32_t l = threadIdx.x & 63;
  for (uint32_t r0 = 0; r0 < nseg; r0 += 64) {
    const uint32_t nj = min(64u, nseg - r0);
    const uint32_t c = l < nj ? count_of(r0 + l) : 0u;
    const uint32_t inc = wave_incl_scan(c);
    const uint32_t total = uni(__builtin_amdgcn_readlane(inc, 63));
    const uint32_t off = inc - c;   // segment l's first event in the stream
    // chunk [g0, g0 + 64): lane l loads stream event g0 + l
    auto load = [&](uint32_t g0, double* sc, int32_t* dc) {
      *sc = 0.0;
      *dc = 0;
      const uint32_t g = g0 + l;
      uint64_t m = __ballot(l < nj && c > 0 && off < g0 + 64u && off + c > g0);
      uint32_t rs = 0, ro = 0;
      while (m) {
        const int r = __builtin_ctzll(m);
        m &= m - 1;
        const uint32_t o = __builtin_amdgcn_readlane(off, r);
        const uint32_t cc = __builtin_amdgcn_readlane(c, r);
        if (g >= o && g - o < cc) { rs = static_cast<uint32_t>(r); ro = o; }
      }
      if (g < total) load_event<kCoherent>(base_of(r0 + rs) + (g - ro), sc, dc);
    };
    double sc, nsc;
    int32_t dc, ndc;
    load(0, &sc, &dc);
    for (uint32_t c0 = 0; c0 < total; c0 += 64) {
      load(c0 + 64, &nsc, &ndc);
      F.step(sc, dc, c0 + l < total, emit);
      sc = nsc;
      dc = ndc;
    }
  }
}

// Every event, in order (wide queries: the shard reduce keeps all of them).
struct PassFilter {
  template <class Emit>
  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&& emit) {
    uint64_t cm = __ballot(valid);
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      emit(readlane_f64(sc, fl),
           static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(dc), fl)));
    }
  }
};

// The libstdc++ heap of a wide query (k up to kMaxKWide) in LDS: the same
// __push_heap / __adjust_heap walks as WaveHeap, as wave-uniform code (every
// lane reads the same LDS word, lane 0 writes), then RankDoc / SortHeap.
struct LdsHeapSink {
  double* hs;
  int32_t* hd;
  uint32_t n = 0, k = 0;
  __device__ __forceinline__ double at(uint32_t i) const { return hs[i]; }
  __device__ __forceinline__ void set(uint32_t i, double vs, int32_t vd) {
    __builtin_amdgcn_wave_barrier();
    if ((threadIdx.x & 63) == 0) { hs[i] = vs; hd[i] = vd; }
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void push_hole(uint32_t hole, double vs, int32_t vd) {
    while (hole > 0) {
      const uint32_t parent = (hole - 1) >> 1;
      const double ps = at(parent);
      if (!(ps > vs)) break;
      set(hole, ps, hd[parent]);
      hole = parent;
    }
    set(hole, vs, vd);
  }
  __device__ __forceinline__ void pop() {
    if (n > 1) {
      const uint32_t len = n - 1;
      const double vs = at(len);
      const int32_t vd = hd[len];
      uint32_t hole = 0, child = 0;
      while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (at(child) > at(child - 1)) --child;
        set(hole, at(child), hd[child]);
        hole = child;
      }
      if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        set(hole, at(child - 1), hd[child - 1]);
        hole = child - 1;
      }
      push_hole(hole, vs, vd);
    }
    --n;
  }
  // RankDoc (query_processing.h:595-602)
  __device__ __forceinline__ void insert(double sv, int32_t dv) {
    if (n < k) { push_hole(n, sv, dv); ++n; }
    else if (sv > at(0)) { pop(); push_hole(n, sv, dv); ++n; }
  }
  // candidates of a chunk: those that beat the heap's minimum as it stands
  // (it only grows), each applied in doc order through insert
  template <class Emit>
  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&&) {
    const double mn = n < k ? -1.0 : at(0);
    uint64_t cm = __ballot(valid && sc > mn);
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      insert(readlane_f64(sc, fl),
             static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(dc), fl)));
    }
  }
  // SortHeap (query_processing.h:551-562): pop into LDS in descending order, one store
  __device__ __forceinline__ void finish(HitDev* out, int32_t* n_out) {
    const uint32_t l = threadIdx.x & 63;
    const uint32_t m = n;
    for (uint32_t i = 0; i < m; ++i) {
      const double ts = at(0);
      const int32_t td = hd[0];
      pop();
      // slot m-1-i is past the live heap (size m-1-i after the pop): free
      set(m - 1 - i, ts, td);
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = l; i < m; i += 64) {
      HitDev h;
      h.doc = hd[i];
      h.pad = 0;
      h.score = hs[i];
      out[i] = h;
    }
    if (l == 0) *n_out = static_cast<int32_t>(m);
  }
};

// RankDoc (query_processing.h:595-602) on the restated heap, then SortHeap
// (query_processing.h:551-562): results leave with one coalesced store.
// As a stream consumer (step) it needs no separate insertion filter: the
// reference's test is the heap's own (size < k, or score > its top, the k-th
// best), and the heap's state after any prefix of the event stream is the
// reference heap's at that doc (only insertions change it, and every
// insertion is an event), so an event that is not an insertion is rejected
// here exactly as its survivor was.
struct HeapSink {
  WaveHeap H;
  uint32_t k = 0;
  __device__ __forceinline__ void insert(double sv, int32_t dv) {
    if (H.n < k) H.push(sv, dv);
    else if (sv > H.at(0)) { H.pop(); H.push(sv, dv); }
    else return;
  }
  // one chunk of up to 64 events in doc order (lane order): the candidates
  // beat the heap's top as it stands (it only grows), each applied in turn
  template <class Emit>
  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&&) {
    const double top = H.n < k ? -1.0 : H.at(0);
    uint64_t cm = __ballot(valid && sc > top);
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      insert(readlane_f64(sc, fl),
             static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(dc), fl)));
    }
  }
  __device__ __forceinline__ void finish(HitDev* out, int32_t* n_out) {
    const uint32_t l = threadIdx.x & 63;
    const uint32_t m = H.n;
    double os = 0.0;
    int32_t od = 0;
    for (uint32_t i = 0; i < m; ++i) {
      const double ts = H.at(0);
      const int32_t td = __builtin_amdgcn_readlane(H.hd, 0);
      if (l == m - 1 - i) { os = ts; od = td; }
      H.pop();
    }
    if (l < m) {
      HitDev h;
      h.doc = od;
      h.pad = 0;
      h.score = os;
      out[l] = h;
    }
    if (l == 0) *n_out = static_cast<int32_t>(m);
  }
};

// One wave per query: the events of its segments (doc-id order) through the
// restated heap (Sink::step: the heap's own insertion test).
template <bool kCoherent, class Sink>
__device__ __forceinline__ void replay_query_sink(const QueryPlan& P, uint32_t k, const Event* events,
                                                  const uint32_t* ev_cnt, HitDev* out, int32_t* n_out) {
  Sink sink;
  sink.k = k;
  consume_stream<kCoherent>(
      sink, P.n_items, [&](uint32_t r) { return load_count<kCoherent>(ev_cnt + P.item_base + r); },
      [&](uint32_t r) { return events + P.ev_base + static_cast<uint64_t>(r) * P.seg_blocks * 128; },
      [](double, int32_t) {});
  sink.finish(out, n_out);
}
template <bool kCoherent>
__device__ __forceinline__ void replay_query(const QueryIn* __restrict__ qs,
                                             const QueryPlan* __restrict__ plan, int qi,
                                             const Event* events, const uint32_t* ev_cnt,
                                             HitDev* __restrict__ hits, int hit_stride,
                                             int32_t* __restrict__ n_hits) {
  const QueryPlan P = plan[qi];
  const uint32_t k = uni(qs[qi].k > 0 ? static_cast<uint32_t>(qs[qi].k) : 0u);
  HitDev* out = hits + static_cast<int64_t>(qi) * hit_stride;
  replay_query_sink<kCoherent, HeapSink>(P, k, events, ev_cnt, out, &n_hits[qi]);
}

// A one-item query's events straight from the lean kernel's LDS buffer (lane
// i = event i, doc order, n <= 64) through the restated heap.  Out of line, so
// the lean kernel's registers are its own; every uniform argument is made
// wave-uniform at entry (a callee's arguments arrive in VGPRs: the heap's
// loops must not compile as divergent ones).
__device__ __noinline__ void replay_lds_call(double sc, int32_t dc, uint32_t n, uint32_t k, HitDev* out,
                                             int32_t* n_out) {
  const uint64_t o = reinterpret_cast<uint64_t>(out), no = reinterpret_cast<uint64_t>(n_out);
  out = reinterpret_cast<HitDev*>(static_cast<uint64_t>(uni(static_cast<uint32_t>(o))) |
                                  (static_cast<uint64_t>(uni(static_cast<uint32_t>(o >> 32))) << 32));
  n_out = reinterpret_cast<int32_t*>(static_cast<uint64_t>(uni(static_cast<uint32_t>(no))) |
                                     (static_cast<uint64_t>(uni(static_cast<uint32_t>(no >> 32))) << 32));
  n = uni(n);
  k = uni(k);
  HeapSink sink;
  sink.k = k;
  sink.step(sc, dc, (threadIdx.x & 63) < n, [](double, int32_t) {});
  sink.finish(out, n_out);
}

// out-of-line copy for the segment kernel (keeps its register allocation
// independent of the replay code; called once per query)
__device__ __noinline__ void replay_query_call(const QueryIn* qs, const QueryPlan* plan, int qi,
                                               const Event* events, const uint32_t* ev_cnt,
                                               HitDev* hits, int hit_stride, int32_t* n_hits) {
  replay_query<true>(qs, plan, qi, events, ev_cnt, hits, hit_stride, n_hits);
}

// Wide queries (k > kMaxK): their segments emitted every survivor; one wave
// per query applies the whole stream, in doc order, to the heap in LDS.
__global__ __launch_bounds__(64) void wide_replay_kernel(const QueryIn* __restrict__ qs,
                                                         const QueryPlan* __restrict__ plan, int nq,
                                                         const Event* __restrict__ events,
                                                         const uint32_t* __restrict__ ev_cnt,
                                                         HitDev* __restrict__ hits, int hit_stride,
                                                         int32_t* __restrict__ n_hits) {
  __shared__ double s_hs[kMaxKWide];
  __shared__ int32_t s_hd[kMaxKWide];
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const int32_t kq = qs[qi].k;
  if (kq <= kMaxK) return;
  const QueryPlan P = plan[qi];
  LdsHeapSink sink;
  sink.hs = s_hs;
  sink.hd = s_hd;
  sink.k = static_cast<uint32_t>(kq);
  consume_stream<false>(
      sink, P.n_items, [&](uint32_t r) { return ev_cnt[P.item_base + r]; },
      [&](uint32_t r) { return events + P.ev_base + static_cast<uint64_t>(r) * P.seg_blocks * 128; },
      [](double, int32_t) {});
  sink.finish(hits + static_cast<int64_t>(qi) * hit_stride, &n_hits[qi]);
}

// Fused shard emission (FusedReplay::x_send): the query's events, reduced as
// shard_reduce_kernel does (compacted in place, coherent: other workers wrote
// them), then appended to the owner's slot and described in x_meta.
// (the exchange fields come as values: a FusedReplay passed by reference would
// be copied to every wave's stack at kernel entry, 6 KB of scratch per wave)
__device__ __noinline__ void shard_emit_call(const QueryIn* qs, const QueryPlan* plan, int qi, Event* events,
                                             const uint32_t* ev_cnt, Event* x_send, int32_t* x_meta,
                                             uint32_t* x_fill, uint32_t* x_err, uint64_t x_slot,
                                             uint64_t x_stride, uint64_t x_meta_stride, int32_t x_qpr) {
  FusedReplay fr{};
  fr.x_send = x_send; fr.x_meta = x_meta; fr.x_fill = x_fill; fr.x_err = x_err;
  fr.x_slot = x_slot; fr.x_stride = x_stride; fr.x_meta_stride = x_meta_stride; fr.x_qpr = x_qpr;
  const uint32_t l = threadIdx.x & 63;
  const QueryPlan P = plan[qi];
  const uint32_t k = uni(qs[qi].k > 0 ? static_cast<uint32_t>(qs[qi].k) : 0u);
  Event* out = events + P.ev_base;
  uint32_t n = 0;
  // writes land at out[n], below every event not yet read (see shard_reduce_kernel)
  auto emit = [&](double sv, int32_t dv) {
    if (l == 0) {
      Event e;
      e.score = sv;
      e.doc = dv;
      e.pad = 0;
      store_event_coherent(&out[n], e);
    }
    ++n;
  };
  auto count_of = [&](uint32_t r) { return load_count<true>(ev_cnt + P.item_base + r); };
  auto base_of = [&](uint32_t r) { return events + P.ev_base + static_cast<uint64_t>(r) * P.seg_blocks * 128; };
  if (k > static_cast<uint32_t>(kMaxK)) {
    PassFilter F;
    consume_stream<true>(F, P.n_items, count_of, base_of, emit);
  } else {
    EventFilter F;
    F.k = k;
    consume_stream<true>(F, P.n_items, count_of, base_of, emit);
  }
  __builtin_amdgcn_s_waitcnt(0);
  const uint32_t o = static_cast<uint32_t>(qi) / static_cast<uint32_t>(fr.x_qpr);
  uint32_t off = 0;
  if (l == 0 && n) off = atomicAdd(&fr.x_fill[o], n);
  off = uni(off);
  int32_t cnt = static_cast<int32_t>(n);
  if (static_cast<uint64_t>(off) + n > fr.x_slot) {
    cnt = -1;
    if (l == 0) atomicOr(fr.x_err, static_cast<uint32_t>(kErrExchange));
  } else {
    Event* dst = fr.x_send + static_cast<uint64_t>(o) * fr.x_stride + off;
    for (uint32_t i = l; i < n; i += 64) {
      double sc;
      int32_t dc;
      load_event<true>(&out[i], &sc, &dc);
      Event e;
      e.score = sc;
      e.doc = dc;
      e.pad = 0;
      dst[i] = e;
    }
  }
  if (l == 0) {
    int32_t* m = fr.meta_of(static_cast<uint32_t>(qi));
    m[0] = cnt;
    m[1] = static_cast<int32_t>(off);
  }
}

// ------------------------------------------------------ item plumbing --
// Score floors of the earlier items of a query.  pub[i] is backed by k
// survivors at or before item i (its running k-th best, or the floor it had),
// so the largest pub of the items before this one bounds the k-th best before
// it as well, and is at least the predecessor's alone: items of one query run
// at once, and the predecessor's value reaches a later item only one refresh
// per hop.  prev_pub = pub + item - 1, n_prev = the items before this one; lane
// l loads pub[item - 1 - l] (the nearest 64), floor_max reduces over the wave.
__device__ __forceinline__ uint64_t floor_lanes(const uint64_t* prev_pub, uint32_t n_prev) {
  const uint32_t l = threadIdx.x & 63;
  return (prev_pub && l < n_prev) ? __hip_atomic_load(prev_pub - l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0ull;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  uint32_t y;
  y = dpp<kRowShr1>(x); x = umax(x, y);
  y = dpp<kRowShr2>(x); x = umax(x, y);
  y = dpp<kRowShr4>(x); x = umax(x, y);
  y = dpp<kRowShr8>(x); x = umax(x, y);
  y = dpp<kRowBcast15, 0xA>(x); x = umax(x, y);
  y = dpp<kRowBcast31, 0xC>(x); x = umax(x, y);
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint64_t floor_max(uint64_t x) {
  // (volatile: the reduction stays inside the caller's refresh branch; the
  // compiler would otherwise run it speculatively on every driver block)
  asm volatile("" : "+v"(x));
  const uint32_t hi = wave_max(static_cast<uint32_t>(x >> 32));
  const uint32_t lo = wave_max(static_cast<uint32_t>(x >> 32) == hi ? static_cast<uint32_t>(x) : 0u);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Next work item of a persistent worker over items [lo, hi), split into
// kQueueShards round-robin shards (relative index i in shard i % kQueueShards),
// each with its own head on its own 64-byte line; a worker starts with its own
// shard and steals from the others.  Returns hi when the range is drained.
__device__ __forceinline__ uint32_t next_item(uint32_t* heads, uint32_t lo, uint32_t hi,
                                              uint32_t& shard, uint32_t& tried) {
  const uint32_t n = hi - lo;
  const uint32_t l = threadIdx.x & 63;
  while (tried < kQueueShards) {
    // the current shard: a load first, so that drained heads see no
    // read-modify-write from thousands of finishing workers
    const uint32_t limit = (n + kQueueShards - 1 - shard) / kQueueShards;
    uint32_t local = 0;
    if (l == 0) {
      local = __hip_atomic_load(&heads[16 * shard], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (local < limit) local = atomicAdd(&heads[16 * shard], 1u);
    }
    local = uni(local);
    if (local < limit) return lo + shard + kQueueShards * local;
    // drained (a drained shard stays drained): read all heads in one round
    // and move to the next shard that still has work
    uint32_t h = 0, lim = 0;
    if (l < kQueueShards) {
      h = __hip_atomic_load(&heads[16 * l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lim = (n + kQueueShards - 1 - l) / kQueueShards;
    }
    const uint32_t avail = static_cast<uint32_t>(__ballot(l < kQueueShards && h < lim));
    if (!avail) break;
    const uint32_t rot = ((avail >> shard) | (avail << (kQueueShards - shard))) & ((1u << kQueueShards) - 1u);
    shard = (shard + __builtin_ctz(rot)) % kQueueShards;
    ++tried;
  }
  tried = kQueueShards;
  return hi;
}

// End of a work item: re-filter its events against the earlier segments'
// floor as it stands now (it only grows, and every value it takes is backed by
// k survivors before this segment), keeping the doc order; publish the count;
// with fused replay, the worker that completes a query's last item replays the
// query (its coherent event stores complete before the counter moves, and the
// replay reads the other items' events with coherent loads).
template <bool kWave>
__device__ __forceinline__ void finish_item(const QueryIn* qs, const QueryPlan* plan, uint32_t qi,
                                            uint32_t n_items, uint32_t item,
                                            const uint64_t* prev_pub, uint32_t n_prev, Event* ev_out, uint32_t ev_n,
                                            const Event* events, uint32_t* ev_cnt,
                                            const FusedReplay& fr) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  if (prev_pub && ev_n > 0) {
    const double fl_end = __longlong_as_double(static_cast<long long>(floor_max(floor_lanes(prev_pub, n_prev))));
    uint32_t kept = 0;
    for (uint32_t c = 0; c < ev_n; c += 64) {
      double sc = 0.0;
      int32_t dc = 0;
      const bool in = c + l < ev_n;
      if (in) load_event<true>(&ev_out[c + l], &sc, &dc);
      const bool keep = in && sc > fl_end;
      const uint64_t km = __ballot(keep);
      if (keep) {
        Event e;
        e.score = sc;
        e.doc = dc;
        e.pad = 0;
        store_event_coherent(&ev_out[kept + __popcll(km & lt)], e);
      }
      kept += __popcll(km);
    }
    ev_n = kept;
  }
  // The hand-off, stated against the LLVM AMDGPU memory model's code
  // sequences for GFX942/GFX950 (AMDGPUUsage, "Memory Model GFX942"):
  //  * every byte the replay reads (events, counts) is written here with
  //    `store atomic monotonic agent` = global_store sc1: written through to
  //    the agent's point of coherence (no XCD's L2 keeps it dirty);
  //  * `s_waitcnt vmcnt(0)` below returns only when those stores are acked at
  //    that point, and the counter RMW (`atomicrmw monotonic agent`, sc1) is
  //    issued after it, so it is ordered after them in the memory system;
  //  * the finisher's loads depend on the RMW's value (control dependence, no
  //    speculation of vector loads on GFX9) and are `load atomic monotonic
  //    agent` = global_load sc1, which miss every non-coherent L2 line.
  // The acquire-release RMW (the C++-model form) adds `buffer_wbl2 sc1` before
  // and `buffer_inv sc1` after the RMW: a write-back / invalidate of the whole
  // L2 of the issuing XCD that has nothing to do here (the only data handed
  // over is sc1-coherent), on every item.  Measured: 0.88 against 0.49 ms for
  // the C2 high x high class, 5.8 against 10.6 M q/s on the C3 headline,
  // parity green both ways (profiles/r03_handoff_ab.txt).
  if (l == 0) __hip_atomic_store(&ev_cnt[item], ev_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // wide queries (k > kMaxK) are replayed by wide_replay_kernel after the
  // segments; in a shard step every query is emitted here
  if (fr.q_done && (fr.x_send || uni(static_cast<uint32_t>(qs[qi].k)) <= static_cast<uint32_t>(kMaxK))) {
    __builtin_amdgcn_s_waitcnt(0);
    block_sync<kWave>();
    uint32_t old = 0;
    if (l == 0)
      old = __hip_atomic_fetch_add(&fr.q_done[qi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = uni(old);
    if (old + 1 == n_items) {
      if (fr.x_send)
        shard_emit_call(qs, plan, static_cast<int>(qi), const_cast<Event*>(events), ev_cnt, fr.x_send,
                        fr.x_meta, fr.x_fill, fr.x_err, fr.x_slot, fr.x_stride, fr.x_meta_stride, fr.x_qpr);
      else
        replay_query_call(qs, plan, static_cast<int>(qi), events, ev_cnt, fr.hits, fr.hit_stride,
                          fr.n_hits);
    }
  }
}

// PosStream keeps the pack dwords it last read and takes a bag's next
// positions from them while they cover them (one load per bag of small
// deltas instead of one per position).
constexpr bool kPosWindow = true;
// PosStream takes its first pack record from the bag's word pair (pos_start)
// instead of a dependent pos_pk load.
constexpr bool kPosBag = true;
// phrase_match2 primes both bags' first windows before the merge pops
constexpr bool kPosPrime = true;

// waves per SIMD the segment kernel is compiled for (register budget)
constexpr int kSegWaves = 3;

// ---------------------------------------------------------- phrase check --
// Per general workgroup (kPhraseScratch words), per query term s: the image
// posting slot of value v (= 2l or 2l+1 of the driver block) at [s*256 + v],
// its tf at [s*256 + 128 + v] (phrase queries only).

// Does the doc hold the query's terms at consecutive positions?  Term i's bag
// (query order) = tf_i positions delta coded from 0 starting at entry
// pos_start[slot_i] of its box.  True iff some a has a + i in bag i for every
// i, which is PhraseQueryProcessor2::NumOfMatches() > 0 (query_processing.h:
// 264-336: the 2-term merge and the general max-adjusted walk both find every
// such a).  One lane per survivor; term state stays in registers (the term
// loop is unrolled, so every index is static).
// One position bag read as a stream: entry e of the box sits in pack e / 128
// (offset and width from the pack directory, reloaded only when the pack
// changes) or in the decoded VInts remainder; positions are prefix sums of
// the bag's deltas.
struct PosStream {
  const uint8_t* data;   // current pack's values
  uint32_t bits, pk;     // its width and index (pk = ~0: none yet)
  uint32_t e, end;       // next entry, one past the bag
  int32_t cur;           // last position popped
  // the last two aligned dwords read from the pack, from bit wb of the pack's
  // data (kPosWindow): a bag's next values usually lie in them, so a bag of
  // small deltas costs one load instead of one per position
  uint32_t w0, w1;
  int32_t wb;
  // (P: the list's box; the record of the bag's first pack comes with the
  // bag's start, in one 8-byte word, so the first position needs no pos_pk load)
  __device__ __forceinline__ void init(const IndexArgs& ix, const PosDev& P, uint32_t slot, uint32_t tf) {
    const uint2 sb = ix.pos_start[slot];
    e = sb.x;
    const uint32_t g = kPosBag ? sb.y : 0u;
    end = e + tf;
    cur = 0;
    pk = 0xFFFFFFFFu;
    data = ix.pos_blob;
    bits = 1;
    if (g) {
      pk = e >> 7;
      data = ix.pos_blob + P.base + (g >> 6) + 2;
      bits = g & 63u;
    }
    w0 = w1 = 0;
    wb = -(1 << 30);
  }
  // (kPosPrime) the window of the bag's first position, loaded before either
  // stream of a pair pops, so the two bags' first pack reads share one round
  // trip (the pack record came with the start; without it, next() loads it)
  __device__ __forceinline__ void prime() {
    if (!kPosWindow || e >= end || pk != (e >> 7)) return;
    const int32_t bit = static_cast<int32_t>((e & 127u) * bits);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(__builtin_align_down(data + (bit >> 3), 4));
    w0 = w[0];
    w1 = w[1];
    wb = static_cast<int32_t>(reinterpret_cast<const uint8_t*>(w) - data) * 8;
  }
  // pop the next position (false past the bag's end)
  __device__ __forceinline__ bool next(const IndexArgs& ix, const PosDev& P) {
    if (e >= end) return false;
    const uint32_t p = e >> 7;
    uint32_t v;
    if (p < P.npk) {
      if (p != pk) {
        const uint2 w = ix.pos_pk[P.pk0 + p];
        data = ix.pos_blob + P.base + w.x + 2;
        bits = w.y;
        pk = p;
        wb = -(1 << 30);
      }
      const int32_t bit = static_cast<int32_t>((e & 127u) * bits);
      if (kPosWindow) {
        if (bit - wb < 0 || bit - wb + static_cast<int32_t>(bits) > 64) {
          const uint8_t* a = data + (bit >> 3);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(__builtin_align_down(a, 4));
          w0 = w[0];
          w1 = w[1];
          wb = static_cast<int32_t>(reinterpret_cast<const uint8_t*>(w) - data) * 8;
        }
        const uint32_t sh = static_cast<uint32_t>(bit - wb);
        const uint64_t x = ((static_cast<uint64_t>(w1) << 32) | w0) >> sh;
        v = static_cast<uint32_t>(x) & (bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u));
      } else {
        v = pack_value(data, bits, e & 127u);
      }
    } else {
      v = ix.pos_tail[P.tail + (e - (P.npk << 7))];
    }
    ++e;
    cur += static_cast<int32_t>(v);
    return true;
  }
};

// Does the doc hold the query's terms at consecutive positions?  Term i's bag
// (query order) = tf_i positions delta coded from 0 starting at entry
// pos_start[slot_i] of its box (slot_i, tf_i in the caller's scratch ph at
// [i*256 + v], [i*256 + 128 + v]).  True iff some a has a + i in bag i for
// every i, which is PhraseQueryProcessor2::NumOfMatches() > 0
// (query_processing.h:264-336: the 2-term merge and the general max-adjusted
// walk both find every such a).  One lane per survivor.
// bloom_check (libbloom/bloom.c:48-75) of list `elem`'s term in the bit array
// `side` (0 prior, 1 next) of posting slot `slot`: false = not present (an
// all-zero array, as for a posting without one, answers false).  Bit x of the
// array is bit x % 8 of byte x / 8, i.e. bit x % 32 of little-endian dword x / 32.
__device__ __forceinline__ bool bloom_may(const IndexArgs& ix, uint32_t slot, uint32_t side, int32_t elem) {
  const uint2 h = ix.blm_hash[elem];
  const uint4 w = ix.blm[2 * slot + side];
  for (uint32_t i = 0; i < ix.blm_hashes; ++i) {
    const uint32_t x = (h.x + i * h.y) % ix.blm_bits;
    const uint32_t q = x >> 5;
    const uint32_t d = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    if (!((d >> (x & 31u)) & 1u)) return false;
  }
  return true;
}

// QueryProcessor::IsPossibleToPresent (query_processing.h:873-884): two terms,
// CheckBloomWithEnableFactor (:796-807) -- the shorter list's filter, by the
// lists' full sizes; more terms, CheckBloomFallBack (:784-794) -- every term's
// "next" filter holds the following term.
__device__ __forceinline__ bool bloom_possible(const IndexArgs& ix, const int32_t* qlist, uint32_t nt,
                                               const uint32_t* ph, uint32_t v) {
  if (nt == 2) {
    const uint64_t f = ix.bloom_factor;
    const uint64_t s1 = ix.lists[qlist[0]].df, s2 = ix.lists[qlist[1]].df;
    if (f * s1 <= s2) return bloom_may(ix, ph[v], 1, qlist[1]);
    if (f * s2 < s1) return bloom_may(ix, ph[256 + v], 0, qlist[0]);
    return true;
  }
  for (uint32_t i = 0; i + 1 < nt; ++i)
    if (!bloom_may(ix, ph[i * 256 + v], 1, qlist[i + 1])) return false;
  return true;
}

// Two-term phrase of a lean item: terms (query order) list l0 / l1, their
// posting slots and tfs in registers.  The bloom rule of bloom_possible's
// two-term case, then ProcessTwoTerm's merge (bag 0 shifted by one against
// bag 1).  Inlined: the lean kernel keeps no phrase scratch.
__device__ __forceinline__ bool phrase_match2(const IndexArgs& ix, uint32_t l0, uint32_t l1, uint32_t slot0,
                                              uint32_t tf0, uint32_t slot1, uint32_t tf1) {
  if (ix.bloom_factor) {
    const uint64_t f = ix.bloom_factor;
    const uint64_t s1 = ix.lists[l0].df, s2 = ix.lists[l1].df;
    if (f * s1 <= s2) {
      if (!bloom_may(ix, slot0, 1, static_cast<int32_t>(l1))) return false;
    } else if (f * s2 < s1) {
      if (!bloom_may(ix, slot1, 0, static_cast<int32_t>(l0))) return false;
    }
  }
  const PosDev P0 = ix.pos_lists[l0], P1 = ix.pos_lists[l1];
  PosStream s0, s1;
  s0.init(ix, P0, slot0, tf0);
  s1.init(ix, P1, slot1, tf1);
  if (kPosPrime) {
    s0.prime();
    s1.prime();
  }
  if (!s0.next(ix, P0) || !s1.next(ix, P1)) return false;
  for (;;) {
    const int32_t a = s0.cur + 1, b = s1.cur;
    if (a == b) return true;
    if (a < b) { if (!s0.next(ix, P0)) return false; }
    else if (!s1.next(ix, P1)) return false;
  }
}

__device__ __noinline__ bool phrase_match(const IndexArgs& ix, const int32_t* qlist, uint32_t nt,
                                          const uint32_t* ph, uint32_t v) {
  if (ix.bloom_factor && !bloom_possible(ix, qlist, nt, ph, v)) return false;
  if (nt == 2) {   // ProcessTwoTerm: a merge of bag 0 against bag 1 shifted by one
    const PosDev P0 = ix.pos_lists[qlist[0]], P1 = ix.pos_lists[qlist[1]];
    PosStream s0, s1;
    s0.init(ix, P0, ph[v], ph[128 + v]);
    s1.init(ix, P1, ph[256 + v], ph[384 + v]);
    if (!s0.next(ix, P0) || !s1.next(ix, P1)) return false;
    for (;;) {
      const int32_t a = s0.cur + 1, b = s1.cur;
      if (a == b) return true;
      if (a < b) { if (!s0.next(ix, P0)) return false; }
      else if (!s1.next(ix, P1)) return false;
    }
  }
  PosStream st[kMaxPhraseTerms];
#pragma unroll
  for (uint32_t i = 0; i < kMaxPhraseTerms; ++i) {
    const PosDev Pi = ix.pos_lists[i < nt ? qlist[i] : qlist[0]];
    st[i].init(ix, Pi, i < nt ? ph[i * 256 + v] : 0u, i < nt ? ph[i * 256 + 128 + v] : 0u);
    if (i < nt && !st[i].next(ix, Pi)) return false;
  }
  int32_t a = 0;
  for (;;) {
    bool moved = false;
#pragma unroll
    for (uint32_t i = 0; i < kMaxPhraseTerms; ++i) {
      if (i < nt) {
        const int32_t ii = static_cast<int32_t>(i);
        if (st[i].cur - ii < a) {
          const PosDev P = ix.pos_lists[qlist[i]];
          do {
            if (!st[i].next(ix, P)) return false;
          } while (st[i].cur - ii < a);
        }
        if (st[i].cur - ii > a) {
          a = st[i].cur - ii;
          moved = true;
        }
      }
    }
    if (!moved) return true;
  }
}

// ------------------------------------------------- lean bitmap segment --
// Byte loads of the pipeline are whole aligned dwords, kept raw until the
// consuming stage extracts the byte (an extraction next to the load would make
// the loop wait for it in the iteration that issued it).
__device__ __forceinline__ uint32_t byte_word(const uint8_t* p, uint32_t* sh) {
  *sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3) << 3;
  return *reinterpret_cast<const uint32_t*>(__builtin_align_down(p, 4));
}

// Three dwords covering values 2l and 2l+1 of a 128-value pack whose data
// starts at d (bit width b <= 32): one load per lane for both values.
__device__ __forceinline__ void pair_words(const uint8_t* d, uint32_t b, uint32_t l, uint32_t& w0,
                                           uint32_t& w1, uint32_t& w2, uint32_t& sh) {
  const uint32_t bit = 2 * l * b;
  const uint8_t* a = d + (bit >> 3);
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a) & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(__builtin_align_down(a, 4));
  w0 = w[0];
  w1 = w[1];
  w2 = w[2];
  sh = (mis << 3) + (bit & 7);
}

__device__ __forceinline__ void pair_values(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t sh,
                                            uint32_t b, uint32_t& v0, uint32_t& v1) {
  const uint32_t mask = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
  v0 = __builtin_amdgcn_alignbit(w1, w0, sh) & mask;   // sh <= 31
  const uint32_t s2 = sh + b;                           // <= 63
  const bool up = s2 >= 32;
  v1 = __builtin_amdgcn_alignbit(up ? w2 : w1, up ? w1 : w0, s2 & 31u) & mask;
}

// Segment of an item whose other lists all carry rank bitmaps (the common
// case: a short driver against long lists).  The driver's blocks stream
// through a software pipeline, one block per stage and iteration j:
//   C(j-2)  compaction: the survivors of block j-2 (docs present in the most
//           selective other list O1) are appended, in doc order, to a queue in
//           LDS with their doc-length code and both tfs; every full 64 are
//           scored one per lane (all query terms, query order, the further
//           other lists probed here) and fed to the running top-k;
//   H(j-1)  O1's bitmap words of block j-1 give hits and posting ranks; the
//           hits' 1-byte tfs are loaded;
//   D(j)    block j's doc ids are unpacked and prefix-summed; O1's bitmap
//           words, the doc-length bytes and the driver's tf words are loaded;
//   W(j+1)  the doc-id pack words of block j+1 (and the score floor) are loaded.
// Every load is issued unconditionally (drained stages read index 0) so each
// stage waits only for loads issued one iteration earlier.  Scoring one
// survivor per lane instead of two postings per lane keeps the f64 work
// proportional to the survivors.
// Driver blocks between floor refreshes.  At 8: events per 4,096 C2 queries
// 160 k -> 98 k (high x high 584 k -> 356 k), the most events of one query
// 3,378 -> 1,111, main leg 26.37 -> 26.53 M q/s (4 is no better,
// profiles/r02_sc_ab.txt; 16 and 32 are within the noise, with 6 % and 21 %
// more events: profiles/r02_su_refresh_interval_ab.txt).
constexpr uint32_t kFloorRefresh = 8;
// Extra iterations of slack in the conjunctive lean pipeline (kDeep of
// lean_segment): 0 -- H consumes the O1 probes D issued one iteration
// earlier and C the rank records H issued one iteration earlier; 1 -- H runs
// two blocks behind D (the probes have a whole iteration in flight); 2 -- C
// also runs two blocks behind H.  Each stage of slack keeps one more register
// set live across the loop.
constexpr int kLeanDeep = 0;
// Capacity of the LDS event buffer: flushed after every chunk that added
// events (64 since round 3: C2 leg 31.5 -> 33.2 M q/s, C4 11.8 -> 12.5 M
// against 128, C3 headline unchanged; 4 KB less LDS per workgroup,
// profiles/r03_knob_ab.txt).
constexpr uint32_t kLeanEvs = 64;
// LDS of one wave of the lean kernel (kPh: phrase instance, whose queue also
// carries the driver's posting slot and O1's posting rank of every survivor)
template <bool kPh>
struct LeanLdsT {
  uint32_t q[kPh ? 1536 : 1024];   // survivor queue (4 or 6 rings of 256); at item end the
                                   // replay's segment scan
  Event evs[kLeanEvs];   // events buffered in LDS, stored when a chunk could overflow them
                         // and at the end
  uint4 dblk[64];        // the driver's directory entries of the segment
  uint32_t dmeta[64];
};

// (single-term items run single_segment: every item here has an O1.)
// tdoc/ttf: the driver's VInts tail block (doc ids, tfs; 2 per lane) when
// dtail, used for block b1 - 1.
// kTwo: every item of the launch is a two-term, k <= kMaxK query (the
// headline's, C2's and C5's batches): two terms scored inline, no wide or
// single-term paths, so the instance keeps fewer registers (90 VGPRs, no
// scratch, half the SGPR spill reloads of the general instance).
// kPh: the batch holds phrase queries; a lean one has two terms (the plan
// sends longer phrases to the general class), the driver and O1, whose
// posting slots and tfs ride in the survivor queue, so the position check
// (phrase_match2) runs on registers with no scratch.
// kBk: O1 carries offset buckets (the item's QueryDesc::o_bm has a shift):
// D loads its bucket entry, H matches the offset and loads the hit's tf word,
// C resolves the rare probe past a bucket's fourth posting from its offset
// bytes.  The same pipeline otherwise.
template <bool kPh, bool kTwo = false, bool kBk = false, int kDeep = 0>
__device__ __forceinline__ void lean_segment(const IndexArgs& ix, LeanLdsT<kPh>& S, const double* norm_tab,
                                             const QueryDesc& Q, const int32_t* qlist,
                                             bool phrase, uint32_t b0, uint32_t b1, bool dtail,
                                             uint32_t tdoc0, uint32_t tdoc1, uint32_t ttf0, uint32_t ttf1,
                                             uint64_t floor0, const uint64_t* prev_pub, uint32_t n_prev,
                                             uint64_t* my_pub,
                                             Event* ev_out, uint32_t& ev_n, uint32_t& evb,
                                             double& pt, uint32_t& pt_n,
                                             double& last_pub, uint32_t& n_surv, uint32_t& n_dblk) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  const uint32_t d = kTwo ? (Q.slots & 1u) : (Q.slots & 0xFFFFu);
  const uint32_t o1 = kTwo ? (d ^ 1u) : (Q.slots >> 16);
  const uint32_t nt = kTwo ? 2u : (Q.nt & 0xFFFFu), k = Q.k;
  // k > kMaxK: every survivor is an event; the replay's heap in LDS decides
  const bool wide = !kTwo && k > static_cast<uint32_t>(kMaxK);
  const uint32_t min_last = in_vgpr(Q.min_last);
  // O1's bitmap (buckets: reads go to a valid dummy word; the image may have
  // no bitmaps): the probe reads the mask word alone; a hit reads its rank
  // record (H stage)
  const uint32_t* o_mk = kBk ? ix.blk_last : &ix.dense[Q.o_bm].w;
  const uint2* o_rk = kBk ? reinterpret_cast<const uint2*>(ix.blk_last)
                          : reinterpret_cast<const uint2*>(ix.dense_rk) + Q.o_bm;
  auto o_probe = [&](uint32_t e) __attribute__((always_inline)) { return o_mk[e]; };
  auto probe_bit = [&](uint32_t v, uint32_t sh) __attribute__((always_inline)) { return ((v >> sh) & 1u) != 0u; };
  // posting rank of a hit, without the rank word (added at compaction)
  auto probe_rank = [&](uint32_t v, uint32_t sh) __attribute__((always_inline)) {
    return static_cast<uint32_t>(__popc(v & ((1u << sh) - 1u)));
  };
  const uint8_t* o_tf8 = ix.tf8 + Q.o_tf8;
  // buckets (kBk): entries, shift and offset bytes of O1
  const uint32_t bsh = kBk ? static_cast<uint32_t>(Q.o_bm >> kProbeShiftBit) : 0u;
  const uint2* o_bk = kBk ? ix.bkt + (Q.o_bm & kProbeBaseMask) : nullptr;
  const uint8_t* o_off = kBk ? bucket_offsets(ix, Q.o_bm) : nullptr;
  const uint32_t o_tf8_mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(o_tf8)) & 3u;
  const uint32_t o_off_mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(o_off)) & 3u;
  const uint8_t* a_blob = ix.blob + Q.a_base;
  const uint32_t lo = in_vgpr(ix.doc_lo), span = in_vgpr(ix.dense_span);
  const uint32_t hi_rel = in_vgpr(ix.doc_hi - ix.doc_lo);   // docs a with a - lo < hi_rel are in the image
  const double idf_d = in_vgpr(Q.a_idf), idf_o = in_vgpr(Q.o_idf);
  uint32_t* qdoc = S.q;             // survivor queue (ring of 256)
  uint32_t* qc4 = qdoc + 256;
  uint32_t* qtd = qdoc + 512;
  uint32_t* qto = qdoc + 768;       // tf byte, or 0x80000000 | posting index when escaped
  uint32_t* qpd = qdoc + (kPh ? 1024 : 0);   // phrase: driver posting slot
  uint32_t* qpo = qdoc + (kPh ? 1280 : 0);   //         O1 posting rank
  const uint32_t o_slot0 = (kPh && phrase) ? ix.lists[Q.o_list].blk0 * 128u : 0u;
  uint32_t qhead = 0, qtail = 0;
  uint32_t bend = b1;
  // The loop issues only plain loads: coherent (agent-scope) loads, stores
  // and atomics take longer to complete and, counted in order with the loads,
  // would hold up every wait behind them.  So the score floor is read once,
  // here; the segment's own k-th best is published once, at the end; events
  // stay in LDS until 64 are pending (a chunk adds at most 64).  The final
  // re-filter in finish_item applies the floor as it stands at the end.
  uint64_t floor_bits = prev_pub ? floor_max(floor0) : 0ull;   // (floor0: the caller's floor_lanes)
  double pub_val = 0.0;
  // Floor refresh (every kFloorRefresh driver blocks): the item publishes
  // its floor as it stands (the k-th best of docs before the next item) and
  // reads the earlier items' (floor_lanes), so the items of one query, which
  // run at once, hand their thresholds on while they run instead of at their
  // ends.  The loads are issued just before a block's pack loads, which the
  // next iteration waits for anyway, and consumed one refresh later.
  uint64_t floor_next = 0;   // per lane: one earlier item's pub
  double sent = 0.0;
  // Pre-probe pruning.  A driver posting whose score bound -- its own term,
  // exact, plus QueryDesc's bound of the other terms at its doc length -- is
  // <= the threshold known so far, max(the floor of the query's earlier items,
  // the running k-th best), can be no event: the reference heap inserts only a
  // strictly larger score (query_processing.h:595-602), and both only grow.
  // Such a posting is dropped before its bitmap probe.  The bound is f32 and
  // the threshold carries a 0.2 % margin, far above the bound's rounding, so a
  // dropped posting's f64 score is strictly below the threshold.
  constexpr float kPruneMargin = 0.998f;
  const float b_id = Q.b_id;
  float b_iom = Q.b_iom, b_m = Q.b_m;
  float thr_s = wide ? -1.0f
                     : static_cast<float>(__longlong_as_double(static_cast<long long>(
                           (static_cast<uint64_t>(uni(static_cast<uint32_t>(floor_bits >> 32))) << 32) |
                           uni(static_cast<uint32_t>(floor_bits))))) * kPruneMargin;
  auto bound = [&](uint32_t t, uint32_t c) __attribute__((always_inline)) {
    const float nf = static_cast<float>(norm_tab[c]);
    const float f = static_cast<float>(t);
    return b_id * f * __builtin_amdgcn_rcpf(f + nf) + b_iom * __builtin_amdgcn_rcpf(b_m + nf);
  };

  auto flush = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    if (l < evb) store_event_coherent(&ev_out[ev_n - evb + l], S.evs[l]);
    __builtin_amdgcn_wave_barrier();
    evb = 0;
  };
  // score survivors qhead .. qhead+n (n <= 64, lane = doc order) and run the top-k
  auto score_chunk = [&](uint32_t n) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    const uint32_t e = (qhead + l) & 255u;
    bool alive = l < n;
    const uint32_t doc = qdoc[e];
    const uint32_t c4 = qc4[e];
    const uint32_t td = qtd[e];
    uint32_t to = qto[e];
    const uint32_t pd = kPh ? qpd[e] : 0u, po = kPh ? qpo[e] : 0u;
    __builtin_amdgcn_wave_barrier();
    qhead += n;
    if (__ballot(alive && (to & 0x80000000u))) {   // O1's tf bytes by rank (bit 31: a rank)
      const bool rk = alive && (to & 0x80000000u);
      uint32_t t = load_byte(o_tf8 + (rk ? (to & 0x7FFFFFFFu) : 0u));
      if (__ballot(rk && t == kTf8Escape)) {
        const ListDev O = ix.lists[Q.o_list];
        if (rk && t == kTf8Escape) t = dense_tf_slow(ix, O, to & 0x7FFFFFFFu);
      }
      if (rk) to = t;
    }
    const double norm = norm_tab[c4 & 255u];
    double sc = 0.0;   // BM25 accumulated in query-term order (scoring.h:133-144)
    if constexpr (kTwo) {   // the two terms in query order: the driver's slot first or second
      const double sd = bm25_term(idf_d, alive ? td : 0u, norm), so = bm25_term(idf_o, alive ? to : 0u, norm);
      if (d == 0) { sc += sd; sc += so; } else { sc += so; sc += sd; }
    }
    for (uint32_t s = 0; s < (kTwo ? 0u : nt); ++s) {
      if (s == d) {
        sc += bm25_term(idf_d, alive ? td : 0u, norm);
      } else if (s == o1) {
        sc += bm25_term(idf_o, alive ? to : 0u, norm);
      } else {
        const ListDev B = ix.lists[qlist[s]];
        uint32_t t = 0, x = 0;
        const DenseVal v = dense_load(ix, B, doc, alive);
        alive = alive && dense_resolve(ix, B, doc, v, &t, &x);
        if (__ballot(alive) == 0) break;
        sc += bm25_term(B.idf, alive ? t : 0u, norm);
      }
    }
    // HandleTheFoundDoc: a phrase query ranks only docs that hold the phrase.
    // Only a doc that can still enter the running top-k needs its position
    // check: the chunk's candidates at the k-th best before it (and the floor)
    // are a superset of the chunk's events whatever the phrase matches among
    // them, and a doc that is no candidate is no event either way.
    if (kPh && phrase && __ballot(alive)) {
      bool need = alive;
      if (!wide) {
        const uint64_t fb0 = floor_bits;
        const double flo0 = __longlong_as_double(static_cast<long long>(
            (static_cast<uint64_t>(uni(static_cast<uint32_t>(fb0 >> 32))) << 32) |
            uni(static_cast<uint32_t>(fb0))));
        const double kth0 = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
        need = alive && sc > flo0 && (pt_n < k || sc > kth0);
      }
      if (__ballot(need)) {   // (a lean phrase query has two terms: the driver and O1)
        const uint32_t so = o_slot0 + po;
        if (need)
          need = d == 0 ? phrase_match2(ix, qlist[0], qlist[1], pd, td, so, to)
                        : phrase_match2(ix, qlist[0], qlist[1], so, to, pd, td);
      }
      alive = need;
    }
    const uint64_t am = __ballot(alive);
    if (am == 0) return;
    n_surv += __popcll(am);
    if (wide) {   // all of them, in doc order (lane order), no floor
      if (evb + __popcll(am) > kLeanEvs) flush();
      if (alive) {
        Event ev;
        ev.score = sc;
        ev.doc = static_cast<int32_t>(doc);
        ev.pad = 0;
        S.evs[evb + __popcll(am & lt)] = ev;
      }
      ev_n += __popcll(am);
      evb += __popcll(am);
      return;
    }
    // running top-k: candidates beat the k-th best so far and the floor of the
    // query's earlier segments (scores are > 0, so bits order as values)
    const uint64_t fb = floor_bits;
    const double flo = __longlong_as_double(static_cast<long long>(
        (static_cast<uint64_t>(uni(static_cast<uint32_t>(fb >> 32))) << 32) |
        uni(static_cast<uint32_t>(fb))));
    const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
    uint64_t cm = __ballot(alive && sc > flo && (pt_n < k || sc > kth));
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      const double sv = readlane_f64(sc, fl);
      const uint32_t dv = __builtin_amdgcn_readlane(doc, fl);
      const uint32_t pos = __popcll(__ballot(l < pt_n && pt >= sv));
      if (pos < k) {
        if (evb == kLeanEvs) flush();
        if (l == 0) {
          Event ev;
          ev.score = sv;
          ev.doc = static_cast<int32_t>(dv);
          ev.pad = 0;
          S.evs[evb] = ev;
        }
        ++ev_n;
        ++evb;
        const double up = wave_shr1_f64(pt);
        if (l > pos) pt = up;
        else if (l == pos) pt = sv;
        pt_n = pt_n + 1 > k ? k : pt_n + 1;
      }
    }
    const double kn = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
    const double pv = kn > flo ? kn : flo;
    pub_val = pv > pub_val ? pv : pub_val;
    thr_s = static_cast<float>(pv) * kPruneMargin;
  };

  // Pipeline registers, in two alternating sets: iteration j reads set X
  // (written by iteration j-1) and writes set Y, then j+1 runs with the roles
  // swapped.  No register holding an in-flight load is ever copied (a copy
  // would wait for the load).
  struct Regs {
    // (the block's pack widths and blob offsets are read again from the
    // directory in LDS where they are used, so that no scalar registers hold
    // them across the iteration)
    uint32_t w0 = 0, w1 = 0, w2 = 0;               // doc-id pack words of the next block
    uint32_t wc = 0;                               //   its doc-length codes (2 bytes of a word)
    uint32_t wt0 = 0, wt1 = 0, wt2 = 0;            //   its driver tf pack words
    // D: a decoded block and its loads in flight
    uint32_t da0 = ~0u, da1 = ~0u, dcc = 0;        // docs, doc-length codes (c0 | c1 << 8)
    uint32_t dt0 = 0, dt1 = 0;                     // driver tfs
    std::conditional_t<kBk, uint2, uint32_t> de0{}, de1{};   // O1 bitmap mask words / bucket entries
    // (per-lane flags ride in the values -- a doc of ~0u is a posting past the
    // block, outside the image or pruned, a rank with bit 31 set is an O1 miss
    // -- so that they take no scalar lane-mask registers across the iteration)
    // H: the block decoded one iteration earlier, with its O1 hits
    uint32_t ha0 = 0, ha1 = 0, hc0 = 0, hc1 = 0, ht0 = 0, ht1 = 0;   // docs, length codes, driver tfs
    uint2 hf0 = make_uint2(0, 0), hf1 = make_uint2(0, 0);   // O1 rank records (rank, 4 tfs; in flight)
                                                            // kBk: the hit's tf word, the bucket count
    uint32_t hx0 = 0x80000000u, hx1 = 0x80000000u; // O1 posting ranks (bit 31: no hit; kBk: bit 30,
                                                   // the bucket's rank, its offsets to scan)

  };
  Regs R0, R1;
  // byte shift of a pair's first value inside its aligned dword (pair_words)
  auto pair_shift = [&](uint32_t rel, uint32_t bits) __attribute__((always_inline)) {
    const uint32_t bit = 2 * l * bits;
    const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a_blob)) + rel + 2 +
                       (bit >> 3);
    return ((a & 3u) << 3) + (bit & 7u);
  };

  auto issue_words = [&](uint32_t b, Regs& Y) __attribute__((always_inline)) {
    const uint32_t bi = b < b1 ? b - b0 : 0u;
    const uint32_t m = uni(S.dmeta[bi]);
    const uint4 e = S.dblk[bi];
    // (VInts tail: width 0 -> a harmless dummy read)
    uint32_t sh;
    pair_words(a_blob + uni(e.z) + 2, (m & 0xFF) ? (m & 0xFF) : 1u, l, Y.w0, Y.w1, Y.w2, sh);
    // its doc-length codes (postings 2l, 2l+1: one line per block, plen) and
    // driver tfs, so that D can bound each posting's score before the probe
    Y.wc = reinterpret_cast<const uint32_t*>(ix.plen)[(Q.a_blk0 + (b < b1 ? b : b0)) * 32u + (l >> 1)];
    pair_words(a_blob + uni(e.w) + 2, (m >> 8) ? (m >> 8) : 1u, l, Y.wt0, Y.wt1, Y.wt2, sh);
  };
  auto stage_C = [&](Regs& X, Regs& Y, uint32_t j) __attribute__((always_inline)) {
    // C(j-2-kDeep): compaction of that block (its H fields are in X)
    if (j >= b0 + 2 + kDeep) {
      // O1 posting ranks (hits): rank word + bits below; the tf byte is read by
      // rank when the chunk is scored (flag bit 31)
      // (the record's tf bytes cover the word's first four postings)
      uint32_t rk0, rk1, f0, f1, hx0 = X.hx0, hx1 = X.hx1;
      if constexpr (kBk) {
        // probes past a bucket's fourth posting: the window of its next offset
        // bytes loaded in H (bit 30; count in bits 23-29), a walk past it
        const bool s0 = (hx0 >> 30) == 1u, s1 = (hx1 >> 30) == 1u;
        if (__ballot(s0 || s1)) {
          const uint32_t m = (1u << bsh) - 1u;
          auto resolve = [&](uint32_t hx, uint2 win, uint32_t doc) __attribute__((always_inline)) {
            const uint32_t rk = hx & 0x7FFFFFu, cn = (hx >> 23) & 127u, o = (doc - lo) & m;
            uint32_t next = 0;
            const uint32_t pos = bucket_window(win.x, win.y, (o_off_mis + rk + kBucketInline) & 3u, cn, o, &next);
            if (pos < 8u) return (rk + kBucketInline + pos) | 0x40000000u;
            if (pos == kWindowScan) {   // past the window (the count is exact below 127)
              const uint32_t c = cn < 127u ? cn : (o_bk[(doc - lo) >> bsh].x & 511u);
              uint32_t i = 0;
              if (bucket_scan(o_off, rk, c, o, &i, next)) return i | 0x40000000u;
            }
            return 0x80000000u;
          };
          if (s0) hx0 = resolve(hx0, X.hf0, X.ha0);
          if (s1) hx1 = resolve(hx1, X.hf1, X.ha1);
        }
        // (a scanned hit, bit 30, reads its tf by rank when scored)
        rk0 = hx0 & 0x3FFFFFFFu;
        rk1 = hx1 & 0x3FFFFFFFu;
        f0 = (hx0 & 0x40000000u) ? kTf8Escape : (X.hf0.x >> (((o_tf8_mis + rk0) & 3u) << 3)) & 0xFFu;
        f1 = (hx1 & 0x40000000u) ? kTf8Escape : (X.hf1.x >> (((o_tf8_mis + rk1) & 3u) << 3)) & 0xFFu;
      } else {
        rk0 = X.hf0.x + hx0;
        rk1 = X.hf1.x + hx1;
        f0 = hx0 < 4u ? (X.hf0.y >> ((hx0 & 3u) << 3)) & 0xFFu : kTf8Escape;
        f1 = hx1 < 4u ? (X.hf1.y >> ((hx1 & 3u) << 3)) & 0xFFu : kTf8Escape;
      }
      const uint32_t to0 = f0 != kTf8Escape ? f0 : (0x80000000u | rk0);
      const uint32_t to1 = f1 != kTf8Escape ? f1 : (0x80000000u | rk1);
      const bool hh0 = !(hx0 >> 31), hh1 = !(hx1 >> 31);
      const uint64_t m0 = __ballot(hh0), m1 = __ballot(hh1);
      const uint32_t r0 = qtail + __popcll(m0 & lt) + __popcll(m1 & lt);
      const uint32_t r1 = r0 + (hh0 ? 1u : 0u);
      // branch-free: misses write the free slot before the queue head (at
      // most 63 + 128 entries are live, so it is never one of them)
      const uint32_t spare = (qhead - 1u) & 255u;
      const uint32_t e0 = hh0 ? (r0 & 255u) : spare, e1 = hh1 ? (r1 & 255u) : spare;
      qdoc[e0] = X.ha0; qc4[e0] = X.hc0; qtd[e0] = X.ht0; qto[e0] = to0;
      qdoc[e1] = X.ha1; qc4[e1] = X.hc1; qtd[e1] = X.ht1; qto[e1] = to1;
      if (kPh) {   // block j-2's postings 2l, 2l+1 and their O1 ranks
        const uint32_t pd0 = (Q.a_blk0 + j - 2 - kDeep) * 128u + 2 * l;
        qpd[e0] = pd0; qpo[e0] = rk0;
        qpd[e1] = pd0 + 1; qpo[e1] = rk1;
      }
      qtail += __popcll(m0) + __popcll(m1);
      // (at most two full chunks: fewer than 64 + 128 entries are queued;
      // one call site keeps a single inlined copy of the scoring code)
#pragma nounroll
      for (int c = 0; c < 2 && qtail - qhead >= 64; ++c) score_chunk(64);
    }
  };
  auto stage_H = [&](Regs& X, Regs& Yh, uint32_t j) __attribute__((always_inline)) {
    // H(j-1) (kDeep >= 1: H(j-2)): the block whose D fields are in X: O1 hits,
    // its driver tfs and length codes extracted, into Yh's H fields (kDeep 2:
    // X's, read by C two iterations later)
    Regs& Y = kDeep >= 2 ? X : Yh;
    if constexpr (kBk) {
      const uint32_t q0 = X.da0 - lo, q1 = X.da1 - lo;
      const uint32_t m = (1u << bsh) - 1u;
      const bool v0 = (X.da0 != ~0u) & (q0 < span), v1 = (X.da1 != ~0u) & (q1 < span);
      const uint32_t ps0 = bucket_pos(X.de0, q0 & m), ps1 = bucket_pos(X.de1, q1 & m);
      const bool h0 = v0 & (ps0 < kBucketInline), h1 = v1 & (ps1 < kBucketInline);
      const bool sc0 = v0 & (ps0 == kBucketScan), sc1 = v1 & (ps1 == kBucketScan);
      const uint32_t r0 = X.de0.x >> 9, r1 = X.de1.x >> 9;
      const uint32_t k0 = r0 + (h0 ? ps0 : 0u), k1 = r1 + (h1 ? ps1 : 0u);
      // a hit: its tf byte, as its aligned word; a probe past the fourth
      // posting: the next 8 offset bytes (two aligned words)
      const uint32_t* p0 = reinterpret_cast<const uint32_t*>(
          sc0 ? __builtin_align_down(o_off + r0 + kBucketInline, 4) : __builtin_align_down(o_tf8 + (h0 ? k0 : 0u), 4));
      const uint32_t* p1 = reinterpret_cast<const uint32_t*>(
          sc1 ? __builtin_align_down(o_off + r1 + kBucketInline, 4) : __builtin_align_down(o_tf8 + (h1 ? k1 : 0u), 4));
      Y.hf0.x = p0[0];
      Y.hf1.x = p1[0];
      Y.hf0.y = p0[1];
      Y.hf1.y = p1[1];
      const uint32_t n0 = min(X.de0.x & 511u, 127u), n1 = min(X.de1.x & 511u, 127u);
      Y.hx0 = h0 ? k0 : sc0 ? (0x40000000u | (n0 << 23) | r0) : 0x80000000u;
      Y.hx1 = h1 ? k1 : sc1 ? (0x40000000u | (n1 << 23) | r1) : 0x80000000u;
      Y.ha0 = X.da0; Y.ha1 = X.da1;
      Y.hc0 = X.dcc & 0xFFu;
      Y.hc1 = X.dcc >> 8;
      Y.ht0 = X.dt0;
      Y.ht1 = X.dt1;
    } else {
      const uint32_t q0 = X.da0 - lo, q1 = X.da1 - lo;
      const uint32_t s0 = q0 % kDenseDocs, s1 = q1 % kDenseDocs;
      // (bitwise, not short-circuit: the compiler would branch on each term)
      const bool h0 = (X.da0 != ~0u) & (q0 < span) & probe_bit(X.de0, s0);
      const bool h1 = (X.da1 != ~0u) & (q1 < span) & probe_bit(X.de1, s1);
      const uint32_t x0 = probe_rank(X.de0, s0);
      const uint32_t x1 = probe_rank(X.de1, s1);
      // the hits' rank records (O1's tf bytes past a word's first four postings
      // are read by rank when the chunk is scored)
      Y.hf0 = o_rk[h0 ? q0 / kDenseDocs : 0u];
      Y.hf1 = o_rk[h1 ? q1 / kDenseDocs : 0u];
      // (ranks are < 2^31)
      Y.hx0 = h0 ? (x0 & 0x7FFFFFFFu) : 0x80000000u;
      Y.hx1 = h1 ? (x1 & 0x7FFFFFFFu) : 0x80000000u;

      Y.ha0 = X.da0; Y.ha1 = X.da1;
      Y.hc0 = X.dcc & 0xFFu;
      Y.hc1 = X.dcc >> 8;
      Y.ht0 = X.dt0;
      Y.ht1 = X.dt1;
    }
  };
  auto stage_D = [&](Regs& X, Regs& Yd, uint32_t j) __attribute__((always_inline)) {
    // D(j): decode block j from X's words into Yd (kDeep >= 1: into X, read
    // by H two iterations later), issue its loads
    Regs& Y = kDeep >= 1 ? X : Yd;
    {
      const bool live = j < bend;
      // (the block issue_words loaded: j < b1 there, and the values of a block
      // past bend are discarded below)
      const uint32_t bi = j < b1 ? j - b0 : 0u;
      const uint4 be = S.dblk[bi];
      const uint32_t m = uni(S.dmeta[bi]);
      const uint32_t prev = uni(be.x);
      const uint32_t wbits = (m & 0xFF) ? (m & 0xFF) : 1u, wtb = (m >> 8) ? (m >> 8) : 1u;
      const uint32_t cnt = live ? ((j == Q.a_nblk - 1) ? Q.a_tail_cnt : 128u) : 0u;
      uint32_t x0, x1;
      pair_values(X.w0, X.w1, X.w2, pair_shift(uni(be.z), wbits), wbits, x0, x1);
      const uint32_t sm = x0 + x1;
      const uint32_t inc = wave_incl_scan(sm);
      uint32_t a0 = prev + (inc - sm) + x0;
      uint32_t a1 = a0 + x1;
      const bool tl = live && dtail && j == b1 - 1;
      if (tl) { a0 = tdoc0; a1 = tdoc1; }
      const bool ok0 = (2 * l < cnt) & (a0 - lo < hi_rel);
      const bool ok1 = (2 * l + 1 < cnt) & (a1 - lo < hi_rel);
      uint32_t t0, t1;
      pair_values(X.wt0, X.wt1, X.wt2, pair_shift(uni(be.w), wtb), wtb, t0, t1);
      if (tl) { t0 = ttf0; t1 = ttf1; }
      const uint32_t c0 = (X.wc >> ((l & 1u) << 4)) & 0xFFu;
      const uint32_t c1 = (X.wc >> (((l & 1u) << 4) + 8)) & 0xFFu;
      // pre-probe pruning (above): a dropped posting is never probed
      // (branch-free: the bound of a lane past the block is computed and dropped)
      const bool p0 = ok0 & (bound(t0, c0) > thr_s);
      const bool p1 = ok1 & (bound(t1, c1) > thr_s);
      const bool in0 = p0 & (a0 - lo < span);
      const bool in1 = p1 & (a1 - lo < span);
      if constexpr (kBk) {
        Y.de0 = o_bk[in0 ? (a0 - lo) >> bsh : 0u];
        Y.de1 = o_bk[in1 ? (a1 - lo) >> bsh : 0u];
      } else {
        Y.de0 = o_probe(in0 ? (a0 - lo) / kDenseDocs : 0u);
        Y.de1 = o_probe(in1 ? (a1 - lo) / kDenseDocs : 0u);
      }
      Y.dcc = c0 | (c1 << 8);
      Y.dt0 = t0; Y.dt1 = t1;
      Y.da0 = p0 ? a0 : ~0u; Y.da1 = p1 ? a1 : ~0u;
      if (live) ++n_dblk;
      // past the smallest last doc of the other lists nothing later can match
      const uint64_t past = __ballot((ok0 & (a0 > min_last)) | (ok1 & (a1 > min_last)));
      if (live & (past != 0)) bend = j + 1;
    }
  };
  auto body = [&](Regs& X, Regs& Y, uint32_t j) __attribute__((always_inline)) {
    if (((j - b0) % kFloorRefresh) == kFloorRefresh - 1 && !wide) {
      const uint64_t fb = floor_max(floor_next);
      if (fb > floor_bits) {
        floor_bits = fb;
        const float t = static_cast<float>(__longlong_as_double(static_cast<long long>(fb))) * kPruneMargin;
        thr_s = t > thr_s ? t : thr_s;
      }
      if (my_pub && pub_val > sent) {
        if (l == 0)
          __hip_atomic_fetch_max(my_pub, static_cast<uint64_t>(__double_as_longlong(pub_val)),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sent = pub_val;
      }
      floor_next = floor_lanes(prev_pub, n_prev);
    }
    // W(j+1): the doc-id words of block j+1
    issue_words(j + 1, Y);
    stage_C(X, Y, j);
    stage_H(X, Y, j);
    stage_D(X, Y, j);
  };
  issue_words(b0, R0);
  for (uint32_t j = b0; j < bend + 2 + kDeep; j += 2) {
    body(R0, R1, j);
    if (j + 1 >= bend + 2 + kDeep) break;
    body(R1, R0, j + 1);
  }
  if (qtail != qhead) score_chunk(qtail - qhead);
  // (the last evb events stay in S.evs: the item's end re-filters or replays
  // them from there, finish_lean_item)
  if (my_pub && pub_val > last_pub && l == 0)
    __hip_atomic_fetch_max(my_pub, static_cast<uint64_t>(__double_as_longlong(pub_val)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  last_pub = pub_val;
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------ single-term segment --
// A single-term item (SingleTermQueryProcessor::Process, query_processing.h:
// 620-642: every posting of the list is scored and offered to the heap).
// A posting's score is its own term's, so the threshold known before it -- the
// floor of the query's earlier items and the item's own running k-th best --
// rules whole blocks out: a block whose bound, idf x its largest TfNormLossy
// (IndexArgs::bmax, f32 rounded up at load), is at most that threshold holds no
// heap insertion and is skipped with no load at all.  The blocks that remain
// are read in one round each (doc-id and tf pack words, the doc-length line),
// the next remaining block's loads in flight while one is scored; inside a
// block each posting's own bound (its tf and length, f32) leaves only the
// candidates for the f64 score and the running top-k.  Safety of the f32
// bounds: as the lean pipeline's pre-probe pruning (kPruneMargin).
constexpr bool kSingleQueue = true;
template <bool kPh>
__device__ __forceinline__ void single_segment(const IndexArgs& ix, LeanLdsT<kPh>& S, const double* norm_tab,
                                               const QueryDesc& Q, uint32_t b0, uint32_t b1, bool dtail,
                                               uint32_t tdoc0, uint32_t tdoc1, uint32_t ttf0, uint32_t ttf1,
                                               uint64_t floor0, const uint64_t* prev_pub, uint32_t n_prev,
                                               uint64_t* my_pub, Event* ev_out, uint32_t& ev_n, uint32_t& evb, double& pt,
                                               uint32_t& pt_n, double& last_pub, uint32_t& n_surv,
                                               uint32_t& n_dblk) {
  const uint32_t l = threadIdx.x & 63;
  const uint32_t k = Q.k;
  const bool wide = k > static_cast<uint32_t>(kMaxK);   // every posting is an event
  constexpr float kPruneMargin = 0.998f;
  const uint8_t* a_blob = ix.blob + Q.a_base;
  const uint32_t lo = in_vgpr(ix.doc_lo), hi_rel = in_vgpr(ix.doc_hi - ix.doc_lo);
  const double idf = Q.a_idf;
  const float b_id = Q.b_id, idf_f = static_cast<float>(Q.a_idf);
  // The item runs window by window, 64 blocks each (its first window's
  // directory is in S already); per window the block bounds, one per lane
  // (blocks wb + l), and, for the first, those of the 64 blocks before the
  // item (a floor seed, below).
  uint32_t wb = b0, we = min(b0 + 64u, b1);
  float bmax = wb + l < we ? ix.bmax[Q.a_blk0 + wb + l] * idf_f : 0.0f;
  // the next window's directory and bounds, loaded one window ahead (a
  // window switch is then LDS stores, not a round trip to memory)
  uint4 nx_dblk = {0u, 0u, 0u, 0u};
  uint32_t nx_dmeta = 0u;
  float nx_bmax = 0.0f;
  auto prefetch_window = [&](uint32_t from) __attribute__((always_inline)) {
    const uint32_t to = min(from + 64u, b1);
    if (from + l < to) {
      nx_dblk = reinterpret_cast<const uint4*>(ix.blocks)[Q.a_blk0 + from + l];
      nx_dmeta = ix.blk_meta[Q.a_blk0 + from + l];
      nx_bmax = ix.bmax[Q.a_blk0 + from + l] * idf_f;
    }
  };
  prefetch_window(we);
  const bool pre_in = !wide && b0 > 64u - l;   // block b0 - 64 + l, list block >= 1
  const float pre = ix.bmax[Q.a_blk0 + (pre_in ? b0 - 64u + l : 0u)];
  uint64_t floor_bits = prev_pub ? floor_max(floor0) : 0ull;   // (floor0: the caller's floor_lanes)
  // Floor seed: each block holds a doc whose score is its block max, so the
  // k-th largest block max of k blocks before this item bounds from below the
  // k-th best score before it -- the reference heap's minimum at every doc of
  // the item (the same argument as the floors of earlier items).  Lower bound
  // of a block's f64 max score: idf * bmax * (1 - 2^-21) (bmax is rounded up
  // by at most one f32 ulp; the score's own roundings are f64).  Blocks from
  // the list's second on: their docs lie past the first block's last doc, so
  // inside a doc-range shard's range whenever this item's are.
  if (uni(static_cast<uint32_t>(__ballot(pre_in) != 0)) && k <= 64u) {
    uint32_t v = pre_in ? __float_as_uint(pre) : 0u;   // (positive floats order as their bits)
    uint32_t kth = 0;
    for (uint32_t i = 0; i < k; ++i) {
      kth = wave_max(v);
      const uint64_t at = __ballot(v == kth);
      if (l == static_cast<uint32_t>(__builtin_ctzll(at))) v = 0u;
    }
    const double seed = idf * static_cast<double>(__uint_as_float(kth)) * (1.0 - 0x1.0p-21);
    const uint64_t sb = static_cast<uint64_t>(__double_as_longlong(seed));
    floor_bits = sb > floor_bits ? sb : floor_bits;
  }
  auto as_f64 = [](uint64_t b) __attribute__((always_inline)) {
    return __longlong_as_double(static_cast<long long>(
        (static_cast<uint64_t>(uni(static_cast<uint32_t>(b >> 32))) << 32) | uni(static_cast<uint32_t>(b))));
  };
  double flo = as_f64(floor_bits);
  float thr_s = wide ? -1.0f : static_cast<float>(flo) * kPruneMargin;
  double pub_val = 0.0, sent = 0.0;
  uint64_t floor_next = 0;
  uint32_t n_done = 0;
  // the first block of the window at or after b whose bound passes the
  // threshold (we: none)
  auto next_block = [&](uint32_t b) __attribute__((always_inline)) {
    const uint64_t m = __ballot(wb + l >= b && bmax > thr_s);
    return m ? wb + static_cast<uint32_t>(__builtin_ctzll(m)) : we;
  };
  struct Regs {
    uint32_t w0 = 0, w1 = 0, w2 = 0, t0 = 0, t1 = 0, t2 = 0, wc = 0, b = 0;
  };
  auto issue = [&](uint32_t b, Regs& Y) __attribute__((always_inline)) {
    const uint32_t bi = b < we ? b - wb : 0u;
    const uint32_t m = uni(S.dmeta[bi]);
    const uint4 e = S.dblk[bi];
    uint32_t sh;
    pair_words(a_blob + uni(e.z) + 2, (m & 0xFF) ? (m & 0xFF) : 1u, l, Y.w0, Y.w1, Y.w2, sh);
    pair_words(a_blob + uni(e.w) + 2, (m >> 8) ? (m >> 8) : 1u, l, Y.t0, Y.t1, Y.t2, sh);
    Y.wc = reinterpret_cast<const uint32_t*>(ix.plen)[(Q.a_blk0 + (b < we ? b : wb)) * 32u + (l >> 1)];
    Y.b = b;
  };
  auto pair_shift = [&](uint32_t rel, uint32_t bits) __attribute__((always_inline)) {
    const uint32_t bit = 2 * l * bits;
    const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a_blob)) + rel + 2 + (bit >> 3);
    return ((a & 3u) << 3) + (bit & 7u);
  };
  auto flush = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    if (l < evb) store_event_coherent(&ev_out[ev_n - evb + l], S.evs[l]);
    __builtin_amdgcn_wave_barrier();
    evb = 0;
  };
  // kSingleQueue: survivors wait in a ring of 256 in LDS (doc, tf, length
  // code) and are scored 64 at a time, one per lane: a block keeps ~3 of
  // its 128 postings, so scoring each block's 128 lanes in f64 spent most of
  // its instructions on postings already dropped
  uint32_t* qdoc = S.q;
  uint32_t* qtf = S.q + 256;
  uint32_t* qc4 = S.q + 512;
  uint32_t qhead = 0, qtail = 0;
  auto score_chunk = [&](uint32_t n) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    const uint32_t e = (qhead + l) & 255u;
    const bool alive = l < n;
    const uint32_t doc = qdoc[e], tf = qtf[e], c4 = qc4[e];
    __builtin_amdgcn_wave_barrier();
    qhead += n;
    double sc = 0.0;   // BM25 of the one term (scoring.h:133-144: summed from 0.0)
    sc += bm25_term(idf, alive ? tf : 0u, norm_tab[alive ? (c4 & 255u) : 0u]);
    const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
    uint64_t cm = __ballot(alive && (wide || (sc > flo && (pt_n < k || sc > kth))));
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      const double sv = readlane_f64(sc, fl);
      const uint32_t dv = __builtin_amdgcn_readlane(doc, fl);
      const uint32_t pos = wide ? 0u : __popcll(__ballot(l < pt_n && pt >= sv));
      if (wide || pos < k) {
        if (evb == kLeanEvs) flush();
        if (l == 0) {
          Event ev;
          ev.score = sv;
          ev.doc = static_cast<int32_t>(dv);
          ev.pad = 0;
          S.evs[evb] = ev;
        }
        ++ev_n;
        ++evb;
        if (!wide) {
          const double up = wave_shr1_f64(pt);
          if (l > pos) pt = up;
          else if (l == pos) pt = sv;
          pt_n = pt_n + 1 > k ? k : pt_n + 1;
        }
      }
    }
    if (!wide) {
      const double kn = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
      const double pv = kn > flo ? kn : flo;
      pub_val = pv > pub_val ? pv : pub_val;
      thr_s = static_cast<float>(pv) * kPruneMargin;
    }
  };
  // score block X.b (its loads were issued one block earlier)
  auto score = [&](const Regs& X) __attribute__((always_inline)) {
    const uint32_t b = X.b, bi = b - wb;
    const uint4 be = S.dblk[bi];
    const uint32_t m = uni(S.dmeta[bi]);
    const uint32_t wbits = (m & 0xFF) ? (m & 0xFF) : 1u, wtb = (m >> 8) ? (m >> 8) : 1u;
    const uint32_t cnt = (b == Q.a_nblk - 1) ? Q.a_tail_cnt : 128u;
    uint32_t x0, x1, t0, t1;
    pair_values(X.w0, X.w1, X.w2, pair_shift(uni(be.z), wbits), wbits, x0, x1);
    pair_values(X.t0, X.t1, X.t2, pair_shift(uni(be.w), wtb), wtb, t0, t1);
    const uint32_t sm = x0 + x1;
    const uint32_t inc = wave_incl_scan(sm);
    uint32_t a0 = uni(be.x) + (inc - sm) + x0;
    uint32_t a1 = a0 + x1;
    if (dtail && b == b1 - 1) { a0 = tdoc0; a1 = tdoc1; t0 = ttf0; t1 = ttf1; }
    const uint32_t c0 = (X.wc >> ((l & 1u) << 4)) & 0xFFu;
    const uint32_t c1 = (X.wc >> (((l & 1u) << 4) + 8)) & 0xFFu;
    const float nf0 = static_cast<float>(norm_tab[c0]), nf1 = static_cast<float>(norm_tab[c1]);
    const float f0 = static_cast<float>(t0), f1 = static_cast<float>(t1);
    const bool p0 = (2 * l < cnt) & (a0 - lo < hi_rel) & (b_id * f0 * __builtin_amdgcn_rcpf(f0 + nf0) > thr_s);
    const bool p1 = (2 * l + 1 < cnt) & (a1 - lo < hi_rel) & (b_id * f1 * __builtin_amdgcn_rcpf(f1 + nf1) > thr_s);
    ++n_dblk;
    const uint64_t m0 = __ballot(p0), m1 = __ballot(p1);
    if ((m0 | m1) == 0) return;
    n_surv += __popcll(m0) + __popcll(m1);
    if constexpr (kSingleQueue) {
      // append the block's survivors, in doc order, to the LDS queue (misses
      // write the free slot before its head: at most 63 + 128 are live);
      // every full 64 are scored one per lane
      const uint64_t lt = lanemask_lt();
      const uint32_t r0 = qtail + __popcll(m0 & lt) + __popcll(m1 & lt);
      const uint32_t r1 = r0 + (p0 ? 1u : 0u);
      const uint32_t spare = (qhead - 1u) & 255u;
      const uint32_t e0 = p0 ? (r0 & 255u) : spare, e1 = p1 ? (r1 & 255u) : spare;
      qdoc[e0] = a0; qtf[e0] = t0; qc4[e0] = c0;
      qdoc[e1] = a1; qtf[e1] = t1; qc4[e1] = c1;
      qtail += __popcll(m0) + __popcll(m1);
#pragma nounroll
      for (int c = 0; c < 2 && qtail - qhead >= 64; ++c) score_chunk(64);
      return;
    }
    // BM25 of the one term (scoring.h:133-144: summed from 0.0)
    double s0 = 0.0, s1 = 0.0;
    s0 += bm25_term(idf, p0 ? t0 : 0u, norm_tab[p0 ? c0 : 0u]);
    s1 += bm25_term(idf, p1 ? t1 : 0u, norm_tab[p1 ? c1 : 0u]);
    const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
    // candidates in doc order: lane by lane, posting 2l before 2l + 1
    uint64_t cm0 = __ballot(p0 && (wide || (s0 > flo && (pt_n < k || s0 > kth))));
    uint64_t cm1 = __ballot(p1 && (wide || (s1 > flo && (pt_n < k || s1 > kth))));
    while (cm0 | cm1) {
      const int fl = __builtin_ctzll(cm0 | cm1);
      const bool second = !((cm0 >> fl) & 1);
      if (second) cm1 &= cm1 - 1; else cm0 &= ~(1ull << fl);
      const double sv = readlane_f64(second ? s1 : s0, fl);
      const uint32_t dv = __builtin_amdgcn_readlane(second ? a1 : a0, fl);
      const uint32_t pos = wide ? 0u : __popcll(__ballot(l < pt_n && pt >= sv));
      if (wide || pos < k) {
        if (evb == kLeanEvs) flush();
        if (l == 0) {
          Event e;
          e.score = sv;
          e.doc = static_cast<int32_t>(dv);
          e.pad = 0;
          S.evs[evb] = e;
        }
        ++ev_n;
        ++evb;
        if (!wide) {
          const double up = wave_shr1_f64(pt);
          if (l > pos) pt = up;
          else if (l == pos) pt = sv;
          pt_n = pt_n + 1 > k ? k : pt_n + 1;
        }
      }
    }
    if (!wide) {
      const double kn = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
      const double pv = kn > flo ? kn : flo;
      pub_val = pv > pub_val ? pv : pub_val;
      thr_s = static_cast<float>(pv) * kPruneMargin;
    }
  };
  auto refresh = [&]() __attribute__((always_inline)) {
    if (wide || ++n_done % kFloorRefresh) return;
    // (the queue's partial chunk too: block skipping needs the threshold its
    // survivors raise, at most kFloorRefresh blocks late)
    if (kSingleQueue && qtail != qhead) score_chunk(qtail - qhead);
    const uint64_t fb = floor_max(floor_next);
    if (fb > floor_bits) {
      floor_bits = fb;
      flo = as_f64(fb);
      const float t = static_cast<float>(flo) * kPruneMargin;
      thr_s = t > thr_s ? t : thr_s;
    }
    if (my_pub && pub_val > sent) {
      if (l == 0)
        __hip_atomic_fetch_max(my_pub, static_cast<uint64_t>(__double_as_longlong(pub_val)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      sent = pub_val;
    }
    floor_next = floor_lanes(prev_pub, n_prev);
  };
  Regs R0, R1;
  for (;;) {
    uint32_t b = next_block(wb);
    issue(b, R0);
    while (b < we) {
      b = next_block(b + 1);
      issue(b, R1);
      score(R0);
      refresh();
      if (R1.b >= we) break;
      b = next_block(b + 1);
      issue(b, R0);
      score(R1);
      refresh();
      if (R0.b >= we) break;
    }
    if (we >= b1) break;
    // the next window: its directory and block bounds from the registers
    // loaded a window earlier, and the loads of the one after it
    // (its blocks' survivors go on queueing behind this window's)
    wb = we;
    we = min(wb + 64u, b1);
    __builtin_amdgcn_wave_barrier();
    if (wb + l < we) {
      S.dblk[l] = nx_dblk;
      S.dmeta[l] = nx_dmeta;
    }
    bmax = wb + l < we ? nx_bmax : 0.0f;
    __builtin_amdgcn_wave_barrier();
    prefetch_window(we);
  }
  if (kSingleQueue && qtail != qhead) score_chunk(qtail - qhead);
  // (the last evb events stay in S.evs for finish_lean_item)
  if (my_pub && pub_val > last_pub && l == 0)
    __hip_atomic_fetch_max(my_pub, static_cast<uint64_t>(__double_as_longlong(pub_val)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  last_pub = pub_val;
  __builtin_amdgcn_wave_barrier();
}

// kPhrase: the batch holds phrase queries (their position check is compiled
// only into this instance, so the conjunctive kernel keeps its registers).
template <bool kPhrase>
__global__ __launch_bounds__(64, kSegWaves) void segment_kernel(IndexArgs ix, const QueryIn* __restrict__ qs,
                                                     const QueryPlan* __restrict__ plan, int nq,
                                                     uint32_t* __restrict__ counters,
                                                     Event* __restrict__ events,
                                                     uint32_t* __restrict__ ev_cnt,
                                                     uint32_t* __restrict__ stats, FusedReplay fr,
                                                     const uint32_t* __restrict__ item_q,
                                                     uint64_t* __restrict__ pub,
                                                     uint32_t* __restrict__ ph_all) {
  __shared__ WaveLds S;
  const uint32_t l = threadIdx.x & 63;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) S.norm[l + 64 * i] = ix.cache[l + 64 * i];
  const uint64_t lt = lanemask_lt();
  // general items are [lean end, total): the lean kernel takes the others
  const uint32_t total = uni(__hip_atomic_load(&counters[kCtrItems], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t n_lean = uni(__hip_atomic_load(&counters[kCtrLean], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
  uint32_t n_surv = 0, n_dblk = 0, n_oblk = 0;
  // first item: this workgroup's own index; then the shard heads
  uint32_t shard = blockIdx.x % kQueueShards;
  uint32_t tried = 0;
  uint32_t item = n_lean + blockIdx.x;
  for (;;) {
    if (item >= total) item = next_item(&counters[kCtrGHead0], n_lean, total, shard, tried);
    if (item >= total) break;
    const uint32_t qi = uni(item_q[item]);   // written by plan_fill_kernel
    const QueryPlan P = plan[qi];
    const int32_t* qlist = qlist_of(qs, static_cast<int>(qi));
    const uint32_t r = item - P.item_base;
    const uint32_t d = uni(P.driver & kPlanSlotMask);
    const uint32_t nt = uni(static_cast<uint32_t>(qs[qi].n_terms));
    const uint32_t k = uni(static_cast<uint32_t>(qs[qi].k));
    const bool wide = k > static_cast<uint32_t>(kMaxK);   // every survivor is an event
    const ListDev A = ix.lists[qlist[d]];
    const uint32_t seg = uni(P.seg_blocks);
    // phrase query: every term's posting of each candidate is recorded in this
    // workgroup's slice of ph_all, then the positions are checked
    const bool phrase = kPhrase && nt > 1 && (uni(static_cast<uint32_t>(qs[qi].flags)) & kQueryPhrase);
    // (the conjunctive instance runs a batch whose phrase queries are all lean,
    // by the host's restatement of the class rule: a general phrase item here
    // would lose its position check, so it fails the batch loudly instead)
    if (!kPhrase && nt > 1 && (uni(static_cast<uint32_t>(qs[qi].flags)) & kQueryPhrase)) {
      if (l == 0) atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrClass));
      finish_item<false>(qs, plan, qi, P.n_items, item, nullptr, r, events + P.ev_base, 0, events, ev_cnt, fr);
      item = 0xFFFFFFFFu;
      continue;
    }
    uint32_t* ph = kPhrase ? ph_all + static_cast<uint64_t>(blockIdx.x) * kPhraseScratch : nullptr;
    const uint32_t b0 = r * seg;
    const uint32_t b1 = min(b0 + seg, A.nblk);
    Event* ev_out = events + P.ev_base + static_cast<uint64_t>(r) * seg * 128;
    uint32_t ev_n = 0;
    // Score floor from the earlier segments of the query: pub[item] holds the
    // largest k-th best score known from survivors at or before this segment
    // (max of this segment's running k-th best and its predecessor's floor).
    // k survivors before this segment score >= the floor, so nothing at or
    // below it can be a heap insertion of the reference run.
    uint64_t* my_pub = pub ? pub + item : nullptr;
    const uint64_t* prev_pub = (pub && r > 0) ? pub + item - 1 : nullptr;
    double last_pub = 0.0;

    // the driver's directory entries of this segment, one per lane (seg <= kSegCost < 64)
    __syncthreads();
    if (b0 + l < b1) {
      S.dblk[l] = reinterpret_cast<const uint4*>(ix.blocks)[A.blk0 + b0 + l];
      S.dmeta[l] = ix.blk_meta[A.blk0 + b0 + l];
    }
    __syncthreads();
    const uint32_t first_doc = b0 == 0 ? 0u : uni(S.dblk[0].x) + 1u;
    bool done = false;   // some other list has no doc >= the next driver doc
    uint32_t fo = kNoSlot;   // first other slot in query order
    // (cursors into the block directories of the first kMaxTerms slots live in
    // LDS; a slot past them, in the rare longer query, finds its block from
    // the segment's first doc at every driver block instead)
    for (uint32_t s = 0; s < nt; ++s) {
      if (s != d) {
        const ListDev B = ix.lists[qlist[s]];
        if (fo == kNoSlot) fo = s;
        if (use_dense(ix, B.bm != kNoDense, B.nblk, A.nblk)) {
          // probed through its bitmap: no cursor, only its end matters
          if (first_doc > ix.blk_last[B.blk0 + B.nblk - 1]) done = true;
        } else {
          const uint32_t c0 = uni(find_block(ix.blk_last + B.blk0, 0, B.nblk, first_doc));
          if (l == 0 && s < kMaxTerms) S.cur[s] = c0;
          if (c0 >= B.nblk) done = true;
        }
      }
    }
    // the first other list's bitmap entries are fetched one block ahead
    ListDev F = A;
    bool fo_dense = false;
    if (fo != kNoSlot) {
      F = ix.lists[qlist[fo]];
      fo_dense = use_dense(ix, F.bm != kNoDense, F.nblk, A.nblk);
    }
    const uint64_t f_bm = fo_dense ? F.bm : 0ull;
    const uint8_t* f_tf8 = ix.tf8 + (fo_dense ? F.tf8 : 0ull);
    const uint32_t f_last = fo_dense ? uni(ix.blk_last[F.blk0 + F.nblk - 1]) : 0u;

    // The driver's VInts tail block (docs and tfs) is decoded into LDS once,
    // so that the per-block loads below have the same count on every path
    // (the compiler's vmcnt accounting then lets the next block's loads stay
    // in flight while this block is scored).
    bool dtail = false;
    if (b0 < b1) {
      const uint32_t mt = uni(S.dmeta[b1 - 1 - b0]);
      dtail = (mt & 0xFF) == 0;
      if (dtail) {
        const int bi = static_cast<int>(b1 - 1 - b0);
        const uint32_t cnt = A.tail_cnt;
        decode_block(ix.blob + A.base + uni(S.dblk[bi].z), 0, cnt, true,
                     uni(S.dblk[bi].x), S.dtd);
        __syncthreads();
        decode_block(ix.blob + A.base + uni(S.dblk[bi].w), mt >> 8, cnt,
                     false, 0, S.dtt);
        __syncthreads();
      }
    }

    double pt = 0.0;     // running top-k scores, lane t holds rank t (descending)
    uint32_t pt_n = 0;   // valid entries (uniform)
    uint32_t evb = 0;    // events buffered in S.evs (flushed 64 at a time)

    // Stage of one driver block: doc ids, in-range flags and the loads scoring
    // needs (doc lengths, the driver's tf, the first other list's bitmap
    // entries), issued one block before the block is scored.  Every load is
    // unconditional (masked lanes read index 0) so the count is static.
    // (Loaded values are kept raw; selects on them happen where they are
    // consumed, so the fetch itself never waits for its own loads.)
    struct Stage {
      uint32_t a0, a1, c0, c1, ta0, ta1;
      bool al0, al1, ok0, ok1;
      DenseVal p0, p1;
    };
    // raw pack words of the driver block to decode next (issued a block ahead)
    uint32_t nx0 = 0, nx1 = 0;
    auto issue_words = [&](uint32_t b) __attribute__((always_inline)) {
      const int bi = static_cast<int>(b - b0);
      const uint32_t m = uni(S.dmeta[bi]);
      const uint32_t rel = uni(S.dblk[bi].z);
      const uint32_t bits = (m & 0xFF) ? (m & 0xFF) : 1u;   // VInts tail: harmless dummy read
      nx0 = pack_value(ix.blob + A.base + rel + 2, bits, 2 * l);
      nx1 = pack_value(ix.blob + A.base + rel + 2, bits, 2 * l + 1);
    };
    auto fetch = [&](uint32_t b, Stage& g) __attribute__((always_inline)) {
      const int bi = static_cast<int>(b - b0);
      const uint32_t prev = uni(S.dblk[bi].x);
      const uint32_t tf_rel = uni(S.dblk[bi].w);
      const uint32_t m = uni(S.dmeta[bi]);
      const uint32_t cnt = (b == A.nblk - 1) ? A.tail_cnt : 128u;
      const bool is_tail = dtail && b == b1 - 1;
      {
        const uint32_t x0 = nx0, x1 = nx1;
        const uint32_t sm = x0 + x1;
        const uint32_t inc = wave_incl_scan(sm);
        const uint32_t p0 = prev + (inc - sm) + x0;
        g.a0 = is_tail ? S.dtd[2 * l] : p0;
        g.a1 = is_tail ? S.dtd[2 * l + 1] : p0 + x1;
      }
      issue_words(b + 1 < b1 ? b + 1 : b);
      g.al0 = 2 * l < cnt && g.a0 >= ix.doc_lo && g.a0 < ix.doc_hi;
      g.al1 = 2 * l + 1 < cnt && g.a1 >= ix.doc_lo && g.a1 < ix.doc_hi;
      g.ok0 = g.al0 && g.a0 < ix.n_c4;
      g.ok1 = g.al1 && g.a1 < ix.n_c4;
      // doc-length codes of postings 2l, 2l+1 (plen word, bytes picked at use)
      g.c0 = reinterpret_cast<const uint32_t*>(ix.plen)[(A.blk0 + b) * 32u + (l >> 1)];
      g.c1 = g.c0;
      const uint32_t tbits = (m >> 8) ? (m >> 8) : 1u;
      const uint8_t* tp = ix.blob + A.base + tf_rel;
      g.ta0 = pack_tf(tp, tbits, 2 * l);
      g.ta1 = pack_tf(tp, tbits, 2 * l + 1);
      const uint32_t r0 = g.a0 - ix.doc_lo, r1 = g.a1 - ix.doc_lo;
      const bool d0 = fo_dense && g.al0 && r0 < ix.dense_span;
      const bool d1 = fo_dense && g.al1 && r1 < ix.dense_span;
      g.p0 = probe_at(ix, f_bm, r0, d0);
      g.p1 = probe_at(ix, f_bm, r1, d1);
    };
    auto flush_events = [&](uint32_t n) __attribute__((always_inline)) {
      __builtin_amdgcn_wave_barrier();
      if (l < n) store_event_coherent(&ev_out[ev_n - evb + l], S.evs[l]);
      __builtin_amdgcn_wave_barrier();
    };

    // Score driver block b (stage cs) while the loads of block b+1 (stage ns) fly.
    auto step = [&](Stage& cs, Stage& ns, uint32_t b) __attribute__((always_inline)) {
      // first other list through its bitmap: hits, and their tf bytes, issued
      // before the next block's loads so that waiting for them does not wait
      // for those
      bool fh0 = false, fh1 = false;
      uint32_t fi0 = 0, fi1 = 0;
      if (fo_dense) {
        fh0 = cs.al0 && probe_hit(ix, f_bm, cs.a0, cs.p0, &fi0);
        fh1 = cs.al1 && probe_hit(ix, f_bm, cs.a1, cs.p1, &fi1);
      }
      const uint32_t ft0 = f_tf8[fh0 ? fi0 : 0u], ft1 = f_tf8[fh1 ? fi1 : 0u];
      const uint64_t floor_bits =
          prev_pub ? __hip_atomic_load(prev_pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      fetch(b + 1 < b1 ? b + 1 : b, ns);
      ++n_dblk;
      const uint32_t a0 = cs.a0, a1 = cs.a1;
      bool al0 = cs.al0, al1 = cs.al1;
      double s0 = 0.0, s1 = 0.0;   // BM25 accumulated in query-term order (scoring.h:133-144)
      const double nrm0 = S.norm[cs.ok0 ? (cs.c0 >> ((l & 1u) << 4)) & 0xFFu : 0u];
      const double nrm1 = S.norm[cs.ok1 ? (cs.c1 >> (((l & 1u) << 4) + 8)) & 0xFFu : 0u];
      const bool is_tail = dtail && b == b1 - 1;
      const uint32_t ta0 = is_tail ? S.dtt[2 * l] : cs.ta0;
      const uint32_t ta1 = is_tail ? S.dtt[2 * l + 1] : cs.ta1;

      // phrase: image posting slot and tf of term s for values 2l, 2l+1
      auto rec = [&](uint32_t s, uint32_t sl0, uint32_t sl1, uint32_t tf0, uint32_t tf1)
          __attribute__((always_inline)) {
        if (phrase) {
          if (al0) { ph[s * 256 + 2 * l] = sl0; ph[s * 256 + 128 + 2 * l] = tf0; }
          if (al1) { ph[s * 256 + 2 * l + 1] = sl1; ph[s * 256 + 128 + 2 * l + 1] = tf1; }
        }
      };
      for (uint32_t s = 0; s < nt; ++s) {
        if (__ballot(al0 || al1) == 0) break;
        const ListDev L = ix.lists[qlist[s]];
        if (s == d) {  // the driver's own tf
          if (al0) s0 += bm25_term(L.idf, ta0, nrm0);
          if (al1) s1 += bm25_term(L.idf, ta1, nrm1);
          rec(s, (A.blk0 + b) * 128u + 2 * l, (A.blk0 + b) * 128u + 2 * l + 1, ta0, ta1);
          continue;
        }
        const ListDev& B = L;
        if (s == fo && fo_dense) {
          // past B's last doc nothing later in the segment can match
          if (__ballot((al0 && a0 > f_last) || (al1 && a1 > f_last))) done = true;
          uint32_t t0 = ft0, t1 = ft1;
          if (fh0 && t0 == kTf8Escape) t0 = dense_tf_slow(ix, B, fi0);
          if (fh1 && t1 == kTf8Escape) t1 = dense_tf_slow(ix, B, fi1);
          al0 = al0 && fh0;
          al1 = al1 && fh1;
          if (al0) s0 += bm25_term(B.idf, t0, nrm0);
          if (al1) s1 += bm25_term(B.idf, t1, nrm1);
          rec(s, B.blk0 * 128u + fi0, B.blk0 * 128u + fi1, t0, t1);
          continue;
        }
        if (use_dense(ix, B.bm != kNoDense, B.nblk, A.nblk)) {
          uint32_t t0 = 0, t1 = 0, x0 = 0, x1 = 0;
          const DenseVal v0 = dense_load(ix, B, a0, al0);
          const DenseVal v1 = dense_load(ix, B, a1, al1);
          const bool h0 = al0 && dense_resolve(ix, B, a0, v0, &t0, &x0);
          const bool h1 = al1 && dense_resolve(ix, B, a1, v1, &t1, &x1);
          const uint32_t blast = ix.blk_last[B.blk0 + B.nblk - 1];
          if (__ballot((al0 && a0 > blast) || (al1 && a1 > blast))) done = true;
          al0 = h0;
          al1 = h1;
          if (al0) s0 += bm25_term(B.idf, t0, nrm0);
          if (al1) s1 += bm25_term(B.idf, t1, nrm1);
          rec(s, B.blk0 * 128u + x0, B.blk0 * 128u + x1, t0, t1);
          continue;
        }
        const uint32_t* last = ix.blk_last + B.blk0;
        const uint32_t c = s < kMaxTerms ? uni(S.cur[s])
                                         : uni(find_block(last, 0, B.nblk, uni(S.dblk[b - b0].x) + (b > 0 ? 1u : 0u)));
        // directory window cur..cur+63 into LDS (one coalesced round)
        const uint32_t wn = min(kWin, B.nblk - c);
        uint32_t wl = 0;
        __syncthreads();
        if (l < wn) {
          wl = last[c + l];
          S.wlast[l] = wl;
          S.wblk[l] = ix.blocks[B.blk0 + c + l];
          S.wmeta[l] = ix.blk_meta[B.blk0 + c + l];
        }
        const uint32_t wmax = uni(__builtin_amdgcn_readlane(wl, static_cast<int>(wn) - 1));
        __syncthreads();
        uint32_t j0 = kNoBlock, j1 = kNoBlock;
        if (al0) j0 = a0 <= wmax ? c + lds_lower_bound(S.wlast, wn, a0) : find_block(last, c + wn, B.nblk, a0);
        if (al1) j1 = a1 <= wmax ? c + lds_lower_bound(S.wlast, wn, a1) : find_block(last, c + wn, B.nblk, a1);
        // a doc beyond the list's last block cannot match, nor can any later doc
        if (__ballot((al0 && j0 >= B.nblk) || (al1 && j1 >= B.nblk))) done = true;
        al0 = al0 && j0 < B.nblk;
        al1 = al1 && j1 < B.nblk;
        // distinct blocks probed, in order (probe blocks are non-decreasing)
        const uint32_t k0 = al0 ? j0 + 1 : 0u, k1 = al1 ? j1 + 1 : 0u;
        const uint32_t pre = wave_excl_max(k0 > k1 ? k0 : k1);
        const bool st0 = k0 && k0 > pre;
        const bool st1 = k1 && k1 > (pre > k0 ? pre : k0);
        const uint64_t m0 = __ballot(st0), m1 = __ballot(st1);
        const uint32_t nd = __popcll(m0) + __popcll(m1);
        const uint32_t before = __popcll(m0 & lt) + __popcll(m1 & lt);
        const uint32_t r0 = before + (st0 ? 1u : 0u) - 1u;              // rank of value (l,0)'s block
        const uint32_t r1 = before + (st0 ? 1u : 0u) + (st1 ? 1u : 0u) - 1u;
        if (st0) S.dl[before] = j0;
        if (st1) S.dl[before + (st0 ? 1u : 0u)] = j1;
        __syncthreads();
        // the list's VInts tail (if probed) is the last distinct block
        const uint32_t jlast = nd ? uni(S.dl[nd - 1]) : 0u;
        const bool tail_vints = nd && B.tail_cnt < 128u && jlast == B.nblk - 1;
        const uint32_t npk = tail_vints ? nd - 1 : nd;
        uint32_t t0 = 0, t1 = 0;
        bool h0 = false, h1 = false;
        uint32_t p0 = 0, p1 = 0;
        for (uint32_t base = 0; base < npk;) {
          const uint32_t rem = npk - base;
#define WSR_PROBE(GG)                                                             \
  {                                                                               \
    grouped_decode<GG>(ix, B, S, c, wn, base, npk);                               \
    n_oblk += min(static_cast<uint32_t>(GG), rem);                                \
    __syncthreads();                                                              \
    if (al0 && r0 >= base && r0 < base + GG) {                                    \
      p0 = grouped_lower_bound<GG>(S, r0 - base, a0);                             \
      h0 = p0 < 128 && grouped_at<GG>(S, r0 - base, p0) == a0;                    \
    }                                                                             \
    if (al1 && r1 >= base && r1 < base + GG) {                                    \
      p1 = grouped_lower_bound<GG>(S, r1 - base, a1);                             \
      h1 = p1 < 128 && grouped_at<GG>(S, r1 - base, p1) == a1;                    \
    }                                                                             \
    __syncthreads();                                                              \
    base += GG;                                                                   \
  }
          if (rem >= 8) WSR_PROBE(8)
          else if (rem >= 4) WSR_PROBE(4)
          else if (rem >= 2) WSR_PROBE(2)
          else WSR_PROBE(1)
#undef WSR_PROBE
        }
        if (tail_vints) {
          const uint32_t jt = B.nblk - 1;
          BlockDev bb;
          uint32_t bm;
          dir_entry(ix, B, S, c, wn, jt, &bb, &bm);
          decode_block(ix.blob + B.base + bb.doc_rel, 0, B.tail_cnt, true, bb.prev, S.mb[0]);
          ++n_oblk;
          if (al0 && r0 == nd - 1) {
            p0 = lds_lower_bound(S.mb[0], B.tail_cnt, a0);
            h0 = p0 < B.tail_cnt && S.mb[0][p0] == a0;
          }
          if (al1 && r1 == nd - 1) {
            p1 = lds_lower_bound(S.mb[0], B.tail_cnt, a1);
            h1 = p1 < B.tail_cnt && S.mb[0][p1] == a1;
          }
          const bool tv0 = h0 && r0 == nd - 1, tv1 = h1 && r1 == nd - 1;
          if (__ballot(tv0 || tv1)) {
            __syncthreads();
            decode_block(ix.blob + B.base + bb.tf_rel, bm >> 8, B.tail_cnt, false, 0, S.tf);
            if (tv0) t0 = S.tf[p0];
            if (tv1) t1 = S.tf[p1];
          }
          __syncthreads();
        }
        // tf of matched postings held in packs: direct per-lane read
        if (h0 && !(tail_vints && r0 == nd - 1)) {
          BlockDev bb;
          uint32_t bm;
          dir_entry(ix, B, S, c, wn, j0, &bb, &bm);
          t0 = pack_tf(ix.blob + B.base + bb.tf_rel, bm >> 8, p0);
        }
        if (h1 && !(tail_vints && r1 == nd - 1)) {
          BlockDev bb;
          uint32_t bm;
          dir_entry(ix, B, S, c, wn, j1, &bb, &bm);
          t1 = pack_tf(ix.blob + B.base + bb.tf_rel, bm >> 8, p1);
        }
        al0 = h0;
        al1 = h1;
        if (al0) s0 += bm25_term(B.idf, t0, nrm0);
        if (al1) s1 += bm25_term(B.idf, t1, nrm1);
        rec(s, (B.blk0 + j0) * 128u + p0, (B.blk0 + j1) * 128u + p1, t0, t1);
        // advance the cursor to the furthest block queried (docs only increase)
        if (l == 0 && nd && jlast > c && s < kMaxTerms) S.cur[s] = jlast;
      }
      if (__ballot(al0 || al1) == 0) return;
      if (phrase) {   // HandleTheFoundDoc: rank only docs that hold the phrase
        // (only the block's top-k candidates are checked, as in lean_segment)
        if (!wide) {
          const double flo0 = __longlong_as_double(static_cast<long long>(
              (static_cast<uint64_t>(uni(static_cast<uint32_t>(floor_bits >> 32))) << 32) |
              uni(static_cast<uint32_t>(floor_bits))));
          const double kth0 = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
          al0 = al0 && s0 > flo0 && (pt_n < k || s0 > kth0);
          al1 = al1 && s1 > flo0 && (pt_n < k || s1 > kth0);
        }
        // the candidates of both halves compacted onto the wave's lanes, one
        // check each (two passes of divergent position walks become one when
        // they are at most 64); two-term phrases take the inline check
        const uint64_t m0 = __ballot(al0), m1 = __ballot(al1);
        const uint32_t n0 = __popcll(m0), nc = n0 + __popcll(m1);
        const uint32_t c0 = __popcll(m0 & lanemask_lt()), c1 = n0 + __popcll(m1 & lanemask_lt());
        bool r0 = false, r1 = false;
        for (uint32_t base = 0; base < nc; base += 64) {
          const uint32_t c = base + l;
          bool ok = false;
          if (c < nc) {
            // value of candidate c: the (c)-th set lane of m0 (value 2l), else of m1 (2l + 1)
            const uint64_t m = c < n0 ? m0 : m1;
            uint32_t want = c < n0 ? c : c - n0, pos = 0;
            for (uint32_t step = 32; step; step >>= 1) {   // lowest pos with want + 1 set bits at or below
              const uint32_t below = __popcll(m & ((2ull << (pos + step - 1)) - 1ull));
              if (below <= want) pos += step;
            }
            const uint32_t v = 2 * pos + (c < n0 ? 0u : 1u);
            ok = nt == 2 ? phrase_match2(ix, static_cast<uint32_t>(qlist[0]), static_cast<uint32_t>(qlist[1]), ph[v],
                                         ph[128 + v], ph[256 + v], ph[384 + v])
                         : phrase_match(ix, qlist, nt, ph, v);
          }
          const uint64_t res = __ballot(ok);
          if (al0 && c0 >= base && c0 < base + 64) r0 = (res >> (c0 - base)) & 1ull;
          if (al1 && c1 >= base && c1 < base + 64) r1 = (res >> (c1 - base)) & 1ull;
        }
        al0 = r0;
        al1 = r1;
        if (__ballot(al0 || al1) == 0) return;
      }
      n_surv += __popcll(__ballot(al0)) + __popcll(__ballot(al1));

      // running top-k: candidates beat the k-th best at block start and the
      // floor of the earlier segments (scores are > 0, so bits order as values)
      const double flo = __longlong_as_double(static_cast<long long>(
          (static_cast<uint64_t>(uni(static_cast<uint32_t>(floor_bits >> 32))) << 32) |
          uni(static_cast<uint32_t>(floor_bits))));
      const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
      uint64_t cm0 = __ballot(al0 && (wide || (s0 > flo && (pt_n < k || s0 > kth))));
      uint64_t cm1 = __ballot(al1 && (wide || (s1 > flo && (pt_n < k || s1 > kth))));
      while (cm0 | cm1) {
        const int fl = __builtin_ctzll(cm0 | cm1);
        const bool second = !((cm0 >> fl) & 1);
        if (second) cm1 &= cm1 - 1; else cm0 &= ~(1ull << fl);
        const double sv = readlane_f64(second ? s1 : s0, fl);
        const uint32_t dv = __builtin_amdgcn_readlane(second ? a1 : a0, fl);
        const uint32_t pos = wide ? 0u : __popcll(__ballot(l < pt_n && pt >= sv));
        if (wide || pos < k) {
          if (l == 0) {
            Event e;
            e.score = sv;
            e.doc = static_cast<int32_t>(dv);
            e.pad = 0;
            S.evs[evb] = e;
          }
          ++ev_n;
          if (++evb == 64) { flush_events(64); evb = 0; }
          if (!wide) {
            const double up = wave_shr1_f64(pt);
            if (l > pos) pt = up;
            else if (l == pos) pt = sv;
            pt_n = pt_n + 1 > k ? k : pt_n + 1;
          }
        }
      }
      if (my_pub && !wide) {
        const double kn = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
        const double pv = kn > flo ? kn : flo;
        if (pv > last_pub) {
          if (l == 0)
            __hip_atomic_fetch_max(my_pub, static_cast<uint64_t>(__double_as_longlong(pv)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last_pub = pv;
        }
      }
    };

    Stage sa, sb;
    if (b0 < b1) {
      issue_words(b0);
      fetch(b0, sa);
    }
    for (uint32_t b = b0; b < b1 && !done; b += 2) {
      step(sa, sb, b);
      if (b + 1 >= b1 || done) break;
      step(sb, sa, b + 1);
    }
    if (evb) flush_events(evb);
    finish_item<false>(qs, plan, qi, P.n_items, item, prev_pub, r, ev_out, ev_n, events, ev_cnt, fr);
    item = 0xFFFFFFFFu;
  }
  if (l == 0) {
    stats[blockIdx.x * kStatStride + 0] = n_surv;
    stats[blockIdx.x * kStatStride + 1] = n_dblk;
    stats[blockIdx.x * kStatStride + 2] = n_oblk;
  }
}


// (below, with the owner replay kernel)
__device__ __noinline__ void owner_replay_tail(const QueryIn* qs, const int32_t* meta, const Event* recv,
                                               HitDev* hits, int32_t* n_hits, uint32_t* counters,
                                               uint32_t wave, uint32_t waves, uint64_t meta_stride,
                                               uint64_t stride, int32_t q0, int32_t nq, int32_t n_shards,
                                               int32_t hit_stride);

// ----------------------------------------------------------- lean kernel --
// Items whose other lists all carry rank bitmaps (and single-term items).
// Workgroups of kLeanWaves independent waves: each wave dequeues and runs its
// own items, so the only workgroup barrier is the norm-table fill at start.
// Small LDS (LeanLds per wave + one shared norm table) and a register budget
// of kLeanWgs workgroups per CU keep several waves per SIMD resident, which
// is what hides the dependent loads of short items and of the probe chains.
// 5 workgroups (the conjunctive instance: 96 VGPRs, 27.7 KB LDS, 5 waves per
// SIMD): with the pre-probe bound the main leg went 23.5 -> 24.9 M q/s against
// 4 (profiles/r02_pr2_ab.txt).  The phrase instance: 4 (kLeanWgsPhrase).
constexpr int kLeanWgs = kLeanDeep ? 4 : 5;   // (a deeper pipeline's register sets: 4)
constexpr int kLeanWgsPhrase = 4;
// kOne: every item of the launch is a single-term query's (single_high,
// single_low, a batch former's single-term batches): only single_segment is
// compiled in, so the instance keeps its registers for it (no spills).
template <bool kPh, bool kTwo = false, bool kOne = false>
__global__ __launch_bounds__(64 * kLeanWaves, kPh ? kLeanWgsPhrase : kLeanWgs) void lean_kernel(
    IndexArgs ix, const QueryIn* __restrict__ qs, const QueryPlan* __restrict__ plan, int nq,
    uint32_t* __restrict__ counters, Event* __restrict__ events, uint32_t* __restrict__ ev_cnt,
    uint32_t* __restrict__ stats, FusedReplay fr, const uint32_t* __restrict__ item_q,
    uint64_t* __restrict__ pub, const QueryDesc* __restrict__ desc) {
  __shared__ LeanLdsT<kPh> SW[kLeanWaves];
  __shared__ double norm[256];
  const uint32_t l = threadIdx.x & 63;
  // (wave-uniform; said so, so that the item indices, segment bounds and the
  // pipeline's loop counter derived from it are scalar, not per-lane values)
  const uint32_t w = uni(threadIdx.x >> 6);
  for (uint32_t i = threadIdx.x; i < 256; i += 64 * kLeanWaves) norm[i] = ix.cache[i];
  __syncthreads();
  LeanLdsT<kPh>& S = SW[w];
  const uint32_t wid = blockIdx.x * kLeanWaves + w;
  // this instance's items: the conjunctive lean ones [0, lean conj), or (kPh)
  // the lean phrase queries' [lean conj, lean)
  const uint32_t n_conj = uni(__hip_atomic_load(&counters[kCtrLeanConj], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t lo = kPh ? n_conj : 0u;
  const uint32_t n_lean = kPh ? uni(__hip_atomic_load(&counters[kCtrLean], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT))
                              : n_conj;
  uint32_t* heads = &counters[kPh ? kCtrPHead0 : kCtrHead0];
  uint32_t n_surv = 0, n_dblk = 0;
  uint32_t shard = wid % kQueueShards, tried = 0;
  uint32_t item = lo + wid;
  for (;;) {
    if (item >= n_lean) item = next_item(heads, lo, n_lean, shard, tried);
    if (item >= n_lean) break;
    const uint32_t qi = uni(item_q[item]);
    const QueryDesc Q = desc[qi];   // everything the item's setup needs, one record
    const uint32_t r = item - Q.item_base;
    const uint32_t seg = Q.seg;
    const uint32_t b0 = r * seg;
    const uint32_t b1 = min(b0 + seg, Q.a_nblk);
    Event* ev_out = events + Q.ev_base + static_cast<uint64_t>(r) * seg * 128;
    uint64_t* my_pub = pub ? pub + item : nullptr;
    const uint64_t* prev_pub = (pub && r > 0) ? pub + item - 1 : nullptr;

    // the segment's directory entries, the driver's decoded VInts tail and
    // the earlier items' score floors (floor_lanes): one round of loads
    const uint64_t floor0 = floor_lanes(prev_pub, r);
    __builtin_amdgcn_wave_barrier();
    if (b0 + l < b1) {
      S.dblk[l] = reinterpret_cast<const uint4*>(ix.blocks)[Q.a_blk0 + b0 + l];
      S.dmeta[l] = ix.blk_meta[Q.a_blk0 + b0 + l];
    }
    const bool dtail = b0 < b1 && b1 == Q.a_nblk && Q.a_tail != kNoTail;
    uint32_t tdoc0 = 0, tdoc1 = 0, ttf0 = 0, ttf1 = 0;
    if (dtail) {
      const uint32_t cnt = Q.a_tail_cnt;
      const uint32_t* t = ix.tails + Q.a_tail;
      if (2 * l < cnt) { tdoc0 = t[2 * l]; ttf0 = t[cnt + 2 * l]; }
      if (2 * l + 1 < cnt) { tdoc1 = t[2 * l + 1]; ttf1 = t[cnt + 2 * l + 1]; }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t first_doc = b0 == 0 ? 0u : uni(S.dblk[0].x) + 1u;
    // an other list ends before this segment: nothing in it can match
    const bool done = first_doc > Q.min_last;
    // a query of one item with fused replay: the heap runs here, no events
    double pt = 0.0, last_pub = 0.0;
    uint32_t pt_n = 0, ev_n = 0, evb = 0;   // events of the item; the last evb of them still in S.evs
    if (!done && b0 < b1) {
      const bool phrase =
          kPh && (Q.nt & 0xFFFFu) > 1 && (uni(static_cast<uint32_t>(qs[qi].flags)) & kQueryPhrase);
      const int32_t* ql = qlist_of(qs, static_cast<int>(qi));
      if constexpr (kOne) {
        single_segment<kPh>(ix, S, norm, Q, b0, b1, dtail, tdoc0, tdoc1, ttf0, ttf1, floor0, prev_pub, r, my_pub,
                            ev_out, ev_n, evb, pt, pt_n, last_pub, n_surv, n_dblk);
      } else {
      if (!kTwo && !kPh && (Q.slots >> 16) == kNoSlot)   // one term (never a phrase instance's item)
        single_segment<kPh>(ix, S, norm, Q, b0, b1, dtail, tdoc0, tdoc1, ttf0, ttf1, floor0, prev_pub, r, my_pub,
                            ev_out,
                            ev_n, evb, pt, pt_n, last_pub, n_surv, n_dblk);
      else if (uni(static_cast<uint32_t>(Q.o_bm >> kProbeShiftBit)))   // O1 has offset buckets
        lean_segment<kPh, kTwo, true, kPh ? 0 : kLeanDeep>(ix, S, norm, Q, ql, phrase, b0, b1, dtail, tdoc0, tdoc1, ttf0, ttf1,
                                      floor0, prev_pub, r, my_pub, ev_out, ev_n, evb, pt, pt_n, last_pub, n_surv, n_dblk);
      else
        lean_segment<kPh, kTwo, false, kPh ? 0 : kLeanDeep>(ix, S, norm, Q, ql, phrase, b0, b1, dtail, tdoc0, tdoc1, ttf0, ttf1,
                                       floor0, prev_pub, r, my_pub, ev_out, ev_n, evb, pt, pt_n, last_pub, n_surv, n_dblk);
      }
    }
    // The item's end from the events still in LDS where it can (finish_item
    // otherwise): every event of the item is there when ev_n == evb.
    __builtin_amdgcn_wave_barrier();
    const bool in_lds = ev_n == evb;
    double esc = 0.0;
    int32_t edc = 0;
    if (l < evb) {
      esc = S.evs[l].score;
      edc = S.evs[l].doc;
    }
    __builtin_amdgcn_wave_barrier();
    if (in_lds && Q.n_items == 1 && fr.q_done && !fr.x_send && Q.k <= static_cast<uint32_t>(kMaxK)) {
      // a query of one item: its events are the query's whole stream, in doc
      // order; the restated heap replays them here (replay_query's HeapSink)
      // with no store, count hand-off or reload
      replay_lds_call(esc, edc, evb, Q.k, fr.hits + static_cast<int64_t>(qi) * fr.hit_stride, &fr.n_hits[qi]);
      if (l == 0) ev_cnt[item] = ev_n;   // (batch statistics)
    } else {
      const uint64_t* refilter = prev_pub;
      if (in_lds && prev_pub && ev_n > 0) {
        // finish_item's re-filter against the earlier items' floor, on the
        // LDS copy: only the kept events are stored
        const double fl_end =
            __longlong_as_double(static_cast<long long>(floor_max(floor_lanes(prev_pub, r))));
        const bool keep = l < evb && esc > fl_end;
        const uint64_t km = __ballot(keep);
        if (keep) {
          Event e;
          e.score = esc;
          e.doc = edc;
          e.pad = 0;
          store_event_coherent(&ev_out[__popcll(km & lanemask_lt())], e);
        }
        ev_n = __popcll(km);
        refilter = nullptr;
      } else if (l < evb) {   // the rest of the item's events, after those stored before
        Event e;
        e.score = esc;
        e.doc = edc;
        e.pad = 0;
        store_event_coherent(&ev_out[ev_n - evb + l], e);
      }
      finish_item<true>(qs, plan, qi, Q.n_items, item, refilter, r, ev_out, ev_n, events, ev_cnt, fr);
    }
    item = 0xFFFFFFFFu;
  }
  if (fr.oj.nq > 0)   // an earlier step group's owner replay, deferred into this kernel's tail
    owner_replay_tail(fr.oj.qs, fr.oj.meta, fr.oj.recv, fr.oj.hits, fr.oj.n_hits, fr.oj.counters, wid,
                      gridDim.x * kLeanWaves, fr.oj.meta_stride, fr.oj.stride, fr.oj.q0, fr.oj.nq,
                      fr.oj.n_shards, fr.oj.hit_stride);
  if (l == 0) {
    stats[wid * kStatStride + 0] = n_surv;
    stats[wid * kStatStride + 1] = n_dblk;
    stats[wid * kStatStride + 2] = 0;
  }
}

// ------------------------------------------------------ doc-range shards --
// Owner side of the fused exchange (wsr_shard_step): meta[g * meta_stride +
// 2 * i] = {count, offset} shard g sent for owned query i (count -1: the
// sender's slot overflowed: flagged, read as empty); its events at recv +
// g * stride + offset.
// kWide: the queries with k > kMaxK, heap in LDS (a separate instance, so the
// common one reserves no LDS for it).
template <bool kWide>
__device__ __forceinline__ void owner_replay_query(const QueryIn* __restrict__ qs, int qi, int q0, int n_shards,
                                                   const int32_t* __restrict__ meta, uint64_t meta_stride,
                                                   uint64_t stride, const Event* __restrict__ recv,
                                                   HitDev* __restrict__ hits, int hit_stride,
                                                   int32_t* __restrict__ n_hits, uint32_t* __restrict__ counters) {
  const int gq = q0 + qi;
  const uint32_t k = uni(qs[gq].k > 0 ? static_cast<uint32_t>(qs[gq].k) : 0u);
  if ((k > static_cast<uint32_t>(kMaxK)) != kWide) return;
  const uint32_t l = threadIdx.x & 63;
  auto meta_of = [&](uint32_t g) { return meta + g * meta_stride + 2ull * static_cast<uint32_t>(qi); };
  for (uint32_t g = l; g < static_cast<uint32_t>(n_shards); g += 64)   // (up to kMaxOwners shards)
    if (meta_of(g)[0] < 0) atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrExchange));
  auto count_of = [&](uint32_t g) {
    const int32_t c = meta_of(g)[0];
    return static_cast<uint32_t>(c > 0 ? c : 0);
  };
  auto base_of = [&](uint32_t g) { return recv + g * stride + static_cast<uint32_t>(meta_of(g)[1]); };
  if constexpr (kWide) {
    __shared__ double s_hs[kMaxKWide];
    __shared__ int32_t s_hd[kMaxKWide];
    LdsHeapSink sink;
    sink.hs = s_hs;
    sink.hd = s_hd;
    sink.k = k;
    consume_stream(sink, static_cast<uint32_t>(n_shards), count_of, base_of, [](double, int32_t) {});
    sink.finish(hits + static_cast<int64_t>(gq) * hit_stride, &n_hits[gq]);
  } else {
    HeapSink sink;
    sink.k = k;
    consume_stream(sink, static_cast<uint32_t>(n_shards), count_of, base_of, [](double, int32_t) {});
    sink.finish(hits + static_cast<int64_t>(gq) * hit_stride, &n_hits[gq]);
  }
}

template <bool kWide>
__global__ __launch_bounds__(64) void owner_replay_meta_kernel(const QueryIn* __restrict__ qs, int q0, int nq,
                                                               int n_shards, const int32_t* __restrict__ meta,
                                                               uint64_t meta_stride, uint64_t stride,
                                                               const Event* __restrict__ recv,
                                                               HitDev* __restrict__ hits, int hit_stride,
                                                               int32_t* __restrict__ n_hits,
                                                               uint32_t* __restrict__ counters) {
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  owner_replay_query<kWide>(qs, qi, q0, n_shards, meta, meta_stride, stride, recv, hits, hit_stride, n_hits,
                            counters);
}

// The deferred form (OwnerJob): a lean kernel's waves, their items done,
// replay owned queries wave, wave + waves, ...  Out of line, fields as values
// (see shard_emit_call), so the lean kernel's registers are its own; the
// arguments come in VGPRs and are made wave-uniform first (readfirstlane), so
// the loop is a scalar one.  (A first form claimed queries with lane 0's
// atomicAdd + readfirstlane on VGPR arguments: the loop compiled as a
// divergent one and never ended on the GPU; a static stride needs neither.)
__device__ __forceinline__ const void* uni_ptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  return reinterpret_cast<const void*>(static_cast<uint64_t>(uni(static_cast<uint32_t>(v))) |
                                       (static_cast<uint64_t>(uni(static_cast<uint32_t>(v >> 32))) << 32));
}
__device__ __noinline__ void owner_replay_tail(const QueryIn* qs, const int32_t* meta, const Event* recv,
                                               HitDev* hits, int32_t* n_hits, uint32_t* counters,
                                               uint32_t wave, uint32_t waves, uint64_t meta_stride,
                                               uint64_t stride, int32_t q0, int32_t nq, int32_t n_shards,
                                               int32_t hit_stride) {
  qs = static_cast<const QueryIn*>(uni_ptr(qs));
  meta = static_cast<const int32_t*>(uni_ptr(meta));
  recv = static_cast<const Event*>(uni_ptr(recv));
  hits = static_cast<HitDev*>(const_cast<void*>(uni_ptr(hits)));
  n_hits = static_cast<int32_t*>(const_cast<void*>(uni_ptr(n_hits)));
  counters = static_cast<uint32_t*>(const_cast<void*>(uni_ptr(counters)));
  const uint32_t w0 = uni(wave), nw = uni(waves), n = uni(static_cast<uint32_t>(nq));
  const uint64_t ms = static_cast<uint64_t>(uni(static_cast<uint32_t>(meta_stride))) |
                      (static_cast<uint64_t>(uni(static_cast<uint32_t>(meta_stride >> 32))) << 32);
  const uint64_t st = static_cast<uint64_t>(uni(static_cast<uint32_t>(stride))) |
                      (static_cast<uint64_t>(uni(static_cast<uint32_t>(stride >> 32))) << 32);
  const int32_t b0 = static_cast<int32_t>(uni(static_cast<uint32_t>(q0)));
  const int32_t ns = static_cast<int32_t>(uni(static_cast<uint32_t>(n_shards)));
  const int32_t hs = static_cast<int32_t>(uni(static_cast<uint32_t>(hit_stride)));
  for (uint32_t qi = w0; qi < n; qi += nw)
    owner_replay_query<false>(qs, static_cast<int>(qi), b0, ns, meta, ms, st, recv, hits, hs, n_hits, counters);
}

// ------------------------------------------------------------ launchers --
hipError_t launch_plan(const IndexArgs& ix, const QueryIn* q, int nq, QueryPlan* plan,
                       uint32_t* counters, uint64_t ev_capacity, uint32_t item_capacity,
                       int lean_grid, int lean_grid_ph, int seg_grid, const FusedReplay& fr, uint32_t* item_q,
                       uint64_t* pub, QueryDesc* desc, PlanPart* part, hipStream_t st) {
  const int n_part = std::max(1, (nq + kPlanThreads - 1) / kPlanThreads);
  hipLaunchKernelGGL(plan_query_kernel, dim3(n_part), dim3(kPlanThreads), 0, st, ix, q, nq, plan,
                     counters, fr, desc, part);
  hipLaunchKernelGGL(plan_fill_kernel, dim3(n_part), dim3(kPlanThreads), 0, st, nq, plan, part, n_part,
                     counters, ev_capacity, item_capacity, static_cast<uint32_t>(lean_grid),
                     static_cast<uint32_t>(lean_grid_ph), static_cast<uint32_t>(seg_grid), item_q, pub, desc);
  return hipGetLastError();
}

hipError_t launch_segments(const IndexArgs& ix, const QueryIn* q, const QueryPlan* plan, int nq,
                           uint32_t* counters, Event* events, uint32_t* ev_cnt, uint32_t* stats,
                           int grid, const FusedReplay& fr, const uint32_t* item_q,
                           uint64_t* pub, uint32_t* ph, hipStream_t st) {
  if (ph)
    hipLaunchKernelGGL(segment_kernel<true>, dim3(grid), dim3(64), 0, st, ix, q, plan, nq, counters,
                       events, ev_cnt, stats, fr, item_q, pub, ph);
  else
    hipLaunchKernelGGL(segment_kernel<false>, dim3(grid), dim3(64), 0, st, ix, q, plan, nq, counters,
                       events, ev_cnt, stats, fr, item_q, pub, ph);
  return hipGetLastError();
}

hipError_t launch_lean(const IndexArgs& ix, const QueryIn* q, const QueryPlan* plan, int nq,
                       uint32_t* counters, Event* events, uint32_t* ev_cnt, uint32_t* stats,
                       int lean_wgs, const FusedReplay& fr, const uint32_t* item_q,
                       uint64_t* pub, const QueryDesc* desc, bool phrase, bool two, bool one,
                       hipStream_t st) {
  // (a persistent grid sized for the conjunctive instance: waves of a larger
  // instance that find no room start later and find the queue drained)
  const dim3 g(lean_wgs), b(64 * kLeanWaves);
  if (!phrase && one)
    hipLaunchKernelGGL((lean_kernel<false, false, true>), g, b, 0, st, ix, q, plan, nq, counters, events, ev_cnt,
                       stats, fr, item_q, pub, desc);
  else if (phrase && two)
    hipLaunchKernelGGL((lean_kernel<true, true>), g, b, 0, st, ix, q, plan, nq, counters, events, ev_cnt,
                       stats, fr, item_q, pub, desc);
  else if (phrase)
    hipLaunchKernelGGL((lean_kernel<true, false>), g, b, 0, st, ix, q, plan, nq, counters, events, ev_cnt,
                       stats, fr, item_q, pub, desc);
  else if (two)
    hipLaunchKernelGGL((lean_kernel<false, true>), g, b, 0, st, ix, q, plan, nq, counters, events, ev_cnt,
                       stats, fr, item_q, pub, desc);
  else
    hipLaunchKernelGGL((lean_kernel<false, false>), g, b, 0, st, ix, q, plan, nq, counters, events, ev_cnt,
                       stats, fr, item_q, pub, desc);
  return hipGetLastError();
}

int lean_kernel_occupancy(bool phrase) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, phrase ? lean_kernel<true, true> : lean_kernel<false>,
                                                   64 * kLeanWaves, 0) != hipSuccess)
    return 1;
  return n;
}

hipError_t launch_wide_replay(const QueryIn* q, const QueryPlan* plan, int nq, const Event* events,
                              const uint32_t* ev_cnt, HitDev* hits, int hit_stride, int32_t* n_hits,
                              hipStream_t st) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(wide_replay_kernel, dim3(nq), dim3(64), 0, st, q, plan, nq, events, ev_cnt, hits,
                     hit_stride, n_hits);
  return hipGetLastError();
}

int segment_kernel_occupancy() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, segment_kernel<false>, 64, 0) != hipSuccess) return 1;
  return n;
}

hipError_t launch_owner_replay_meta(const QueryIn* q, int q0, int nq, int n_shards, const int32_t* meta,
                                    uint64_t meta_stride, uint64_t stride, const Event* recv, HitDev* hits,
                                    int hit_stride, int32_t* n_hits, uint32_t* counters, bool any_wide,
                                    hipStream_t st) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(owner_replay_meta_kernel<false>, dim3(nq), dim3(64), 0, st, q, q0, nq, n_shards, meta,
                     meta_stride, stride, recv, hits, hit_stride, n_hits, counters);
  if (any_wide)
    hipLaunchKernelGGL(owner_replay_meta_kernel<true>, dim3(nq), dim3(64), 0, st, q, q0, nq, n_shards, meta,
                       meta_stride, stride, recv, hits, hit_stride, n_hits, counters);
  return hipGetLastError();
}

// Test hook: decode one block of the image on the device (wave-cooperative).
__global__ __launch_bounds__(64) void decode_probe_kernel(const uint8_t* p, uint32_t bits,
                                                          uint32_t cnt, uint32_t delta,
                                                          uint32_t seed, uint32_t* out) {
  __shared__ uint32_t buf[128];
  decode_block(p, bits, cnt, delta != 0, seed, buf);
  out[2 * threadIdx.x] = buf[2 * threadIdx.x];
  out[2 * threadIdx.x + 1] = buf[2 * threadIdx.x + 1];
}

hipError_t launch_decode_probe(const uint8_t* p, uint32_t bits, uint32_t cnt, bool delta,
                               uint32_t seed, uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(decode_probe_kernel, dim3(1), dim3(64), 0, st, p, bits, cnt, delta ? 1u : 0u,
                     seed, out);
  return hipGetLastError();
}

}  // namespace wiser
