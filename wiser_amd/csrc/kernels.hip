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
// Three launches per query batch:
//   plan_kernel     one workgroup: per query pick the shortest list as driver,
//                   cut its blocks into segments of similar cost, exclusive-scan
//                   segment counts and event capacities.
//   segment_kernel  persistent, one wave per workgroup, segments pulled from an
//                   atomic queue.  Per driver block (128 postings): wave-decode
//                   doc ids (2 per lane; bit-unpack or ballot-parallel varint),
//                   gallop each other list's block directory per lane, decode the
//                   touched blocks into LDS once, lower_bound in LDS, decode the
//                   tf blocks only where something matched, score survivors in
//                   fp64 in query-term order, and keep a running top-k (one f64
//                   per lane) to emit the survivors a heap started empty at the
//                   segment start would insert ("events", in doc-id order).
//   replay_kernel   one lane per query: replays the events of its segments, in
//                   doc-id order, through a restatement of libstdc++'s
//                   push_heap/pop_heap with the reference comparator, then SortHeap.
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

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (l >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    uint32_t y = __shfl_xor(x, d, 64);
    x = x > y ? x : y;
  }
  return x;
}

// Value j of a 128-value pack whose data bytes start at d (bit width b):
// bits [j*b, j*b+b) of an LSB-first little-endian stream.  Reads the two
// aligned dwords that cover the value (the blob is padded at its end).
__device__ __forceinline__ uint32_t pack_value(const uint8_t* d, uint32_t b, uint32_t j) {
  const uint32_t bit = j * b;
  const uintptr_t a = reinterpret_cast<uintptr_t>(d) + (bit >> 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
  const uint32_t sh = static_cast<uint32_t>((a & 3) << 3) + (bit & 7);
  const uint64_t v = (static_cast<uint64_t>(w[1]) << 32) | w[0];
  const uint32_t mask = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
  return static_cast<uint32_t>(v >> sh) & mask;
}

__device__ __forceinline__ uint32_t load_byte(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t w = *reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
  return (w >> ((a & 3) << 3)) & 0xFFu;
}

// Wave-cooperative decode of one block (pack of 128 or VInts tail of cnt) into
// out[0..cnt); delta blocks are prefix-summed from `seed` (doc ids), raw blocks
// are term frequencies.  Values past cnt are written as the last value (delta)
// or 0 (raw).  Ends with the wave's LDS writes visible to every lane.
__device__ void decode_block(const uint8_t* p, uint32_t cnt, bool delta, uint32_t seed,
                             uint32_t* out) {
  const uint32_t l = threadIdx.x & 63;
  uint32_t x0, x1;
  const uint32_t magic = uni(load_byte(p));
  if (magic == 0xD6) {
    const uint32_t b = uni(load_byte(p + 1));
    x0 = pack_value(p + 2, b, 2 * l);
    x1 = pack_value(p + 2, b, 2 * l + 1);
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
    __syncthreads();
    x0 = 2 * l < cnt ? out[2 * l] : 0;
    x1 = 2 * l + 1 < cnt ? out[2 * l + 1] : 0;
    __syncthreads();
  }
  if (delta) {
    const uint32_t s = x0 + x1;
    const uint32_t inc = wave_incl_scan(s);
    x0 = seed + (inc - s) + x0;
    x1 = x0 + x1;
  }
  out[2 * l] = x0;
  out[2 * l + 1] = x1;
  __syncthreads();
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
// the block DocIdIterator::GetBlobIndexToGo walks to (flash_iterators.h:218-227),
// found by galloping from the cursor.
__device__ __forceinline__ uint32_t find_block(const uint32_t* last, uint32_t cur, uint32_t nblk,
                                               uint32_t x) {
  if (cur >= nblk) return nblk;
  if (last[cur] >= x) return cur;
  uint32_t lo = cur + 1, step = 1, hi;
  for (;;) {
    const uint32_t probe = cur + step;
    if (probe >= nblk) { hi = nblk; break; }
    if (last[probe] >= x) { hi = probe; break; }
    lo = probe + 1;
    step <<= 1;
  }
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (last[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// ----------------------------------------------------------------- plan --
__global__ __launch_bounds__(1024) void plan_kernel(IndexArgs ix, const QueryIn* __restrict__ qs,
                                                    int nq, QueryPlan* __restrict__ plan,
                                                    uint32_t* __restrict__ counters,
                                                    uint64_t ev_capacity, uint32_t item_capacity) {
  __shared__ uint32_t s_items[1024];
  __shared__ uint64_t s_cap[1024];
  const int t = threadIdx.x, T = blockDim.x;
  const int per = (nq + T - 1) / T;
  const int q0 = t * per, q1 = min(nq, q0 + per);
  uint32_t items = 0;
  uint64_t cap = 0;
  uint32_t err = 0;
  for (int i = q0; i < q1; ++i) {
    const QueryIn q = qs[i];
    QueryPlan p{0, 0, 1, 0, 0};
    bool ok = q.n_terms > 0 && q.k > 0;
    if (q.n_terms > kMaxTerms || q.k > kMaxK) { ok = false; err |= kErrLimit; }
    uint32_t nb[kMaxTerms];
    for (int s = 0; ok && s < q.n_terms; ++s) {
      const int32_t id = q.list[s];
      if (id < 0 || static_cast<uint32_t>(id) >= ix.n_lists) { ok = false; break; }
      nb[s] = ix.lists[id].nblk;
      if (nb[s] == 0) ok = false;  // no docs of this list in this shard: empty AND
    }
    if (ok) {
      uint32_t d = 0;
      for (int s = 1; s < q.n_terms; ++s) if (nb[s] < nb[d]) d = s;
      float cost = 1.0f;
      for (int s = 0; s < q.n_terms; ++s)
        if (s != static_cast<int>(d)) cost += fminf(static_cast<float>(nb[s]) / nb[d], 64.0f);
      uint32_t seg = static_cast<uint32_t>(kSegCost / cost);
      seg = seg < 1 ? 1 : (seg > nb[d] ? nb[d] : seg);
      p.driver = d;
      p.seg_blocks = seg;
      p.n_items = (nb[d] + seg - 1) / seg;
    }
    p.item_base = items;          // local, made global after the scan
    p.ev_base = cap;
    items += p.n_items;
    cap += static_cast<uint64_t>(p.n_items) * p.seg_blocks * 128;
    plan[i] = p;
  }
  s_items[t] = items;
  s_cap[t] = cap;
  __syncthreads();
  // exclusive scan over threads (Hillis-Steele on LDS; 1024 entries)
  for (int d = 1; d < T; d <<= 1) {
    uint32_t a = 0; uint64_t c = 0;
    if (t >= d) { a = s_items[t - d]; c = s_cap[t - d]; }
    __syncthreads();
    s_items[t] += a; s_cap[t] += c;
    __syncthreads();
  }
  const uint32_t ib = s_items[t] - items;
  const uint64_t cb = s_cap[t] - cap;
  for (int i = q0; i < q1; ++i) { plan[i].item_base += ib; plan[i].ev_base += cb; }
  if (err) atomicOr(&counters[kCtrError], err);
  if (t == T - 1) {
    const bool fits = s_cap[t] <= ev_capacity && s_items[t] <= item_capacity;
    if (!fits) atomicOr(&counters[kCtrError], static_cast<uint32_t>(kErrCapacity));
    counters[kCtrItems] = fits ? s_items[t] : 0u;  // never write past the workspace
    counters[kCtrHead] = 0;
    counters[kCtrEvCap] = static_cast<uint32_t>(s_cap[t] > 0xFFFFFFFFull ? 0xFFFFFFFFull : s_cap[t]);
    counters[kCtrSurvivors] = 0;
    counters[kCtrDriverBlocks] = 0;
    counters[kCtrOtherBlocks] = 0;
  }
}

// -------------------------------------------------------------- segment --
struct WaveLds {
  uint32_t doc[128];                 // decoded doc ids of the current other-list block
  uint32_t tf[128];                  // decoded tf block (other list, then driver)
  uint32_t tfq[kMaxTerms][128];      // tf per query slot per driver posting of the block
};

__global__ __launch_bounds__(64) void segment_kernel(IndexArgs ix, const QueryIn* __restrict__ qs,
                                                     const QueryPlan* __restrict__ plan, int nq,
                                                     uint32_t* __restrict__ counters,
                                                     Event* __restrict__ events,
                                                     uint32_t* __restrict__ ev_cnt) {
  __shared__ WaveLds S;
  const uint32_t l = threadIdx.x & 63;
  const uint32_t total = uni(__hip_atomic_load(&counters[kCtrItems], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
  uint32_t n_surv = 0, n_dblk = 0, n_oblk = 0;
  for (;;) {
    uint32_t item = 0;
    if (l == 0) item = atomicAdd(&counters[kCtrHead], 1u);
    item = uni(__shfl(item, 0, 64));
    if (item >= total) break;
    // query of this item: last q with plan[q].item_base <= item
    uint32_t lo = 0, hi = static_cast<uint32_t>(nq);
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (plan[mid].item_base <= item) lo = mid; else hi = mid;
    }
    const uint32_t qi = uni(lo);
    const QueryPlan P = plan[qi];
    const int32_t* qlist = qs[qi].list;
    const uint32_t r = item - P.item_base;
    const uint32_t d = uni(P.driver);
    const uint32_t nt = uni(static_cast<uint32_t>(qs[qi].n_terms));
    const uint32_t k = uni(static_cast<uint32_t>(qs[qi].k));
    const ListDev A = ix.lists[qlist[d]];
    const uint32_t seg = uni(P.seg_blocks);
    const uint32_t b0 = r * seg;
    const uint32_t b1 = min(b0 + seg, A.nblk);
    Event* ev_out = events + P.ev_base + static_cast<uint64_t>(r) * seg * 128;
    uint32_t ev_n = 0;

    // per other slot: cursor into its block directory, seeded at the segment's first doc
    uint32_t cur[kMaxTerms];
    const uint32_t first_doc = b0 == 0 ? 0u : ix.blocks[A.blk0 + b0].prev + 1u;
    bool done = false;   // some other list has no doc >= the next driver doc
#pragma unroll
    for (uint32_t s = 0; s < kMaxTerms; ++s) {
      cur[s] = 0;
      if (s < nt && s != d) {
        const ListDev B = ix.lists[qlist[s]];
        cur[s] = uni(find_block(ix.blk_last + B.blk0, 0, B.nblk, first_doc));
        if (cur[s] >= B.nblk) done = true;
      }
    }

    double pt = 0.0;     // running top-k scores, lane t holds rank t (descending)
    uint32_t pt_n = 0;   // valid entries (uniform)

    for (uint32_t b = b0; b < b1 && !done; ++b) {
      const BlockDev blk = ix.blocks[A.blk0 + b];
      const uint32_t cnt = (b == A.nblk - 1) ? A.tail_cnt : 128u;
      decode_block(ix.blob + A.base + blk.doc_rel, cnt, true, blk.prev, S.tfq[d]);
      ++n_dblk;
      const uint32_t a0 = S.tfq[d][2 * l], a1 = S.tfq[d][2 * l + 1];
      __syncthreads();
      bool al0 = 2 * l < cnt && a0 >= ix.doc_lo && a0 < ix.doc_hi;
      bool al1 = 2 * l + 1 < cnt && a1 >= ix.doc_lo && a1 < ix.doc_hi;

      for (uint32_t s = 0; s < nt; ++s) {
        if (s == d) continue;
        if (__ballot(al0 || al1) == 0) break;
        const ListDev B = ix.lists[qlist[s]];
        const uint32_t* last = ix.blk_last + B.blk0;
        uint32_t c = 0;
#pragma unroll
        for (uint32_t u = 0; u < kMaxTerms; ++u) if (u == s) c = cur[u];
        const uint32_t j0 = al0 ? find_block(last, c, B.nblk, a0) : kNoBlock;
        const uint32_t j1 = al1 ? find_block(last, c, B.nblk, a1) : kNoBlock;
        bool pd0 = al0 && j0 < B.nblk, pd1 = al1 && j1 < B.nblk;
        // a doc beyond the list's last block cannot match, nor can any later doc
        if (__ballot((al0 && j0 >= B.nblk) || (al1 && j1 >= B.nblk))) done = true;
        al0 = pd0; al1 = pd1;
        uint32_t t0 = 0, t1 = 0;
        for (;;) {
          const uint64_t any0 = __ballot(pd0), any1 = __ballot(pd1);
          if ((any0 | any1) == 0) break;
          const int fl = __builtin_ctzll(any0 | any1);
          const uint32_t cand = ((any0 >> fl) & 1) ? j0 : j1;
          const uint32_t jj = uni(__builtin_amdgcn_readlane(cand, fl));
          const BlockDev bb = ix.blocks[B.blk0 + jj];
          const uint32_t bc = (jj == B.nblk - 1) ? B.tail_cnt : 128u;
          decode_block(ix.blob + B.base + bb.doc_rel, bc, true, bb.prev, S.doc);
          ++n_oblk;
          uint32_t p0 = 0, p1 = 0;
          bool h0 = false, h1 = false;
          if (pd0 && j0 == jj) {
            p0 = lds_lower_bound(S.doc, bc, a0);
            h0 = p0 < bc && S.doc[p0] == a0;
            pd0 = false;
            al0 = h0;
          }
          if (pd1 && j1 == jj) {
            p1 = lds_lower_bound(S.doc, bc, a1);
            h1 = p1 < bc && S.doc[p1] == a1;
            pd1 = false;
            al1 = h1;
          }
          __syncthreads();
          if (__ballot(h0 || h1)) {
            decode_block(ix.blob + B.base + bb.tf_rel, bc, false, 0, S.tf);
            if (h0) t0 = S.tf[p0];
            if (h1) t1 = S.tf[p1];
            __syncthreads();
          }
        }
        if (al0) S.tfq[s][2 * l] = t0;
        if (al1) S.tfq[s][2 * l + 1] = t1;
        // advance the cursor to the furthest block queried (docs only increase)
        const uint32_t q0 = j0 != kNoBlock ? j0 : 0u, q1 = j1 != kNoBlock ? j1 : 0u;
        const uint32_t jm = uni(wave_max(q0 > q1 ? q0 : q1));
#pragma unroll
        for (uint32_t u = 0; u < kMaxTerms; ++u)
          if (u == s && jm > cur[u]) cur[u] = jm;
      }
      __syncthreads();
      if (__ballot(al0 || al1) == 0) continue;

      // driver tf
      decode_block(ix.blob + A.base + blk.tf_rel, cnt, false, 0, S.tf);
      const uint32_t ta0 = S.tf[2 * l], ta1 = S.tf[2 * l + 1];
      __syncthreads();
      // BM25 in query-term order (scoring.h:124-145), fp64, no contraction
      double s0 = 0.0, s1 = 0.0;
      const uint32_t c0 = al0 && a0 < ix.n_c4 ? ix.c4[a0] : 0u;
      const uint32_t c1 = al1 && a1 < ix.n_c4 ? ix.c4[a1] : 0u;
      const double cache0 = ix.cache[c0], cache1 = ix.cache[c1];
      for (uint32_t s = 0; s < nt; ++s) {
        const double idf = ix.lists[qlist[s]].idf;
        const uint32_t f0 = s == d ? ta0 : S.tfq[s][2 * l];
        const uint32_t f1 = s == d ? ta1 : S.tfq[s][2 * l + 1];
        const double k1p1 = 1.2 + 1;
        const double n0 = (static_cast<double>(static_cast<int32_t>(f0)) * k1p1) /
                          (static_cast<double>(static_cast<int32_t>(f0)) + cache0);
        const double n1 = (static_cast<double>(static_cast<int32_t>(f1)) * k1p1) /
                          (static_cast<double>(static_cast<int32_t>(f1)) + cache1);
        s0 += idf * n0;
        s1 += idf * n1;
      }
      n_surv += __popcll(__ballot(al0)) + __popcll(__ballot(al1));

      // running top-k: candidates beat the k-th best at block start
      const double kth = pt_n >= k ? readlane_f64(pt, static_cast<int>(k) - 1) : 0.0;
      uint64_t cm0 = __ballot(al0 && (pt_n < k || s0 > kth));
      uint64_t cm1 = __ballot(al1 && (pt_n < k || s1 > kth));
      while (cm0 | cm1) {
        const int fl = __builtin_ctzll(cm0 | cm1);
        const bool second = !((cm0 >> fl) & 1);
        if (second) cm1 &= cm1 - 1; else cm0 &= ~(1ull << fl);
        const double sv = readlane_f64(second ? s1 : s0, fl);
        const uint32_t dv = __builtin_amdgcn_readlane(second ? a1 : a0, fl);
        const uint32_t pos = __popcll(__ballot(l < pt_n && pt >= sv));
        if (pos < k) {
          if (l == 0) {
            Event e;
            e.score = sv;
            e.doc = static_cast<int32_t>(dv);
            e.pad = 0;
            ev_out[ev_n] = e;
          }
          ++ev_n;
          const double up = __shfl_up(pt, 1, 64);
          if (l > pos) pt = up;
          else if (l == pos) pt = sv;
          pt_n = pt_n + 1 > k ? k : pt_n + 1;
        }
      }
    }
    if (l == 0) ev_cnt[item] = ev_n;
  }
  if (l == 0) {
    atomicAdd(&counters[kCtrSurvivors], n_surv);
    atomicAdd(&counters[kCtrDriverBlocks], n_dblk);
    atomicAdd(&counters[kCtrOtherBlocks], n_oblk);
  }
}

// --------------------------------------------------------------- replay --
// libstdc++ std::priority_queue<unique_ptr<ResultDocEntry>, vector, EntryGreater>
// (query_processing.h:510-524): push = push_back + __push_heap, pop = __pop_heap
// (+ __adjust_heap) + pop_back, with comp(a, b) = a.score > b.score.
struct HeapView {
  double* sc;
  int32_t* dc;
  uint32_t stride;
  __device__ double& s(uint32_t i) { return sc[i * stride]; }
  __device__ int32_t& d(uint32_t i) { return dc[i * stride]; }
  __device__ void push_hole(uint32_t hole, uint32_t top, double vs, int32_t vd) {
    uint32_t parent = hole ? (hole - 1) / 2 : 0;
    while (hole > top && s(parent) > vs) {
      s(hole) = s(parent); d(hole) = d(parent);
      hole = parent;
      parent = hole ? (hole - 1) / 2 : 0;
    }
    s(hole) = vs; d(hole) = vd;
  }
  __device__ void push(uint32_t& n, double vs, int32_t vd) { push_hole(n, 0, vs, vd); ++n; }
  __device__ void pop(uint32_t& n) {
    if (n > 1) {
      const uint32_t len = n - 1;
      const double vs = s(len); const int32_t vd = d(len);
      s(len) = s(0); d(len) = d(0);
      // __adjust_heap(first, 0, len, value)
      uint32_t hole = 0, child = 0;
      while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (s(child) > s(child - 1)) --child;
        s(hole) = s(child); d(hole) = d(child);
        hole = child;
      }
      if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        s(hole) = s(child - 1); d(hole) = d(child - 1);
        hole = child - 1;
      }
      push_hole(hole, 0, vs, vd);
    }
    --n;
  }
};

__global__ __launch_bounds__(64) void replay_kernel(const QueryIn* __restrict__ qs,
                                                    const QueryPlan* __restrict__ plan, int nq,
                                                    const Event* __restrict__ events,
                                                    const uint32_t* __restrict__ ev_cnt,
                                                    HitDev* __restrict__ hits, int hit_stride,
                                                    int32_t* __restrict__ n_hits) {
  __shared__ double s_sc[kMaxK * 64];
  __shared__ int32_t s_dc[kMaxK * 64];
  const int t = threadIdx.x;
  const int qi = blockIdx.x * 64 + t;
  if (qi >= nq) return;
  const QueryIn Q = qs[qi];
  const QueryPlan P = plan[qi];
  HeapView H{s_sc + t, s_dc + t, 64};
  uint32_t n = 0;
  const uint32_t k = Q.k > 0 ? static_cast<uint32_t>(Q.k) : 0u;
  for (uint32_t r = 0; r < P.n_items; ++r) {
    const Event* ev = events + P.ev_base + static_cast<uint64_t>(r) * P.seg_blocks * 128;
    const uint32_t ne = ev_cnt[P.item_base + r];
    for (uint32_t i = 0; i < ne; ++i) {
      const double sc = ev[i].score;
      const int32_t dc = ev[i].doc;
      if (n < k) {
        H.push(n, sc, dc);
      } else if (sc > H.s(0)) {
        H.pop(n);
        H.push(n, sc, dc);
      }
    }
  }
  // SortHeap (query_processing.h:551-562): pop to ascending, then reverse
  const uint32_t m = n;
  HitDev* out = hits + static_cast<int64_t>(qi) * hit_stride;
  for (uint32_t i = 0; i < m; ++i) {
    HitDev h;
    h.doc = H.d(0);
    h.pad = 0;
    h.score = H.s(0);
    out[m - 1 - i] = h;
    H.pop(n);
  }
  n_hits[qi] = static_cast<int32_t>(m);
}

// ------------------------------------------------------------ launchers --
hipError_t launch_plan(const IndexArgs& ix, const QueryIn* q, int nq, QueryPlan* plan,
                       uint32_t* counters, uint64_t ev_capacity, uint32_t item_capacity,
                       hipStream_t st) {
  hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(1024), 0, st, ix, q, nq, plan, counters,
                     ev_capacity, item_capacity);
  return hipGetLastError();
}

hipError_t launch_segments(const IndexArgs& ix, const QueryIn* q, const QueryPlan* plan, int nq,
                           uint32_t* counters, Event* events, uint32_t* ev_cnt, int grid,
                           hipStream_t st) {
  hipLaunchKernelGGL(segment_kernel, dim3(grid), dim3(64), 0, st, ix, q, plan, nq, counters,
                     events, ev_cnt);
  return hipGetLastError();
}

hipError_t launch_replay(const QueryIn* q, const QueryPlan* plan, int nq, const Event* events,
                         const uint32_t* ev_cnt, HitDev* hits, int hit_stride, int32_t* n_hits,
                         hipStream_t st) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(replay_kernel, dim3((nq + 63) / 64), dim3(64), 0, st, q, plan, nq, events,
                     ev_cnt, hits, hit_stride, n_hits);
  return hipGetLastError();
}

int segment_kernel_occupancy() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, segment_kernel, 64, 0) != hipSuccess) return 1;
  return n;
}

// Test hook: decode one block of the image on the device (wave-cooperative).
__global__ __launch_bounds__(64) void decode_probe_kernel(const uint8_t* p, uint32_t cnt,
                                                          uint32_t delta, uint32_t seed,
                                                          uint32_t* out) {
  __shared__ uint32_t buf[128];
  decode_block(p, cnt, delta != 0, seed, buf);
  out[2 * threadIdx.x] = buf[2 * threadIdx.x];
  out[2 * threadIdx.x + 1] = buf[2 * threadIdx.x + 1];
}

hipError_t launch_decode_probe(const uint8_t* p, uint32_t cnt, bool delta, uint32_t seed,
                               uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(decode_probe_kernel, dim3(1), dim3(64), 0, st, p, cnt, delta ? 1u : 0u, seed,
                     out);
  return hipGetLastError();
}

}  // namespace wiser
