// RegHeap: the reference's top-k heap for k <= kRegHeapK, held in registers.
//
// The reference keeps its top-k in MinPointerHeap = std::priority_queue<...,
// EntryGreater> (src/qq_mem/src/query_processing.h:510-524): libstdc++'s
// binary heap with comp(a, b) = a.score > b.score; RankDoc (:590-602) pushes
// while size < k, else pops and pushes iff the score beats the top; SortHeap
// (:551-562) pops everything and reverses.  Docs of equal score leave in the
// order that heap's exact walks put them in, so the walks are restated, not
// replaced:
//   push  = __push_heap(first, hole = n, top = 0, value)
//   pop   = value = first[len]; __adjust_heap(first, 0, len, value), len = n - 1
//
// One replay wave holds one heap, every lane the same copy.  Every array
// index below is a compile-time constant (the hole of a walk is a template
// argument, a runtime position is dispatched once through a switch), so the
// arrays live in registers and no step is a permute, a readlane or an LDS
// access; each level of a walk is one f64 compare and a uniform branch.  (The
// lane-per-entry WaveHeap costs ~1,300 cycles per insertion in chains of
// ds_bpermute / readlane, profiles/r05/heap_bench_r05an.txt.)
//
// Host-compilable (no device intrinsics outside rh_uniform), so the CPU test
// (tests/test_regheap.py) runs this very code against libstdc++'s own
// std::push_heap / std::pop_heap.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define RH_FN __host__ __device__ __forceinline__
#else
#define RH_FN inline
#endif

namespace wiser {

constexpr int kRegHeapK = 16;

// A condition every lane agrees on, as a scalar (uniform) branch condition.
RH_FN bool rh_uniform(bool c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(c)) != 0u;
#else
  return c;
#endif
}

struct RegHeap {
  double s[kRegHeapK];
  int32_t d[kRegHeapK];
  uint32_t n = 0;

  template <int H>
  RH_FN void put(double vs, int32_t vd) {
    s[H] = vs;
    d[H] = vd;
  }
  template <int H, int F>
  RH_FN void move() {
    s[H] = s[F];
    d[H] = d[F];
  }

  // __push_heap(first, H, 0, value): while the parent's score > value's, the
  // parent moves down into the hole
  template <int H>
  RH_FN void sift(double vs, int32_t vd) {
    if constexpr (H == 0) {
      put<0>(vs, vd);
    } else {
      constexpr int P = (H - 1) / 2;
      if (rh_uniform(s[P] > vs)) {
        move<H, P>();
        sift<P>(vs, vd);
      } else {
        put<H>(vs, vd);
      }
    }
  }

  // sift<hole>, the hole known only at run time (< kRegHeapK)
  RH_FN void sift_at(uint32_t hole, double vs, int32_t vd) {
    switch (hole) {
#define RH_CASE(i) \
  case i: sift<i>(vs, vd); break;
      RH_CASE(0) RH_CASE(1) RH_CASE(2) RH_CASE(3) RH_CASE(4) RH_CASE(5) RH_CASE(6) RH_CASE(7)
      RH_CASE(8) RH_CASE(9) RH_CASE(10) RH_CASE(11) RH_CASE(12) RH_CASE(13) RH_CASE(14) RH_CASE(15)
#undef RH_CASE
      default: break;
    }
  }

  // first[i], i known only at run time
  RH_FN void at(uint32_t i, double& vs, int32_t& vd) const {
    switch (i) {
#define RH_CASE(j) \
  case j: vs = s[j]; vd = d[j]; break;
      RH_CASE(0) RH_CASE(1) RH_CASE(2) RH_CASE(3) RH_CASE(4) RH_CASE(5) RH_CASE(6) RH_CASE(7)
      RH_CASE(8) RH_CASE(9) RH_CASE(10) RH_CASE(11) RH_CASE(12) RH_CASE(13) RH_CASE(14) RH_CASE(15)
#undef RH_CASE
      default: vs = 0.0; vd = 0; break;
    }
  }

  // __adjust_heap(first, 0, len, value) from hole H (== libstdc++'s
  // `__secondChild`): the larger-indexed child unless it is > the other, so
  // the child whose score is not greater, moves up; at the end the value
  // sifts up from the hole.
  template <int H>
  RH_FN void adjust(uint32_t len, double vs, int32_t vd) {
    constexpr int C = 2 * (H + 1);
    if constexpr (C < kRegHeapK) {
      if (static_cast<uint32_t>(H) < (len - 1) / 2) {
        if (rh_uniform(s[C] > s[C - 1])) {
          move<H, C - 1>();
          adjust<C - 1>(len, vs, vd);
        } else {
          move<H, C>();
          adjust<C>(len, vs, vd);
        }
        return;
      }
      if ((len & 1u) == 0u && static_cast<uint32_t>(H) == (len - 2) / 2) {
        move<H, C - 1>();
        sift<C - 1>(vs, vd);
        return;
      }
    }
    sift<H>(vs, vd);
  }

  // std::priority_queue::pop (pop_heap + pop_back)
  RH_FN void pop() {
    if (n > 1) {
      const uint32_t len = n - 1;
      double vs;
      int32_t vd;
      at(len, vs, vd);
      adjust<0>(len, vs, vd);
    }
    --n;
  }
  // std::priority_queue::push (push_back + push_heap)
  RH_FN void push(double vs, int32_t vd) {
    sift_at(n, vs, vd);
    ++n;
  }
  // RankDoc (query_processing.h:595-602), k <= kRegHeapK
  RH_FN void insert(uint32_t k, double sv, int32_t dv) {
    if (n < k) {
      push(sv, dv);
    } else if (rh_uniform(sv > s[0])) {
      pop();
      push(sv, dv);
    }
  }
};

}  // namespace wiser
