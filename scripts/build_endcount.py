#!/usr/bin/env python3
"""Build the `endcount` diagnostic variant (scripts/build_variant.py): like
`endphase` (scripts/build_endphase.py) but for each lean wave's longest query
replay it writes the replayed events (stats word 0), the heap insertions among
them (word 1), the summed replay ticks (word 2) and the longest replay's ticks
(word 3).  Read with scripts/gpu_lean_phase.sh TAG --count."""
import subprocess
s = open('/root/repo/wiser_amd/csrc/kernels.hip').read()
subs = [
("""struct HeapSink {
  WaveHeap H;
  uint32_t k = 0;
  __device__ __forceinline__ void insert(double sv, int32_t dv) {
    if (H.n < k) H.push(sv, dv);
    else if (sv > H.at(0)) { H.pop(); H.push(sv, dv); }
    else return;
  }""",
"""struct HeapSink {
  WaveHeap H;
  uint32_t k = 0;
  uint32_t n_ins = 0, n_ev = 0;
  __device__ __forceinline__ void insert(double sv, int32_t dv) {
    if (H.n < k) { H.push(sv, dv); ++n_ins; }
    else if (sv > H.at(0)) { H.pop(); H.push(sv, dv); ++n_ins; }
    else return;
  }"""),
("""  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&&) {
    const double top = H.n < k ? -1.0 : H.at(0);""",
"""  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid, Emit&&) {
    n_ev += __popcll(__ballot(valid));
    const double top = H.n < k ? -1.0 : H.at(0);"""),
("""template <bool kCoherent>
__device__ __forceinline__ void replay_query(const QueryIn* __restrict__ qs,""",
"""template <bool kCoherent>
__device__ __forceinline__ uint64_t replay_query(const QueryIn* __restrict__ qs,"""),
("""  sink.finish(hits + static_cast<int64_t>(qi) * hit_stride, &n_hits[qi]);
}

// A one-item query's events""",
"""  sink.finish(hits + static_cast<int64_t>(qi) * hit_stride, &n_hits[qi]);
  return (static_cast<uint64_t>(sink.n_ev) << 32) | sink.n_ins;
}

// A one-item query's events"""),
("""__device__ __noinline__ void replay_query_call(const QueryIn* qs, const QueryPlan* plan, int qi,""",
"""__device__ __noinline__ uint64_t replay_query_call(const QueryIn* qs, const QueryPlan* plan, int qi,"""),
("""                                               HitDev* hits, int hit_stride, int32_t* n_hits) {
  replay_query<true>(qs, plan, qi, events, ev_cnt, hits, hit_stride, n_hits);""",
"""                                               HitDev* hits, int hit_stride, int32_t* n_hits) {
  return replay_query<true>(qs, plan, qi, events, ev_cnt, hits, hit_stride, n_hits);"""),
("""                                            const Event* events, uint32_t* ev_cnt,
                                            const FusedReplay& fr) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  if (prev_pub && ev_n > 0) {""",
"""                                            const Event* events, uint32_t* ev_cnt,
                                            const FusedReplay& fr, uint64_t* tb = nullptr) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  if (prev_pub && ev_n > 0) {"""),
("""      else
        replay_query_call(qs, plan, static_cast<int>(qi), events, ev_cnt, fr.hits, fr.hit_stride,
                          fr.n_hits);
    }
  }
}""",
"""      else {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t rv = replay_query_call(qs, plan, static_cast<int>(qi), events, ev_cnt, fr.hits,
                                              fr.hit_stride, fr.n_hits);
        const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
        if (tb) {
          tb[2] += dt;
          if (dt > tb[3]) { tb[3] = dt; tb[0] = rv >> 32; tb[1] = rv & 0xFFFFFFFFull; }
        }
      }
    }
  }
}"""),
("""  uint32_t n_surv = 0, n_dblk = 0;
  uint32_t shard = wid % kQueueShards, tried = 0;""",
"""  uint32_t n_surv = 0, n_dblk = 0;
  uint64_t tb[4] = {0, 0, 0, 0};
  uint32_t shard = wid % kQueueShards, tried = 0;"""),
("""      finish_item<true>(qs, plan, qi, Q.n_items, item, refilter, r, ev_out, ev_n, events, ev_cnt, fr);""",
"""      finish_item<true>(qs, plan, qi, Q.n_items, item, refilter, r, ev_out, ev_n, events, ev_cnt, fr, tb);"""),
("""    stats[wid * kStatStride + 0] = n_surv;
    stats[wid * kStatStride + 1] = n_dblk;
    stats[wid * kStatStride + 2] = 0;""",
"""    stats[wid * kStatStride + 0] = static_cast<uint32_t>(tb[0]) + 0u * n_surv + 0u * n_dblk;
    stats[wid * kStatStride + 1] = static_cast<uint32_t>(tb[1]);
    stats[wid * kStatStride + 2] = static_cast<uint32_t>(tb[2]);
    stats[wid * kStatStride + 3] = static_cast<uint32_t>(tb[3]);"""),
]
# optional: NAME and further FILE OLD NEW substitutions (applied after these)
import sys
extra = sys.argv[2:]
args = ['python3', '/root/repo/scripts/build_variant.py', sys.argv[1] if len(sys.argv) > 1 else 'endcount']
for a, b in subs:
    assert s.count(a) == 1, a[:80]
    args += ['kernels.hip', a, b]
args += extra
r = subprocess.run(args, capture_output=True, text=True, timeout=1200)
print(r.stdout[-300:], r.stderr[-1500:])
