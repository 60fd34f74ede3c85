#!/usr/bin/env python3
"""Build the `endphase` diagnostic variant (scripts/build_variant.py): lean waves
write the ticks of their item ends split into re-filter, count hand-off and
query replay, and the longest replay (stats words 0-3; read by
scripts/lean_phase.py --end via scripts/gpu_lean_phase.sh TAG --end)."""
import subprocess
s = open('/root/repo/wiser_amd/csrc/kernels.hip').read()
subs = [
("""                                            const Event* events, uint32_t* ev_cnt,
                                            const FusedReplay& fr) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  if (prev_pub && ev_n > 0) {""",
"""                                            const Event* events, uint32_t* ev_cnt,
                                            const FusedReplay& fr, uint64_t* tb = nullptr) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  const uint64_t ta = __builtin_amdgcn_s_memrealtime();
  if (prev_pub && ev_n > 0) {"""),
("""  if (l == 0) __hip_atomic_store(&ev_cnt[item], ev_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // wide queries""",
"""  const uint64_t tb1 = __builtin_amdgcn_s_memrealtime();
  if (tb) tb[0] += tb1 - ta;
  if (l == 0) __hip_atomic_store(&ev_cnt[item], ev_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // wide queries"""),
("""    old = uni(old);
    if (old + 1 == n_items) {
      if (fr.x_send)""",
"""    old = uni(old);
    const uint64_t tb2 = __builtin_amdgcn_s_memrealtime();
    if (tb) tb[1] += tb2 - tb1;
    if (old + 1 == n_items) {
      if (fr.x_send)"""),
("""        replay_query_call(qs, plan, static_cast<int>(qi), events, ev_cnt, fr.hits, fr.hit_stride,
                          fr.n_hits);
    }
  }
}""",
"""        replay_query_call(qs, plan, static_cast<int>(qi), events, ev_cnt, fr.hits, fr.hit_stride,
                          fr.n_hits);
      const uint64_t tb3 = __builtin_amdgcn_s_memrealtime();
      if (tb) { tb[2] += tb3 - tb2; tb[3] = tb3 - tb2 > tb[3] ? tb3 - tb2 : tb[3]; }
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
args = ['python3', '/root/repo/scripts/build_variant.py', 'endphase']
for a, b in subs:
    assert s.count(a) == 1, a[:80]
    args += ['kernels.hip', a, b]
r = subprocess.run(args, capture_output=True, text=True, timeout=1200)
print(r.stdout[-300:], r.stderr[-1500:])
