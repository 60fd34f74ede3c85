// Cost of one heap insertion of the query replay (HeapSink over WaveHeap),
// one wave alone on the device (diagnostic for DESIGN §5.00: a heavy query's
// replay inside the lean kernel costs ~0.7 us per insertion).  Scores rise, so
// every event past the first k is an insertion (a pop and a push).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//          -Iinclude -Iwiser_amd/csrc scripts/heap_bench.hip -o /tmp/heap_bench
#include "../wiser_amd/csrc/kernels.hip"
#include <cstdio>
#include <vector>

namespace wiser {
__global__ void heap_bench_kernel(const double* vals, int n, uint32_t k, uint64_t* ticks, HitDev* out,
                                  int32_t* nout) {
  HeapSink sink;
  sink.k = uni(k);
  const uint32_t l = threadIdx.x & 63;
  double sc = vals[l];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (int c = 0; c < n; c += 64) {
    const double nx = c + 64 < n ? vals[c + 64 + l] : 0.0;
    sink.step(sc, c + static_cast<int32_t>(l), true, [](double, int32_t) {});
    sc = nx;
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  sink.finish(out, nout);
  if (l == 0) { ticks[0] = t1 - t0; ticks[1] = c1 - c0; }
}
}  // namespace wiser

namespace wiser {
// the replay heap walked as uniform scalar code over lane registers (readlane
// reads, lane-select writes): the form measured in-kernel in r05ae
struct LaneHeapB {
  uint32_t lo = 0, hi = 0;
  int32_t hd = 0;
  uint32_t n = 0;
  __device__ __forceinline__ double at(uint32_t i) const {
    const uint32_t a = __builtin_amdgcn_readlane(lo, static_cast<int>(i));
    const uint32_t b = __builtin_amdgcn_readlane(hi, static_cast<int>(i));
    return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(b) << 32) | a));
  }
  __device__ __forceinline__ int32_t doc(uint32_t i) const {
    return static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(hd), static_cast<int>(i)));
  }
  __device__ __forceinline__ void set(uint32_t i, double vs, int32_t vd) {
    const uint64_t u = static_cast<uint64_t>(__double_as_longlong(vs));
    const bool me = (threadIdx.x & 63) == i;
    lo = me ? static_cast<uint32_t>(u) : lo;
    hi = me ? static_cast<uint32_t>(u >> 32) : hi;
    hd = me ? vd : hd;
  }
  __device__ __forceinline__ void push_hole(uint32_t hole, double vs, int32_t vd) {
    while (hole > 0) {
      const uint32_t parent = (hole - 1) >> 1;
      const double ps = at(parent);
      if (!(ps > vs)) break;
      set(hole, ps, doc(parent));
      hole = parent;
    }
    set(hole, vs, vd);
  }
  __device__ __forceinline__ void push(double vs, int32_t vd) { push_hole(n, vs, vd); ++n; }
  __device__ __forceinline__ void pop() {
    if (n > 1) {
      const uint32_t len = n - 1;
      const double vs = at(len);
      const int32_t vd = doc(len);
      uint32_t hole = 0, child = 0;
      while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (at(child) > at(child - 1)) --child;
        set(hole, at(child), doc(child));
        hole = child;
      }
      if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        set(hole, at(child - 1), doc(child - 1));
        hole = child - 1;
      }
      push_hole(hole, vs, vd);
    }
    --n;
  }
};
struct LaneSink {
  LaneHeapB H;
  uint32_t k = 0;
  __device__ __forceinline__ void step(double sc, int32_t dc, bool valid) {
    const double top = H.n < k ? -1.0 : H.at(0);
    uint64_t cm = __ballot(valid && sc > top);
    while (cm) {
      const int fl = __builtin_ctzll(cm);
      cm &= cm - 1;
      const double sv = readlane_f64(sc, fl);
      const int32_t dv = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(dc), fl));
      if (H.n < k) H.push(sv, dv);
      else if (sv > H.at(0)) { H.pop(); H.push(sv, dv); }
    }
  }
};
__global__ void lane_bench_kernel(const double* vals, int n, uint32_t k, uint64_t* ticks, double* out) {
  LaneSink sink;
  sink.k = uni(k);
  const uint32_t l = threadIdx.x & 63;
  double sc = vals[l];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int c = 0; c < n; c += 64) {
    const double nx = c + 64 < n ? vals[c + 64 + l] : 0.0;
    sink.step(sc, c + static_cast<int32_t>(l), true);
    sc = nx;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  out[l] = sink.H.at(0) + sink.H.lo;
  if (l == 0) ticks[0] = t1 - t0;
}
}  // namespace wiser

namespace wiser {
// Where an insertion's cycles go: the candidate loop alone
// (readlanes and the top test, no heap operation), pushes alone (into a heap
// emptied every k), pops alone (of a heap refilled every k), and the LDS heap
// of the wide queries (LdsHeapSink: a wave-uniform walk over LDS) at k = 10.
__global__ void parts_bench_kernel(const double* vals, int n, uint32_t k, uint32_t mode, uint64_t* ticks,
                                   double* out) {
  __shared__ double s_hs[kMaxKWide];
  __shared__ int32_t s_hd[kMaxKWide];
  k = uni(k);
  mode = uni(mode);
  const uint32_t l = threadIdx.x & 63;
  double sc = vals[l];
  WaveHeap H;
  LdsHeapSink L;
  L.hs = s_hs;
  L.hd = s_hd;
  L.k = k;
  double acc = 0.0;
  uint32_t cnt = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int c = 0; c < n; c += 64) {
    const double nx = c + 64 < n ? vals[c + 64 + l] : 0.0;
    if (mode == 3) {
      L.step(sc, c + static_cast<int32_t>(l), true, [](double, int32_t) {});
    } else {
      const double top = H.n < k ? -1.0 : H.at(0);
      uint64_t cm = __ballot(sc > top || mode != 0);
      while (cm) {
        const int fl = __builtin_ctzll(cm);
        cm &= cm - 1;
        const double sv = readlane_f64(sc, fl);
        const int32_t dv = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(c + l), fl));
        if (mode == 0) {            // the loop alone
          acc += sv;
          ++cnt;
        } else if (mode == 1) {     // pushes alone
          if (H.n == k) H.n = 0;
          H.push(sv, dv);
        } else {                    // pops alone (refilled by pushes, not timed apart)
          if (H.n <= 1) {
            for (uint32_t i = 0; i < k; ++i) H.push(sv + i, dv);
          }
          H.pop();
        }
      }
    }
    sc = nx;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  out[l] = acc + H.hs + cnt + (L.n ? L.at(0) : 0.0);
  if (l == 0) ticks[0] = t1 - t0;
}
}  // namespace wiser

int main() {
  const int n = 64 * 64;   // 4,096 events, rising: 4,096 insertions
  std::vector<double> h(n);
  for (int i = 0; i < n; ++i) h[i] = 1.0 + i * 1e-3;
  double* d; uint64_t* t; wiser::HitDev* o; int32_t* no;
  hipMalloc(&d, n * sizeof(double)); hipMalloc(&t, 16); hipMalloc(&o, 64 * sizeof(wiser::HitDev)); hipMalloc(&no, 4);
  hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
  for (uint32_t k : {10u, 64u}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(wiser::heap_bench_kernel, dim3(1), dim3(64), 0, 0, d, n, k, t, o, no);
      uint64_t ht[2];
      hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost);
      std::printf("k %u: %d insertions, %.3f us (%.1f ns each), %.1f s_memtime ticks each\n", k, n,
                  ht[0] / 100.0, ht[0] * 10.0 / n, static_cast<double>(ht[1]) / n);
    }
  }
  double* od; hipMalloc(&od, 64 * sizeof(double));
  {
    std::vector<double> h2(n);
    for (int i = 0; i < n; ++i) h2[i] = 1.0 + i * 1e-3;
    hipMemcpy(d, h2.data(), n * sizeof(double), hipMemcpyHostToDevice);
    const char* names[] = {"candidate loop alone", "pushes alone", "pops alone (+1 refill push per pop... see note)",
                           "LDS heap (LdsHeapSink)"};
    for (uint32_t mode = 0; mode < 4; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(wiser::parts_bench_kernel, dim3(1), dim3(64), 0, 0, d, n, 10u, mode, t, od);
        uint64_t ht[2];
        hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost);
        std::printf("parts k 10 mode %u (%s): %.1f ns per event\n", mode, names[mode], ht[0] * 10.0 / n);
      }
    }
  }
  for (uint32_t k : {10u, 64u}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(wiser::lane_bench_kernel, dim3(1), dim3(64), 0, 0, d, n, k, t, od);
      uint64_t ht[2];
      hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost);
      std::printf("lane heap k %u: %.1f ns per insertion\n", k, ht[0] * 10.0 / n);
    }
  }
  return 0;
}
