// Micro-benchmark (diagnostics): cycles per RankDoc insertion of the wave heap
// (kernels.hip WaveHeap) against the previous scalar-walk form, one wave per
// workgroup, grid of 1 and of 4096 workgroups, k = 10, 256 insertions of
// increasing scores (every one replaces the top).  Built by hand:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I wiser_amd/csrc scripts/heap_bench.hip
#include "../wiser_amd/csrc/kernels.hip"

#include <cstdio>

namespace wiser {
#include "serial_heap.inc"

template <class H>
__global__ __launch_bounds__(64) void heap_bench_kernel(uint64_t* cycles, double* sink, int n_ins) {
  H h;
  const uint32_t k = 10;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n_ins; ++i) {
    const double sv = 1.0 + i * 0.001 + (blockIdx.x & 7) * 1e-6;
    if (h.n < k) h.push(sv, i);
    else if (sv > h.at(0)) { h.pop(); h.push(sv, i); }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = h.hs + h.hd;
}
}  // namespace wiser

int main() {
  using namespace wiser;
  uint64_t* cyc;
  double* sink;
  const int grid = 4096, n_ins = 256;
  (void)hipMalloc(&cyc, sizeof(uint64_t) * grid);
  (void)hipMalloc(&sink, sizeof(double) * grid * 64);
  uint64_t h[grid];
  for (int form = 0; form < 2; ++form)
    for (int g : {1, grid}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (form == 0) hipLaunchKernelGGL(heap_bench_kernel<WaveHeap>, dim3(g), dim3(64), 0, 0, cyc, sink, n_ins);
        else hipLaunchKernelGGL(heap_bench_kernel<WaveHeapSerial>, dim3(g), dim3(64), 0, 0, cyc, sink, n_ins);
        (void)hipDeviceSynchronize();
      }
      (void)hipMemcpy(h, cyc, sizeof(uint64_t) * g, hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < g; ++i) s += h[i];
      std::printf("%s heap, grid %4d: %.0f cycles per insertion\n", form == 0 ? "wave-parallel" : "scalar-walk",
                  g, s / g / n_ins);
    }
  return 0;
}
