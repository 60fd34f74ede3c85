// Calibration of the L2 -> fabric read counters (TCC_EA0_RDREQ*) on gfx950 for
// the engine's access shapes (MI355X_MICROARCH.md, HBM section: "calibrate on
// a known byte count in your own access pattern").  Each kernel is launched
// once over a 1 GiB buffer (past the 256 MiB Infinity Cache) and reads a
// known set of 128-byte lines:
//   stream16   every byte once, 16 B per lane, coalesced        (bytes known)
//   gather4    one 4 B load per lane, each lane a distinct line  (lines known)
//   gather8    the same with an 8 B load (the rank-bitmap probe)
//   gather12   three dwords (the pair_words load of a pack)
//   halves4    two lanes per line, at byte 0 and byte 64
// The program prints the known counts as one JSON line; rocprofv3 --pmc
// passes give the counters per dispatch (scripts/pmc_bytes.py pairs them).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void stream16(const uint4* __restrict__ p, size_t n, uint4* __restrict__ out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x9E3779B9u && acc.y == 1u) out[0] = acc;   // never true: keeps the loads
}

// line of lane i: a bijection of [0, n_lines) (n_lines a power of two)
__device__ __forceinline__ size_t line_of(size_t i, size_t n_lines) {
  return (i * 0x9E3779B1ull) & (n_lines - 1);
}

template <int W>
__global__ void gather(const uint32_t* __restrict__ base, size_t n_lines, size_t n, uint32_t off_dw,
                       uint32_t* __restrict__ out) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  const uint32_t* a = base + line_of(i, n_lines) * 32 + off_dw;
  uint32_t v;
  if (W == 1) v = a[0];
  else if (W == 2) { const uint2 x = *reinterpret_cast<const uint2*>(a); v = x.x ^ x.y; }
  else v = a[0] ^ a[1] ^ a[2];
  if (v == 0x9E3779B9u) out[0] = v;
}

__global__ void halves4(const uint32_t* __restrict__ base, size_t n_lines, size_t n,
                        uint32_t* __restrict__ out) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i >= 2 * n) return;
  const uint32_t v = base[line_of(i >> 1, n_lines) * 32 + (i & 1) * 16];
  if (v == 0x9E3779B9u) out[0] = v;
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
  } while (0)

int main() {
  const size_t bytes = size_t{1} << 30, n_lines = bytes / 128, n = n_lines / 2;
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, bytes));
  CK(hipDeviceSynchronize());
  const uint32_t* b = static_cast<const uint32_t*>(buf);
  const int T = 256;
  const unsigned G = static_cast<unsigned>((n + T - 1) / T);
  hipLaunchKernelGGL(stream16, dim3(4096), dim3(T), 0, 0, static_cast<const uint4*>(buf), bytes / 16,
                     reinterpret_cast<uint4*>(out));
  hipLaunchKernelGGL(gather<1>, dim3(G), dim3(T), 0, 0, b, n_lines, n, 0u, out);
  hipLaunchKernelGGL(gather<2>, dim3(G), dim3(T), 0, 0, b, n_lines, n, 2u, out);
  hipLaunchKernelGGL(gather<3>, dim3(G), dim3(T), 0, 0, b, n_lines, n, 5u, out);
  hipLaunchKernelGGL(halves4, dim3(2 * G), dim3(T), 0, 0, b, n_lines, n, out);
  CK(hipDeviceSynchronize());
  std::printf("{\"buffer_bytes\": %zu, \"stream16_bytes\": %zu, \"gather_lines\": %zu, "
              "\"halves4_lines\": %zu, \"halves4_loads\": %zu}\n",
              bytes, bytes, n, n, 2 * n);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
