// Diagnostics only: the rate of the lean kernel's rank-bitmap probe pattern
// on its own.  Every wave walks "items" of 63 driver blocks of 128 postings,
// posting p of a block at doc start + p*G + jitter(p) (jitter < G, so doc
// order holds), and probes a 1.375 MB bitmap (8 bytes per 32 docs, the C3
// stand-in's span) picked per item from a large pool, as the lean kernel probes
// O1.  Loads of block j are consumed in iteration j+1 (the kernel's pipeline
// depth).  Layouts: 0 = lane l probes postings 2l and 2l+1 (the lean kernel's
// pair decode), 1 = lane l probes postings l and l+64 (each instruction covers
// 64 consecutive postings, so it touches about half as many distinct lines).
// Usage: probe_bench LAYOUT GAP POOL_MB [WGS_PER_CU] [VALU]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

constexpr uint32_t kSpanWords = 171875;   // 5.5 M docs / 32
constexpr uint32_t kBlocks = 63;

template <int kLayout>
__global__ __launch_bounds__(256) void probe_kernel(const uint2* __restrict__ pool, uint32_t nregions,
                                                    uint32_t gap, uint32_t items, uint32_t valu,
                                                    uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t acc = 0;
  for (uint32_t it = 0; it < items; ++it) {
    const uint32_t h = mix(wave * 7919u + it * 104729u);
    const uint2* bm = pool + static_cast<uint64_t>(h % nregions) * kSpanWords;
    const uint32_t span_docs = kSpanWords * 32u;
    const uint32_t need = kBlocks * 128u * gap;
    const uint32_t start = need < span_docs ? mix(h) % (span_docs - need) : 0u;
    uint2 e0 = make_uint2(0, 0), e1 = make_uint2(0, 0);
    float f = static_cast<float>(l);
    for (uint32_t j = 0; j <= kBlocks; ++j) {
      // consume the previous block's probes
      acc += e0.x ^ e1.y;
      if (j == kBlocks) break;
      uint32_t p0, p1;
      if (kLayout == 0) { p0 = 2 * l; p1 = 2 * l + 1; }
      else { p0 = l; p1 = l + 64; }
      const uint32_t q0 = j * 128u + p0, q1 = j * 128u + p1;
      const uint32_t d0 = start + q0 * gap + mix(q0 ^ h) % gap;
      const uint32_t d1 = start + q1 * gap + mix(q1 ^ h) % gap;
      e0 = bm[(d0 / 32u) % kSpanWords];
      e1 = bm[(d1 / 32u) % kSpanWords];
      for (uint32_t v = 0; v < valu; ++v) f = f * 1.0001f + 0.5f;   // VALU filler
    }
    acc += static_cast<uint32_t>(f) & 1u;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const int layout = argc > 1 ? std::atoi(argv[1]) : 0;
  const uint32_t gap = argc > 2 ? std::atoi(argv[2]) : 183;
  const uint64_t pool_mb = argc > 3 ? std::atoll(argv[3]) : 8192;
  const int wgs = argc > 4 ? std::atoi(argv[4]) : 5;
  const uint32_t valu = argc > 5 ? std::atoi(argv[5]) : 0;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const uint64_t region_bytes = static_cast<uint64_t>(kSpanWords) * 8;
  uint32_t nregions = static_cast<uint32_t>((pool_mb << 20) / region_bytes);
  if (nregions == 0) nregions = 1;
  uint2* pool;
  uint32_t* out;
  CHECK(hipMalloc(&pool, nregions * region_bytes + 64));
  CHECK(hipMemset(pool, 0x5a, nregions * region_bytes + 64));
  CHECK(hipMalloc(&out, 64));
  const uint32_t items = 8;
  const dim3 grid(cus * wgs), block(256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto run = [&]() {
    if (layout == 0) probe_kernel<0><<<grid, block>>>(pool, nregions, gap, items, valu, out);
    else probe_kernel<1><<<grid, block>>>(pool, nregions, gap, items, valu, out);
  };
  run();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a));
    run();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double blocks = static_cast<double>(grid.x) * 4 * items * kBlocks;
  std::printf("{\"layout\": %d, \"gap\": %u, \"pool_mb\": %llu, \"wgs_per_cu\": %d, \"valu\": %u, "
              "\"ms\": %.4f, \"driver_blocks\": %.0f, \"gblocks_per_s\": %.4f, \"cu_cycles_per_block_2p4ghz\": %.1f}\n",
              layout, gap, static_cast<unsigned long long>(pool_mb), wgs, valu, best, blocks,
              blocks / best / 1e6, best * 1e-3 * 2.4e9 * cus / blocks);
  return 0;
}
