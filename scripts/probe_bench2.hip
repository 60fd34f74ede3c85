// Diagnostics only: a two-level probe against the one-level 16-byte bitmap
// probe (96 docs per entry), on the lean kernel's pattern (scripts/probe_bench.hip).
// Level 1 is a summary of one bit per G docs (32-bit words); a posting whose
// summary bit is set -- with probability 1-(1-rho)^G for a list of density rho,
// drawn here by a hash -- then loads its 16-byte entry (level 2) one iteration
// later; the others read a shared dummy entry.  Loads of block j are consumed
// one iteration after they are issued at each level.
// Usage: probe_bench2 GAP RHO G [POOL_MB] [WGS_PER_CU]   (G = 0: one level)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

constexpr uint32_t kSpanDocs = 5500000;
constexpr uint32_t kBlocks = 63;
constexpr uint32_t kEnts = kSpanDocs / 96 + 1;
constexpr uint64_t kRegion = static_cast<uint64_t>(kEnts) * 16;

__global__ __launch_bounds__(256) void probe2_kernel(const uint8_t* __restrict__ pool, const uint32_t* __restrict__ sum,
                                                     uint32_t nregions, uint32_t gap, uint32_t g, uint32_t pass_thr,
                                                     uint32_t items, uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t swords = g ? kSpanDocs / (32u * g) + 1 : 1;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < items; ++it) {
    const uint32_t h = mix(wave * 7919u + it * 104729u);
    const uint32_t reg = h % nregions;
    const uint4* bm = reinterpret_cast<const uint4*>(pool + static_cast<uint64_t>(reg) * kRegion);
    const uint32_t* sm = sum + static_cast<uint64_t>(reg) * swords;
    const uint32_t need = kBlocks * 128u * gap;
    const uint32_t start = need < kSpanDocs ? mix(h) % (kSpanDocs - need) : 0u;
    uint32_t s0 = 0, s1 = 0, d0p = 0, d1p = 0;   // level 1 in flight and its docs
    uint4 e0 = make_uint4(0, 0, 0, 0), e1 = make_uint4(0, 0, 0, 0);
    for (uint32_t j = 0; j <= kBlocks + 1; ++j) {
      acc += e0.x ^ e1.w;   // level 2 of block j-2
      if (g) {
        // level 1 of block j-1 -> level 2 issue
        const bool p0 = j >= 1 && (mix(d0p ^ s0 ^ 0x9e3779b9u) < pass_thr);
        const bool p1 = j >= 1 && (mix(d1p ^ s1 ^ 0x85ebca6bu) < pass_thr);
        e0 = bm[p0 ? (d0p / 96u) % kEnts : 0u];
        e1 = bm[p1 ? (d1p / 96u) % kEnts : 0u];
      }
      if (j >= kBlocks) continue;
      const uint32_t q0 = j * 128u + 2 * l, q1 = q0 + 1;
      const uint32_t d0 = start + q0 * gap + mix(q0 ^ h) % gap;
      const uint32_t d1 = start + q1 * gap + mix(q1 ^ h) % gap;
      if (g) {
        s0 = sm[(d0 / (32u * g)) % swords];
        s1 = sm[(d1 / (32u * g)) % swords];
        d0p = d0; d1p = d1;
      } else {
        e0 = bm[(d0 / 96u) % kEnts];
        e1 = bm[(d1 / 96u) % kEnts];
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint32_t gap = argc > 1 ? std::atoi(argv[1]) : 183;
  const double rho = argc > 2 ? std::atof(argv[2]) : 0.01;
  const uint32_t g = argc > 3 ? std::atoi(argv[3]) : 4;
  const uint64_t pool_mb = argc > 4 ? std::atoll(argv[4]) : 8192;
  const int wgs = argc > 5 ? std::atoi(argv[5]) : 5;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t nregions = static_cast<uint32_t>((pool_mb << 20) / kRegion);
  if (nregions == 0) nregions = 1;
  const uint32_t swords = g ? kSpanDocs / (32u * g) + 1 : 1;
  uint8_t* pool;
  uint32_t *sum, *out;
  CHECK(hipMalloc(&pool, nregions * kRegion + 64));
  CHECK(hipMemset(pool, 0x5a, nregions * kRegion + 64));
  CHECK(hipMalloc(&sum, static_cast<uint64_t>(nregions) * swords * 4 + 64));
  CHECK(hipMemset(sum, 0x33, static_cast<uint64_t>(nregions) * swords * 4 + 64));
  CHECK(hipMalloc(&out, 64));
  const double pass = g ? 1.0 - std::pow(1.0 - rho, static_cast<double>(g)) : 1.0;
  const uint32_t thr = static_cast<uint32_t>(std::min(4294967295.0, pass * 4294967296.0));
  const uint32_t items = 8;
  const dim3 grid(cus * wgs), block(256);
  auto run = [&]() { probe2_kernel<<<grid, block>>>(pool, sum, nregions, gap, g, thr, items, out); };
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
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
  std::printf("{\"gap\": %u, \"rho\": %g, \"g\": %u, \"pass\": %.3f, \"pool_mb\": %llu, \"wgs_per_cu\": %d, "
              "\"ms\": %.4f, \"cu_cycles_per_block_2p4ghz\": %.1f}\n",
              gap, rho, g, pass, static_cast<unsigned long long>(pool_mb), wgs, best,
              best * 1e-3 * 2.4e9 * cus / blocks);
  return 0;
}
