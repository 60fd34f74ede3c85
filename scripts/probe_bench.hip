// Diagnostics only: the rate of the lean kernel's rank-bitmap probe pattern
// on its own.  Every wave walks "items" of 63 driver blocks of 128 postings,
// posting p of a block at doc start + p*G + jitter(p) (jitter < G, so doc
// order holds), and probes a bitmap over 5.5 M docs (the C3 stand-in's span)
// picked per item from a large pool, as the lean kernel probes O1.  Loads of
// block j are consumed in iteration j+1 (the kernel's pipeline depth).
// Layouts: 0 = lane l probes postings 2l and 2l+1 (the lean kernel's pair
// decode), 1 = lane l probes postings l and l+64.
// Element forms (FORM): 0 = 8 B per 32 docs (the rank bitmap), 1 = 8 B per 48
// docs, 2 = 16 B per 112 docs, 3 = 8 B per 32 docs read non-temporal, 4 = 8 B
// per 32 docs from uncached (fine-grained) memory.
// Usage: probe_bench LAYOUT GAP POOL_MB [WGS_PER_CU] [VALU] [FORM]
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

constexpr uint32_t kSpanDocs = 5500000;
constexpr uint32_t kBlocks = 63;

template <int kForm> struct FormOf;
template <> struct FormOf<0> { static constexpr uint32_t docs = 32, bytes = 8; };
template <> struct FormOf<1> { static constexpr uint32_t docs = 48, bytes = 8; };
template <> struct FormOf<2> { static constexpr uint32_t docs = 112, bytes = 16; };
template <> struct FormOf<3> { static constexpr uint32_t docs = 32, bytes = 8; };
template <> struct FormOf<4> { static constexpr uint32_t docs = 32, bytes = 8; };

__host__ __device__ constexpr uint64_t region_bytes(uint32_t docs, uint32_t bytes) {
  return (static_cast<uint64_t>(kSpanDocs / docs) + 1) * bytes;
}

template <int kLayout, int kForm>
__global__ __launch_bounds__(256) void probe_kernel(const uint8_t* __restrict__ pool, uint32_t nregions,
                                                    uint32_t gap, uint32_t items, uint32_t valu,
                                                    uint32_t* __restrict__ out) {
  using F = FormOf<kForm>;
  const uint32_t l = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nelem = kSpanDocs / F::docs + 1;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < items; ++it) {
    const uint32_t h = mix(wave * 7919u + it * 104729u);
    const uint8_t* bm = pool + static_cast<uint64_t>(h % nregions) * region_bytes(F::docs, F::bytes);
    const uint32_t need = kBlocks * 128u * gap;
    const uint32_t start = need < kSpanDocs ? mix(h) % (kSpanDocs - need) : 0u;
    uint4 e0 = make_uint4(0, 0, 0, 0), e1 = make_uint4(0, 0, 0, 0);
    float f = static_cast<float>(l);
    for (uint32_t j = 0; j <= kBlocks; ++j) {
      acc += e0.x ^ e1.y ^ e0.z ^ e1.w;   // consume the previous block's probes
      if (j == kBlocks) break;
      uint32_t p0, p1;
      if (kLayout == 0) { p0 = 2 * l; p1 = 2 * l + 1; }
      else { p0 = l; p1 = l + 64; }
      const uint32_t q0 = j * 128u + p0, q1 = j * 128u + p1;
      const uint32_t d0 = start + q0 * gap + mix(q0 ^ h) % gap;
      const uint32_t d1 = start + q1 * gap + mix(q1 ^ h) % gap;
      const uint32_t i0 = (d0 / F::docs) % nelem, i1 = (d1 / F::docs) % nelem;
      if (F::bytes == 16) {
        e0 = reinterpret_cast<const uint4*>(bm)[i0];
        e1 = reinterpret_cast<const uint4*>(bm)[i1];
      } else if (kForm == 3) {
        const uint64_t a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(bm) + i0);
        const uint64_t b = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(bm) + i1);
        e0 = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), 0, 0);
        e1 = make_uint4(static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32), 0, 0);
      } else {
        const uint2 a = reinterpret_cast<const uint2*>(bm)[i0];
        const uint2 b = reinterpret_cast<const uint2*>(bm)[i1];
        e0 = make_uint4(a.x, a.y, 0, 0);
        e1 = make_uint4(b.x, b.y, 0, 0);
      }
      for (uint32_t v = 0; v < valu; ++v) f = f * 1.0001f + 0.5f;   // VALU filler
    }
    acc += static_cast<uint32_t>(f) & 1u;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int kLayout, int kForm>
void launch(dim3 grid, const uint8_t* pool, uint32_t nregions, uint32_t gap, uint32_t items, uint32_t valu,
            uint32_t* out) {
  probe_kernel<kLayout, kForm><<<grid, dim3(256)>>>(pool, nregions, gap, items, valu, out);
}

int main(int argc, char** argv) {
  const int layout = argc > 1 ? std::atoi(argv[1]) : 0;
  const uint32_t gap = argc > 2 ? std::atoi(argv[2]) : 183;
  const uint64_t pool_mb = argc > 3 ? std::atoll(argv[3]) : 8192;
  const int wgs = argc > 4 ? std::atoi(argv[4]) : 5;
  const uint32_t valu = argc > 5 ? std::atoi(argv[5]) : 0;
  const int form = argc > 6 ? std::atoi(argv[6]) : 0;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  static const uint32_t docs[] = {32, 48, 112, 32, 32}, bytes[] = {8, 8, 16, 8, 8};
  const uint64_t rb = region_bytes(docs[form], bytes[form]);
  uint32_t nregions = static_cast<uint32_t>((pool_mb << 20) / rb);
  if (nregions == 0) nregions = 1;
  uint8_t* pool;
  uint32_t* out;
  if (form == 4) CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&pool), nregions * rb + 64,
                                             hipDeviceMallocUncached));
  else CHECK(hipMalloc(&pool, nregions * rb + 64));
  CHECK(hipMemset(pool, 0x5a, nregions * rb + 64));
  CHECK(hipMalloc(&out, 64));
  const uint32_t items = 8;
  const dim3 grid(cus * wgs);
  auto run = [&]() {
#define L(LA, FO) launch<LA, FO>(grid, pool, nregions, gap, items, valu, out)
    if (layout == 0) {
      switch (form) { case 0: L(0, 0); break; case 1: L(0, 1); break; case 2: L(0, 2); break;
                      case 3: L(0, 3); break; default: L(0, 4); }
    } else {
      switch (form) { case 0: L(1, 0); break; case 1: L(1, 1); break; case 2: L(1, 2); break;
                      case 3: L(1, 3); break; default: L(1, 4); }
    }
#undef L
  };
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
  std::printf("{\"layout\": %d, \"form\": %d, \"docs_per_elem\": %u, \"elem_bytes\": %u, \"gap\": %u, "
              "\"pool_mb\": %llu, \"wgs_per_cu\": %d, \"valu\": %u, \"ms\": %.4f, \"driver_blocks\": %.0f, "
              "\"gblocks_per_s\": %.4f, \"cu_cycles_per_block_2p4ghz\": %.1f}\n",
              layout, form, docs[form], bytes[form], gap, static_cast<unsigned long long>(pool_mb), wgs, valu,
              best, blocks, blocks / best / 1e6, best * 1e-3 * 2.4e9 * cus / blocks);
  return 0;
}
