// Two-way phrase bloom filters of the Vacuum layout (writer side).
//
// Each posting of a list may carry two small bloom filters over the terms that
// follow ("end") and precede ("begin") the list's term in that doc
// (BloomFilterStore::Add, bloom_filter.h:277-300; fixture columns "bloom" /
// "bloom_before" of testdata/iter_test_3_docs_tf_bi-bloom).  The filter is
// libbloom's (src/libbloom/bloom.c:48-75,84-115) sized for a fixed number of
// entries at a float error ratio, hashed with MurmurHash2
// (libbloom/murmur2/MurmurHash2.c:15-64).  The query path only prunes with
// them (QueryProcessor::IsPossibleToPresent, query_processing.h:766-884); the
// GPU phrase path applies the same check before reading positions
// (HostImage::blm, kernels.hip bloom_may).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace wiser {

// MurmurHash2 (little-endian 4-byte reads, as on x86-64)
inline uint32_t murmurhash2(const void* key, int len, uint32_t seed) {
  const uint32_t m = 0x5bd1e995;
  const int r = 24;
  uint32_t h = seed ^ static_cast<uint32_t>(len);
  const unsigned char* data = static_cast<const unsigned char*>(key);
  while (len >= 4) {
    uint32_t k;
    std::memcpy(&k, data, 4);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
    data += 4;
    len -= 4;
  }
  switch (len) {
    case 3: h ^= static_cast<uint32_t>(data[2]) << 16; [[fallthrough]];
    case 2: h ^= static_cast<uint32_t>(data[1]) << 8; [[fallthrough]];
    case 1: h ^= data[0]; h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

// bloom_init / bloom_set / bloom_bytes sizing (bloom.c:84-138); `error` is the
// float ratio of the Vacuum header widened to double, as the reference does.
struct BloomShape {
  int bits = 0, bytes = 0, hashes = 0;
  BloomShape(int entries, float ratio) {
    const double error = static_cast<double>(ratio);
    const double bpe = -(std::log(error) / 0.480453013918201);
    bits = static_cast<int>(static_cast<double>(entries) * bpe);
    bytes = bits % 8 ? bits / 8 + 1 : bits / 8;
    hashes = static_cast<int>(std::ceil(0.693147180559945 * bpe));
  }
};

// bloom_add (bloom.c:48-75 with add = 1) into a bit array of shape s
inline void bloom_add(const BloomShape& s, std::string* bf, const std::string& elem) {
  const uint32_t a = murmurhash2(elem.data(), static_cast<int>(elem.size()), 0x9747b28c);
  const uint32_t b = murmurhash2(elem.data(), static_cast<int>(elem.size()), a);
  for (int i = 0; i < s.hashes; ++i) {
    const uint32_t x = (a + static_cast<uint32_t>(i) * b) % static_cast<uint32_t>(s.bits);
    (*bf)[x >> 3] = static_cast<char>(static_cast<uint8_t>((*bf)[x >> 3]) | (1u << (x % 8)));
  }
}

// The bit array of one posting: empty when the term has no neighbour on that
// side (BloomFilterStore::Add keeps no filter for an empty list, and the box
// bitmap then marks the posting absent).
inline std::string make_bloom(const BloomShape& s, const std::vector<std::string>& elems) {
  if (elems.empty()) return std::string();
  std::string bf(static_cast<size_t>(s.bytes), '\0');
  for (const auto& e : elems) bloom_add(s, &bf, e);
  return bf;
}

}  // namespace wiser
