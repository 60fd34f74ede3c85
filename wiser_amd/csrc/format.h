// Vacuum on-disk format: constants and byte-level codecs shared by the host
// side of the HIP engine (index writer, index loader, work planner).
//
// Layout contract (restated from the reference, file:line in
// /root/reference/src/qq_mem/src):
//   magic bytes ............................ types.h:44-52
//   LEB128 varint (0 -> one 0x00 byte) ...... utils.cc:257-270, utils.h:249-266
//   1-byte lossy length "Char4" ............. utils.h:301-329
//   128-value bit pack, value j at bit j*b
//   of an LSB-first little-endian stream .... packed_value.h:87-128,
//                                              LittleIntPacker/scripts/turbopacking32.py:83-112
//   VInts blob = 0x9B | varint nbytes | data packed_value.h:372-397
//   skip list row = 7 varints, delta coded .. flash_containers.h:282-299,354-391
//   .tip entry = u32 len | bytes | i64 (pages<<48 | off)
//                                              file_dumper.h:82-86, flash_engine_dumper.h:44-49
//   .doc_length = i32 n | f64 avg | n*(i32 id, i8 char4)
//                                              doc_length_store.h:140-161
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace wiser {

constexpr uint8_t kSkipListMagic = 0xA3;
constexpr uint8_t kPostingListMagic = 0xF4;
constexpr uint8_t kPackMagic = 0xD6;
constexpr uint8_t kVIntsMagic = 0x9B;
constexpr uint8_t kVacuumMagic = 0x88;
constexpr uint8_t kBloomSkipListMagic = 0xA4;   // types.h:44
constexpr uint8_t kBloomBoxMagic = 0xF5;        // types.h:48
constexpr int kPackSize = 128;          // values per pack == postings per skip row
constexpr int kVacuumHeaderBytes = 100; // first posting list starts here

// ---------------------------------------------------------------- varints --
inline void put_varint(std::string* out, uint64_t v) {
  do {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if (v) b |= 0x80;
    out->push_back(static_cast<char>(b));
  } while (v);
}

inline int varint_len(uint64_t v) {
  int n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}

// Returns bytes consumed; never reads past `end` (returns 0 on truncation).
inline int get_varint(const uint8_t* p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  int i = 0;
  while (p + i < end && i < 10) {
    uint8_t b = p[i];
    r |= static_cast<uint64_t>(b & 0x7f) << (7 * i);
    ++i;
    if (!(b & 0x80)) { *v = r; return i; }
  }
  return 0;
}

// ------------------------------------------------------- lossy doc length --
inline int num_bits(uint32_t v) {
  int n = 0;
  while (v) { v >>= 1; ++n; }
  return n;
}

inline uint8_t length_to_char4(uint32_t len) {
  if (len < 8) return static_cast<uint8_t>(len);
  int shift = num_bits(len) - 4;
  uint32_t mant = (len >> shift) & 0x07;
  return static_cast<uint8_t>(mant | ((shift + 1) << 3));
}

inline uint32_t char4_to_length(uint8_t c) {
  uint32_t mant = c & 0x07;
  int shift = (c >> 3) - 1;
  if (shift < 0) return mant;
  return (mant | 0x08) << shift;  // wraps to 0 for shift >= 29, as the reference
}

// ------------------------------------------------------------ bit packing --
// Serialised pack: 0xD6 | b | 16*b data bytes, b in [1, 32].
inline int pack_bits_for(const uint32_t* v, int n) {
  int b = 1;
  for (int i = 0; i < n; ++i) {
    int nb = num_bits(v[i]);
    if (nb > b) b = nb;
  }
  return b;
}

inline void append_pack(std::string* out, const uint32_t* v /*128*/) {
  const int b = pack_bits_for(v, kPackSize);
  out->push_back(static_cast<char>(kPackMagic));
  out->push_back(static_cast<char>(b));
  // value j at bits [j*b, j*b+b) of a little-endian stream of 64-bit words
  uint64_t w[2 * 32 + 1] = {0};
  for (int j = 0; j < kPackSize; ++j) {
    const uint32_t bit = static_cast<uint32_t>(j) * b;
    const uint64_t val = v[j];
    const uint32_t at = bit >> 6, sh = bit & 63;
    w[at] |= val << sh;
    if (sh + b > 64) w[at + 1] |= val >> (64 - sh);
  }
  const size_t base = out->size();
  out->resize(base + 16 * b, 0);
  std::memcpy(&(*out)[base], w, 16 * b);   // (x86 and gfx950 hosts: little-endian)
}

inline void append_vints(std::string* out, const uint32_t* v, int n) {
  std::string body;
  for (int i = 0; i < n; ++i) put_varint(&body, v[i]);
  out->push_back(static_cast<char>(kVIntsMagic));
  put_varint(out, body.size());
  out->append(body);
}

// Size in bytes of the blob (pack or VInts) starting at p.
inline uint64_t blob_bytes(const uint8_t* p, const uint8_t* end) {
  if (p >= end) return 0;
  if (p[0] == kPackMagic) return 2 + 16ull * p[1];
  if (p[0] == kVIntsMagic) {
    uint64_t nb = 0;
    int l = get_varint(p + 1, end, &nb);
    if (!l) return 0;
    return 1 + l + nb;
  }
  return 0;
}

// Offsets packed in .tip: (n_pages_of_prefetch_zone << 48) | posting list start.
inline int64_t encode_tip_value(uint32_t pages, uint64_t off) {
  return static_cast<int64_t>((static_cast<uint64_t>(pages) << 48) | off);
}
inline uint64_t tip_offset(int64_t v) {
  return static_cast<uint64_t>(v) & ((1ull << 48) - 1);
}
inline uint32_t tip_pages(int64_t v) { return static_cast<uint64_t>(v) >> 48; }

}  // namespace wiser
