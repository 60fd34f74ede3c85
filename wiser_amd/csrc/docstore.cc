// Chunked LZ4 doc store (see docstore.h).
#include "docstore.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <iterator>
#include <stdexcept>

#include "format.h"

extern "C" {
int LZ4_compress_default(const char* src, char* dst, int src_size, int dst_capacity);
int LZ4_decompress_safe(const char* src, char* dst, int compressed_size, int dst_capacity);
}

namespace wiser {

constexpr uint8_t kDocMagic = 0x33;   // COMPRESSED_DOC_MAGIC (types.h:41)

void DocStoreWriter::open(const std::string& dir, bool align) {
  dir_ = dir;
  align_ = align;
  ::mkdir(dir.c_str(), 0755);   // (the index writer may not have created it yet)
  fdt_.open(dir + "/my.fdt", std::ios::binary | std::ios::trunc);
  if (!fdt_) throw std::runtime_error("cannot write my.fdt");
  at_ = 0;
  offs_.clear();
  buf_.assign(kBufBytes, 0);
}

void DocStoreWriter::add(const std::string& text) {
  // CompressText (doc_store.h:83-103): LZ4 chunks of at most half the buffer
  std::string sizes, blocks;
  size_t done = 0;
  uint64_t n_chunks = 0;
  while (done < text.size()) {
    const size_t len = std::min(text.size() - done, static_cast<size_t>(kBufBytes / 2));
    const int got = LZ4_compress_default(text.data() + done, buf_.data(), static_cast<int>(len), kBufBytes);
    if (got <= 0) throw std::runtime_error("LZ4 compression failed");
    put_varint(&sizes, static_cast<uint64_t>(got));
    blocks.append(buf_.data(), got);
    done += len;
    ++n_chunks;
  }
  std::string rec(1, static_cast<char>(kDocMagic));
  put_varint(&rec, n_chunks);
  rec += sizes;
  rec += blocks;
  // DumpDocAligned (:327-341) with ShouldAlign (:72-77) as written
  const uint64_t off = at_;
  bool pad = false;
  if (align_) {
    const uint64_t kb = 1024, page = 4 * kb;
    const uint64_t whole = (rec.size() + page - 1) / page;
    const uint64_t shifted = ((off % 4) * kb + rec.size() + page - 1) / page;
    pad = shifted > whole;
  }
  if (pad) {
    const uint64_t to = (off / 4096 + 1) * 4096;
    const std::string zeros(to - off, '\0');
    fdt_.write(zeros.data(), static_cast<std::streamsize>(zeros.size()));
    at_ = to;
  }
  fdt_.write(rec.data(), static_cast<std::streamsize>(rec.size()));
  at_ += rec.size();
  offs_.push_back(static_cast<int64_t>((off << 1) | (pad ? 1u : 0u)));
}

void DocStoreWriter::close() {
  fdt_.close();
  std::ofstream fdx(dir_ + "/my.fdx", std::ios::binary | std::ios::trunc);
  if (!fdx) throw std::runtime_error("cannot write my.fdx");
  std::string hdr;   // DumpHeader (:306-318)
  put_varint(&hdr, offs_.size());
  put_varint(&hdr, static_cast<uint64_t>(kBufBytes));
  fdx.write(hdr.data(), static_cast<std::streamsize>(hdr.size()));
  fdx.write(reinterpret_cast<const char*>(offs_.data()),
            static_cast<std::streamsize>(offs_.size() * sizeof(int64_t)));
  if (!fdx) throw std::runtime_error("short write of my.fdx");
}

DocStore::~DocStore() {
  if (map_) munmap(map_, len_);
}

bool DocStore::open(const std::string& dir) {
  std::ifstream f(dir + "/my.fdx", std::ios::binary);
  if (!f) return false;
  const std::string raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const uint8_t* p = reinterpret_cast<const uint8_t*>(raw.data());
  const uint8_t* end = p + raw.size();
  uint64_t n = 0, bs = 0;
  int l = get_varint(p, end, &n);
  if (!l) throw std::runtime_error("my.fdx: bad header");
  p += l;
  l = get_varint(p, end, &bs);
  if (!l) throw std::runtime_error("my.fdx: bad header");
  p += l;
  if (static_cast<uint64_t>(end - p) < n * 8) throw std::runtime_error("my.fdx: truncated");
  offs_.resize(n);
  std::memcpy(offs_.data(), p, n * 8);
  n_ = static_cast<int32_t>(n);
  buf_bytes_ = static_cast<int32_t>(bs);
  const int fd = ::open((dir + "/my.fdt").c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("my.fdx without my.fdt");
  struct stat sb;
  fstat(fd, &sb);
  len_ = static_cast<uint64_t>(sb.st_size);
  if (len_) {
    void* m = mmap(nullptr, len_, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { ::close(fd); throw std::runtime_error("cannot map my.fdt"); }
    map_ = static_cast<uint8_t*>(m);
  }
  ::close(fd);
  loaded_ = true;
  return true;
}

std::string DocStore::get(int32_t doc) const {
  if (!loaded_) throw std::runtime_error("the index has no doc store (my.fdx / my.fdt)");
  if (doc < 0 || doc >= n_) throw std::runtime_error("doc id outside the doc store");
  const int64_t e = offs_[doc];
  uint64_t at = static_cast<uint64_t>(e >> 1);
  if (e & 1) at = (at / 4096 + 1) * 4096;   // the record was moved to the next page
  if (at >= len_ || map_[at] != kDocMagic) throw std::runtime_error("doc store record: bad magic");
  const uint8_t* p = map_ + at + 1;
  const uint8_t* end = map_ + len_;
  uint64_t n_chunks = 0;
  int l = get_varint(p, end, &n_chunks);
  if (!l) throw std::runtime_error("doc store record: bad header");
  p += l;
  std::vector<uint64_t> sizes(n_chunks);
  for (auto& s : sizes) {
    l = get_varint(p, end, &s);
    if (!l) throw std::runtime_error("doc store record: bad header");
    p += l;
  }
  std::string text;
  thread_local std::vector<char> buf;   // (one decode buffer per thread, no zero fill per call)
  if (buf.size() < static_cast<size_t>(buf_bytes_)) buf.resize(buf_bytes_);
  for (uint64_t s : sizes) {
    if (static_cast<uint64_t>(end - p) < s) throw std::runtime_error("doc store record: truncated");
    const int got = LZ4_decompress_safe(reinterpret_cast<const char*>(p), buf.data(),
                                        static_cast<int>(s), buf_bytes_);
    if (got < 0) throw std::runtime_error("doc store record: LZ4 decode failed");
    text.append(buf.data(), got);
    p += s;
  }
  return text;
}

}  // namespace wiser
