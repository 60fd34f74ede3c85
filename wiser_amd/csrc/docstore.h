// Doc store in the reference's chunked layout (my.fdx / my.fdt), host side.
//
// Written by the index writer (FlashEngineDumper::Dump -> ChunkedDocStoreDumper,
// doc_store.h:277-363, flash_engine_dumper.h:717,743) and read by the snippet
// stage (ChunkedDocStoreReader::Get, doc_store.h:365-455):
//   my.fdx : varint n_doc_ids | varint buffer size (16 KB) | n x int64 (off << 1 | aligned)
//   my.fdt : per doc 0x33 | varint n_chunks | varint chunk bytes... | LZ4 blocks, each
//            block <= buffer/2 bytes of text; a doc whose chunks would straddle
//            one more 4 KB block than necessary starts on the next 4 KB boundary
//            (ShouldAlign, doc_store.h:72-77, whose "% 4*KB" binds as (off % 4) * KB).
// LZ4 is the reference's own codec; the system liblz4 (1.9.3) is linked.
#pragma once

#include <cstdint>
#include <fstream>
#include <string>
#include <vector>

namespace wiser {

class DocStoreWriter {
 public:
  static constexpr int kBufBytes = 16 * 1024;   // dump_buf_size_ (doc_store.h:360)
  void open(const std::string& dir, bool align = true);
  void add(const std::string& text);           // doc ids are consecutive from 0
  void close();                                 // writes my.fdx

 private:
  std::string dir_;
  std::ofstream fdt_;
  uint64_t at_ = 0;
  bool align_ = true;
  std::vector<int64_t> offs_;
  std::vector<char> buf_;
};

class DocStore {
 public:
  DocStore() = default;
  ~DocStore();
  DocStore(const DocStore&) = delete;
  DocStore& operator=(const DocStore&) = delete;
  // false when the index has no doc store (synthetic corpora)
  bool open(const std::string& dir);
  bool is_open() const { return loaded_; }
  int32_t size() const { return n_; }
  std::string get(int32_t doc) const;   // throws on a corrupt record

 private:
  bool loaded_ = false;
  int32_t n_ = 0;
  int32_t buf_bytes_ = 0;
  std::vector<int64_t> offs_;
  uint8_t* map_ = nullptr;
  uint64_t len_ = 0;
};

}  // namespace wiser
