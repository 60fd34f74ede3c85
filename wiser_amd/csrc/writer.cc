// Vacuum index writer.  Restates the byte layout produced by the reference's
// VacuumInvertedIndexDumper (flash_engine_dumper.h:288-411) and friends:
//
//   my.vacuum : 0x88 | 2 x (varint has_bloom, varint bit_array_bytes,
//               varint expected_entries, f32 ratio) | zero pad to byte 100,
//               then one posting list per term:
//               0xF4 | varint df | 8 reserved bytes (two varint 0s, zero pad)
//               | skip list | gap | docid box | tf box | position box | offset box
//   my.tip    : per term u32 len | bytes | i64 (prefetch pages << 48 | list offset)
//   my.doc_length : i32 n | f64 incremental-mean avg | n x (i32 doc, i8 char4)
//
// A "box" (GeneralTermEntry::GetCozyBoxWriter, flash_engine_dumper.h:78-104) is
// floor(n/128) bit packs followed by one VInts blob holding the n mod 128 rest.
// Doc ids are delta coded over the whole list (utils.h:573-584); tf raw;
// positions / offsets delta coded inside each posting's bag.
//
// The skip list is first sized as if the data began 512 KiB later (the
// reference's FakeFileDumper estimate, flash_engine_dumper.h:528-537), the data
// is placed after that estimate, and the real (possibly shorter) skip list is
// written in front, leaving a zero gap -- exactly the reference's placement.
#include "writer.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <queue>
#include <cmath>
#include <fstream>
#include <map>
#include <memory>
#include <random>
#include <stdexcept>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "bloom.h"
#include "docstore.h"
#include "format.h"

namespace wiser {
namespace {

// The "begin" or "end" bloom bit arrays of a list's postings (bloom on):
// has[i] = posting i has one (BloomFilterStore keeps none for a posting with no
// neighbour on that side); the arrays of the postings that have one, each
// `bytes` long, back to back in posting order.
struct BloomBits {
  bool on = false;
  size_t bytes = 0;
  std::vector<uint8_t> has;
  std::vector<uint8_t> bits;
  void push(const std::string& a) {
    has.push_back(a.empty() ? 0 : 1);
    bits.insert(bits.end(), a.begin(), a.end());
  }
};

// ------------------------------------------------------------ term input --
struct TermPostings {
  std::vector<uint32_t> docs;
  std::vector<uint32_t> tfs;
  std::vector<uint32_t> pos_vals;   // per-bag delta coded
  std::vector<uint32_t> pos_sizes;
  std::vector<uint32_t> off_vals;   // per-bag delta coded [s0,e0,s1,e1..]
  std::vector<uint32_t> off_sizes;
  BloomBits blm[2];                 // begin, end filters (bloom on)
};

// One encoded box: the bytes plus, for every skip row, where the row's first
// posting lives (blob offset relative to box start, in-blob index).
struct Box {
  std::string bytes;
  std::vector<uint64_t> row_off;
  std::vector<uint32_t> row_idx;
};

// values + per-posting bag sizes -> packs + vints; rows every 128 postings.
void encode_box(const std::vector<uint32_t>& vals, const std::vector<uint32_t>* sizes,
                size_t n_postings, bool delta, Box* box) {
  const size_t nv = vals.size();
  std::vector<uint32_t> v(nv);
  if (delta) {
    uint32_t prev = 0;
    for (size_t i = 0; i < nv; ++i) { v[i] = vals[i] - prev; prev = vals[i]; }
  } else {
    v = vals;
  }
  const size_t n_packs = nv / kPackSize;
  std::vector<uint64_t> blob_off;
  blob_off.reserve(n_packs + 1);
  for (size_t p = 0; p < n_packs; ++p) {
    blob_off.push_back(box->bytes.size());
    append_pack(&box->bytes, &v[p * kPackSize]);
  }
  const size_t rest = nv - n_packs * kPackSize;
  if (rest) {
    blob_off.push_back(box->bytes.size());
    append_vints(&box->bytes, &v[n_packs * kPackSize], static_cast<int>(rest));
  }
  // value index of posting p = sum of bag sizes before p
  uint64_t vi = 0;
  for (size_t p = 0; p < n_postings; ++p) {
    if (p % kPackSize == 0) {
      const size_t blob = vi / kPackSize;
      if (blob >= blob_off.size())
        throw std::runtime_error("posting bag points past the last blob (empty bags at list end)");
      box->row_off.push_back(blob_off[blob]);
      box->row_idx.push_back(static_cast<uint32_t>(vi % kPackSize));
    }
    vi += sizes ? (*sizes)[p] : 1;
  }
}

struct EncodedList {
  uint32_t df = 0;
  std::vector<uint32_t> prev_doc;  // per row
  Box doc, tf, pos, off;
  const BloomBits* blm[2] = {nullptr, nullptr};   // begin, end (bloom on)
};

// One bloom section (flash_engine_dumper.h:620-646): the bloom skip list
// (0xA4 | varint n_boxes | delta varints of box offsets relative to the list
// start, flash_containers.h:640-660), then the boxes of 128 postings each
// (0xF5 | varint n | MSB-first presence bitmap | the non-empty bit arrays,
// flash_containers.h:499-558).  `at` = offset of the section from the list
// start; the skip list is sized with offsets 512 KB further out, as the
// reference does, and the gap after it is padding.
std::string bloom_section(const BloomBits& arrays, uint64_t at) {
  std::vector<std::string> boxes;
  const size_t np = arrays.has.size();
  const uint8_t* src = arrays.bits.data();
  for (size_t i = 0; i < np; i += kPackSize) {
    const size_t n = std::min<size_t>(kPackSize, np - i);
    std::string b;
    b.push_back(static_cast<char>(kBloomBoxMagic));
    put_varint(&b, n);
    size_t present = 0;
    for (size_t c = 0; c < n; c += 8) {
      uint8_t bits = 0;
      for (size_t o = 0; o < 8 && c + o < n; ++o)
        if (arrays.has[i + c + o]) { bits |= static_cast<uint8_t>(1u << (7 - o)); ++present; }
      b.push_back(static_cast<char>(bits));
    }
    b.append(reinterpret_cast<const char*>(src), present * arrays.bytes);
    src += present * arrays.bytes;
    boxes.push_back(std::move(b));
  }
  auto skip = [&](uint64_t first) {
    std::string sl;
    sl.push_back(static_cast<char>(kBloomSkipListMagic));
    put_varint(&sl, boxes.size());
    uint64_t prev = 0, o = first;
    for (auto& b : boxes) { put_varint(&sl, o - prev); prev = o; o += b.size(); }
    return sl;
  };
  const size_t est = skip(at + 512 * 1024).size();
  std::string sec = skip(at + est);
  if (sec.size() > est) throw std::runtime_error("bloom skip list estimate too small");
  sec.append(est - sec.size(), '\0');
  for (auto& b : boxes) sec += b;
  return sec;
}

void encode_list(const TermPostings& t, EncodedList* e) {
  const size_t n = t.docs.size();
  e->df = static_cast<uint32_t>(n);
  if (t.blm[0].on) { e->blm[0] = &t.blm[0]; e->blm[1] = &t.blm[1]; }
  for (size_t r = 0; r * kPackSize < n; ++r)
    e->prev_doc.push_back(r == 0 ? 0 : t.docs[r * kPackSize - 1]);
  encode_box(t.docs, nullptr, n, true, &e->doc);
  encode_box(t.tfs, nullptr, n, false, &e->tf);
  encode_box(t.pos_vals, &t.pos_sizes, n, false, &e->pos);
  encode_box(t.off_vals, &t.off_sizes, n, false, &e->off);
}

// Skip list with the data sections starting at absolute file offset `data0`
// (`bloom_bytes` of bloom sections sit between the tf and position boxes).
std::string encode_skip_list(const EncodedList& e, uint64_t data0, uint64_t bloom_bytes = 0) {
  const uint64_t d0 = data0;
  const uint64_t t0 = d0 + e.doc.bytes.size();
  const uint64_t p0 = t0 + e.tf.bytes.size() + bloom_bytes;
  const uint64_t o0 = p0 + e.pos.bytes.size();
  std::string s;
  s.push_back(static_cast<char>(kSkipListMagic));
  const size_t rows = e.prev_doc.size();
  put_varint(&s, rows);
  uint32_t pd = 0;
  uint64_t pdo = 0, pto = 0, ppo = 0, poo = 0;
  for (size_t r = 0; r < rows; ++r) {
    const uint64_t dof = d0 + e.doc.row_off[r], tof = t0 + e.tf.row_off[r];
    const uint64_t pof = p0 + e.pos.row_off[r], oof = o0 + e.off.row_off[r];
    put_varint(&s, static_cast<uint32_t>(e.prev_doc[r] - pd));
    put_varint(&s, dof - pdo);
    put_varint(&s, tof - pto);
    put_varint(&s, pof - ppo);
    put_varint(&s, e.pos.row_idx[r]);
    put_varint(&s, oof - poo);
    put_varint(&s, e.off.row_idx[r]);
    pd = e.prev_doc[r]; pdo = dof; pto = tof; ppo = pof; poo = oof;
  }
  return s;
}

class VacuumFileWriter {
 public:
  explicit VacuumFileWriter(const std::string& dir, const BloomSpec& bloom = BloomSpec())
      : dir_(dir), bloom_(bloom.on) {
    ::mkdir(dir.c_str(), 0777);
    vac_.open(dir + "/my.vacuum", std::ios::binary | std::ios::trunc);
    tip_.open(dir + "/my.tip", std::ios::binary | std::ios::trunc);
    if (!vac_ || !tip_) throw std::runtime_error("cannot create index files in " + dir);
    // has_bloom, bit array bytes, expected entries, f32 ratio, for the "begin"
    // and the "end" filter (flash_engine_dumper.h:288-316); zeros without bloom
    std::string h;
    h.push_back(static_cast<char>(kVacuumMagic));
    for (int i = 0; i < 2; ++i) {
      if (bloom.on) {
        put_varint(&h, 1);
        put_varint(&h, static_cast<uint64_t>(BloomShape(bloom.entries, bloom.ratio).bytes));
        put_varint(&h, static_cast<uint64_t>(bloom.entries));
        h.append(reinterpret_cast<const char*>(&bloom.ratio), 4);
      } else {
        put_varint(&h, 0); put_varint(&h, 0); put_varint(&h, 0);
        h.append(4, '\0');
      }
    }
    h.resize(kVacuumHeaderBytes, '\0');
    vac_.write(h.data(), h.size());
    off_ = kVacuumHeaderBytes;
  }

  void add(const std::string& term, const EncodedList& e) {
    const uint64_t start = off_;
    std::string head;
    head.push_back(static_cast<char>(kPostingListMagic));
    put_varint(&head, e.df);
    const size_t resv = head.size();
    put_varint(&head, 0);
    put_varint(&head, 0);
    head.resize(resv + 8, '\0');
    const uint64_t skip_start = start + head.size();
    if (bloom_ && !e.blm[0]) throw std::runtime_error("bloom index: list of '" + term + "' has no filters");
    // bloom sections are sized from their offsets, which follow the skip list:
    // size the skip list for bloom sections 512 KB larger than any real one
    std::string blm[2];
    if (bloom_) {
      // upper bound of both sections: every posting's array + box / skip overheads
      uint64_t ub = 0;
      for (int i = 0; i < 2; ++i) ub += e.blm[i]->bits.size();
      ub += 2 * (e.df / kPackSize + 1) * (kPackSize / 8 + 2 * 10 + 4) + 64;
      const uint64_t est0 = encode_skip_list(e, skip_start + 512 * 1024, ub + 1024 * 1024).size();
      uint64_t at = skip_start + est0 + e.doc.bytes.size() + e.tf.bytes.size() - start;
      for (int i = 0; i < 2; ++i) { blm[i] = bloom_section(*e.blm[i], at); at += blm[i].size(); }
      const uint64_t bb = blm[0].size() + blm[1].size();
      // the skip list written below is no larger than est0, so the sections
      // keep their offsets: pad the skip list gap to est0
      const std::string skip = encode_skip_list(e, skip_start + est0, bb);
      if (skip.size() > est0) throw std::runtime_error("skip list estimate too small");
      const uint64_t s0 = skip_start + est0 + e.doc.bytes.size() + e.tf.bytes.size() - start;
      std::string ptr;   // the 8 reserved bytes: section offsets from the list start
      put_varint(&ptr, s0);
      put_varint(&ptr, s0 + blm[0].size());
      if (ptr.size() > 8) throw std::runtime_error("bloom section pointers exceed 8 bytes");
      head.replace(resv, ptr.size(), ptr);
      head += skip;
      head.append(est0 - skip.size(), '\0');
    } else {
      const size_t est = encode_skip_list(e, skip_start + 512 * 1024).size();
      const std::string skip = encode_skip_list(e, skip_start + est);
      if (skip.size() > est) throw std::runtime_error("skip list estimate too small");
      head += skip;
      head.append(est - skip.size(), '\0');
    }
    vac_.write(head.data(), head.size());
    vac_.write(e.doc.bytes.data(), e.doc.bytes.size());
    vac_.write(e.tf.bytes.data(), e.tf.bytes.size());
    for (auto& b : blm) vac_.write(b.data(), b.size());
    vac_.write(e.pos.bytes.data(), e.pos.bytes.size());
    vac_.write(e.off.bytes.data(), e.off.bytes.size());
    const uint64_t tf_end = start + head.size() + e.doc.bytes.size() + e.tf.bytes.size();
    off_ = tf_end + blm[0].size() + blm[1].size() + e.pos.bytes.size() + e.off.bytes.size();
    const uint32_t pages = static_cast<uint32_t>((tf_end - start) / 4096);
    const int64_t v = encode_tip_value(pages, start);
    const uint32_t len = static_cast<uint32_t>(term.size());
    tip_.write(reinterpret_cast<const char*>(&len), 4);
    tip_.write(term.data(), term.size());
    tip_.write(reinterpret_cast<const char*>(&v), 8);
    ++n_terms_;
  }

  uint64_t bytes() const { return off_; }
  int64_t terms() const { return n_terms_; }
  void close() { vac_.close(); tip_.close(); }

 private:
  std::string dir_;
  bool bloom_ = false;
  std::ofstream vac_, tip_;
  uint64_t off_ = 0;
  int64_t n_terms_ = 0;
};

// Incremental mean exactly as DocLengthCharStore::AddLength (doc_length_store.h:104-112).
struct DocLengths {
  std::vector<uint8_t> c4;
  double avg = 0;
  int64_t cnt = 0, big = 0;
  void add(uint32_t len) {
    avg = avg + (static_cast<int>(len) - avg) / (cnt + 1);
    uint8_t c = length_to_char4(len);
    if (c >= 0x80) ++big;
    c4.push_back(c);
    ++cnt;
  }
  void write(const std::string& dir) const {
    std::ofstream f(dir + "/my.doc_length", std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write my.doc_length");
    int32_t n = static_cast<int32_t>(c4.size());
    f.write(reinterpret_cast<const char*>(&n), 4);
    f.write(reinterpret_cast<const char*>(&avg), 8);
    std::string rec(5 * c4.size(), '\0');
    for (int32_t i = 0; i < n; ++i) {
      std::memcpy(&rec[5 * i], &i, 4);
      rec[5 * i + 4] = static_cast<char>(c4[i]);
    }
    f.write(rec.data(), rec.size());
  }
};

// ------------------------------------------------------- linedoc parsing --
// utils::explode (utils.cc:29-42): split, dropping empty pieces.
std::vector<std::string> explode(const std::string& s, char c) {
  std::vector<std::string> v;
  std::string cur;
  for (char ch : s) {
    if (ch != c) cur += ch;
    else if (!cur.empty()) { v.push_back(cur); cur.clear(); }
  }
  if (!cur.empty()) v.push_back(cur);
  return v;
}

// utils::explode_strict (utils.cc:52-67): split, keeping empty pieces.
std::vector<std::string> explode_strict(const std::string& s, char c) {
  std::vector<std::string> v;
  std::string cur;
  for (char ch : s) {
    if (ch != c) cur += ch;
    else { v.push_back(cur); cur.clear(); }
  }
  v.push_back(cur);
  return v;
}

// utils::parse_offsets (utils.cc:105-141): "s,e;s,e;." groups per term.
std::vector<std::vector<std::pair<uint32_t, uint32_t>>> parse_offsets(const std::string& s) {
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> res;
  std::string grp;
  auto flush_group = [&](const std::string& g) {
    std::vector<std::pair<uint32_t, uint32_t>> term;
    std::string buf;
    for (char ch : g) {
      if (ch != ';') buf += ch;
      else if (!buf.empty()) {
        size_t c = buf.find(',');
        term.emplace_back(std::stoul(buf.substr(0, c)), std::stoul(buf.substr(c + 1)));
        buf.clear();
      }
    }
    res.push_back(term);
  };
  for (char ch : s) {
    if (ch != '.') grp += ch;
    else if (!grp.empty()) { flush_group(grp); grp.clear(); }
  }
  return res;
}

}  // namespace

// ----------------------------------------------- streaming linedoc writer --
// The reference's dumper holds the whole inverted index in memory before it
// writes (FlashEngineDumper::LoadQqMemDump / Dump, flash_engine_dumper.h:735-808).
// This writer keeps host memory bounded by the chunk size instead:
//   pass 1 (parallel): rows are cut into chunks; a worker parses a chunk into
//     one record per (term, doc) and spills the chunk as a run file, terms
//     ascending, each term's records in doc order;
//   pass 2: a k-way merge of the runs by term concatenates a term's records
//     run by run (= doc order), batches of terms are encoded in parallel
//     and appended in term order.
// The output is byte-identical to the one-map writer it replaces
// (tests/golden/writer_sha256.json) at every chunk size and thread count.
namespace {

// utils::explode_strict (utils.cc:52-67) restricted to counting: the column
// `col` of a tab-separated row, or false when the row has too few columns.
bool column_of(const std::string& line, size_t col, size_t need, std::string* out) {
  size_t at = 0, c = 0, begin = 0, end = std::string::npos;
  for (;;) {
    const size_t tab = line.find('\t', at);
    const size_t stop = tab == std::string::npos ? line.size() : tab;
    if (c == col) { begin = at; end = stop; }
    ++c;
    if (tab == std::string::npos) break;
    at = tab + 1;
  }
  if (c < need) return false;
  out->assign(line, begin, end - begin);
  return true;
}

// One record: doc | tf | n_pos | position deltas | n_off | offset deltas
// [| flags (1 begin, 2 end) | begin array | end array], varints.
void put_record(std::string* o, uint32_t doc, uint32_t tf, const std::vector<uint32_t>& pos,
                const std::vector<uint32_t>& off, const std::string* blm) {
  put_varint(o, doc);
  put_varint(o, tf);
  put_varint(o, pos.size());
  uint32_t prev = 0;
  for (uint32_t x : pos) { put_varint(o, static_cast<uint32_t>(x - prev)); prev = x; }
  put_varint(o, off.size());
  prev = 0;
  for (uint32_t x : off) { put_varint(o, static_cast<uint32_t>(x - prev)); prev = x; }
  if (blm) {
    o->push_back(static_cast<char>((blm[0].empty() ? 0 : 1) | (blm[1].empty() ? 0 : 2)));
    *o += blm[0];
    *o += blm[1];
  }
}

struct TermRun {
  std::string bytes;
  uint32_t n = 0;
};

// "begin" / "end" bloom arrays of every token of a doc from its positions
// (the fixture columns bloom_before / bloom: the terms before / after each
// occurrence, testdata/iter_test_3_docs_tf_bi-bloom)
void doc_blooms(const std::vector<const std::string*>& toks, const std::vector<std::vector<uint32_t>>& pos,
                const BloomShape& shape, std::vector<std::array<std::string, 2>>* out) {
  std::unordered_map<uint32_t, const std::string*> at;
  for (size_t t = 0; t < toks.size(); ++t)
    for (uint32_t p : pos[t]) at[p] = toks[t];
  out->resize(toks.size());
  for (size_t t = 0; t < toks.size(); ++t) {
    std::vector<std::string> before, after;
    for (uint32_t p : pos[t]) {
      if (p > 0) { auto it = at.find(p - 1); if (it != at.end()) before.push_back(*it->second); }
      auto it = at.find(p + 1);
      if (it != at.end()) after.push_back(*it->second);
    }
    (*out)[t][0] = make_bloom(shape, before);
    (*out)[t][1] = make_bloom(shape, after);
  }
}

struct ChunkOut {
  std::vector<uint32_t> lens;
  std::string path;
  int64_t err_row = -1;
  std::string err;
};

// Parse rows [doc0, doc0 + lines.size()) into one run file.
void parse_chunk(const std::vector<std::string>& lines, uint32_t doc0, bool token_only, const BloomSpec& bloom,
                 const BloomShape& shape, const std::string& path, ChunkOut* res) {
  std::unordered_map<std::string, TermRun> runs;
  res->lens.reserve(lines.size());
  std::vector<std::array<std::string, 2>> blm;
  std::vector<uint32_t> pos, flat;
  for (size_t r = 0; r < lines.size(); ++r) {
    const uint32_t doc = doc0 + static_cast<uint32_t>(r);
    std::vector<std::string> items = explode_strict(lines[r], '\t');
    if (token_only) {
      // Body = tokens = column 2; tf = token count; positions = token ordinals;
      // offsets = char span (end inclusive) of each occurrence in column 2.
      const std::string& toks = items[2];
      std::map<std::string, std::pair<std::vector<uint32_t>, std::vector<uint32_t>>> occ;
      uint32_t ordinal = 0;
      size_t i = 0;
      while (i < toks.size()) {
        if (toks[i] == ' ') { ++i; continue; }
        size_t j = i;
        while (j < toks.size() && toks[j] != ' ') ++j;
        auto& o = occ[toks.substr(i, j - i)];
        o.first.push_back(ordinal++);
        o.second.push_back(static_cast<uint32_t>(i));
        o.second.push_back(static_cast<uint32_t>(j - 1));
        i = j;
      }
      if (bloom.on) {
        std::vector<const std::string*> dt;
        std::vector<std::vector<uint32_t>> dp;
        for (auto& kv : occ) { dt.push_back(&kv.first); dp.push_back(kv.second.first); }
        doc_blooms(dt, dp, shape, &blm);
      }
      size_t t = 0;
      for (auto& kv : occ) {
        TermRun& tr = runs[kv.first];
        put_record(&tr.bytes, doc, static_cast<uint32_t>(kv.second.first.size()), kv.second.first,
                   kv.second.second, bloom.on ? blm[t].data() : nullptr);
        ++tr.n;
        ++t;
      }
      res->lens.push_back(ordinal);
    } else {
      std::vector<std::string> toks = explode(items[2], ' ');
      auto offsets = parse_offsets(items[3]);
      std::vector<std::string> groups = explode(items[4], '.');
      if (offsets.size() != toks.size() || groups.size() != toks.size()) {
        res->err_row = doc;
        res->err = "linedoc row " + std::to_string(doc) + ": token/offset/position column mismatch";
        return;
      }
      std::unordered_set<std::string> seen;
      std::vector<std::vector<uint32_t>> dpos(toks.size());
      for (size_t t = 0; t < toks.size(); ++t) {
        if (!seen.insert(toks[t]).second) {
          res->err_row = doc;
          res->err = "duplicate token '" + toks[t] + "' in row " + std::to_string(doc);
          return;
        }
        for (auto& p : explode(groups[t], ';')) dpos[t].push_back(static_cast<uint32_t>(std::stoul(p)));
      }
      if (bloom.on) {
        std::vector<const std::string*> dt;
        for (auto& t : toks) dt.push_back(&t);
        doc_blooms(dt, dpos, shape, &blm);
      }
      for (size_t t = 0; t < toks.size(); ++t) {
        flat.clear();
        for (auto& pr : offsets[t]) { flat.push_back(pr.first); flat.push_back(pr.second); }
        TermRun& tr = runs[toks[t]];
        put_record(&tr.bytes, doc, static_cast<uint32_t>(offsets[t].size()), dpos[t], flat,
                   bloom.on ? blm[t].data() : nullptr);
        ++tr.n;
      }
      res->lens.push_back(static_cast<uint32_t>(explode(items[1], ' ').size()));
    }
  }
  // spill: term length | term | record count | record bytes | records, terms ascending
  std::vector<std::pair<const std::string*, TermRun*>> order;
  order.reserve(runs.size());
  for (auto& kv : runs) order.emplace_back(&kv.first, &kv.second);
  std::sort(order.begin(), order.end(), [](const auto& a, const auto& b) { return *a.first < *b.first; });
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot create run file " + path);
  std::string head;
  bool ok = true;
  for (auto& e : order) {
    head.clear();
    put_varint(&head, e.first->size());
    head += *e.first;
    put_varint(&head, e.second->n);
    put_varint(&head, e.second->bytes.size());
    ok = ok && std::fwrite(head.data(), 1, head.size(), f) == head.size();
    ok = ok && std::fwrite(e.second->bytes.data(), 1, e.second->bytes.size(), f) == e.second->bytes.size();
    std::string().swap(e.second->bytes);
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("cannot write run file " + path);
  res->path = path;
}

// Sequential reader of one run file.
class RunReader {
 public:
  explicit RunReader(const std::string& path) : buf_(1 << 20) {
    f_ = std::fopen(path.c_str(), "rb");
    if (!f_) throw std::runtime_error("cannot open run file " + path);
    std::setvbuf(f_, buf_.data(), _IOFBF, buf_.size());
    advance();
  }
  ~RunReader() { if (f_) std::fclose(f_); }
  RunReader(const RunReader&) = delete;
  RunReader& operator=(const RunReader&) = delete;
  bool done() const { return done_; }
  const std::string& term() const { return term_; }
  // the current term's records appended to tp; then the next term
  void take(TermPostings* tp, bool blooms, size_t bloom_bytes) {
    payload_.resize(nbytes_);
    if (nbytes_ && std::fread(&payload_[0], 1, nbytes_, f_) != nbytes_) throw std::runtime_error("short run file");
    const uint8_t* p = reinterpret_cast<const uint8_t*>(payload_.data());
    const uint8_t* end = p + payload_.size();
    auto next = [&]() -> uint32_t {
      uint64_t v;
      const int n = get_varint(p, end, &v);
      if (n <= 0) throw std::runtime_error("corrupt run file");
      p += n;
      return static_cast<uint32_t>(v);
    };
    for (uint64_t r = 0; r < n_; ++r) {
      tp->docs.push_back(next());
      tp->tfs.push_back(next());
      const uint32_t np = next();
      for (uint32_t i = 0; i < np; ++i) tp->pos_vals.push_back(next());
      tp->pos_sizes.push_back(np);
      const uint32_t no = next();
      for (uint32_t i = 0; i < no; ++i) tp->off_vals.push_back(next());
      tp->off_sizes.push_back(no);
      if (blooms) {
        if (p >= end) throw std::runtime_error("corrupt run file");
        const uint8_t fl = *p++;
        for (int s = 0; s < 2; ++s) {
          BloomBits& b = tp->blm[s];
          const bool has = fl & (1u << s);
          b.has.push_back(has ? 1 : 0);
          if (has) {
            if (static_cast<size_t>(end - p) < bloom_bytes) throw std::runtime_error("corrupt run file");
            b.bits.insert(b.bits.end(), p, p + bloom_bytes);
            p += bloom_bytes;
          }
        }
      }
    }
    advance();
  }

 private:
  bool read_varint(uint64_t* v) {
    uint64_t x = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      const int c = std::getc(f_);
      if (c == EOF) return false;
      x |= static_cast<uint64_t>(c & 0x7F) << sh;
      if (!(c & 0x80)) { *v = x; return true; }
    }
    return false;
  }
  void advance() {
    uint64_t len;
    if (!read_varint(&len)) { done_ = true; return; }
    term_.resize(len);
    if (len && std::fread(&term_[0], 1, len, f_) != len) throw std::runtime_error("short run file");
    if (!read_varint(&n_) || !read_varint(&nbytes_)) throw std::runtime_error("short run file");
  }
  std::vector<char> buf_;
  FILE* f_ = nullptr;
  std::string term_, payload_;
  uint64_t n_ = 0, nbytes_ = 0;
  bool done_ = false;
};

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

}  // namespace

BuildStats build_from_linedoc(const std::string& linedoc, int64_t n_rows,
                              const std::string& format, const std::string& out_dir,
                              const BloomSpec& bloom) {
  const BloomShape shape(bloom.entries, bloom.ratio);
  const bool token_only = format == "TOKEN_ONLY";
  if (!token_only && format != "WITH_POSITIONS")
    throw std::runtime_error("unsupported linedoc format " + format);
  std::ifstream in(linedoc);
  if (!in) throw std::runtime_error("cannot open linedoc " + linedoc);
  const size_t need = token_only ? 3u : 5u;
  const int hw = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  const int threads = std::max(1, env_int("WSR_WRITER_THREADS", std::min(hw, 16)));
  const size_t chunk_docs = static_cast<size_t>(std::max(1, env_int("WSR_WRITER_CHUNK_DOCS", 8192)));
  ::mkdir(out_dir.c_str(), 0777);
  const std::string run_dir = out_dir + "/.wsr_runs";
  ::mkdir(run_dir.c_str(), 0777);
  std::vector<std::unique_ptr<ChunkOut>> chunks;
  auto cleanup = [&] {
    for (auto& c : chunks) if (c && !c->path.empty()) ::unlink(c->path.c_str());
    ::rmdir(run_dir.c_str());
  };

  // ---- pass 1: rows -> doc store (in order, this thread) + run files (workers)
  struct Job {
    std::vector<std::string> lines;
    uint32_t doc0;
    ChunkOut* out;
    std::string path;
  };
  std::mutex mu;
  std::condition_variable cv_job, cv_room;
  std::deque<Job> jobs;
  bool closing = false;
  std::exception_ptr fatal;
  auto worker = [&] {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_job.wait(lk, [&] { return closing || !jobs.empty(); });
        if (jobs.empty()) return;
        j = std::move(jobs.front());
        jobs.pop_front();
      }
      cv_room.notify_one();
      try {
        parse_chunk(j.lines, j.doc0, token_only, bloom, shape, j.path, j.out);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        if (!fatal) fatal = std::current_exception();
      }
    }
  };
  std::vector<std::thread> pool;
  for (int i = 0; i < threads; ++i) pool.emplace_back(worker);
  // doc store: DocInfo::Body() = column 2 for TOKEN_ONLY, column 1 otherwise
  // (engine_loader.h:63-65,91-93), added by FlashEngineDumper (flash_engine_dumper.h:717)
  DocStoreWriter store;
  std::string line, body;
  uint32_t doc = 0;
  int64_t col_err = -1;
  try {
    store.open(out_dir);
    std::getline(in, line);  // header row
    std::vector<std::string> cur;
    auto submit = [&] {
      if (cur.empty()) return;
      chunks.push_back(std::make_unique<ChunkOut>());
      Job j;
      j.doc0 = doc - static_cast<uint32_t>(cur.size());
      j.lines = std::move(cur);
      j.out = chunks.back().get();
      j.path = run_dir + "/run_" + std::to_string(chunks.size() - 1);
      cur.clear();
      std::unique_lock<std::mutex> lk(mu);
      cv_room.wait(lk, [&] { return jobs.size() < static_cast<size_t>(threads); });
      jobs.push_back(std::move(j));
      lk.unlock();
      cv_job.notify_one();
    };
    while ((n_rows < 0 || doc < n_rows) && std::getline(in, line)) {
      if (!column_of(line, token_only ? 2 : 1, need, &body)) { col_err = doc; break; }
      store.add(body);
      cur.push_back(std::move(line));
      ++doc;
      if (cur.size() == chunk_docs) submit();
    }
    submit();
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu);
    if (!fatal) fatal = std::current_exception();
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    closing = true;
  }
  cv_job.notify_all();
  for (auto& t : pool) t.join();
  if (fatal) { cleanup(); std::rethrow_exception(fatal); }
  // the first bad row in doc order, as a one-pass reader would report it
  for (auto& c : chunks)
    if (c->err_row >= 0 && (col_err < 0 || c->err_row < col_err)) { cleanup(); throw std::runtime_error(c->err); }
  if (col_err >= 0) {
    cleanup();
    throw std::runtime_error("linedoc row " + std::to_string(col_err) + " has too few columns");
  }
  store.close();
  DocLengths lens;
  lens.c4.reserve(doc);
  for (auto& c : chunks) {
    for (uint32_t x : c->lens) lens.add(x);
    std::vector<uint32_t>().swap(c->lens);
  }

  // ---- pass 2: merge the runs by term; encode batches in parallel, append in order
  BuildStats st;
  try {
    VacuumFileWriter w(out_dir, bloom);
    std::vector<std::unique_ptr<RunReader>> rd;
    for (auto& c : chunks) rd.push_back(std::make_unique<RunReader>(c->path));
    using Head = std::pair<std::string, size_t>;   // (term, run): runs of one term pop in run order
    std::priority_queue<Head, std::vector<Head>, std::greater<Head>> heap;
    for (size_t i = 0; i < rd.size(); ++i)
      if (!rd[i]->done()) heap.emplace(rd[i]->term(), i);
    std::vector<std::pair<std::string, TermPostings>> batch;
    uint64_t batch_bytes = 0;
    auto flush = [&] {
      std::vector<EncodedList> enc(batch.size());
      std::atomic<size_t> next{0};
      auto work = [&] {
        for (size_t i; (i = next++) < batch.size();) encode_list(batch[i].second, &enc[i]);
      };
      std::vector<std::thread> ts;
      const int nt = static_cast<int>(std::min<size_t>(threads, batch.size()));
      for (int i = 1; i < nt; ++i) ts.emplace_back(work);
      work();
      for (auto& t : ts) t.join();
      for (size_t i = 0; i < batch.size(); ++i) {
        w.add(batch[i].first, enc[i]);
        st.n_postings += enc[i].df;
      }
      batch.clear();
      batch_bytes = 0;
    };
    while (!heap.empty()) {
      const std::string term = heap.top().first;
      TermPostings tp;
      if (bloom.on)
        for (auto& b : tp.blm) { b.on = true; b.bytes = static_cast<size_t>(shape.bytes); }
      while (!heap.empty() && heap.top().first == term) {
        const size_t r = heap.top().second;
        heap.pop();
        rd[r]->take(&tp, bloom.on, static_cast<size_t>(shape.bytes));
        if (!rd[r]->done()) heap.emplace(rd[r]->term(), r);
      }
      batch_bytes += 4 * (tp.docs.size() * 2 + tp.pos_vals.size() + tp.off_vals.size()) +
                     tp.blm[0].bits.size() + tp.blm[1].bits.size();
      batch.emplace_back(term, std::move(tp));
      if (batch.size() >= 4096 || batch_bytes >= (64u << 20)) flush();
    }
    flush();
    w.close();
    st.n_terms = w.terms();
    st.vacuum_bytes = static_cast<int64_t>(w.bytes());
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  lens.write(out_dir);
  st.n_docs = doc;
  st.docs_char4_ge_0x80 = lens.big;
  st.avg_length = lens.avg;
  return st;
}

// ------------------------------------------------------ synthetic corpus --
namespace {

std::string synth_term(int64_t id) {
  char b[32];
  std::snprintf(b, sizeof b, "t%07lld", static_cast<long long>(id));
  return b;
}

// Vose alias table for P(rank r) ~ r^-s, r = 1..V (term id = r - 1).
struct Alias {
  std::vector<double> prob;
  std::vector<uint32_t> alias;
  explicit Alias(int64_t V, double s) : prob(V), alias(V) {
    std::vector<double> w(V);
    double tot = 0;
    for (int64_t r = 0; r < V; ++r) { w[r] = std::pow(static_cast<double>(r + 1), -s); tot += w[r]; }
    std::vector<int64_t> small, large;
    for (int64_t r = 0; r < V; ++r) {
      w[r] = w[r] * V / tot;
      (w[r] < 1.0 ? small : large).push_back(r);
    }
    while (!small.empty() && !large.empty()) {
      int64_t a = small.back(); small.pop_back();
      int64_t g = large.back();
      prob[a] = w[a]; alias[a] = static_cast<uint32_t>(g);
      w[g] = (w[g] + w[a]) - 1.0;
      if (w[g] < 1.0) { large.pop_back(); small.push_back(g); }
    }
    for (int64_t g : large) { prob[g] = 1.0; alias[g] = static_cast<uint32_t>(g); }
    for (int64_t a : small) { prob[a] = 1.0; alias[a] = static_cast<uint32_t>(a); }
  }
  uint32_t draw(std::mt19937_64& g) const {
    const uint64_t V = prob.size();
    uint64_t col = g() % V;
    double u = static_cast<double>(g() >> 11) * 0x1.0p-53;
    return u < prob[col] ? static_cast<uint32_t>(col) : alias[col];
  }
};

double unit(std::mt19937_64& g) { return (static_cast<double>(g() >> 11) + 0.5) * 0x1.0p-53; }

}  // namespace

BuildStats build_synthetic(const SyntheticSpec& sp, const std::string& out_dir) {
  const int64_t N = sp.n_docs, V = sp.vocab;
  int threads = sp.threads > 0 ? sp.threads : static_cast<int>(std::thread::hardware_concurrency());
  if (threads < 1) threads = 1;
  Alias alias(V, sp.zipf_s);

  // 1) doc lengths (one stream, so they do not depend on the thread count)
  std::vector<uint32_t> len(N);
  {
    std::mt19937_64 g(sp.seed);
    for (int64_t d = 0; d < N; ++d) {
      double z = std::sqrt(-2.0 * std::log(unit(g))) * std::cos(2.0 * M_PI * unit(g));
      double l = std::round(std::exp(sp.len_mu + sp.len_sigma * z));
      if (l < 1) l = 1;
      if (l > sp.len_max) l = static_cast<double>(sp.len_max);
      len[d] = static_cast<uint32_t>(l);
    }
  }
  std::vector<uint64_t> doc_start(N + 1, 0);
  for (int64_t d = 0; d < N; ++d) doc_start[d + 1] = doc_start[d] + len[d];
  const uint64_t T = doc_start[N];

  // 2) tokens, chunked by 4096 docs with per-chunk seeds
  std::vector<uint32_t> tok(T);
  const int64_t CH = 4096, nch = (N + CH - 1) / CH;
  {
    std::atomic<int64_t> next{0};
    auto work = [&] {
      for (int64_t c; (c = next++) < nch;) {
        std::mt19937_64 g(sp.seed ^ (0x9E3779B97F4A7C15ull * static_cast<uint64_t>(c + 1)));
        for (int64_t d = c * CH; d < std::min(N, (c + 1) * CH); ++d)
          for (uint64_t i = doc_start[d]; i < doc_start[d + 1]; ++i) tok[i] = alias.draw(g);
      }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
  }

  // 3) term-major occurrence lists (doc order, then position order)
  std::vector<uint64_t> term_start(V + 1, 0);
  for (uint64_t i = 0; i < T; ++i) ++term_start[tok[i] + 1];
  for (int64_t v = 0; v < V; ++v) term_start[v + 1] += term_start[v];
  std::vector<uint32_t> occ_doc(T), occ_pos(T);
  {
    std::vector<uint64_t> fill(term_start.begin(), term_start.end() - 1);
    for (int64_t d = 0; d < N; ++d)
      for (uint64_t i = doc_start[d]; i < doc_start[d + 1]; ++i) {
        uint64_t at = fill[tok[i]]++;
        occ_doc[at] = static_cast<uint32_t>(d);
        occ_pos[at] = static_cast<uint32_t>(i - doc_start[d]);
      }
  }
  // 3b) phrase pool (tools/gen_synthetic_log.py:216-240 find_all_unique_phrases
  // over the corpus's own bigrams instead of an English phrase list): bigrams
  // at uniformly drawn token positions, first come first kept, no term in two
  // phrases, no "a a"; written to <out_dir>/phrases.txt for gen_phrase_log
  if (sp.with_positions) {
    std::mt19937_64 g(sp.seed ^ 0x0000000000000007ull);
    std::vector<uint8_t> used(V, 0);
    ::mkdir(out_dir.c_str(), 0777);
    std::ofstream pf(out_dir + "/phrases.txt", std::ios::trunc);
    if (!pf) throw std::runtime_error("cannot write " + out_dir + "/phrases.txt");
    const int64_t want = std::min<int64_t>(50000, V / 2);
    int64_t got = 0;
    for (int64_t tries = 0; got < want && tries < 100 * want && T > 1; ++tries) {
      const int64_t d = static_cast<int64_t>(g() % static_cast<uint64_t>(N));
      if (len[d] < 2) continue;
      const uint64_t i = doc_start[d] + g() % (len[d] - 1);
      const uint32_t a = tok[i], b = tok[i + 1];
      if (a == b || used[a] || used[b]) continue;
      used[a] = used[b] = 1;
      pf << synth_term(a) << ' ' << synth_term(b) << '\n';
      ++got;
    }
  }
  std::vector<uint32_t>().swap(tok);

  // 4) encode lists in parallel batches, append in term-id order
  VacuumFileWriter w(out_dir);
  BuildStats st;
  const int64_t BATCH = 8192;
  for (int64_t b0 = 0; b0 < V; b0 += BATCH) {
    const int64_t b1 = std::min(V, b0 + BATCH);
    std::vector<std::unique_ptr<EncodedList>> enc(b1 - b0);
    std::atomic<int64_t> next{b0};
    auto work = [&] {
      for (int64_t v; (v = next++) < b1;) {
        const uint64_t s = term_start[v], e = term_start[v + 1];
        if (s == e) continue;
        TermPostings tp;
        for (uint64_t i = s; i < e;) {
          uint64_t j = i;
          while (j < e && occ_doc[j] == occ_doc[i]) ++j;
          tp.docs.push_back(occ_doc[i]);
          tp.tfs.push_back(static_cast<uint32_t>(j - i));
          if (sp.with_positions) {
            uint32_t pp = 0, po = 0;
            for (uint64_t k = i; k < j; ++k) {
              uint32_t p = occ_pos[k];
              tp.pos_vals.push_back(p - pp); pp = p;
              // 8-char term + 1 space per token: span [9p, 9p + 7]
              tp.off_vals.push_back(9 * p - po); tp.off_vals.push_back(7); po = 9 * p + 7;
            }
            tp.pos_sizes.push_back(static_cast<uint32_t>(j - i));
            tp.off_sizes.push_back(static_cast<uint32_t>(2 * (j - i)));
          } else {
            // minimal bags: one position (the first) and one offset pair per posting
            tp.pos_vals.push_back(occ_pos[i]);
            tp.pos_sizes.push_back(1);
            tp.off_vals.push_back(9 * occ_pos[i]); tp.off_vals.push_back(7);
            tp.off_sizes.push_back(2);
          }
          i = j;
        }
        auto el = std::make_unique<EncodedList>();
        encode_list(tp, el.get());
        enc[v - b0] = std::move(el);
      }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    for (int64_t v = b0; v < b1; ++v)
      if (enc[v - b0]) { w.add(synth_term(v), *enc[v - b0]); st.n_postings += enc[v - b0]->df; }
  }
  w.close();
  DocLengths lens;
  lens.c4.reserve(N);
  for (int64_t d = 0; d < N; ++d) lens.add(len[d]);
  lens.write(out_dir);
  st.n_docs = N;
  st.n_terms = w.terms();
  st.vacuum_bytes = static_cast<int64_t>(w.bytes());
  st.docs_char4_ge_0x80 = lens.big;
  st.avg_length = lens.avg;
  return st;
}

// ------------------------------------------------ Wikipedia-shaped stand-in --
namespace {
// terms per df decade of the reference's en-Wikipedia index (gen_synthetic_log.py:8-16)
constexpr int64_t kWikiDecades[7] = {4996891, 520675, 94721, 22139, 5717, 1434, 38};
constexpr double kWikiAlpha = 1.6;   // df density ~ df^-alpha inside a decade

std::string wiki_term(int64_t id) {
  char b[32];
  std::snprintf(b, sizeof b, "w%08lld", static_cast<long long>(id));
  return b;
}

// df drawn from density ~ x^-alpha on [lo, hi) (inverse CDF), as an integer
uint32_t powerlaw_df(std::mt19937_64& g, double lo, double hi) {
  const double a = 1.0 - kWikiAlpha;
  const double u = unit(g);
  const double x = std::pow(std::pow(lo, a) + u * (std::pow(hi, a) - std::pow(lo, a)), 1.0 / a);
  const double f = std::floor(x);
  return static_cast<uint32_t>(f < lo ? lo : (f >= hi ? hi - 1 : f));
}

// splitmix64: the stand-in's per-(term, doc) position stream
uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

BuildStats build_wiki_standin(const WikiSpec& sp, const std::string& out_dir) {
  const int64_t N = sp.n_docs;
  if (N < 16 || N > (1ll << 31) - 1) throw std::runtime_error("wiki stand-in: n_docs out of range");
  int threads = sp.threads > 0 ? sp.threads : static_cast<int>(std::thread::hardware_concurrency());
  if (threads < 1) threads = 1;
  // 1) df of every term: decade by decade, then shuffled over the term ids (so
  //    that sorted term strings are not sorted by df, as in a real dictionary)
  std::vector<uint32_t> dfs;
  {
    std::mt19937_64 g(sp.seed);
    for (int e = 0; e < 7; ++e) {
      const double lo = std::pow(10.0, e);
      const double hi = std::min(std::pow(10.0, e + 1), static_cast<double>(N) + 1);
      if (lo >= hi) break;
      const int64_t n = std::llround(kWikiDecades[e] * sp.term_scale);
      for (int64_t i = 0; i < n; ++i) dfs.push_back(powerlaw_df(g, lo, hi));
    }
    for (size_t i = dfs.size(); i > 1; --i) std::swap(dfs[i - 1], dfs[g() % i]);
  }
  const int64_t V = static_cast<int64_t>(dfs.size());
  if (V == 0) throw std::runtime_error("wiki stand-in: empty vocabulary");
  // 2) per-doc verbosity (lognormal): longer docs repeat their terms more
  std::vector<float> verb(N);
  {
    std::mt19937_64 g(sp.seed ^ 0x5151515151515151ull);
    for (int64_t d = 0; d < N; ++d) {
      const double z = std::sqrt(-2.0 * std::log(unit(g))) * std::cos(2.0 * M_PI * unit(g));
      verb[d] = static_cast<float>(std::exp(0.6 * z));
    }
  }
  // 3) phrase pool (the stand-in for tools/gen_synthetic_log.py:216-252
  //    find_all_unique_phrases over an English phrase list): pairs (a, b) of
  //    distinct terms with df in [1e3, 1e6), no term in two pairs.  As a real
  //    phrase's two words, b co-occurs with a: half of the smaller list's size
  //    of b's docs are drawn from a's docs (b's df is kept), and in 60 % of
  //    the docs holding both, b occurs right after a's first occurrence.
  std::vector<int64_t> partner(V, -1);   // b -> a
  std::vector<std::pair<int64_t, int64_t>> pool;
  {
    std::vector<int64_t> cand;
    for (int64_t v = 0; v < V; ++v)
      if (dfs[v] >= 1000 && dfs[v] < 1000000 && dfs[v] < static_cast<uint64_t>(N) / 2) cand.push_back(v);
    std::mt19937_64 g(sp.seed ^ 0x0000000000000007ull);
    for (size_t i = cand.size(); i > 1; --i) std::swap(cand[i - 1], cand[g() % i]);
    for (size_t i = 0; i + 1 < cand.size(); i += 2) {
      pool.emplace_back(cand[i], cand[i + 1]);
      partner[cand[i + 1]] = cand[i];
    }
  }
  constexpr double kPhraseRate = 0.6;

  // df distinct uniform doc ids, sorted: by rejection for rare terms, by
  // selection sampling (Knuth's algorithm S) for common ones
  // (topic-clustered variant: a draw lands in one of the term's home topics
  // with probability `affinity`; the term's topics come from its id)
  const int64_t T = sp.topics > 0 ? sp.topics : 0;
  const int K = std::max(1, sp.topics_per_term);
  auto uniform_docs = [&](uint32_t df, std::mt19937_64& g, std::vector<uint32_t>* out, int64_t id) {
    std::vector<uint32_t>& docs = *out;
    docs.clear();
    if (static_cast<int64_t>(df) * 16 < N) {
      // home-topic draws only while the topics' ranges stay at most half full
      const bool clustered = T > 0 && static_cast<double>(df) * sp.affinity <= 0.5 * K * (N / T);
      uint64_t home[16];
      for (int j = 0; j < std::min(K, 16); ++j)
        home[j] = mix64(sp.seed ^ (static_cast<uint64_t>(id + 1) * 0xC2B2AE3D27D4EB4Full) ^ static_cast<uint64_t>(j)) %
                  static_cast<uint64_t>(T > 0 ? T : 1);
      auto draw = [&]() -> uint32_t {
        if (clustered && unit(g) < sp.affinity) {
          const uint64_t t = home[g() % static_cast<uint64_t>(std::min(K, 16))];
          const int64_t lo = static_cast<int64_t>(t) * N / T, hi = (static_cast<int64_t>(t) + 1) * N / T;
          return static_cast<uint32_t>(lo + static_cast<int64_t>(g() % static_cast<uint64_t>(hi - lo)));
        }
        return static_cast<uint32_t>(g() % static_cast<uint64_t>(N));
      };
      while (docs.size() < df) {
        const size_t need = df - docs.size();
        for (size_t i = 0; i < need; ++i) docs.push_back(draw());
        std::sort(docs.begin(), docs.end());
        docs.erase(std::unique(docs.begin(), docs.end()), docs.end());
      }
    } else {
      docs.reserve(df);
      uint64_t need = df;
      for (int64_t d = 0; d < N && need; ++d)
        if (static_cast<double>(N - d) * unit(g) < static_cast<double>(need)) { docs.push_back(static_cast<uint32_t>(d)); --need; }
    }
  };
  // one term's docs and tfs, from its own seed (independent of the thread count)
  auto make_list = [&](int64_t id, std::vector<uint32_t>* docs_out, std::vector<uint32_t>* tfs_out) {
    std::mt19937_64 g(sp.seed ^ (0x9E3779B97F4A7C15ull * static_cast<uint64_t>(id + 1)));
    const uint32_t df = dfs[id];
    std::vector<uint32_t>& docs = *docs_out;
    docs.clear();
    const int64_t a = partner[id];
    if (a >= 0) {
      // a phrase's second word: c of its docs come from a's docs, the rest
      // are uniform (distinct from them)
      std::vector<uint32_t> ad;
      std::mt19937_64 ga(sp.seed ^ 0xA5A5A5A5A5A5A5A5ull ^ static_cast<uint64_t>(id));
      {
        // (a is never a pool b itself, so this does not recurse)
        std::mt19937_64 gg(sp.seed ^ (0x9E3779B97F4A7C15ull * static_cast<uint64_t>(a + 1)));
        uniform_docs(dfs[a], gg, &ad, a);
      }
      const uint32_t c = std::min<uint32_t>(df, static_cast<uint32_t>(ad.size())) / 2;
      // c of a's docs (partial Fisher-Yates), then uniform docs not yet taken
      for (uint32_t i = 0; i < c; ++i) std::swap(ad[i], ad[i + ga() % (ad.size() - i)]);
      docs.assign(ad.begin(), ad.begin() + c);
      std::sort(docs.begin(), docs.end());
      while (docs.size() < df) {
        const size_t have = docs.size();
        for (size_t i = have; i < df; ++i) docs.push_back(static_cast<uint32_t>(g() % static_cast<uint64_t>(N)));
        std::sort(docs.begin(), docs.end());
        docs.erase(std::unique(docs.begin(), docs.end()), docs.end());
      }
      if (docs.size() > df) docs.resize(df);   // (never: unique keeps at most df)
    } else {
      uniform_docs(df, g, &docs, id);
    }
    const double base = 0.3 + 5.0 * static_cast<double>(df) / static_cast<double>(N);
    tfs_out->resize(docs.size());
    for (size_t i = 0; i < docs.size(); ++i) {
      const double lam = base * verb[docs[i]];
      const double t = 1.0 + std::floor(-std::log(unit(g)) * lam);
      (*tfs_out)[i] = static_cast<uint32_t>(t > 60000.0 ? 60000.0 : t);
    }
  };

  auto run_parallel = [&](int64_t b0, int64_t b1, auto&& fn) {
    std::atomic<int64_t> next{b0};
    std::atomic<bool> failed{false};
    std::string err;
    auto work = [&] {
      try {
        for (int64_t v; (v = next++) < b1 && !failed;) fn(v);
      } catch (const std::exception& ex) {
        if (!failed.exchange(true)) err = ex.what();
      }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    if (failed) throw std::runtime_error(err);
  };

  // 4) doc lengths = the sum of each doc's tfs (pass 1: lists without positions)
  std::unique_ptr<std::atomic<uint32_t>[]> lenA(new std::atomic<uint32_t>[N]);
  for (int64_t d = 0; d < N; ++d) lenA[d].store(0, std::memory_order_relaxed);
  run_parallel(0, V, [&](int64_t v) {
    thread_local std::vector<uint32_t> docs, tfs;
    make_list(v, &docs, &tfs);
    for (size_t i = 0; i < docs.size(); ++i) lenA[docs[i]].fetch_add(tfs[i], std::memory_order_relaxed);
  });
  std::vector<uint32_t> len(N);
  for (int64_t d = 0; d < N; ++d) len[d] = lenA[d].load(std::memory_order_relaxed);
  lenA.reset();

  // the positions of term t in doc d: tf distinct values in [0, len[d]) from
  // the (t, d) stream, sorted; `forced` (if < len) is one of them
  auto positions = [&](int64_t t, uint32_t d, uint32_t tf, int64_t forced, std::vector<uint32_t>* out) {
    const uint32_t L = len[d];
    out->clear();
    if (tf >= L) {   // every position of the doc
      for (uint32_t p = 0; p < L; ++p) out->push_back(p);
      return;
    }
    uint64_t st = mix64(sp.seed ^ (static_cast<uint64_t>(t) * 0xD1B54A32D192ED03ull) ^
                        (static_cast<uint64_t>(d) << 1));
    if (forced >= 0 && forced < L) out->push_back(static_cast<uint32_t>(forced));
    if (tf <= 64) {
      while (out->size() < tf) {
        st = mix64(st);
        const uint32_t p = static_cast<uint32_t>(st % L);
        if (std::find(out->begin(), out->end(), p) == out->end()) out->push_back(p);
      }
    } else {
      std::unordered_set<uint32_t> seen(out->begin(), out->end());
      while (out->size() < tf) {
        st = mix64(st);
        const uint32_t p = static_cast<uint32_t>(st % L);
        if (seen.insert(p).second) out->push_back(p);
      }
    }
    std::sort(out->begin(), out->end());
  };

  // 5) pass 2: lists with positions, encoded in parallel batches, appended in
  //    term-id order (lists are streamed: host memory does not grow with the corpus)
  VacuumFileWriter w(out_dir);
  BuildStats st;
  const int64_t BATCH = 16384;
  for (int64_t b0 = 0; b0 < V; b0 += BATCH) {
    const int64_t b1 = std::min(V, b0 + BATCH);
    std::vector<std::unique_ptr<EncodedList>> enc(b1 - b0);
    run_parallel(b0, b1, [&](int64_t v) {
      TermPostings tp;
      make_list(v, &tp.docs, &tp.tfs);
      // a phrase's second word: in kPhraseRate of the docs it shares with a,
      // it occurs right after a's first occurrence
      const int64_t a = partner[v];
      std::vector<uint32_t> adocs, atfs;
      if (a >= 0) make_list(a, &adocs, &atfs);
      std::vector<uint32_t> pos, apos;
      size_t ai = 0;
      for (size_t i = 0; i < tp.docs.size(); ++i) {
        const uint32_t d = tp.docs[i], tf = tp.tfs[i];
        int64_t forced = -1;
        if (a >= 0) {
          while (ai < adocs.size() && adocs[ai] < d) ++ai;
          if (ai < adocs.size() && adocs[ai] == d &&
              (mix64(sp.seed ^ 0x7777ull ^ (static_cast<uint64_t>(v) << 32) ^ d) >> 11) * 0x1.0p-53 < kPhraseRate) {
            positions(a, d, atfs[ai], -1, &apos);
            forced = static_cast<int64_t>(apos[0]) + 1;
          }
        }
        positions(v, d, tf, forced, &pos);
        // bag: delta coded positions, offset pairs [9p, 9p + 7] delta coded
        // inside the bag (an 8-char term and a space per token)
        uint32_t pp = 0, po = 0;
        for (uint32_t p : pos) {
          tp.pos_vals.push_back(p - pp);
          pp = p;
          tp.off_vals.push_back(9 * p - po);
          tp.off_vals.push_back(7);
          po = 9 * p + 7;
        }
        tp.pos_sizes.push_back(tf);
        tp.off_sizes.push_back(2 * tf);
      }
      auto el = std::make_unique<EncodedList>();
      encode_list(tp, el.get());
      enc[v - b0] = std::move(el);
    });
    for (int64_t v = b0; v < b1; ++v) { w.add(wiki_term(v), *enc[v - b0]); st.n_postings += enc[v - b0]->df; }
  }
  w.close();
  DocLengths lens;
  lens.c4.reserve(N);
  for (int64_t d = 0; d < N; ++d) lens.add(len[d]);
  lens.write(out_dir);
  {
    std::ofstream pf(out_dir + "/phrases.txt", std::ios::trunc);
    if (!pf) throw std::runtime_error("cannot write " + out_dir + "/phrases.txt");
    for (const auto& pr : pool) pf << wiki_term(pr.first) << ' ' << wiki_term(pr.second) << '\n';
  }
  st.n_docs = N;
  st.n_terms = w.terms();
  st.vacuum_bytes = static_cast<int64_t>(w.bytes());
  st.docs_char4_ge_0x80 = lens.big;
  st.avg_length = lens.avg;
  return st;
}

// --------------------------------------------------------- query log gen --
namespace {
// The df groups of tools/gen_synthetic_log.py:21-28 over an index's df table:
// "low" = floor(log10 df) in 0..3, "high" = 4..6.  (my.vacuum is mapped: an
// index of millions of terms would cost a seek per term through a stream.)
void df_groups(const std::string& dir, std::vector<std::string>* low, std::vector<std::string>* high) {
  std::ifstream tip(dir + "/my.tip", std::ios::binary);
  if (!tip) throw std::runtime_error("cannot open index in " + dir);
  const int fd = ::open((dir + "/my.vacuum").c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + dir + "/my.vacuum");
  struct stat sb;
  if (::fstat(fd, &sb) != 0) { ::close(fd); throw std::runtime_error("stat my.vacuum"); }
  const uint64_t flen = static_cast<uint64_t>(sb.st_size);
  void* mp = flen ? ::mmap(nullptr, flen, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
  ::close(fd);
  if (mp == MAP_FAILED) throw std::runtime_error("mmap my.vacuum failed");
  const uint8_t* file = static_cast<const uint8_t*>(mp);
  std::string all((std::istreambuf_iterator<char>(tip)), std::istreambuf_iterator<char>());
  for (size_t at = 0; at + 4 <= all.size();) {
    uint32_t len;
    std::memcpy(&len, &all[at], 4);
    if (at + 4 + len + 8 > all.size()) break;
    std::string term = all.substr(at + 4, len);
    int64_t v;
    std::memcpy(&v, &all[at + 4 + len], 8);
    at += 4 + len + 8;
    const uint64_t off = tip_offset(v);
    uint64_t df = 0;
    if (off + 2 > flen || file[off] != kPostingListMagic || !get_varint(file + off + 1, file + flen, &df)) {
      ::munmap(mp, flen);
      throw std::runtime_error("bad posting list header for " + term);
    }
    if (df >= 1 && df < 10000) low->push_back(std::move(term));
    else if (df >= 10000 && df < 10000000) high->push_back(std::move(term));
  }
  ::munmap(mp, flen);
  if (low->empty() || high->empty() || low->size() + high->size() < 2)
    throw std::runtime_error("df table has an empty low or high group");
}

// One query per line; a file that cannot be opened or written fails the call.
void write_log(const std::string& out_path, const std::vector<std::string>& lines) {
  std::ofstream f(out_path, std::ios::trunc);
  if (!f) throw std::runtime_error("cannot open query log " + out_path);
  for (auto& q : lines) f << q << "\n";
  f.close();
  if (!f) throw std::runtime_error("cannot write query log " + out_path);
}
}  // namespace

int64_t gen_two_term_log(const std::string& dir, int64_t n_queries, uint64_t seed,
                         const std::string& out_path) {
  std::vector<std::string> low, high;
  df_groups(dir, &low, &high);
  std::mt19937_64 g(seed);
  std::unordered_set<std::string> seen;
  std::vector<std::string> out;
  int64_t guard = 0;
  while (static_cast<int64_t>(out.size()) < n_queries) {
    if (++guard > 1000 * n_queries + 1000000) throw std::runtime_error("cannot find enough distinct queries");
    const auto& g1 = (g() & 1) ? high : low;
    const auto& g2 = (g() & 1) ? high : low;
    std::string t1 = g1[g() % g1.size()];
    std::string t2 = g2[g() % g2.size()];
    int spins = 0;
    while (t2 == t1 && spins++ < 1000) t2 = g2[g() % g2.size()];
    if (t2 == t1) continue;
    if (t2 < t1) std::swap(t1, t2);
    std::string q = t1 + " " + t2;
    if (seen.insert(q).second) out.push_back(q);
  }
  write_log(out_path, out);
  return static_cast<int64_t>(out.size());
}

int64_t gen_mixed_log(const std::string& dir, int64_t n_queries, uint64_t seed,
                      const std::string& out_path) {
  std::vector<std::string> low, high;
  df_groups(dir, &low, &high);
  // terms per query: the AOL log's shares of 1..5-term queries
  // (data/AOL_QueryLog_analysis/stat.txt), renormalised
  const double share[5] = {36.8, 25.2, 17.3, 10.0, 5.3};
  double tot = 0;
  for (double x : share) tot += x;
  std::mt19937_64 g(seed);
  std::unordered_set<std::string> seen;
  std::vector<std::string> out;
  int64_t guard = 0;
  while (static_cast<int64_t>(out.size()) < n_queries) {
    if (++guard > 1000 * n_queries + 1000000) throw std::runtime_error("cannot find enough distinct queries");
    const double u = (static_cast<double>(g() >> 11) * 0x1.0p-53) * tot;
    int n = 1;
    for (double acc = share[0]; n < 5 && u >= acc; acc += share[n], ++n) {}
    std::vector<std::string> terms;
    int spins = 0;
    while (static_cast<int>(terms.size()) < n && spins++ < 10000) {
      const auto& grp = (g() & 1) ? high : low;   // as two_term_queries: group, then term
      std::string t = grp[g() % grp.size()];
      if (std::find(terms.begin(), terms.end(), t) == terms.end()) terms.push_back(t);
    }
    if (static_cast<int>(terms.size()) < n) continue;
    std::sort(terms.begin(), terms.end());
    std::string q;
    for (auto& t : terms) q += (q.empty() ? "" : " ") + t;
    if (seen.insert(q).second) out.push_back(q);
  }
  write_log(out_path, out);
  return static_cast<int64_t>(out.size());
}

int64_t gen_single_term_log(const std::string& dir, bool high, int64_t n_queries, uint64_t seed,
                            const std::string& out_path) {
  std::vector<std::string> low, hi;
  df_groups(dir, &low, &hi);
  const auto& grp = high ? hi : low;
  std::mt19937_64 g(seed);
  if (grp.empty()) throw std::runtime_error("no terms in the requested df group");
  std::vector<std::string> out;
  out.reserve(static_cast<size_t>(std::max<int64_t>(n_queries, 0)));
  for (int64_t i = 0; i < n_queries; ++i) out.push_back(grp[g() % grp.size()]);
  write_log(out_path, out);
  return n_queries;
}

int64_t gen_phrase_log(const std::string& dir, int64_t n_queries, uint64_t seed,
                       const std::string& out_path) {
  std::ifstream in(dir + "/phrases.txt");
  if (!in) throw std::runtime_error("no phrase pool " + dir + "/phrases.txt (a synthetic index "
                                    "built with positions writes one)");
  std::vector<std::string> pool;
  for (std::string line; std::getline(in, line);)
    if (!line.empty()) pool.push_back(line);
  // rand_items_from_set: n distinct phrases (partial Fisher-Yates)
  std::mt19937_64 g(seed);
  const int64_t n = std::min<int64_t>(n_queries, static_cast<int64_t>(pool.size()));
  for (int64_t i = 0; i < n; ++i)
    std::swap(pool[i], pool[i + static_cast<int64_t>(g() % (pool.size() - i))]);
  std::vector<std::string> out;
  for (int64_t i = 0; i < n; ++i) out.push_back('"' + pool[i] + '"');   // gen_synthetic_log.py:262
  write_log(out_path, out);
  return n;
}

}  // namespace wiser
