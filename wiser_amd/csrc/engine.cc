// C ABI (include/wiser_hip.h) over the HIP engine: index load + HBM upload,
// resident query batches, kernel launches, result download.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <cstdio>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <cstdlib>
#include <deque>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wiser_hip.h"
#include "engine_types.h"
#include "index.h"
#include "kernels.h"
#include "snippet.h"
#include "writer.h"

namespace wiser {
constexpr int kSegCostMax = kSegCost;
}  // namespace wiser

using namespace wiser;

namespace {
thread_local std::string g_err;

// the list ids of a query in query order (list_ids, then more_ids)
std::vector<int32_t> query_terms(const wsr_query& q) {
  std::vector<int32_t> t(q.n_terms > 0 ? static_cast<size_t>(q.n_terms) : 0u);
  for (int i = 0; i < q.n_terms; ++i) t[i] = i < WSR_MAX_TERMS ? q.list_ids[i] : q.more_ids[i - WSR_MAX_TERMS];
  return t;
}


int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace

namespace wiser {
// (server.cc: a request failed on the dispatcher thread; its caller's thread
// gets the message)
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace wiser

namespace {

#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

template <class T, class A>
uint64_t dev_upload(T** dst, const std::vector<T, A>& src) {
  const size_t n = std::max<size_t>(src.size(), 1) * sizeof(T);
  HIP_OK(hipMalloc(reinterpret_cast<void**>(dst), n));
  if (!src.empty()) HIP_OK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return n;
}

// tuning knobs read once per wsr_open (unset or unparsable: the default)
double env_number(const char* name, double dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const double x = std::strtod(v, &end);
  return (end && *end == 0 && x >= 0) ? x : dflt;
}

}  // namespace

struct wsr_handle {
  std::mutex mu;
  int device = 0;
  hipStream_t stream = nullptr;
  VacuumIndex idx;
  DocStore docs;                    // my.fdx / my.fdt when the index has them (snippets)
  std::unique_ptr<SkipRowCache> rows;   // decoded skip rows for the snippet stage
  std::mutex pool_mu;                   // wsr_search_batch's reusable batches
  std::vector<wsr_batch*> pool;
  IndexArgs args{};
  uint8_t* d_blob = nullptr;
  ListDev* d_lists = nullptr;
  BlockDev* d_blocks = nullptr;
  uint32_t* d_last = nullptr;
  uint32_t* d_meta = nullptr;
  uint8_t* d_c4 = nullptr;
  double* d_cache = nullptr;
  DenseEnt* d_dense = nullptr;
  uint32_t* d_dense_rk = nullptr;   // the bitmap entries' rank records
  uint32_t* d_bkt = nullptr;        // offset buckets (entries and offset bytes)
  uint8_t* d_tf8 = nullptr;
  uint8_t* d_plen = nullptr;
  float* d_bmax = nullptr;
  uint32_t* d_tails = nullptr;
  uint8_t* d_pos_blob = nullptr;    // positions (opened with wsr_open_opts::positions)
  PosDev* d_pos_lists = nullptr;
  uint32_t* d_pos_pk = nullptr;
  uint32_t* d_pos_tail = nullptr;
  uint32_t* d_pos_start = nullptr;
  uint8_t* d_blm = nullptr;
  uint32_t* d_blm_hash = nullptr;
  bool positions = false;
  uint32_t dense_lists = 0;
  wsr_image_info info{};            // HBM bytes of the image's buffers
  std::vector<ListDev> lists;       // host copy of the directory heads
  std::vector<uint64_t> list_bytes; // docid+tf span bytes per list in this image
  std::vector<uint64_t> pos_bytes;  // position box bytes per list (positions on)
  std::vector<BlockDev> blocks;     // host copy (debug decode)
  std::vector<uint32_t> meta;
  // host-exchange owner replays deferred into a later batch run's lean kernel
  // (wsr_shard_step_replay_deferred), oldest first
  std::mutex hdef_mu;
  std::deque<wsr_batch*> hdef_q;
  int grid = 0;        // general segment kernel: workgroups (one wave each)
  int lean_wgs = 0;    // lean kernel: workgroups of kLeanWaves waves
  int lean_wgs_ph = 0; // ... its phrase instance's
  int lean_wgs_two = 0; // ... its two-term instance's (one workgroup per CU past residency)
  int gen_cap = 0;     // general workgroups launched at most
};

struct wsr_batch {
  int max_q = 0, stride = 0, nq = 0;
  QueryIn* d_q = nullptr;          // QueryIn[nq], then the term table of queries over kMaxTerms
  size_t q_cap = 0;                // bytes of d_q
  QueryPlan* d_plan = nullptr;
  QueryDesc* d_desc = nullptr;     // lean queries' work records
  PlanPart* d_part = nullptr;      // plan pass 1 -> 2 partial sums, per kPlanThreads queries
  uint32_t* d_ctr = nullptr;
  uint32_t* h_ctr = nullptr;       // pinned host copy of the counters (fetch)
  Event* d_events = nullptr;
  uint64_t ev_cap = 0;
  uint32_t* d_evcnt = nullptr;
  uint64_t item_cap = 0;
  HitDev* d_hits = nullptr;
  int32_t* d_nhits = nullptr;
  uint32_t* d_qdone = nullptr;   // fused replay: completed items per query
  uint32_t* d_itemq = nullptr;   // item -> query (capacity item_cap)
  uint64_t* d_pub = nullptr;     // per item score floor (capacity item_cap)
  uint32_t* d_stats = nullptr;   // per general workgroup, then per lean wave: survivors, blocks
  uint32_t* d_ph = nullptr;      // phrase scratch, gen_cap * kPhraseScratch (lazily)
  bool has_phrase = false;       // the uploaded queries include a phrase query
  bool gen_phrase = false;       // ... one of the general class (segment_kernel's phrase instance)
  bool has_conj_lean = true;     // the host's class rule found a conjunctive lean query
  bool has_gen = true;           // ... a general one
  bool ran_conj = true, ran_gen = true;   // the last run launched them (their stats rows are its own)
  bool has_wide = false;         // ... a query with k > kMaxK (wide_replay_kernel)
  bool two_conj = false;         // every conjunctive query: two terms (or empty), k <= kMaxK
  bool two_ph = false;           // every phrase query: k <= kMaxK (a lean one has two terms)
  bool one_conj = false;         // every conjunctive query: one term (or empty)
  uint32_t seg_cap = kSegCost;   // driver blocks per work item at most (wsr_batch_set_item_blocks)
  int seg_grid = 0;
  int lean_wgs = 0;      // the conjunctive lean instance's grid
  int lean_wgs_ph = 0;   // the phrase instance's (batches with phrase queries)
  // doc-range shard exchange (wsr_shard_step): per owner a region of {count,
  // offset} pairs + an event slot, owner-major to send, shard-major received;
  // allocated on first use
  Event* d_xsend = nullptr;
  Event* d_xrecv = nullptr;
  uint64_t x_slots = 0;     // region events * pairs the two exchange buffers were sized for
  int x_pairs = 0;
  hipEvent_t xev[2] = {nullptr, nullptr};   // emission done -> comm stream; exchange done -> replay
  std::atomic<bool> x_pending{false};   // a shard step's exchange + owner replay (xev[1]) not yet joined
  // exchanges asked of the communicator's worker thread for this batch, and
  // those it has enqueued (xev[1] recorded): xev[1] is only waited on once
  // they agree (x_join)
  std::atomic<uint64_t> x_req{0};
  std::atomic<uint64_t> x_enq{0};
  // a step group's owner replay of this batch deferred (wsr_shard_steps) and
  // not yet enqueued: x_join has x_comm enqueue it first (atomic: a fetch on
  // one thread may race a step group on another; the communicator's pend_mu
  // orders what the two do with the group)
  std::atomic<wsr_comm*> x_comm{nullptr};
  bool x_fused = false;     // the last run emitted into the exchange regions (fill counters after d_ctr)
  // a host-exchange owner replay of this batch waiting for another batch's
  // run to carry it (wsr_shard_step_replay_deferred); its regions are in
  // d_xrecv once xev[0] (recorded after their copy on st) has passed.  Set and
  // cleared under the handle's hdef_mu; a run that takes it counts it in
  // x_req before clearing it, so x_join waits for its enqueue
  std::atomic<wsr_handle*> hdef{nullptr};
  int32_t hdef_rank = 0;
  int x_world = 0, x_qpr = 0;   // ... for this world and q_per_owner
  int64_t x_slot = 0;           //     and slot (the replay half must match them)
  uint64_t algo_static = 0;  // sum of list spans + k*12 over the uploaded queries
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};   // [4]: lean kernel end
  // Each batch runs on its own streams, so consecutive batches overlap on the
  // device (one's plan and first items under the other's last items); the
  // general kernel goes to st2, forked from and joined back into st.  HIP maps
  // streams to its hardware queues (GPU_MAX_HW_QUEUES, 4) round-robin in
  // creation order, and kernels of one queue run in order: a batch creates
  // three streams (st_pad carries only the conjunctive lean kernel of batches
  // with phrase queries, beside the other two), so the lean kernels of consecutive
  // batches land on queues 3 apart, i.e. on all four in turn, instead of
  // alternating between two (with two streams per batch the C3 headline fell
  // from 21.7 to 18.9 M q/s and C2 from 35.0 to 29.6 M at unchanged per-batch
  // kernel times, profiles/r04a_bench.json).
  hipStream_t st = nullptr, st2 = nullptr, st_pad = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, join_ph = nullptr;
  bool ran = false;
};
static void replay_flush(wsr_comm* c, const wsr_batch* upto);
static void host_replay_flush(wsr_batch* b);
// Is a shard step's exchange of b outstanding?  First wait until every
// exchange and owner replay asked for b is enqueued (by the communicator's
// worker, or, deferred, by a later step group or batch run: enqueued now if
// still pending), so that xev[1] is the record to wait on.
static bool x_join(wsr_batch* b) {
  if (b->hdef) host_replay_flush(b);
  if (wsr_comm* c = b->x_comm.load(std::memory_order_acquire)) replay_flush(c, b);
  while (b->x_enq.load(std::memory_order_acquire) != b->x_req.load(std::memory_order_acquire))
    std::this_thread::yield();
  return b->x_pending;
}

namespace {
// bytes dev_upload allocates for a host array (at least one element)
template <class V>
uint64_t dev_bytes(const V& v) {
  return std::max<uint64_t>(v.size(), 1) * sizeof(typename V::value_type);
}

// the image's HBM buffers, per kind, as wsr_open allocates them
wsr_image_info image_info_of(const HostImage& img, size_t n_c4) {
  wsr_image_info o{};
  if (img.has_blooms) o.pos_bytes += dev_bytes(img.blm) + dev_bytes(img.blm_hash);
  if (img.has_positions)
    o.pos_bytes += dev_bytes(img.pos_blob) + dev_bytes(img.pos_lists) + dev_bytes(img.pos_pk) +
                   dev_bytes(img.pos_tail) + dev_bytes(img.pos_start);
  o.dense_bytes = dev_bytes(img.dense) + dev_bytes(img.dense_rank) + dev_bytes(img.bkt);
  o.tf8_bytes = dev_bytes(img.tf8);
  o.blob_bytes = dev_bytes(img.blob);
  o.plen_bytes = dev_bytes(img.plen);
  o.dir_bytes = dev_bytes(img.tails) + dev_bytes(img.lists) + dev_bytes(img.blocks) + dev_bytes(img.blk_last) +
                dev_bytes(img.blk_meta) + dev_bytes(img.bmax) + std::max<uint64_t>(n_c4, 1);
  o.dense_lists = img.dense_lists;
  o.n_lists = static_cast<uint32_t>(img.lists.size());
  o.total_bytes = o.blob_bytes + o.dense_bytes + o.tf8_bytes + o.plen_bytes + o.dir_bytes + o.pos_bytes;
  return o;
}

// the load-time knobs of wsr_open (environment)
uint32_t dense_div_knob() { return static_cast<uint32_t>(env_number("WSR_DENSE_DIV", 8192)); }
uint64_t dense_budget_knob() { return static_cast<uint64_t>(env_number("WSR_DENSE_BUDGET_GB", 48) * 1e9); }
}  // namespace

extern "C" {

const char* wsr_last_error(void) { return g_err.c_str(); }
const char* wsr_version(void) { return "wiser-hip 0.2 (gfx950)"; }

int wsr_image_info_get(wsr_handle* h, wsr_image_info* out) {
  if (!h || !out) return fail(WSR_E_INVALID, "null argument");
  *out = h->info;
  out->total_bytes = out->blob_bytes + out->dense_bytes + out->tf8_bytes + out->plen_bytes + out->dir_bytes +
                     out->pos_bytes;
  return WSR_OK;
}


int wsr_image_size(const char* dir, uint32_t doc_lo, uint32_t doc_hi, int32_t positions, int32_t bloom_factor,
                   int32_t threads, wsr_image_info* out) {
  if (!dir || !out) return fail(WSR_E_INVALID, "null argument");
  try {
    VacuumIndex idx;
    idx.open(dir);
    const int t = threads > 0 ? threads : static_cast<int>(std::thread::hardware_concurrency());
    const HostImage img = build_image(idx, doc_lo, doc_hi ? doc_hi : 0xFFFFFFFFu, std::min(t, 32), dense_div_knob(),
                                      positions != 0, dense_budget_knob(), positions && bloom_factor > 0);
    *out = image_info_of(img, idx.char4_lengths().size());
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_runtime_info(char* buf, int32_t cap) {
  if (!buf || cap <= 0) return fail(WSR_E_INVALID, "null argument");
  int ver = 0;
  (void)hipRuntimeGetVersion(&ver);
  Dl_info hip{}, rccl{};
  const char* hp = dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &hip) && hip.dli_fname ? hip.dli_fname : "?";
  const char* rp = dladdr(reinterpret_cast<void*>(&ncclGetUniqueId), &rccl) && rccl.dli_fname ? rccl.dli_fname : "?";
  std::snprintf(buf, static_cast<size_t>(cap), "hipRuntimeGetVersion=%d libamdhip64=%s librccl=%s", ver, hp, rp);
  return WSR_OK;
}

int wsr_open(const char* dir, const wsr_open_opts* opts, wsr_handle** out) {
  if (!dir || !out) return fail(WSR_E_INVALID, "null argument");
  *out = nullptr;
  std::unique_ptr<wsr_handle> h(new wsr_handle());
  try {
    h->idx.open(dir);
    h->docs.open(dir);
    h->rows.reset(new SkipRowCache(h->idx));
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  try {
    const int dev = opts ? opts->device : 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= dev)
      return fail(WSR_E_HIP, "no HIP device " + std::to_string(dev) + " (MI355X required; no CPU fallback)");
    HIP_OK(hipSetDevice(dev));
    h->device = dev;
    uint32_t lo = opts ? opts->doc_lo : 0, hi = opts ? opts->doc_hi : 0;
    if (hi == 0) hi = 0xFFFFFFFFu;
    int threads = opts && opts->threads > 0 ? opts->threads : static_cast<int>(std::thread::hardware_concurrency());
    // probe structures (bitmaps, offset buckets): lists with >= span/div
    // postings (WSR_DENSE_DIV, 0 = off), probed when >= ratio x the driver's
    // blocks (WSR_DENSE_RATIO).  8192 since round 4's buckets made a sparse
    // list's structure cheap (~6 B per posting + 8 B per 256 docs): on the C3
    // stand-in C5 6.1 -> 10.1 M q/s against 2048 (its phrases' lists become
    // lean), headline and C4 within 1 %, image 10.1 -> 14.0 GB (16384 and
    // 32768: C5 the same, headline +0.4 %, 17.6 / 23.0 GB;
    // profiles/r04k/, r04l/).  WSR_DENSE_BUDGET_GB caps their HBM, longest
    // lists first (48 GB)
    const uint32_t dense_div = dense_div_knob();
    const uint64_t dense_budget = dense_budget_knob();
    const float dense_ratio = static_cast<float>(env_number("WSR_DENSE_RATIO", 1.0));
    h->positions = opts && opts->positions;
    const uint32_t bloom_factor = opts && opts->bloom_factor > 0 ? static_cast<uint32_t>(opts->bloom_factor) : 0u;
    // (the bitmaps are sized to what the device has free: an image larger than
    // the free HBM drops the bitmaps of its shortest dense lists first)
    size_t hbm_free = 0, hbm_total = 0;
    HIP_OK(hipMemGetInfo(&hbm_free, &hbm_total));
    HostImage img = build_image(h->idx, lo, hi, std::min(threads, 32), dense_div, h->positions, dense_budget,
                                bloom_factor > 0, hbm_free);
    if (img.has_blooms) {   // (counted with the position boxes)
      h->info.pos_bytes += dev_upload(&h->d_blm, img.blm);
      h->info.pos_bytes += dev_upload(&h->d_blm_hash, img.blm_hash);
      h->args.blm = reinterpret_cast<const uint4*>(h->d_blm);
      h->args.blm_hash = reinterpret_cast<const uint2*>(h->d_blm_hash);
      h->args.blm_bits = img.blm_bits;
      h->args.blm_hashes = img.blm_hashes;
      h->args.bloom_factor = bloom_factor;
      big_vector<uint8_t>().swap(img.blm);
    }
    if (h->positions) {
      h->info.pos_bytes += dev_upload(&h->d_pos_blob, img.pos_blob);
      h->info.pos_bytes += dev_upload(&h->d_pos_lists, img.pos_lists);
      h->info.pos_bytes += dev_upload(&h->d_pos_pk, img.pos_pk);
      h->info.pos_bytes += dev_upload(&h->d_pos_tail, img.pos_tail);
      h->info.pos_bytes += dev_upload(&h->d_pos_start, img.pos_start);
      h->args.pos_blob = h->d_pos_blob;
      h->args.pos_lists = h->d_pos_lists;
      h->args.pos_pk = reinterpret_cast<const uint2*>(h->d_pos_pk);
      h->args.pos_tail = h->d_pos_tail;
      h->args.pos_start = reinterpret_cast<const uint2*>(h->d_pos_start);
      h->pos_bytes = img.pos_list_bytes;
      std::vector<uint8_t>().swap(img.pos_blob);
      std::vector<uint32_t>().swap(img.pos_start);
    }
    h->info.dense_bytes = dev_upload(&h->d_dense, img.dense);
    h->info.dense_bytes += dev_upload(&h->d_dense_rk, img.dense_rank);
    h->info.dense_bytes += dev_upload(&h->d_bkt, img.bkt);
    h->info.tf8_bytes = dev_upload(&h->d_tf8, img.tf8);
    h->dense_lists = img.dense_lists;
    h->info.dense_lists = img.dense_lists;
    h->info.n_lists = static_cast<uint32_t>(img.lists.size());
    h->args.dense = h->d_dense;
    h->args.dense_rk = h->d_dense_rk;
    h->args.bkt = reinterpret_cast<const uint2*>(h->d_bkt);
    h->args.tf8 = h->d_tf8;
    h->args.dense_span = img.dense_span;
    h->args.dense_ratio = dense_ratio;
    h->args.seg_cap = kSegCost;
    h->info.blob_bytes = dev_upload(&h->d_blob, img.blob);
    h->info.plen_bytes = dev_upload(&h->d_plen, img.plen);
    h->args.plen = h->d_plen;
    h->info.dir_bytes += dev_upload(&h->d_bmax, img.bmax);
    h->args.bmax = h->d_bmax;
    h->info.dir_bytes += dev_upload(&h->d_tails, img.tails);
    h->args.tails = h->d_tails;
    h->info.dir_bytes += dev_upload(&h->d_lists, img.lists);
    h->info.dir_bytes += dev_upload(&h->d_blocks, img.blocks);
    h->info.dir_bytes += dev_upload(&h->d_last, img.blk_last);
    h->info.dir_bytes += dev_upload(&h->d_meta, img.blk_meta);
    h->info.dir_bytes += dev_upload(&h->d_c4, h->idx.char4_lengths());
    std::vector<double> cache(h->idx.bm25_cache(), h->idx.bm25_cache() + 256);
    dev_upload(&h->d_cache, cache);
    h->lists = img.lists;
    h->blocks.assign(img.blocks.begin(), img.blocks.end());
    h->meta.assign(img.blk_meta.begin(), img.blk_meta.end());
    h->list_bytes = img.list_bytes;
    h->args.blob = h->d_blob;
    h->args.lists = h->d_lists;
    h->args.blocks = h->d_blocks;
    h->args.blk_last = h->d_last;
    h->args.blk_meta = h->d_meta;
    h->args.c4 = h->d_c4;
    h->args.cache = h->d_cache;
    h->args.n_c4 = static_cast<uint32_t>(h->idx.char4_lengths().size());
    h->args.n_lists = static_cast<uint32_t>(img.lists.size());
    h->args.doc_lo = lo;
    h->args.doc_hi = hi;
    h->args.avg = h->idx.avg_length();
    HIP_OK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));

    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, dev));
    int occ = segment_kernel_occupancy();
    if (occ < 1) occ = 1;
    h->grid = prop.multiProcessorCount * std::min(occ, 32);
    // general workers hold 12 KB of LDS each: at most 4 per CU, so that the
    // concurrent lean kernel keeps its occupancy
    // (one workgroup per CU past that: it starts as the first resident ones
    // leave; C4 +1.6 %, the mixed log +0.6 %, the rest unchanged,
    // profiles/r05/leg_ab.txt r05ar / r05as)
    const int gen_per_cu = static_cast<int>(env_number("WSR_GEN_PER_CU", 4));
    h->gen_cap = prop.multiProcessorCount * std::max(1, std::min(std::min(occ, 32), gen_per_cu) + 1);
    int locc = lean_kernel_occupancy(false);
    if (locc < 1) locc = 1;
    h->lean_wgs = prop.multiProcessorCount * std::min(locc, 16);
    // the phrase instance holds more registers: its resident grid is smaller
    // (workgroups past it would start only as resident ones leave)
    int pocc = lean_kernel_occupancy(true);
    if (pocc < 1) pocc = 1;
    h->lean_wgs_ph = prop.multiProcessorCount * std::min(std::min(pocc, locc), 16);
    // Batches whose conjunctive items are all two-term (the headline's) run one
    // workgroup per CU past the resident grid: it starts as the first resident
    // waves leave and takes items from the queue's tail (C3 24.0 -> 24.5 M q/s,
    // C2 and C4 unchanged; 2 to 11 more: no better, 11 -6 %; single-term
    // batches -2 %, so they keep the resident grid: profiles/r05/leg_ab.txt r05u-w)
    h->lean_wgs_two = prop.multiProcessorCount * std::min(locc + 1, 16);
  } catch (const std::exception& e) {
    wsr_close(h.release());
    return fail(WSR_E_HIP, e.what());
  }
  *out = h.release();
  return WSR_OK;
}

void wsr_close(wsr_handle* h) {
  if (!h) return;
  for (wsr_batch* b : h->pool) wsr_batch_destroy(h, b);
  h->pool.clear();
  if (h->stream) { (void)hipStreamSynchronize(h->stream); (void)hipStreamDestroy(h->stream); }

  for (void* p : {static_cast<void*>(h->d_blob), static_cast<void*>(h->d_lists),
                  static_cast<void*>(h->d_blocks), static_cast<void*>(h->d_last),
                  static_cast<void*>(h->d_meta),
                  static_cast<void*>(h->d_c4), static_cast<void*>(h->d_cache),
                  static_cast<void*>(h->d_dense), static_cast<void*>(h->d_dense_rk),
                  static_cast<void*>(h->d_bkt), static_cast<void*>(h->d_tf8),
                  static_cast<void*>(h->d_plen), static_cast<void*>(h->d_bmax), static_cast<void*>(h->d_tails),
                  static_cast<void*>(h->d_pos_blob), static_cast<void*>(h->d_pos_lists),
                  static_cast<void*>(h->d_pos_pk), static_cast<void*>(h->d_pos_tail),
                  static_cast<void*>(h->d_pos_start), static_cast<void*>(h->d_blm),
                  static_cast<void*>(h->d_blm_hash)})
    if (p) (void)hipFree(p);
  delete h;
}

int wsr_term_count(wsr_handle* h, int32_t* out) {
  if (!h || !out) return fail(WSR_E_INVALID, "null argument");
  *out = h->idx.n_lists();
  return WSR_OK;
}

int wsr_n_docs(wsr_handle* h, int32_t* out) {
  if (!h || !out) return fail(WSR_E_INVALID, "null argument");
  *out = h->idx.n_docs();
  return WSR_OK;
}

int wsr_lookup(wsr_handle* h, const char* term, int32_t* list_id, int32_t* df) {
  if (!h || !term) return fail(WSR_E_INVALID, "null argument");
  const int32_t id = h->idx.find(term);
  if (list_id) *list_id = id;
  if (df) *df = id < 0 ? 0 : static_cast<int32_t>(h->idx.df(id));
  return WSR_OK;
}

// ------------------------------------------------------------ snippets ----
// Host stage after the top-k, as in the reference (vacuum_engine.h:243-253).
struct wsr_docs {
  VacuumIndex idx;
  DocStore docs;
  std::unique_ptr<SkipRowCache> rows;
};

namespace {
int copy_out(const std::string& s, char* out, int32_t cap, int32_t* len) {
  if (len) *len = static_cast<int32_t>(s.size());
  if (out && cap > 0) std::memcpy(out, s.data(), std::min<size_t>(s.size(), static_cast<size_t>(cap)));
  return WSR_OK;
}

int check_snippet_query(const VacuumIndex& idx, const DocStore& docs, const wsr_query* q) {
  if (q->n_terms < 1 || q->n_terms > WSR_MAX_QUERY_TERMS) return fail(WSR_E_LIMIT, "bad term count");
  if (q->n_terms > WSR_MAX_TERMS && !q->more_ids) return fail(WSR_E_INVALID, "more_ids missing");
  if (!docs.is_open()) return fail(WSR_E_INVALID, "the index has no doc store (my.fdx / my.fdt)");
  for (int32_t id : query_terms(*q))
    if (id < 0 || id >= idx.n_lists())
      return fail(WSR_E_INVALID, "a query term is not in the index (no result entries)");
  return WSR_OK;
}

int snippet_of(const VacuumIndex& idx, const SkipRowCache& rows, const DocStore& docs, const wsr_query* q,
               int32_t doc, int32_t n_passages, char* out, int32_t cap, int32_t* len) {
  if (!q || !len || n_passages < 0) return fail(WSR_E_INVALID, "bad snippet arguments");
  const int rc = check_snippet_query(idx, docs, q);
  if (rc != WSR_OK) return rc;
  try {
    const std::vector<int32_t> ids = query_terms(*q);
    return copy_out(make_snippet(idx, rows, docs, ids.data(), q->n_terms,
                                 (q->flags & WSR_QUERY_PHRASE) != 0, doc, n_passages),
                    out, cap, len);
  } catch (const std::exception& e) {
    return fail(WSR_E_INVALID, e.what());
  }
}

int doc_text(const DocStore& docs, int32_t doc, char* out, int32_t cap, int32_t* len) {
  if (!len) return fail(WSR_E_INVALID, "null argument");
  try {
    return copy_out(docs.get(doc), out, cap, len);
  } catch (const std::exception& e) {
    return fail(WSR_E_INVALID, e.what());
  }
}
}  // namespace

int wsr_snippet(wsr_handle* h, const wsr_query* q, int32_t doc, int32_t n_passages, char* out,
                int32_t cap, int32_t* len) {
  if (!h) return fail(WSR_E_INVALID, "null argument");
  return snippet_of(h->idx, *h->rows, h->docs, q, doc, n_passages, out, cap, len);
}

int wsr_snippets_batch(wsr_handle* h, const wsr_query* q, int32_t nq, const wsr_hit* hits,
                       const int32_t* n_hits, int32_t stride, int32_t n_passages, int32_t threads,
                       char* buf, uint64_t cap, uint64_t* ends, uint64_t* total) {
  if (!h || (nq > 0 && (!q || !hits || !n_hits || !ends)) || !total || nq < 0 || stride <= 0 ||
      n_passages < 0)
    return fail(WSR_E_INVALID, "bad snippet batch arguments");
  std::vector<std::pair<int32_t, int32_t>> work;   // (query, entry)
  for (int32_t i = 0; i < nq; ++i) {
    if (n_hits[i] < 0 || n_hits[i] > stride) return fail(WSR_E_INVALID, "bad hit count");
    if (n_hits[i] == 0) continue;
    const int rc = check_snippet_query(h->idx, h->docs, &q[i]);
    if (rc != WSR_OK) return rc;
    for (int32_t j = 0; j < n_hits[i]; ++j) work.emplace_back(i, j);
  }
  std::vector<std::string> out(static_cast<size_t>(nq) * stride);
  std::atomic<size_t> next{0};
  std::mutex err_mu;
  std::string err;
  auto run = [&]() {
    for (size_t w; (w = next.fetch_add(1)) < work.size();) {
      const int32_t i = work[w].first, j = work[w].second;
      try {
        const std::vector<int32_t> ids = query_terms(q[i]);
        out[static_cast<size_t>(i) * stride + j] =
            make_snippet(h->idx, *h->rows, h->docs, ids.data(), q[i].n_terms,
                         (q[i].flags & WSR_QUERY_PHRASE) != 0, hits[static_cast<size_t>(i) * stride + j].doc_id,
                         n_passages);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(err_mu);
        if (err.empty()) err = e.what();
      }
    }
  };
  int nt = threads > 0 ? threads : static_cast<int>(std::thread::hardware_concurrency());
  nt = std::max(1, std::min<int>(nt, std::min<size_t>(64, work.size())));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(run);
  run();
  for (auto& t : pool) t.join();
  if (!err.empty()) return fail(WSR_E_INVALID, err);
  uint64_t n = 0;
  for (const auto& s : out) n += s.size();
  *total = n;
  if (n > cap) return fail(WSR_E_LIMIT, "snippet buffer too small (see *total)");
  uint64_t at = 0;
  for (size_t e = 0; e < out.size(); ++e) {
    if (!out[e].empty()) std::memcpy(buf + at, out[e].data(), out[e].size());
    at += out[e].size();
    ends[e] = at;
  }
  return WSR_OK;
}

int wsr_doc_get(wsr_handle* h, int32_t doc, char* out, int32_t cap, int32_t* len) {
  if (!h) return fail(WSR_E_INVALID, "null argument");
  return doc_text(h->docs, doc, out, cap, len);
}

int wsr_docs_open(const char* dir, wsr_docs** out) {
  if (!dir || !out) return fail(WSR_E_INVALID, "null argument");
  *out = nullptr;
  std::unique_ptr<wsr_docs> d(new wsr_docs());
  try {
    d->idx.open(dir);
    if (!d->docs.open(dir)) return fail(WSR_E_IO, std::string("no doc store in ") + dir);
    d->rows.reset(new SkipRowCache(d->idx));
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  *out = d.release();
  return WSR_OK;
}

void wsr_docs_close(wsr_docs* d) { delete d; }

int wsr_docs_lookup(wsr_docs* d, const char* term, int32_t* list_id, int32_t* df) {
  if (!d || !term) return fail(WSR_E_INVALID, "null argument");
  const int32_t id = d->idx.find(term);
  if (list_id) *list_id = id;
  if (df) *df = id < 0 ? 0 : static_cast<int32_t>(d->idx.df(id));
  return WSR_OK;
}

int wsr_docs_snippet(wsr_docs* d, const wsr_query* q, int32_t doc, int32_t n_passages, char* out,
                     int32_t cap, int32_t* len) {
  if (!d) return fail(WSR_E_INVALID, "null argument");
  return snippet_of(d->idx, *d->rows, d->docs, q, doc, n_passages, out, cap, len);
}

int wsr_docs_get(wsr_docs* d, int32_t doc, char* out, int32_t cap, int32_t* len) {
  if (!d) return fail(WSR_E_INVALID, "null argument");
  return doc_text(d->docs, doc, out, cap, len);
}

int wsr_highlight(const int32_t* pairs, const int32_t* counts, int32_t n_terms, int32_t n_passages,
                  const char* text, char* out, int32_t cap, int32_t* len) {
  if ((!pairs && n_terms > 0) || (!counts && n_terms > 0) || !text || !len || n_terms < 0)
    return fail(WSR_E_INVALID, "null argument");
  try {
    std::vector<std::vector<OffsetPair>> t(n_terms);
    for (int32_t i = 0; i < n_terms; ++i)
      for (int32_t j = 0; j < counts[i]; ++j, pairs += 2) t[i].emplace_back(pairs[0], pairs[1]);
    return copy_out(highlight_offsets(t, n_passages, text), out, cap, len);
  } catch (const std::exception& e) {
    return fail(WSR_E_INVALID, e.what());
  }
}

int wsr_list_bytes(wsr_handle* h, int32_t id, uint64_t* out) {
  if (!h || !out) return fail(WSR_E_INVALID, "null argument");
  *out = (id >= 0 && id < static_cast<int32_t>(h->list_bytes.size())) ? h->list_bytes[id] : 0;
  return WSR_OK;
}

int wsr_batch_create(wsr_handle* h, int32_t max_q, int32_t stride, wsr_batch** out) {
  if (!h || !out || max_q <= 0 || stride <= 0 || stride > WSR_MAX_K)
    return fail(WSR_E_INVALID, "bad batch arguments");
  std::lock_guard<std::mutex> g(h->mu);
  std::unique_ptr<wsr_batch> b(new wsr_batch());
  try {
    HIP_OK(hipSetDevice(h->device));
    b->max_q = max_q;
    b->stride = stride;
    b->q_cap = sizeof(QueryIn) * max_q;
    HIP_OK(hipMalloc(&b->d_q, b->q_cap));
    HIP_OK(hipMalloc(&b->d_plan, sizeof(QueryPlan) * max_q));
    HIP_OK(hipMalloc(&b->d_desc, sizeof(QueryDesc) * max_q));
    HIP_OK(hipMalloc(&b->d_part, sizeof(PlanPart) * ((max_q + kPlanThreads - 1) / kPlanThreads + 1)));
    HIP_OK(hipMalloc(&b->d_ctr, sizeof(uint32_t) * (kNumCounters + kMaxOwners)));   // + shard fill counters
    HIP_OK(hipHostMalloc(&b->h_ctr, sizeof(uint32_t) * kNumCounters));
    HIP_OK(hipMalloc(&b->d_hits, sizeof(HitDev) * static_cast<size_t>(max_q) * stride));
    HIP_OK(hipMalloc(&b->d_nhits, sizeof(int32_t) * max_q));
    HIP_OK(hipMalloc(&b->d_qdone, sizeof(uint32_t) * max_q));
    HIP_OK(hipMalloc(&b->d_stats, sizeof(uint32_t) * kStatStride *
                                      (std::max(std::max(h->grid, h->gen_cap), 1) +   // (seg_grid <= gen_cap)
                                       kLeanWaves * (std::max(h->lean_wgs_two, 1) + std::max(h->lean_wgs_ph, 1)))));
    for (auto& e : b->ev) HIP_OK(hipEventCreate(&e));
    HIP_OK(hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&b->st2, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&b->st_pad, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&b->fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&b->join, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&b->join_ph, hipEventDisableTiming));
  } catch (const std::exception& e) {
    wsr_batch_destroy(h, b.release());
    return fail(WSR_E_HIP, e.what());
  }
  *out = b.release();
  return WSR_OK;
}

void wsr_batch_destroy(wsr_handle* h, wsr_batch* b) {
  if (!b) return;
  if (x_join(b)) (void)hipEventSynchronize(b->xev[1]);   // a shard step's exchange reads its buffers
  if (b->st) (void)hipStreamSynchronize(b->st);
  if (b->st2) (void)hipStreamSynchronize(b->st2);
  if (b->st_pad) (void)hipStreamSynchronize(b->st_pad);
  for (void* p : {static_cast<void*>(b->d_q), static_cast<void*>(b->d_plan),
                  static_cast<void*>(b->d_desc), static_cast<void*>(b->d_part),
                  static_cast<void*>(b->d_ctr), static_cast<void*>(b->d_events),
                  static_cast<void*>(b->d_evcnt), static_cast<void*>(b->d_hits),
                  static_cast<void*>(b->d_nhits), static_cast<void*>(b->d_stats),
                  static_cast<void*>(b->d_qdone), static_cast<void*>(b->d_itemq),
                  static_cast<void*>(b->d_pub), static_cast<void*>(b->d_ph),
                  static_cast<void*>(b->d_xsend), static_cast<void*>(b->d_xrecv)})
    if (p) (void)hipFree(p);
  if (b->h_ctr) (void)hipHostFree(b->h_ctr);
  for (auto& e : b->ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : b->xev) if (e) (void)hipEventDestroy(e);
  if (b->fork) (void)hipEventDestroy(b->fork);
  if (b->join) (void)hipEventDestroy(b->join);
  if (b->join_ph) (void)hipEventDestroy(b->join_ph);
  if (b->st) (void)hipStreamDestroy(b->st);
  if (b->st2) (void)hipStreamDestroy(b->st2);
  if (b->st_pad) (void)hipStreamDestroy(b->st_pad);
  delete b;
}

int wsr_check_query(wsr_handle* h, const wsr_query* q) {
  if (!h || !q) return fail(WSR_E_INVALID, "null argument");
  if (q->n_terms > WSR_MAX_QUERY_TERMS || q->k > WSR_MAX_K)
    return fail(WSR_E_LIMIT, "n_terms or k over the limit");
  if (q->n_terms > WSR_MAX_TERMS && !q->more_ids)
    return fail(WSR_E_INVALID, "a query of more than WSR_MAX_TERMS terms needs more_ids");
  if ((q->flags & WSR_QUERY_PHRASE) && q->n_terms > WSR_MAX_PHRASE_TERMS)
    return fail(WSR_E_LIMIT, "a phrase query has at most WSR_MAX_PHRASE_TERMS terms");
  if (q->flags & ~WSR_QUERY_PHRASE) return fail(WSR_E_INVALID, "unknown flags");
  if ((q->flags & WSR_QUERY_PHRASE) && q->n_terms > 1 && !h->positions)
    return fail(WSR_E_INVALID, "phrase query on an engine opened without positions");
  return WSR_OK;
}

int wsr_batch_upload(wsr_handle* h, wsr_batch* b, const wsr_query* q, int32_t nq) {
  if (!h || !b || (nq > 0 && !q) || nq < 0 || nq > b->max_q)
    return fail(WSR_E_INVALID, "bad upload arguments");
  // (no handle lock: the handle's image is read-only after wsr_open and the
  // batch belongs to the caller, so threads with their own batches pipeline)
  std::vector<QueryIn> in(nq);
  std::vector<int32_t> ext;   // term lists of queries over kMaxTerms, after the QueryIn array
  uint64_t ev_need = 0, items_need = 0, algo = 0;
  // the device's class rule (plan_query_kernel), restated to size the two
  // persistent grids: lean items run in lean_kernel, the rest in segment_kernel
  uint64_t lean_need = 0, lean_need_ph = 0, gen_need = 0;
  const float dense_ratio = h->args.dense_ratio;
  bool has_phrase = false, has_wide = false, two_conj = true, two_ph = true, one_conj = true, gen_phrase = false;
  std::vector<int32_t> ids;
  for (int i = 0; i < nq; ++i) {
    const wsr_query& s = q[i];
    if (s.k > b->stride)
      return fail(WSR_E_LIMIT, "query " + std::to_string(i) + ": k over the batch's hit stride");
    const int qrc = wsr_check_query(h, &s);
    if (qrc) return fail(qrc, "query " + std::to_string(i) + ": " + g_err);
    const bool phrase = (s.flags & WSR_QUERY_PHRASE) && s.n_terms > 1;
    has_phrase = has_phrase || phrase;
    has_wide = has_wide || s.k > kMaxK;
    if (phrase) two_ph = two_ph && s.k <= kMaxK;
    else {
      two_conj = two_conj && s.k <= kMaxK && (s.n_terms == 2 || s.n_terms <= 0 || s.k <= 0);
      one_conj = one_conj && (s.n_terms == 1 || s.n_terms <= 0 || s.k <= 0);
    }
    QueryIn& d = in[i];
    d.n_terms = s.n_terms < 0 ? 0 : s.n_terms;
    d.k = s.k < 0 ? 0 : s.k;
    d.flags = phrase ? kQueryPhrase : 0;
    d.ext = 0;
    ids = query_terms(s);
    for (int t = 0; t < kMaxTerms; ++t) d.list[t] = t < d.n_terms ? ids[t] : -1;
    if (d.n_terms > kMaxTerms) {
      d.ext = static_cast<uint32_t>((sizeof(QueryIn) * static_cast<size_t>(nq)) / sizeof(int32_t) + ext.size());
      ext.insert(ext.end(), ids.begin(), ids.end());
    }
    uint32_t nbmin = 0xFFFFFFFFu;
    bool ok = d.n_terms > 0 && d.k > 0;
    for (int t = 0; t < d.n_terms; ++t) {
      const int32_t id = ids[t];
      if (id < 0 || id >= static_cast<int32_t>(h->lists.size())) { ok = false; continue; }
      nbmin = std::min(nbmin, h->lists[id].nblk);
    }
    if (ok && nbmin > 0) {
      // (a single-term item spans up to kSingleWindows items' blocks)
      const uint64_t seg_max = d.n_terms == 1 ? std::min<uint64_t>(nbmin, uint64_t{kSegCostMax} * kSingleWindows)
                                              : uint64_t{kSegCostMax};
      ev_need += (static_cast<uint64_t>(nbmin) + seg_max) * 128;
      items_need += nbmin;
      int drv = 0;
      for (int t = 1; t < d.n_terms; ++t)
        if (h->lists[ids[t]].nblk < h->lists[ids[drv]].nblk) drv = t;
      auto dense = [&](int t) {
        const ListDev& L = h->lists[ids[t]];
        return L.bm != kNoDense && static_cast<float>(L.nblk) >= dense_ratio * static_cast<float>(nbmin);
      };
      bool lean = !(phrase && d.n_terms > 2);   // (longer phrases: general class)
      for (int t = 0; t < d.n_terms; ++t)
        if (t != drv && !dense(t)) lean = false;
      (lean ? (phrase ? lean_need_ph : lean_need) : gen_need) += nbmin;
      gen_phrase = gen_phrase || (phrase && !lean);
      // every term's docid+tf span, and for a phrase query also its
      // position box (the bags the position check reads from)
      for (int t = 0; t < d.n_terms; ++t) {
        algo += h->list_bytes[ids[t]];
        if (phrase && !h->pos_bytes.empty()) algo += h->pos_bytes[ids[t]];
      }
      algo += 12ull * d.k;
    }
  }
  const size_t q_bytes = sizeof(QueryIn) * static_cast<size_t>(nq) + sizeof(int32_t) * ext.size();
  try {
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(b->st));
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));   // a shard step's exchange + replay
    if (ev_need > b->ev_cap) {
      if (b->d_events) HIP_OK(hipFree(b->d_events));
      b->ev_cap = ev_need + ev_need / 4 + 4096;
      HIP_OK(hipMalloc(&b->d_events, sizeof(Event) * b->ev_cap));
    }
    if (items_need > b->item_cap || !b->d_evcnt) {
      if (b->d_evcnt) HIP_OK(hipFree(b->d_evcnt));
      if (b->d_itemq) HIP_OK(hipFree(b->d_itemq));
      if (b->d_pub) HIP_OK(hipFree(b->d_pub));
      b->d_itemq = nullptr;
      b->d_pub = nullptr;
      b->item_cap = items_need + items_need / 4 + 1024;
      HIP_OK(hipMalloc(&b->d_evcnt, sizeof(uint32_t) * b->item_cap));
      HIP_OK(hipMalloc(&b->d_itemq, sizeof(uint32_t) * b->item_cap));
      HIP_OK(hipMalloc(&b->d_pub, sizeof(uint64_t) * b->item_cap));
    }
    if (has_phrase && !b->d_ph)   // one per general workgroup
      HIP_OK(hipMalloc(&b->d_ph, sizeof(uint32_t) * kPhraseScratch * static_cast<size_t>(std::max(h->gen_cap, 1))));
    if (q_bytes > b->q_cap) {   // (the term table of long queries follows the QueryIn array)
      if (b->d_q) HIP_OK(hipFree(b->d_q));
      b->d_q = nullptr;
      b->q_cap = q_bytes + q_bytes / 4;
      HIP_OK(hipMalloc(&b->d_q, b->q_cap));
    }
    if (nq) HIP_OK(hipMemcpy(b->d_q, in.data(), sizeof(QueryIn) * nq, hipMemcpyHostToDevice));
    if (!ext.empty())
      HIP_OK(hipMemcpy(reinterpret_cast<char*>(b->d_q) + sizeof(QueryIn) * nq, ext.data(),
                       sizeof(int32_t) * ext.size(), hipMemcpyHostToDevice));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  b->nq = nq;
  b->has_phrase = has_phrase;
  b->has_wide = has_wide;
  b->two_conj = two_conj;
  b->gen_phrase = gen_phrase;
  b->has_conj_lean = lean_need > 0;
  b->has_gen = gen_need > 0;
  b->two_ph = two_ph;
  b->one_conj = one_conj && !two_conj;   // (a batch of empty queries only: the two-term instance)
  // persistent grid: never more workgroups than work items can exist
  // (at least one worker each: a grid also drains items the estimate missed)
  b->seg_grid = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(h->gen_cap, gen_need)));
  b->lean_wgs = static_cast<int>(std::max<uint64_t>(
      1, std::min<uint64_t>(two_conj ? h->lean_wgs_two : h->lean_wgs, (lean_need + kLeanWaves - 1) / kLeanWaves)));
  b->lean_wgs_ph = static_cast<int>(std::max<uint64_t>(
      1, std::min<uint64_t>(h->lean_wgs_ph, (lean_need_ph + kLeanWaves - 1) / kLeanWaves)));
  b->algo_static = algo;
  b->ran = false;
  return WSR_OK;
}

// Shard emission of a batch run (wsr_shard_step): owners, queries per owner,
// slot, and the send / meta buffers the segment kernels append to.
struct ShardEmit {
  int owners;
  int32_t qpr;
  uint64_t slot;         // capacity of an owner's slot (events)
  Event* send;           // owner 0's slot; owner o's at send + o * stride
  uint64_t stride;
  int32_t* meta;         // owner 0's {count, offset} block; owner o's at meta + o * meta_stride
  uint64_t meta_stride;
};

static int batch_run(wsr_handle* h, wsr_batch* b, const ShardEmit* se = nullptr, const OwnerJob* oj = nullptr);
static wsr_batch* take_host_replay(wsr_handle* h, const wsr_batch* b, OwnerJob* oj);
static void host_replay_enqueue(wsr_batch* pb, wsr_handle* h);


int wsr_batch_run(wsr_handle* h, wsr_batch* b) { return batch_run(h, b); }

// One run of the batch: plan, then the lean and general segment kernels on
// two streams; the worker that finishes a query's last item replays it
// (se == nullptr) or emits its reduced events into the owner's exchange
// region (a shard step).  Wide queries (k > kMaxK) of a plain run are
// replayed by one more launch after the segments.  oj: an earlier step
// group's owner replay for the lean kernel's tail (its exchange is done).
static std::atomic<int32_t> g_fail_runs{0};   // wsr_debug_fail_runs

int wsr_debug_fail_runs(int32_t n) {
  g_fail_runs.store(n > 0 ? n : 0);
  return WSR_OK;
}

static int batch_run(wsr_handle* h, wsr_batch* b, const ShardEmit* se, const OwnerJob* oj) {
  if (!h || !b) return fail(WSR_E_INVALID, "null argument");
  for (int32_t f = g_fail_runs.load(); f > 0;)
    if (g_fail_runs.compare_exchange_weak(f, f - 1)) return fail(WSR_E_HIP, "injected run failure");
  wsr_batch* pb = nullptr;   // (a host replay taken, below)
  bool pb_queued = false;
  try {
    HIP_OK(hipSetDevice(h->device));
    hipStream_t st = b->st;
    // the previous shard step's exchange and owner replay (on the communicator's
    // stream) read this batch's buffers and write its results
    if (x_join(b)) HIP_OK(hipStreamWaitEvent(st, b->xev[1], 0));
    b->x_pending = false;
    // a host-exchange owner replay another batch deferred (wsr_shard_step_
    // replay_deferred) rides in this run's lean kernel, after its regions'
    // copy; its end is recorded on this stream behind the lean kernel
    OwnerJob hoj{};
    if (!oj && (pb = take_host_replay(h, b, &hoj))) {
      HIP_OK(hipStreamWaitEvent(st, pb->xev[0], 0));
      oj = &hoj;
    }
    HIP_OK(hipMemsetAsync(b->d_ctr, 0, sizeof(uint32_t) * (kNumCounters + (se ? se->owners : 0)), st));
    FusedReplay fr{b->d_qdone, b->d_hits, b->stride, b->d_nhits};
    if (se) {
      fr.x_send = se->send;
      fr.x_meta = se->meta;
      fr.x_fill = b->d_ctr + kNumCounters;
      fr.x_err = b->d_ctr + kCtrError;
      fr.x_slot = se->slot;
      fr.x_stride = se->stride;
      fr.x_meta_stride = se->meta_stride;
      fr.x_qpr = se->qpr;
    }
    if (oj) fr.oj = *oj;
    HIP_OK(hipEventRecord(b->ev[0], st));
    IndexArgs pa = h->args;   // (the batch's item length)
    pa.seg_cap = b->seg_cap;
    // A batch with phrase queries launches the conjunctive lean kernel and the
    // general one only when the host's restatement of the class rule found
    // such queries (an empty persistent launch waited for CU slots beside the
    // others: 54 us on C5, profiles/r05p); the plan flags kErrClass if a class
    // without a launch holds items.  (Shard steps launch everything: their
    // owners read every query's emission.)
    // (a taken owner replay rides in the conjunctive launch: it runs then
    // even with no conjunctive lean item of its own)
    const bool run_conj = se || oj || !b->has_phrase || b->has_conj_lean;
    const bool run_gen = se || !b->has_phrase || b->has_gen;
    b->ran_conj = run_conj;
    b->ran_gen = run_gen;
    HIP_OK(launch_plan(pa, b->d_q, b->nq, b->d_plan, b->d_ctr, b->ev_cap,
                       static_cast<uint32_t>(std::min<uint64_t>(b->item_cap, 0xFFFFFFFFull)),
                       run_conj ? kLeanWaves * b->lean_wgs : 0, b->has_phrase ? kLeanWaves * b->lean_wgs_ph : 0,
                       run_gen ? b->seg_grid : 0, fr, b->d_itemq, b->d_pub, b->d_desc, b->d_part, st));
    HIP_OK(hipEventRecord(b->ev[1], st));
    // general items on the second stream, lean items here; both drain their
    // own queue, then the streams join
    HIP_OK(hipEventRecord(b->fork, st));
    HIP_OK(hipStreamWaitEvent(b->st2, b->fork, 0));
    if (run_gen)
      HIP_OK(launch_segments(h->args, b->d_q, b->d_plan, b->nq, b->d_ctr, b->d_events, b->d_evcnt,
                             b->d_stats, b->seg_grid, fr, b->d_itemq, b->d_pub,
                             b->gen_phrase ? b->d_ph : nullptr, b->st2));
    uint32_t* lean_stats = b->d_stats + static_cast<size_t>(kStatStride) * b->seg_grid;
    HIP_OK(hipEventRecord(b->join, b->st2));
    if (b->has_phrase) {
      // The lean phrase queries' items run in the phrase instance (its
      // position check and registers) and the conjunctive lean items keep the
      // conjunctive instance's occupancy: the phrase launch on the batch
      // stream (where a phrase batch's lean kernel has always run, so that
      // consecutive batches' kernels rotate over the hardware queues as
      // before), the conjunctive one on the third stream beside it.  (A
      // deferred owner replay runs in the conjunctive launch only.)
      HIP_OK(hipStreamWaitEvent(b->st_pad, b->fork, 0));
      if (run_conj)
        HIP_OK(launch_lean(h->args, b->d_q, b->d_plan, b->nq, b->d_ctr, b->d_events, b->d_evcnt, lean_stats,
                           b->lean_wgs, fr, b->d_itemq, b->d_pub, b->d_desc, false, b->two_conj, b->one_conj,
                           b->st_pad));
      if (pb) {   // the replay's end: behind the conjunctive launch that carried it
        HIP_OK(hipEventRecord(pb->xev[1], b->st_pad));
        pb_queued = true;
      }
      HIP_OK(hipEventRecord(b->join_ph, b->st_pad));
      FusedReplay frp = fr;
      frp.oj = OwnerJob{};
      HIP_OK(launch_lean(h->args, b->d_q, b->d_plan, b->nq, b->d_ctr, b->d_events, b->d_evcnt,
                         lean_stats + static_cast<size_t>(kStatStride) * kLeanWaves * b->lean_wgs,
                         b->lean_wgs_ph, frp, b->d_itemq, b->d_pub, b->d_desc, true, b->two_ph, false, st));
    } else {
      HIP_OK(launch_lean(h->args, b->d_q, b->d_plan, b->nq, b->d_ctr, b->d_events, b->d_evcnt, lean_stats,
                         b->lean_wgs, fr, b->d_itemq, b->d_pub, b->d_desc, false, b->two_conj, b->one_conj, st));
    }
    HIP_OK(hipEventRecord(b->ev[4], st));
    if (pb && !pb_queued) {
      HIP_OK(hipEventRecord(pb->xev[1], st));
      pb_queued = true;
    }
    if (pb) {
      pb->x_pending = true;
      pb->x_enq.fetch_add(1, std::memory_order_release);   // (take_host_replay counted it in x_req)
      pb = nullptr;
    }
    HIP_OK(hipStreamWaitEvent(st, b->join, 0));
    if (b->has_phrase) HIP_OK(hipStreamWaitEvent(st, b->join_ph, 0));
    HIP_OK(hipEventRecord(b->ev[2], st));
    if (!se && b->has_wide)
      HIP_OK(launch_wide_replay(b->d_q, b->d_plan, b->nq, b->d_events, b->d_evcnt, b->d_hits, b->stride,
                                b->d_nhits, st));
    HIP_OK(hipEventRecord(b->ev[3], st));
  } catch (const std::exception& e) {
    if (pb) {
      if (!pb_queued) host_replay_enqueue(pb, h);   // (its own stream, then)
      else pb->x_pending = true;
      pb->x_enq.fetch_add(1, std::memory_order_release);
    }
    return fail(WSR_E_HIP, e.what());
  }
  b->ran = true;
  b->x_fused = se != nullptr;
  return WSR_OK;
}

int wsr_sync(wsr_handle* h) {
  if (!h) return fail(WSR_E_INVALID, "null argument");
  hipError_t e = hipSetDevice(h->device);
  if (e == hipSuccess) e = hipDeviceSynchronize();   // every batch's streams
  if (e != hipSuccess) return fail(WSR_E_HIP, hipGetErrorString(e));
  return WSR_OK;
}

// Results of the batch's last run: the counters, hit rows and hit counts go
// out as copies queued on the batch stream behind its kernels (and behind a
// shard step's exchange + owner replay), then one wait -- one host round trip
// instead of a synchronize per buffer (pinned destinations; pageable ones are
// copied after the wait).  The error flags are checked after the
// copies; on an error the output buffers hold whatever the run left and the
// call fails.  cols < stride copies the first cols entries of every row.
static bool host_pinned(const void* p) {
  if (!p) return true;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();   // plain pageable memory: not an error of this call
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

static int batch_fetch(wsr_handle* h, wsr_batch* b, wsr_hit* hits, int32_t* n_hits, int32_t cols) {
  try {
    HIP_OK(hipSetDevice(h->device));
    hipStream_t st = b->st;
    if (x_join(b)) HIP_OK(hipStreamWaitEvent(st, b->xev[1], 0));   // a shard step's exchange + replay
    HIP_OK(hipMemcpyAsync(b->h_ctr, b->d_ctr, sizeof(uint32_t) * kNumCounters, hipMemcpyDeviceToHost, st));
    if (b->nq && !(host_pinned(hits) && host_pinned(n_hits))) {
      // pageable destinations: a queued copy into them is staged by the runtime
      // while the stream drains (serialising concurrent callers), so wait
      // first and copy after
      HIP_OK(hipStreamSynchronize(st));
      const uint32_t err = b->h_ctr[kCtrError];
      if (err) return fail(WSR_E_INTERNAL, "device reported error flags " + std::to_string(err));
      if (hits && cols == b->stride)
        HIP_OK(hipMemcpy(hits, b->d_hits, sizeof(HitDev) * b->nq * b->stride, hipMemcpyDeviceToHost));
      else if (hits)
        HIP_OK(hipMemcpy2D(hits, sizeof(HitDev) * cols, b->d_hits, sizeof(HitDev) * b->stride,
                           sizeof(HitDev) * cols, b->nq, hipMemcpyDeviceToHost));
      if (n_hits) HIP_OK(hipMemcpy(n_hits, b->d_nhits, sizeof(int32_t) * b->nq, hipMemcpyDeviceToHost));
      return WSR_OK;
    }
    if (b->nq) {
      if (hits && cols == b->stride)
        HIP_OK(hipMemcpyAsync(hits, b->d_hits, sizeof(HitDev) * b->nq * b->stride, hipMemcpyDeviceToHost, st));
      else if (hits)   // a pitched copy
        HIP_OK(hipMemcpy2DAsync(hits, sizeof(HitDev) * cols, b->d_hits, sizeof(HitDev) * b->stride,
                                sizeof(HitDev) * cols, b->nq, hipMemcpyDeviceToHost, st));
      if (n_hits)
        HIP_OK(hipMemcpyAsync(n_hits, b->d_nhits, sizeof(int32_t) * b->nq, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    const uint32_t err = b->h_ctr[kCtrError];
    if (err) return fail(WSR_E_INTERNAL, "device reported error flags " + std::to_string(err));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_batch_fetch(wsr_handle* h, wsr_batch* b, wsr_hit* hits, int32_t* n_hits) {
  if (!h || !b || !b->ran) return fail(WSR_E_INVALID, "batch has not been run");
  return batch_fetch(h, b, hits, n_hits, b->stride);
}

int wsr_batch_fetch_cols(wsr_handle* h, wsr_batch* b, wsr_hit* hits, int32_t* n_hits, int32_t cols) {
  if (!h || !b || !b->ran) return fail(WSR_E_INVALID, "batch has not been run");
  if (cols < 1 || cols > b->stride) return fail(WSR_E_INVALID, "cols must be in [1, hit stride]");
  return batch_fetch(h, b, hits, n_hits, cols);
}

int wsr_pinned_alloc(uint64_t bytes, void** out) {
  if (!out) return fail(WSR_E_INVALID, "null argument");
  *out = nullptr;
  const hipError_t e = hipHostMalloc(out, bytes ? bytes : 1);
  if (e != hipSuccess) return fail(WSR_E_HIP, hipGetErrorString(e));
  return WSR_OK;
}

void wsr_pinned_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int wsr_batch_ready(wsr_handle* h, wsr_batch* b) {
  if (!h || !b) return fail(WSR_E_INVALID, "null argument");
  if (!b->ran) return 0;
  hipError_t e = hipEventQuery(b->ev[3]);   // recorded after the batch's last kernel
  if (e == hipSuccess && x_join(b)) e = hipEventQuery(b->xev[1]);   // and a shard step's replay
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return fail(WSR_E_HIP, hipGetErrorString(e));
}

int wsr_batch_stats_get(wsr_handle* h, wsr_batch* b, wsr_batch_stats* out) {
  if (!h || !b || !out || !b->ran) return fail(WSR_E_INVALID, "batch has not been run");
  std::lock_guard<std::mutex> g(h->mu);
  try {
    HIP_OK(hipStreamSynchronize(b->st));
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));   // a shard step's exchange + replay
    uint32_t ctr[kNumCounters];
    HIP_OK(hipMemcpy(ctr, b->d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
    const int rows = b->seg_grid + kLeanWaves * (b->lean_wgs + (b->has_phrase ? b->lean_wgs_ph : 0));
    std::vector<uint32_t> ws(static_cast<size_t>(kStatStride) * rows);
    HIP_OK(hipMemcpy(ws.data(), b->d_stats, ws.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    uint64_t sv = 0, db = 0, ob = 0;
    for (int i = 0; i < rows; ++i) {
      // (rows of a kernel the last run did not launch hold an earlier run's values)
      if (i < b->seg_grid ? !b->ran_gen : (i < b->seg_grid + kLeanWaves * b->lean_wgs && !b->ran_conj)) continue;
      sv += ws[kStatStride * i]; db += ws[kStatStride * i + 1]; ob += ws[kStatStride * i + 2];
    }
    out->work_items = ctr[kCtrItems];
    out->survivors = sv;
    out->driver_blocks = db;
    out->other_blocks = ob;
    out->algo_bytes = b->algo_static + sv;
    {
      const uint32_t items = ctr[kCtrItems];
      std::vector<uint32_t> ec(items);
      std::vector<QueryPlan> pl(b->nq);
      if (items) HIP_OK(hipMemcpy(ec.data(), b->d_evcnt, items * sizeof(uint32_t), hipMemcpyDeviceToHost));
      if (b->nq) HIP_OK(hipMemcpy(pl.data(), b->d_plan, pl.size() * sizeof(QueryPlan), hipMemcpyDeviceToHost));
      uint64_t tot = 0, mx = 0;
      for (const QueryPlan& p : pl) {
        uint64_t e = 0;
        for (uint32_t r = 0; r < p.n_items && p.item_base + r < items; ++r) e += ec[p.item_base + r];
        tot += e;
        mx = std::max(mx, e);
      }
      out->events = tot;
      out->max_query_events = mx;
    }
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, b->ev[0], b->ev[1])); out->plan_ms = ms;
    HIP_OK(hipEventElapsedTime(&ms, b->ev[1], b->ev[2])); out->segment_ms = ms;
    HIP_OK(hipEventElapsedTime(&ms, b->ev[2], b->ev[3])); out->replay_ms = ms;
    HIP_OK(hipEventElapsedTime(&ms, b->ev[1], b->ev[4])); out->lean_ms = ms;
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_search_batch(wsr_handle* h, const wsr_query* q, int32_t nq, int32_t stride, wsr_hit* hits,
                     int32_t* n_hits) {
  if (!h || nq < 0 || (nq && (!q || !hits || !n_hits))) return fail(WSR_E_INVALID, "bad arguments");
  if (nq == 0) return WSR_OK;
  // batches are kept in a per-handle pool (one per concurrent caller): creating
  // one allocates its device buffers, which would dominate a small call
  wsr_batch* b = nullptr;
  {
    std::lock_guard<std::mutex> g(h->pool_mu);
    for (size_t i = 0; i < h->pool.size(); ++i)
      if (h->pool[i]->max_q >= nq && h->pool[i]->stride == stride) {
        b = h->pool[i];
        h->pool.erase(h->pool.begin() + i);
        break;
      }
  }
  if (!b) {
    int32_t cap = 64;
    while (cap < nq) cap *= 2;
    const int rc = wsr_batch_create(h, cap, stride, &b);
    if (rc) return rc;
  }
  int rc = wsr_batch_upload(h, b, q, nq);
  if (!rc) rc = wsr_batch_run(h, b);
  if (!rc) rc = wsr_batch_fetch(h, b, hits, n_hits);
  {
    std::lock_guard<std::mutex> g(h->pool_mu);
    if (!rc && h->pool.size() < 8) { h->pool.push_back(b); b = nullptr; }
  }
  if (b) wsr_batch_destroy(h, b);
  return rc;
}

int wsr_resolve_text(wsr_handle* h, const char* text, int64_t len, int32_t k, int32_t max_q,
                     wsr_query* q, int32_t* nq_out, int32_t* more_store, int64_t more_cap) {
  if (!h || (!text && len > 0) || len < 0 || max_q < 0 || (max_q && !q) || !nq_out || k < 0 ||
      more_cap < 0 || (more_cap > 0 && !more_store))
    return fail(WSR_E_INVALID, "bad resolve_text arguments");
  // QueryProducerByLog (query_pool.h:319-378): one query per line, terms
  // separated by spaces, a line in double quotes is a phrase query; each term
  // through the term index (VacuumInvertedIndex::FindIteratorsSolid,
  // vacuum_engine.h:89-99)
  int32_t n = 0;
  // the terms are parsed first and looked up together (find_many: the
  // dictionary's cache misses overlap)
  std::vector<const char*> tp;
  std::vector<uint32_t> tn;
  // (query, slot) of every parsed term; ids land in list_ids, or past 16 in
  // the caller's more_store (more_ids), once every term is looked up
  std::vector<std::pair<int32_t, int32_t>> dst;
  std::vector<size_t> more_at(static_cast<size_t>(max_q), 0);
  size_t n_more = 0;
  tp.reserve(static_cast<size_t>(max_q) * 2);
  tn.reserve(static_cast<size_t>(max_q) * 2);
  dst.reserve(static_cast<size_t>(max_q) * 2);
  for (int64_t at = 0; at < len;) {
    int64_t e = at;
    while (e < len && text[e] != '\n') ++e;
    int64_t a = at, z = e;
    at = e + 1;
    while (a < z && (text[a] == ' ' || text[a] == '\r' || text[a] == '\t')) ++a;
    while (z > a && (text[z - 1] == ' ' || text[z - 1] == '\r' || text[z - 1] == '\t')) --z;
    if (a == z) continue;
    if (n >= max_q) return fail(WSR_E_LIMIT, "more than max_q queries in the text");
    wsr_query& w = q[n];
    std::memset(&w, 0, sizeof w);
    if (z - a >= 2 && text[a] == '"' && text[z - 1] == '"') { w.flags = WSR_QUERY_PHRASE; ++a; --z; }
    w.k = k;
    more_at[n] = n_more;
    for (int64_t i = a; i < z;) {
      while (i < z && text[i] == ' ') ++i;
      int64_t j = i;
      while (j < z && text[j] != ' ') ++j;
      if (j > i) {
        if (w.n_terms >= WSR_MAX_QUERY_TERMS)
          return fail(WSR_E_LIMIT, "query " + std::to_string(n) + ": more than WSR_MAX_QUERY_TERMS terms");
        tp.push_back(text + i);
        tn.push_back(static_cast<uint32_t>(j - i));
        dst.emplace_back(n, w.n_terms++);
        if (w.n_terms > WSR_MAX_TERMS) ++n_more;
      }
      i = j;
    }
    for (int t = w.n_terms; t < WSR_MAX_TERMS; ++t) w.list_ids[t] = -1;
    ++n;
  }
  if (static_cast<int64_t>(n_more) > more_cap)
    return fail(WSR_E_LIMIT, "the text's queries need " + std::to_string(n_more) +
                                 " more_ids entries, more_store holds " + std::to_string(more_cap));
  std::vector<int32_t> ids(tp.size());
  h->idx.find_many(tp.data(), tn.data(), tp.size(), ids.data());
  for (size_t i = 0; i < ids.size(); ++i) {
    const int32_t qi = dst[i].first, slot = dst[i].second;
    if (slot < WSR_MAX_TERMS) q[qi].list_ids[slot] = ids[i];
    else more_store[more_at[qi] + (slot - WSR_MAX_TERMS)] = ids[i];
  }
  for (int32_t i = 0; i < n; ++i)
    if (q[i].n_terms > WSR_MAX_TERMS) q[i].more_ids = more_store + more_at[i];
  *nq_out = n;
  return WSR_OK;
}

int wsr_search_text(wsr_handle* h, const char* text, int64_t len, int32_t k, int32_t hit_stride,
                    int32_t max_q, wsr_hit* hits, int32_t* n_hits, int32_t* nq_out) {
  if (!h || !nq_out || max_q < 0) return fail(WSR_E_INVALID, "bad search_text arguments");
  std::vector<wsr_query> q(static_cast<size_t>(max_q));
  // (at most one more_ids entry per two text bytes: every term has a byte and
  // a separator; the ids are consumed within this call, so a per-thread
  // buffer is safe here)
  thread_local std::vector<int32_t> more;
  if (more.size() < static_cast<size_t>(len / 2 + 1)) more.resize(static_cast<size_t>(len / 2 + 1));
  int rc = wsr_resolve_text(h, text, len, k, max_q, q.data(), nq_out, more.data(),
                            static_cast<int64_t>(more.size()));
  if (rc) return rc;
  return wsr_search_batch(h, q.data(), *nq_out, hit_stride, hits, n_hits);
}

int wsr_class_order(const wsr_query* q, int32_t nq, int32_t* order, int32_t* n_conj) {
  if (nq < 0 || (nq && (!q || !order)) || !n_conj) return fail(WSR_E_INVALID, "bad class_order arguments");
  // (a one-term phrase is a single-term query: the same class as in the plan)
  auto phrase = [&](int32_t i) { return (q[i].flags & WSR_QUERY_PHRASE) != 0 && q[i].n_terms > 1; };
  int32_t n = 0;
  for (int32_t i = 0; i < nq; ++i)
    if (!phrase(i)) order[n++] = i;
  *n_conj = n;
  for (int32_t i = 0; i < nq; ++i)
    if (phrase(i)) order[n++] = i;
  return WSR_OK;
}

int wsr_shard_fill(wsr_handle* h, wsr_batch* b, int32_t n_owners, int64_t* owner_totals) {
  if (!h || !b || !b->x_fused || !owner_totals || n_owners <= 0 || n_owners > b->x_world)
    return fail(WSR_E_INVALID, "call wsr_shard_step (or wsr_shard_step_emit) first");
  try {
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(b->st));
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));   // a shard step's exchange + replay
    // the segment kernels' per-owner fill counters
    std::vector<uint32_t> fill(n_owners);
    HIP_OK(hipMemcpy(fill.data(), b->d_ctr + kNumCounters, sizeof(uint32_t) * n_owners, hipMemcpyDeviceToHost));
    for (int i = 0; i < n_owners; ++i) owner_totals[i] = fill[i];
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_batch_stream(wsr_handle* h, wsr_batch* b, void** stream) {
  if (!h || !b || !stream) return fail(WSR_E_INVALID, "null argument");
  *stream = b->st;
  return WSR_OK;
}

// ---- native RCCL exchange (one process per GPU, no Python in the loop) ----
// Every collective of a communicator runs on its one stream, in issue order
// (the same order on every rank), whatever batch stream it serves: a step's
// pack is joined into it by an event and its replay waits for it by another,
// so consecutive batches still overlap their kernels.
// The exchange half of a step group (the collective and the owner replays)
// is enqueued by the communicator's own worker thread: an ncclAllToAll call
// can hold its caller for milliseconds while the device is busy (RCCL's host
// side waits for its earlier work: 0.13-0.23 ms of host time per step in the
// hybrid rehearsal, the loop host-bound, profiles/r04g/), and the caller's
// next batches must not wait behind it.  Jobs run in submission order, so
// every rank issues its collectives in the same order.
//
// A group's owner replays are deferred (WSR_REPLAY_DEFER, default 1) into the
// lean kernels of the step group kReplayLag groups later: each of its
// batches' lean kernel, its own items done, replays one batch of the earlier
// group (OwnerJob).  A separate owner replay launch -- thousands of one-wave,
// latency-bound workgroups per batch beside the persistent lean kernels --
// cost more than its work (one-rank rehearsal 16.8 M q/s with it, 20.9 M with
// the replay dropped, profiles/r04r/).  Whatever needs a deferred replay's
// results first (a fetch, the batch's next run, wsr_comm_flush) enqueues it
// on the communicator's stream instead (replay_flush).
struct XGroup {
  wsr_handle* h;
  std::vector<wsr_batch*> bs;
  int32_t qpr;
  int64_t slot;
  int xs;                              // its exchange buffers: c->xs[xs]
  bool defer;
  std::vector<hipEvent_t> wait_done;   // the slot's previous replays (before the all-to-all)
  std::vector<uint8_t> queued;         // deferred: bs[i]'s replay enqueued
  std::atomic<bool> enq{false};        // the worker has enqueued the all-to-all (and, not deferred, the replays)
};
using XJob = std::shared_ptr<XGroup>;
constexpr int kXSlots = 4;       // exchange buffer sets in rotation
constexpr size_t kReplayLag = 2;  // groups between a group's exchange and its deferred replays
struct XSlot {
  Event* send = nullptr;
  Event* recv = nullptr;
  uint64_t events = 0;
  hipEvent_t xa = nullptr;            // the last all-to-all out of this slot done (comm stream)
  std::vector<hipEvent_t> done;       // its group's owner replays done, one per batch
  size_t n_done = 0;                  // (recorded)
  std::shared_ptr<XGroup> last;       // the group that used it last
};
// Loopback group (wsr_loopback_create): the all-to-all of W communicators of
// one process by device copies.  Call n of every rank meets in calls[n]:
// each rank records its send buffer ready, waits on the host until all W have
// (phase 1), copies region r of every rank's send buffer into slot g of its
// receive buffer behind that rank's ready event, records its reads done and
// waits until all W have (phase 2), then makes its stream wait for every
// rank's reads -- so a rank's collective completes only once its send buffer
// has been read by all, as ncclAllToAll's does, and no rank records its
// per-communicator events again before every rank has waited on them.
struct wsr_loopback {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  struct Call {
    std::vector<const void*> send;
    std::vector<hipEvent_t> ready, read;
    int arrived = 0, read_done = 0, left = 0;
  };
  std::map<uint64_t, Call> calls;
};

struct wsr_comm {
  ncclComm_t comm = nullptr;
  wsr_loopback* loop = nullptr;   // a loopback communicator (no RCCL)
  uint64_t loop_seq = 0;
  hipEvent_t loop_ready = nullptr, loop_read = nullptr;
  hipStream_t stream = nullptr;
  int world = 0, rank = 0, device = 0;
  // WSR_HOST_TIMING=1: host time per phase of wsr_shard_step (enqueue only),
  // printed to stderr when the communicator closes
  bool timing = false;
  uint64_t steps = 0, t_ns[4] = {0, 0, 0, 0};   // run, submit, rccl (worker), replay (worker)
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<XJob> jobs;   // (FIFO)
  size_t head = 0;
  bool stop = false;
  std::atomic<int> err{WSR_OK};   // the worker's first failure, reported by the next call
  std::string err_msg;
  XSlot xs[kXSlots];
  uint64_t n_groups = 0;
  std::atomic<int64_t> replays_lean{0}, replays_stream{0};   // wsr_comm_stats
  bool defer = true;
  // deferred groups, oldest first.  pend, XGroup::queued and the batches'
  // x_comm are changed by wsr_shard_steps and by whatever flushes a deferred
  // replay (x_join inside a fetch, upload, run or destroy; wsr_comm_flush),
  // which may run on other threads: pend_mu orders them (recursive: a step
  // group flushes its own batches' earlier replays).
  std::deque<std::shared_ptr<XGroup>> pend;
  std::recursive_mutex pend_mu;
};

static void set_comm_err(wsr_comm* c, int rc, const std::string& msg) {
  std::lock_guard<std::mutex> g(c->mu);
  if (c->err.load() == WSR_OK) {
    c->err_msg = msg;
    c->err.store(rc);
  }
}

static uint64_t now_ns() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                   std::chrono::steady_clock::now().time_since_epoch())
                                   .count());
}

static int step_replay_from(wsr_handle* h, wsr_batch* b, int rank, int W, int32_t q_per_owner, const Event* recv,
                            uint64_t owner_stride, hipStream_t st);

// The loopback group's all-to-all (wsr_loopback above): bytes per rank pair.
static void loopback_alltoall(wsr_comm* c, const Event* send, Event* recv, uint64_t bytes) {
  wsr_loopback* L = c->loop;
  const int W = L->world, r = c->rank;
  HIP_OK(hipEventRecord(c->loop_ready, c->stream));
  const uint64_t n = c->loop_seq++;
  wsr_loopback::Call* call;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    call = &L->calls[n];
    if (call->send.empty()) {
      call->send.assign(W, nullptr);
      call->ready.assign(W, nullptr);
      call->read.assign(W, nullptr);
    }
    call->send[r] = send;
    call->ready[r] = c->loop_ready;
    ++call->arrived;
    L->cv.notify_all();
    L->cv.wait(lk, [&] { return call->arrived == W; });
  }
  const uint8_t* src_base = nullptr;
  for (int g = 0; g < W; ++g) {
    HIP_OK(hipStreamWaitEvent(c->stream, call->ready[g], 0));
    src_base = static_cast<const uint8_t*>(call->send[g]);
    HIP_OK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(recv) + g * bytes, src_base + r * bytes, bytes,
                          hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_OK(hipEventRecord(c->loop_read, c->stream));
  {
    std::unique_lock<std::mutex> lk(L->mu);
    call->read[r] = c->loop_read;
    ++call->read_done;
    L->cv.notify_all();
    L->cv.wait(lk, [&] { return call->read_done == W; });
  }
  for (int g = 0; g < W; ++g) HIP_OK(hipStreamWaitEvent(c->stream, call->read[g], 0));
  {
    std::lock_guard<std::mutex> lk(L->mu);
    if (++call->left == W) L->calls.erase(n);
  }
}

// One job: wait for the group's emissions (and for the slot's previous
// replays), one ncclAllToAll of the owners' runs of regions, then -- not
// deferred -- the owner replays and the end event of every batch.
static void run_xjob(wsr_comm* c, const XJob& jp) {
  XGroup& j = *jp;
  XSlot& S = c->xs[j.xs];
  const int W = c->world;
  const uint64_t region = (static_cast<uint64_t>(j.qpr) + 1) / 2 + static_cast<uint64_t>(j.slot);
  const uint64_t run = region * j.bs.size();
  uint64_t t0 = c->timing ? now_ns() : 0;
  int rc = WSR_OK;
  std::string msg;
  try {
    HIP_OK(hipSetDevice(c->device));
    // (the device waits for the emissions, not this thread: waiting on the
    // host first makes the collective's own call short, 2-8 us, but the loop
    // no faster -- the enqueueing thread is held by full hardware queues
    // either way, and the exchange starts later: 16.8 -> 15.3 M q/s every
    // query sharded, profiles/r04t/)
    for (wsr_batch* b : j.bs) HIP_OK(hipStreamWaitEvent(c->stream, b->xev[0], 0));
    for (hipEvent_t e : j.wait_done) HIP_OK(hipStreamWaitEvent(c->stream, e, 0));
    if (c->loop) {
      loopback_alltoall(c, S.send, S.recv, run * sizeof(Event));
    } else {
      const ncclResult_t r = ncclAllToAll(S.send, S.recv, run * (sizeof(Event) / sizeof(uint64_t)),
                                          ncclUint64, c->comm, c->stream);
      if (r != ncclSuccess) throw std::runtime_error(std::string("ncclAllToAll: ") + ncclGetErrorString(r));
    }
    HIP_OK(hipEventRecord(S.xa, c->stream));
  } catch (const std::exception& e) {
    rc = WSR_E_HIP;
    msg = e.what();
  }
  uint64_t t1 = c->timing ? now_ns() : 0;
  if (!j.defer) {
    for (size_t i = 0; i < j.bs.size() && rc == WSR_OK; ++i) {
      rc = step_replay_from(j.h, j.bs[i], c->rank, W, j.qpr, S.recv + region * i, run, c->stream);
      if (rc) msg = g_err;
      else if (hipEventRecord(j.bs[i]->xev[1], c->stream) != hipSuccess ||
               hipEventRecord(S.done[i], c->stream) != hipSuccess) {
        rc = WSR_E_HIP;
        msg = "hipEventRecord failed";
      }
    }
    for (wsr_batch* b : j.bs) {
      b->x_pending = rc == WSR_OK;
      b->x_enq.fetch_add(1, std::memory_order_release);
    }
    c->replays_stream.fetch_add(static_cast<int64_t>(j.bs.size()));
  }
  if (rc != WSR_OK) set_comm_err(c, rc, msg);
  j.enq.store(true, std::memory_order_release);
  if (c->timing) {
    const uint64_t t2 = now_ns();
    c->t_ns[2] += t1 - t0;
    c->t_ns[3] += t2 - t1;
  }
}

static void exchange_worker(wsr_comm* c) {
  for (;;) {
    XJob j;
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv.wait(lk, [&] { return c->stop || c->head < c->jobs.size(); });
      if (c->head == c->jobs.size()) return;   // (stop, and drained)
      j = std::move(c->jobs[c->head++]);
      if (c->head == c->jobs.size()) {
        c->jobs.clear();
        c->head = 0;
      }
    }
    run_xjob(c, j);
  }
}

int wsr_comm_unique_id(uint8_t* id) {
  if (!id) return fail(WSR_E_INVALID, "null argument");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(WSR_E_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  static_assert(sizeof(ncclUniqueId) == WSR_COMM_ID_BYTES, "RCCL unique id size");
  std::memcpy(id, &u, sizeof u);
  return WSR_OK;
}

int wsr_comm_open(const uint8_t* id, int32_t world, int32_t rank, int32_t device, wsr_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return fail(WSR_E_INVALID, "bad comm arguments");
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return fail(WSR_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wsr_comm> c(new wsr_comm());
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) return fail(WSR_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  // exchange stream priority (WSR_COMM_PRIORITY=1: high).  Normal since
  // round 4: at high priority the owner replays' thousands of one-wave
  // workgroups are dispatched ahead of the next batches' persistent kernels;
  // one-rank rehearsal 15.6 -> 16.7 M q/s every query sharded, 12.7 -> 15.4 M
  // hybrid (profiles/r04g/; round 2 had measured +3 % for high)
  // (a stream with a full CU mask, i.e. a hardware queue of its own at normal
  // priority, was slower again: 16.5 / 14.2 M against 17.0 / 15.6 M,
  // profiles/r04n/; low priority was slower still: 16.3 / 12.9 M against
  // 16.7 / 15.3 M, profiles/r04s/)
  int lo_prio = 0, hi_prio = 0;
  const bool prio = env_number("WSR_COMM_PRIORITY", 0) != 0 &&
                    hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) == hipSuccess;
  if ((prio ? hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_prio)
            : hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
    (void)ncclCommDestroy(c->comm);
    return fail(WSR_E_HIP, "hipStreamCreate failed");
  }
  c->world = world;
  c->rank = rank;
  c->device = device;
  const char* ht = std::getenv("WSR_HOST_TIMING");
  c->timing = ht && *ht && *ht != '0';
  c->defer = env_number("WSR_REPLAY_DEFER", 1) != 0;
  wsr_comm* cp = c.get();
  cp->worker = std::thread([cp] { exchange_worker(cp); });
  *out = c.release();
  return WSR_OK;
}

int wsr_loopback_create(int32_t world, wsr_loopback** out) {
  if (!out || world < 1 || world > kMaxOwners) return fail(WSR_E_INVALID, "bad loopback arguments");
  *out = new wsr_loopback();
  (*out)->world = world;
  return WSR_OK;
}

void wsr_loopback_destroy(wsr_loopback* l) { delete l; }

int wsr_comm_open_loopback(wsr_loopback* l, int32_t rank, int32_t device, wsr_comm** out) {
  if (!l || !out || rank < 0 || rank >= l->world) return fail(WSR_E_INVALID, "bad loopback comm arguments");
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return fail(WSR_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wsr_comm> c(new wsr_comm());
  c->loop = l;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->loop_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->loop_read, hipEventDisableTiming) != hipSuccess) {
    if (c->loop_ready) (void)hipEventDestroy(c->loop_ready);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    return fail(WSR_E_HIP, "hipStreamCreate / hipEventCreate failed");
  }
  c->world = l->world;
  c->rank = rank;
  c->device = device;
  c->defer = env_number("WSR_REPLAY_DEFER", 1) != 0;
  wsr_comm* cp = c.get();
  cp->worker = std::thread([cp] { exchange_worker(cp); });
  *out = c.release();
  return WSR_OK;
}

void wsr_comm_close(wsr_comm* c) {
  if (!c) return;
  (void)wsr_comm_flush(c);   // (every deferred replay enqueued before the worker stops)
  {
    std::lock_guard<std::mutex> g(c->mu);
    c->stop = true;
  }
  c->cv.notify_one();
  if (c->worker.joinable()) c->worker.join();
  if (c->timing && c->steps)
    std::fprintf(stderr, "wsr_shard_step host us/step over %llu steps: run %.1f submit %.1f rccl %.1f replay %.1f "
                 "(rccl and replay: the exchange worker)\n",
                 static_cast<unsigned long long>(c->steps), c->t_ns[0] / 1e3 / c->steps,
                 c->t_ns[1] / 1e3 / c->steps, c->t_ns[2] / 1e3 / c->steps, c->t_ns[3] / 1e3 / c->steps);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (XSlot& S : c->xs) {
    for (size_t i = 0; i < S.n_done; ++i) (void)hipEventSynchronize(S.done[i]);   // (replays in lean kernels)
    for (hipEvent_t e : S.done) (void)hipEventDestroy(e);
    if (S.xa) (void)hipEventDestroy(S.xa);
    if (S.send) (void)hipFree(S.send);
    if (S.recv) (void)hipFree(S.recv);
  }
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->loop_ready) (void)hipEventDestroy(c->loop_ready);
  if (c->loop_read) (void)hipEventDestroy(c->loop_read);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int owner_replay_meta_on(wsr_handle* h, wsr_batch* b, int32_t q0, int32_t nq_owned, int32_t n_shards,
                                const int32_t* d_rmeta, uint64_t meta_stride, uint64_t stride,
                                const void* d_recv, hipStream_t st) {
  if (!h || !b || n_shards <= 0 || n_shards > kMaxOwners || nq_owned < 0 || q0 < 0 || q0 + nq_owned > b->nq ||
      stride == 0 || (nq_owned && (!d_rmeta || !d_recv)))
    return fail(WSR_E_INVALID, "bad owner_replay_meta arguments");
  try {
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(launch_owner_replay_meta(b->d_q, q0, nq_owned, n_shards, d_rmeta, meta_stride, stride,
                                    static_cast<const Event*>(d_recv), b->d_hits, b->stride, b->d_nhits,
                                    b->d_ctr, b->has_wide, st));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

// One step of a doc-range sharded batch, all of it enqueued, nothing waited on:
//   batch stream: the plan + segment kernels; the worker that finishes a
//     query reduces its events into the owner's region of the send buffer;
//   communicator stream (joined by xev[0]): one ncclAllToAll of the regions
//     (RCCL's pairwise exchange over xGMI), then the owner replay of this
//     rank's queries; xev[1] marks the end.
// An owner's region is [{count, offset} of its qpr queries, padded to whole
// events][slot of events], so one collective moves both.  The batch stream
// never waits on the exchange inside a step, so the next batches' kernels run
// under it; the next run of this batch waits for xev[1] (long past by then),
// and the fetches join it.
// An owner's region: the meta block (2 int32 per query, 4 per event, so the
// qpr pairs take ceil(qpr / 2) events) followed by the slot.
static uint64_t region_events_of(int32_t q_per_owner, int64_t slot) {
  return (static_cast<uint64_t>(q_per_owner) + 1) / 2 + static_cast<uint64_t>(slot);
}

static int check_step(wsr_handle* h, wsr_batch* b, int W, int32_t q_per_owner, int64_t slot) {
  if (!h || !b || W < 1 || q_per_owner <= 0 || slot <= 0 || static_cast<int64_t>(q_per_owner) * W != b->nq)
    return fail(WSR_E_INVALID, "bad shard_step arguments (the batch must hold world * q_per_owner queries)");
  if (W > kMaxOwners) return fail(WSR_E_LIMIT, "more than kMaxOwners ranks");
  if (static_cast<uint64_t>(slot) > 0xFFFFFFFFull) return fail(WSR_E_LIMIT, "slot over 2^32 events");
  return WSR_OK;
}

// The events that order a shard step's exchange against the batch's runs.
static void ensure_xev(wsr_batch* b) {
  if (!b->xev[0]) {
    HIP_OK(hipEventCreateWithFlags(&b->xev[0], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&b->xev[1], hipEventDisableTiming));
  }
}

// The exchange buffers of b: send and receive, need events each.
static void ensure_xbuf(wsr_batch* b, uint64_t need, int W) {
  if (need > b->x_slots || W != b->x_pairs) {
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));
    if (b->d_xsend) HIP_OK(hipFree(b->d_xsend));
    if (b->d_xrecv) HIP_OK(hipFree(b->d_xrecv));
    b->d_xsend = b->d_xrecv = nullptr;
    HIP_OK(hipMalloc(&b->d_xsend, sizeof(Event) * need));
    HIP_OK(hipMalloc(&b->d_xrecv, sizeof(Event) * need));
    b->x_slots = need;
    b->x_pairs = W;
  }
  ensure_xev(b);
}

// First half of a shard step: run the batch with fused emission into the
// send regions, owner o's region at send + o * owner_stride events (one
// batch: its own buffer, owner_stride = region; a step group: the group's
// buffer, this batch's region within every owner's run of regions).
static int step_emit_into(wsr_handle* h, wsr_batch* b, int W, int32_t q_per_owner, int64_t slot, Event* send,
                          uint64_t owner_stride, const OwnerJob* oj = nullptr) {
  const uint64_t meta_events = (static_cast<uint64_t>(q_per_owner) + 1) / 2;
  const uint64_t meta_stride = owner_stride * (sizeof(Event) / sizeof(int32_t));   // int32 per owner
  const ShardEmit se{W, q_per_owner, static_cast<uint64_t>(slot), send + meta_events, owner_stride,
                     reinterpret_cast<int32_t*>(send), meta_stride};
  const int rc = batch_run(h, b, &se, oj);
  if (rc == WSR_OK) {
    b->x_world = W;
    b->x_qpr = q_per_owner;
    b->x_slot = slot;
  }
  return rc;
}

static int step_emit(wsr_handle* h, wsr_batch* b, int W, int32_t q_per_owner, int64_t slot) {
  if (int rc = check_step(h, b, W, q_per_owner, slot)) return rc;
  const uint64_t region = region_events_of(q_per_owner, slot);
  try {
    HIP_OK(hipSetDevice(h->device));
    ensure_xbuf(b, region * W, W);
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return step_emit_into(h, b, W, q_per_owner, slot, b->d_xsend, region);
}

// Second half: the owner replay of this rank's queries over the receive
// regions (region g = what shard g sent this owner, at recv + g *
// owner_stride events), on stream st.
static int step_replay_from(wsr_handle* h, wsr_batch* b, int rank, int W, int32_t q_per_owner, const Event* recv,
                            uint64_t owner_stride, hipStream_t st) {
  const uint64_t meta_events = (static_cast<uint64_t>(q_per_owner) + 1) / 2;
  const uint64_t meta_stride = owner_stride * (sizeof(Event) / sizeof(int32_t));
  return owner_replay_meta_on(h, b, rank * q_per_owner, q_per_owner, W, reinterpret_cast<const int32_t*>(recv),
                              meta_stride, owner_stride, recv + meta_events, st);
}

static int step_replay(wsr_handle* h, wsr_batch* b, int rank, int W, int32_t q_per_owner, int64_t slot,
                       hipStream_t st) {
  return step_replay_from(h, b, rank, W, q_per_owner, b->d_xrecv, region_events_of(q_per_owner, slot), st);
}

// A deferred group's replays not yet enqueued go to the communicator's
// stream (after its all-to-all, which the worker has enqueued first).
static void flush_group(wsr_comm* c, XGroup& g) {
  while (!g.enq.load(std::memory_order_acquire)) std::this_thread::yield();
  XSlot& S = c->xs[g.xs];
  const uint64_t region = region_events_of(g.qpr, g.slot), run = region * g.bs.size();
  int rc = c->err.load() == WSR_OK ? WSR_OK : WSR_E_HIP;
  for (size_t i = 0; i < g.bs.size(); ++i) {
    if (g.queued[i]) continue;
    g.queued[i] = 1;
    c->replays_stream.fetch_add(1);
    wsr_batch* b = g.bs[i];
    if (rc == WSR_OK) {
      rc = step_replay_from(g.h, b, c->rank, c->world, g.qpr, S.recv + region * i, run, c->stream);
      if (rc) set_comm_err(c, rc, g_err);
      else if (hipEventRecord(b->xev[1], c->stream) != hipSuccess ||
               hipEventRecord(S.done[i], c->stream) != hipSuccess) {
        rc = WSR_E_HIP;
        set_comm_err(c, rc, "hipEventRecord failed");
      }
    }
    b->x_pending = rc == WSR_OK;
    b->x_comm.store(nullptr, std::memory_order_release);
    b->x_enq.fetch_add(1, std::memory_order_release);
  }
  S.n_done = g.bs.size();
}

// Enqueue the deferred replays of every pending group up to the one holding
// `upto` (all of them: upto null), oldest first.
static void replay_flush(wsr_comm* c, const wsr_batch* upto) {
  std::lock_guard<std::recursive_mutex> lk(c->pend_mu);
  if (upto) {
    bool held = false;
    for (const auto& g : c->pend)
      for (size_t i = 0; i < g->bs.size(); ++i) held = held || (!g->queued[i] && g->bs[i] == upto);
    if (!held) return;
  }
  while (!c->pend.empty()) {
    std::shared_ptr<XGroup> g = c->pend.front();
    c->pend.pop_front();
    bool has = false;
    for (size_t i = 0; i < g->bs.size(); ++i) has = has || (!g->queued[i] && g->bs[i] == upto);
    flush_group(c, *g);
    if (has) return;
  }
}

int wsr_comm_flush(wsr_comm* c) {
  if (!c) return fail(WSR_E_INVALID, "null argument");
  try {
    HIP_OK(hipSetDevice(c->device));
    replay_flush(c, nullptr);
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  if (const int e = c->err.load()) {
    std::lock_guard<std::mutex> g(c->mu);
    return fail(e, "exchange: " + c->err_msg);
  }
  return WSR_OK;
}

int wsr_comm_stats_get(wsr_comm* c, wsr_comm_stats* out) {
  if (!c || !out) return fail(WSR_E_INVALID, "null argument");
  std::lock_guard<std::recursive_mutex> lk(c->pend_mu);
  out->groups = static_cast<int64_t>(c->n_groups);
  out->steps = static_cast<int64_t>(c->steps);
  out->replays_in_lean = c->replays_lean.load();
  out->replays_on_stream = c->replays_stream.load();
  return WSR_OK;
}

// A step group: n batches of the same shape, each emitted into its region of
// every owner's run of n regions in one of the communicator's exchange buffer
// sets, then ONE ncclAllToAll of the runs on the communicator's stream.  The
// collective's host cost (~0.1-0.2 ms a call under load, more than a whole
// step's kernels) is paid once per group.  The group's owner replays run on
// the communicator's stream too, or (deferred, the default) in the lean
// kernels of the group kReplayLag groups later: batch i of this group replays
// batch i of that one after its own items.
int wsr_shard_steps(wsr_handle* h, wsr_batch* const* bs, int32_t n, wsr_comm* c, int32_t q_per_owner,
                    int64_t slot) {
  if (!c || !bs || n < 1) return fail(WSR_E_INVALID, "bad shard_steps arguments");
  if (const int e = c->err.load()) {   // an earlier exchange of this communicator failed
    std::lock_guard<std::mutex> g(c->mu);
    return fail(e, "exchange worker: " + c->err_msg);
  }
  const int W = c->world;
  for (int i = 0; i < n; ++i) {
    if (int rc = check_step(h, bs[i], W, q_per_owner, slot)) return rc;
    for (int j = 0; j < i; ++j)
      if (bs[j] == bs[i]) return fail(WSR_E_INVALID, "a batch twice in one step group");
  }
  uint64_t t0 = c->timing ? now_ns() : 0;
  auto lap = [&](int i) {
    if (!c->timing) return;
    const uint64_t t = now_ns();
    c->t_ns[i] += t - t0;
    t0 = t;
  };
  const uint64_t region = region_events_of(q_per_owner, slot);
  const uint64_t run = region * static_cast<uint64_t>(n);   // events per owner
  std::lock_guard<std::recursive_mutex> pend_lock(c->pend_mu);
  const int xs = static_cast<int>(c->n_groups % kXSlots);
  XSlot& S = c->xs[xs];
  std::shared_ptr<XGroup> P;   // the group whose replays this one's lean kernels take
  // Once P is off pend, every exit enqueues what its lean kernels did not
  // take on the communicator's stream: on an early error return its batches
  // would otherwise wait in x_join for replays nobody can find any more.
  struct FlushRest {
    wsr_comm* c;
    std::shared_ptr<XGroup>& P;
    ~FlushRest() {
      if (P) flush_group(c, *P);
    }
  } flush_rest{c, P};
  std::vector<OwnerJob> oj(static_cast<size_t>(n));
  try {
    HIP_OK(hipSetDevice(h->device));
    // this group's batches: their own earlier replays enqueued first
    for (int i = 0; i < n; ++i) {
      ensure_xev(bs[i]);
      if (bs[i]->x_comm.load(std::memory_order_acquire)) replay_flush(c, bs[i]);
    }
    // the slot: its previous group's all-to-all and replays enqueued (their
    // end events are what this group's emission and exchange wait for)
    if (S.last) {
      for (size_t i = 0; i < S.last->queued.size(); ++i)
        if (!S.last->queued[i]) replay_flush(c, S.last->bs[i]);
      while (!S.last->enq.load(std::memory_order_acquire)) std::this_thread::yield();
    }
    const uint64_t need = run * static_cast<uint64_t>(W);
    if (need > S.events) {
      if (S.last) {
        HIP_OK(hipEventSynchronize(S.xa));
        for (size_t i = 0; i < S.n_done; ++i) HIP_OK(hipEventSynchronize(S.done[i]));
        S.last.reset();
        S.n_done = 0;
      }
      if (S.send) HIP_OK(hipFree(S.send));
      if (S.recv) HIP_OK(hipFree(S.recv));
      S.send = S.recv = nullptr;
      S.events = 0;
      HIP_OK(hipMalloc(&S.send, sizeof(Event) * need));
      HIP_OK(hipMalloc(&S.recv, sizeof(Event) * need));
      S.events = need;
    }
    if (!S.xa) HIP_OK(hipEventCreateWithFlags(&S.xa, hipEventDisableTiming));
    while (S.done.size() < static_cast<size_t>(n)) {
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      S.done.push_back(e);
    }
    // the deferred replays this group's lean kernels take
    if (c->defer && c->pend.size() >= kReplayLag) {
      P = c->pend.front();
      c->pend.pop_front();
      while (!P->enq.load(std::memory_order_acquire)) std::this_thread::yield();
      const XSlot& SP = c->xs[P->xs];
      const uint64_t rP = region_events_of(P->qpr, P->slot), runP = rP * P->bs.size();
      const uint64_t meta_events = (static_cast<uint64_t>(P->qpr) + 1) / 2;
      for (size_t i = 0; i < P->bs.size() && i < static_cast<size_t>(n); ++i) {
        const wsr_batch* pb = P->bs[i];
        if (P->queued[i]) continue;
        if (pb->has_wide) continue;   // (the LDS heap: on the communicator's stream)
        const Event* recv = SP.recv + rP * i;
        oj[i] = OwnerJob{pb->d_q, reinterpret_cast<const int32_t*>(recv), recv + meta_events, pb->d_hits,
                         pb->d_nhits, pb->d_ctr, runP * (sizeof(Event) / sizeof(int32_t)), runP,
                         c->rank * P->qpr, P->qpr, W, pb->stride};
      }
    }
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  for (int i = 0; i < n; ++i) {
    wsr_batch* b = bs[i];
    const OwnerJob* job = oj[i].nq > 0 ? &oj[i] : nullptr;
    try {
      if (S.last) HIP_OK(hipStreamWaitEvent(b->st, S.xa, 0));   // the slot's last all-to-all read its send buffer
      if (job) HIP_OK(hipStreamWaitEvent(b->st, c->xs[P->xs].xa, 0));
    } catch (const std::exception& e) {
      return fail(WSR_E_HIP, e.what());
    }
    if (int rc = step_emit_into(h, b, W, q_per_owner, slot, S.send + region * i, run, job)) return rc;
    if (hipEventRecord(b->xev[0], b->st) != hipSuccess) return fail(WSR_E_HIP, "hipEventRecord failed");
    if (job) {
      wsr_batch* pb = P->bs[static_cast<size_t>(i)];
      if (hipEventRecord(pb->xev[1], b->st) != hipSuccess ||
          hipEventRecord(c->xs[P->xs].done[static_cast<size_t>(i)], b->st) != hipSuccess)
        return fail(WSR_E_HIP, "hipEventRecord failed");
      pb->x_pending = true;
      pb->x_comm.store(nullptr, std::memory_order_release);
      P->queued[static_cast<size_t>(i)] = 1;
      c->replays_lean.fetch_add(1);
      pb->x_enq.fetch_add(1, std::memory_order_release);
    }
  }
  // the rest of P (more batches than this group, or wide ones): the
  // communicator's stream
  if (P) flush_group(c, *P);
  P.reset();
  lap(0);
  // the exchange half: the communicator's worker thread enqueues it
  auto g = std::make_shared<XGroup>();
  g->h = h;
  g->bs.assign(bs, bs + n);
  g->qpr = q_per_owner;
  g->slot = slot;
  g->xs = xs;
  g->defer = c->defer;
  g->queued.assign(static_cast<size_t>(n), g->defer ? 0 : 1);
  if (S.last) g->wait_done.assign(S.done.begin(), S.done.begin() + static_cast<std::ptrdiff_t>(S.n_done));
  S.last = g;
  S.n_done = 0;
  ++c->n_groups;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    for (int i = 0; i < n; ++i) {
      bs[i]->x_req.fetch_add(1, std::memory_order_acq_rel);
      if (g->defer) bs[i]->x_comm.store(c, std::memory_order_release);
    }
    c->jobs.push_back(g);
  }
  if (g->defer) c->pend.push_back(g);
  c->cv.notify_one();
  lap(1);
  c->steps += static_cast<uint64_t>(n);
  return WSR_OK;
}

int wsr_shard_step(wsr_handle* h, wsr_batch* b, wsr_comm* c, int32_t q_per_owner, int64_t slot) {
  return wsr_shard_steps(h, &b, 1, c, q_per_owner, slot);
}

int wsr_shard_step_regions(int32_t q_per_owner, int64_t slot, uint64_t* region_bytes) {
  if (q_per_owner <= 0 || slot <= 0 || !region_bytes) return fail(WSR_E_INVALID, "bad arguments");
  *region_bytes = region_events_of(q_per_owner, slot) * sizeof(Event);
  return WSR_OK;
}

static int shard_step_emit(wsr_handle* h, wsr_batch* b, int32_t world, int32_t q_per_owner, int64_t slot,
                           void* host_send, bool wait) {
  if (!host_send) return fail(WSR_E_INVALID, "null host buffer");
  const int rc = step_emit(h, b, world, q_per_owner, slot);
  if (rc) return rc;
  try {
    HIP_OK(hipMemcpyAsync(host_send, b->d_xsend, sizeof(Event) * region_events_of(q_per_owner, slot) * world,
                          hipMemcpyDeviceToHost, b->st));
    if (wait) HIP_OK(hipStreamSynchronize(b->st));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_shard_step_emit(wsr_handle* h, wsr_batch* b, int32_t world, int32_t q_per_owner, int64_t slot,
                        void* host_send) {
  return shard_step_emit(h, b, world, q_per_owner, slot, host_send, true);
}

int wsr_shard_step_emit_async(wsr_handle* h, wsr_batch* b, int32_t world, int32_t q_per_owner, int64_t slot,
                              void* host_send) {
  return shard_step_emit(h, b, world, q_per_owner, slot, host_send, false);
}

int wsr_batch_set_item_blocks(wsr_handle* h, wsr_batch* b, int32_t blocks) {
  if (!h || !b || blocks < 1 || blocks > kSegCost) return fail(WSR_E_INVALID, "item blocks must be 1..63");
  b->seg_cap = static_cast<uint32_t>(blocks);
  return WSR_OK;
}

int wsr_batch_stream_sync(wsr_handle* h, wsr_batch* b) {
  if (!h || !b) return fail(WSR_E_INVALID, "null argument");
  const hipError_t e = hipStreamSynchronize(b->st);
  return e == hipSuccess ? WSR_OK : fail(WSR_E_HIP, hipGetErrorString(e));
}

int wsr_shard_step_replay(wsr_handle* h, wsr_batch* b, int32_t rank, int32_t world, int32_t q_per_owner,
                          int64_t slot, const void* host_recv) {
  // (the regions are read at the strides the emission wrote them with: the
  // arguments must be the ones of the preceding wsr_shard_step_emit)
  if (!h || !b || !host_recv || world < 1 || rank < 0 || rank >= world || q_per_owner <= 0 || slot <= 0 ||
      !b->x_fused || b->x_world != world || b->x_qpr != q_per_owner || b->x_slot != slot ||
      static_cast<int64_t>(q_per_owner) * world != b->nq)
    return fail(WSR_E_INVALID, "call wsr_shard_step_emit with the same world, q_per_owner and slot first");
  try {
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipMemcpyAsync(b->d_xrecv, host_recv, sizeof(Event) * region_events_of(q_per_owner, slot) * world,
                          hipMemcpyHostToDevice, b->st));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return step_replay(h, b, rank, world, q_per_owner, slot, b->st);
}

// Host-exchange owner replays deferred into a later run's lean kernel (the
// counterpart of the communicator's deferral, wsr_shard_steps): a separate
// owner replay launch -- thousands of one-wave workgroups -- costs more than
// its work beside the persistent kernels of the next batches.
int wsr_shard_step_replay_deferred(wsr_handle* h, wsr_batch* b, int32_t rank, int32_t world, int32_t q_per_owner,
                                   int64_t slot, const void* host_recv) {
  if (!h || !b || !host_recv || world < 1 || rank < 0 || rank >= world || q_per_owner <= 0 || slot <= 0 ||
      !b->x_fused || b->x_world != world || b->x_qpr != q_per_owner || b->x_slot != slot ||
      static_cast<int64_t>(q_per_owner) * world != b->nq)
    return fail(WSR_E_INVALID, "call wsr_shard_step_emit with the same world, q_per_owner and slot first");
  if (b->has_wide)   // (the LDS heap: the replay launch of its own)
    return wsr_shard_step_replay(h, b, rank, world, q_per_owner, slot, host_recv);
  try {
    HIP_OK(hipSetDevice(h->device));
    if (b->hdef) host_replay_flush(b);   // (an earlier one still waiting: first)
    ensure_xev(b);
    HIP_OK(hipMemcpyAsync(b->d_xrecv, host_recv, sizeof(Event) * region_events_of(q_per_owner, slot) * world,
                          hipMemcpyHostToDevice, b->st));
    HIP_OK(hipEventRecord(b->xev[0], b->st));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  std::lock_guard<std::mutex> g(h->hdef_mu);
  b->hdef_rank = rank;
  b->hdef.store(h);
  h->hdef_q.push_back(b);
  return WSR_OK;
}

// The oldest deferred host replay that a run of b can carry (not b's own),
// off the queue; its OwnerJob in *oj.
static wsr_batch* take_host_replay(wsr_handle* h, const wsr_batch* b, OwnerJob* oj) {
  std::lock_guard<std::mutex> g(h->hdef_mu);
  for (auto it = h->hdef_q.begin(); it != h->hdef_q.end(); ++it) {
    wsr_batch* pb = *it;
    if (pb == b) continue;
    h->hdef_q.erase(it);
    // counted before hdef is cleared: an x_join that sees it cleared waits
    // until the taking run has recorded xev[1] (x_enq)
    pb->x_req.fetch_add(1, std::memory_order_acq_rel);
    pb->hdef.store(nullptr);
    const uint64_t region = region_events_of(pb->x_qpr, pb->x_slot);
    const uint64_t meta_events = (static_cast<uint64_t>(pb->x_qpr) + 1) / 2;
    *oj = OwnerJob{pb->d_q, reinterpret_cast<const int32_t*>(pb->d_xrecv), pb->d_xrecv + meta_events, pb->d_hits,
                   pb->d_nhits, pb->d_ctr, region * (sizeof(Event) / sizeof(int32_t)), region,
                   pb->hdef_rank * pb->x_qpr, pb->x_qpr, pb->x_world, pb->stride};
    return pb;
  }
  return nullptr;
}

// A taken (or still queued, via host_replay_flush) replay on pb's own stream.
static void host_replay_enqueue(wsr_batch* pb, wsr_handle* h) {
  if (step_replay(h, pb, pb->hdef_rank, pb->x_world, pb->x_qpr, pb->x_slot, pb->st) == WSR_OK &&
      hipEventRecord(pb->xev[1], pb->st) == hipSuccess)
    pb->x_pending = true;
}

static void host_replay_flush(wsr_batch* b) {
  wsr_handle* h = b->hdef.load();
  if (!h) return;
  {
    std::lock_guard<std::mutex> g(h->hdef_mu);
    if (!b->hdef.load()) return;   // (taken by a run meanwhile; x_join waits for its enqueue)
    for (auto it = h->hdef_q.begin(); it != h->hdef_q.end(); ++it)
      if (*it == b) {
        h->hdef_q.erase(it);
        break;
      }
    b->hdef.store(nullptr);
  }
  host_replay_enqueue(b, h);
}

int wsr_batch_fetch_range(wsr_handle* h, wsr_batch* b, int32_t q0, int32_t nq, wsr_hit* hits,
                          int32_t* n_hits) {
  if (!h || !b || q0 < 0 || nq < 0 || q0 + nq > b->nq) return fail(WSR_E_INVALID, "bad range");
  try {
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(b->st));
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));   // a shard step's exchange + replay
    uint32_t ctr[kNumCounters];
    HIP_OK(hipMemcpy(ctr, b->d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
    if (ctr[kCtrError])
      return fail(WSR_E_INTERNAL, "device reported error flags " + std::to_string(ctr[kCtrError]) +
                                      (ctr[kCtrError] & kErrExchange ? " (an exchange slot overflowed)" : ""));
    if (nq && hits)
      HIP_OK(hipMemcpy(hits, b->d_hits + static_cast<size_t>(q0) * b->stride,
                       sizeof(HitDev) * static_cast<size_t>(nq) * b->stride, hipMemcpyDeviceToHost));
    if (nq && n_hits)
      HIP_OK(hipMemcpy(n_hits, b->d_nhits + q0, sizeof(int32_t) * nq, hipMemcpyDeviceToHost));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_stream(wsr_handle* h, void** stream) {
  if (!h || !stream) return fail(WSR_E_INVALID, "null argument");
  *stream = h->stream;
  return WSR_OK;
}

int wsr_debug_decode_block(wsr_handle* h, int32_t id, int32_t block, int32_t which, uint32_t* out,
                           int32_t* count) {
  if (!h || !out || id < 0 || id >= static_cast<int32_t>(h->lists.size()))
    return fail(WSR_E_INVALID, "bad list id");
  const ListDev& L = h->lists[id];
  if (block < 0 || static_cast<uint32_t>(block) >= L.nblk) return fail(WSR_E_INVALID, "bad block");
  std::lock_guard<std::mutex> g(h->mu);
  const BlockDev& bd = h->blocks[L.blk0 + block];
  const uint32_t cnt = static_cast<uint32_t>(block) == L.nblk - 1 ? L.tail_cnt : 128u;
  try {
    uint32_t* d_out = nullptr;
    HIP_OK(hipMalloc(&d_out, 128 * sizeof(uint32_t)));
    const uint8_t* p = h->d_blob + L.base + (which ? bd.tf_rel : bd.doc_rel);
    const uint32_t bits = which ? (h->meta[L.blk0 + block] >> 8) : (h->meta[L.blk0 + block] & 0xFF);
    hipError_t e = launch_decode_probe(p, bits, cnt, which == 0, bd.prev, d_out, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d_out, 128 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    HIP_OK(e);
  } catch (const std::exception& ex) {
    return fail(WSR_E_HIP, ex.what());
  }
  if (count) *count = static_cast<int32_t>(cnt);
  return WSR_OK;
}

int wsr_debug_wg_stats(wsr_handle* h, wsr_batch* b, uint32_t* out, int32_t max_words,
                       int32_t* n_wg, int32_t* stride) {
  if (!h || !b) return fail(WSR_E_INVALID, "null argument");
  std::lock_guard<std::mutex> g(h->mu);
  // general workgroups, then lean waves (the conjunctive instance's, then the phrase instance's);
  // the rows of a kernel the last run did not launch (b->ran_conj / ran_gen) are stale
  const int rows = b->seg_grid + kLeanWaves * (b->lean_wgs + (b->has_phrase ? b->lean_wgs_ph : 0));
  if (n_wg) *n_wg = rows;
  if (stride) *stride = kStatStride;
  if (!out) return WSR_OK;
  const size_t n = std::min<size_t>(static_cast<size_t>(std::max(max_words, 0)),
                                    static_cast<size_t>(kStatStride) * rows);
  try {
    HIP_OK(hipStreamSynchronize(b->st));
    if (x_join(b)) HIP_OK(hipEventSynchronize(b->xev[1]));   // a shard step's exchange + replay
    HIP_OK(hipMemcpy(out, b->d_stats, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  } catch (const std::exception& e) {
    return fail(WSR_E_HIP, e.what());
  }
  return WSR_OK;
}

int wsr_debug_dense_lookup(const char* dir, uint32_t doc_lo, uint32_t doc_hi, uint32_t dense_div,
                           const char* term, const uint32_t* docs, int32_t n, int32_t* tf_out,
                           int32_t* is_dense) {
  if (!dir || !term || (n > 0 && (!docs || !tf_out))) return fail(WSR_E_INVALID, "null argument");
  try {
    VacuumIndex idx;
    idx.open(dir);
    const HostImage img = build_image(idx, doc_lo, doc_hi ? doc_hi : 0xFFFFFFFFu, 4, dense_div);
    const int32_t id = idx.find(term);
    const bool dense = id >= 0 && img.lists[id].bm != kNoDense;
    if (is_dense) *is_dense = dense ? 1 : 0;
    for (int32_t i = 0; i < n; ++i)
      tf_out[i] = dense ? static_cast<int32_t>(dense_lookup_host(img, img.lists[id], docs[i])) : -1;
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

// ------------------------------------------------------------ building --
static void fill_stats(const BuildStats& s, wsr_build_stats* st) {
  if (!st) return;
  st->n_docs = s.n_docs;
  st->n_terms = s.n_terms;
  st->n_postings = s.n_postings;
  st->vacuum_bytes = s.vacuum_bytes;
  st->docs_char4_ge_0x80 = s.docs_char4_ge_0x80;
  st->avg_length = s.avg_length;
}

int wsr_build_from_linedoc(const char* linedoc, int64_t n_rows, const char* format,
                           const char* out_dir, wsr_build_stats* st) {
  if (!linedoc || !format || !out_dir) return fail(WSR_E_INVALID, "null argument");
  try {
    fill_stats(build_from_linedoc(linedoc, n_rows, format, out_dir), st);
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_build_from_linedoc_bloom(const char* linedoc, int64_t n_rows, const char* format,
                                 const char* out_dir, float ratio, int32_t expected_entries,
                                 wsr_build_stats* st) {
  if (!linedoc || !format || !out_dir) return fail(WSR_E_INVALID, "null argument");
  if (!(ratio > 0.0f && ratio < 1.0f) || expected_entries < 1)
    return fail(WSR_E_INVALID, "bloom ratio must be in (0, 1) and expected entries >= 1");
  try {
    BloomSpec b;
    b.on = true;
    b.ratio = ratio;
    b.entries = expected_entries;
    fill_stats(build_from_linedoc(linedoc, n_rows, format, out_dir, b), st);
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_build_synthetic(const char* out_dir, int64_t n_docs, int64_t vocab, double zipf_s,
                        uint64_t seed, int32_t with_positions, int32_t threads,
                        wsr_build_stats* st) {
  if (!out_dir || n_docs <= 0 || vocab <= 0) return fail(WSR_E_INVALID, "bad arguments");
  try {
    SyntheticSpec sp;
    sp.n_docs = n_docs;
    sp.vocab = vocab;
    sp.zipf_s = zipf_s;
    sp.seed = seed;
    sp.with_positions = with_positions != 0;
    sp.threads = threads;
    fill_stats(build_synthetic(sp, out_dir), st);
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_build_wiki_standin(const char* out_dir, int64_t n_docs, double term_scale, uint64_t seed,
                           int32_t threads, wsr_build_stats* st) {
  if (!out_dir || n_docs < 16 || !(term_scale > 0)) return fail(WSR_E_INVALID, "bad arguments");
  try {
    WikiSpec sp;
    sp.n_docs = n_docs;
    sp.term_scale = term_scale;
    sp.seed = seed;
    sp.threads = threads;
    fill_stats(build_wiki_standin(sp, out_dir), st);
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_build_wiki_standin_topics(const char* out_dir, int64_t n_docs, double term_scale, uint64_t seed,
                                  int32_t threads, int32_t topics, int32_t topics_per_term, double affinity,
                                  wsr_build_stats* st) {
  if (!out_dir || n_docs < 16 || !(term_scale > 0) || topics < 1 || topics_per_term < 1 || topics_per_term > 16 ||
      !(affinity >= 0 && affinity <= 1) || topics > n_docs)
    return fail(WSR_E_INVALID, "bad arguments");
  try {
    WikiSpec sp;
    sp.n_docs = n_docs;
    sp.term_scale = term_scale;
    sp.seed = seed;
    sp.threads = threads;
    sp.topics = topics;
    sp.topics_per_term = topics_per_term;
    sp.affinity = affinity;
    fill_stats(build_wiki_standin(sp, out_dir), st);
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_gen_two_term_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                         const char* out_path, int64_t* n_written) {
  if (!index_dir || !out_path) return fail(WSR_E_INVALID, "null argument");
  try {
    int64_t n = gen_two_term_log(index_dir, n_queries, seed, out_path);
    if (n_written) *n_written = n;
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_gen_mixed_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                      const char* out_path, int64_t* n_written) {
  if (!index_dir || !out_path) return fail(WSR_E_INVALID, "null argument");
  try {
    int64_t n = gen_mixed_log(index_dir, n_queries, seed, out_path);
    if (n_written) *n_written = n;
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_gen_single_term_log(const char* index_dir, int32_t high, int64_t n_queries, uint64_t seed,
                      const char* out_path, int64_t* n_written) {
  if (!index_dir || !out_path) return fail(WSR_E_INVALID, "null argument");
  try {
    int64_t n = gen_single_term_log(index_dir, high != 0, n_queries, seed, out_path);
    if (n_written) *n_written = n;
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

int wsr_gen_phrase_log(const char* index_dir, int64_t n_queries, uint64_t seed,
                       const char* out_path, int64_t* n_written) {
  if (!index_dir || !out_path) return fail(WSR_E_INVALID, "null argument");
  try {
    int64_t n = gen_phrase_log(index_dir, n_queries, seed, out_path);
    if (n_written) *n_written = n;
  } catch (const std::exception& e) {
    return fail(WSR_E_IO, e.what());
  }
  return WSR_OK;
}

}  // extern "C"
