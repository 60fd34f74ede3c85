// Serving front end over one engine handle: a micro-batcher that coalesces
// concurrent single-query Search() calls into GPU batches, plus a closed-loop
// load generator that measures QPS and latency percentiles through it.
//
// Reference: the gRPC server shares one read-only engine between N worker
// threads, each calling engine->Search() for one request at a time
// (grpc_server_impl.h:104-107,260-263,382-389); the benchmark client keeps
// several requests in flight per thread (grpc_client_impl.h:448-459,557-620).
// On the GPU one query is far too little work, so the dispatcher thread here
// collects requests for a short window (or until a batch is full), runs them
// as one resident batch (wsr_batch_*), and hands each caller its own entries.
// Up to four batches are in flight: the dispatcher collects, uploads and
// launches, a completer thread retires them in launch order and hands out the
// results, so the next batch is launched while earlier ones run and return.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "../../include/wiser_hip.h"

namespace wiser {
void set_last_error(const std::string& msg);   // engine.cc
}

namespace {

using Clock = std::chrono::steady_clock;

// Completion flag of one request: 0 pending, 1 done, 2 pending with its
// caller asleep on the flag (a futex), so the dispatcher wakes exactly the
// callers that sleep and never takes a lock to do it.
constexpr int kPending = 0, kDone = 1, kSleeping = 2;

struct Req {
  wsr_hit* out = nullptr;
  int32_t* n_out = nullptr;
  int rc = WSR_OK;
  std::string err;   // wsr_last_error() of the thread the request failed on
  std::atomic<int> done{kPending};
  void reset() {
    out = nullptr; n_out = nullptr; rc = WSR_OK; err.clear();
    done.store(kPending, std::memory_order_relaxed);
  }
  void fail_with(int code) {
    rc = code;
    if (code != WSR_OK) err = wsr_last_error();
  }
  void signal() {
    if (done.exchange(kDone, std::memory_order_acq_rel) == kSleeping)
      syscall(SYS_futex, reinterpret_cast<int*>(&done), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
  }
  void wait() {
    const auto spin_until = Clock::now() + std::chrono::microseconds(10);
    while (done.load(std::memory_order_acquire) != kDone && Clock::now() < spin_until) {}
    int v = kPending;
    while (done.load(std::memory_order_acquire) != kDone) {
      if (v == kPending && !done.compare_exchange_strong(v, kSleeping, std::memory_order_acq_rel)) {
        if (v == kDone) break;
      }
      syscall(SYS_futex, reinterpret_cast<int*>(&done), FUTEX_WAIT_PRIVATE, kSleeping, nullptr, nullptr, 0);
      v = kSleeping;
    }
  }
};
static_assert(sizeof(std::atomic<int>) == sizeof(int), "futex word");

// One submitted query in the ring: the query itself (so the dispatcher copies
// a batch from consecutive entries instead of chasing every caller's stack),
// its caller's request, its submit time; seq = index + 1 once it is published.
struct alignas(64) Entry {
  wsr_query q;
  Req* r;
  int64_t t_enq;   // steady-clock ns
  std::atomic<uint64_t> seq{0};
};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

struct Slot {
  wsr_batch* b = nullptr;
  std::vector<Req*> reqs;
  std::atomic<bool> busy{false};
  uint64_t seq = 0;   // launch order
  int64_t t_launch = 0;
  int32_t kmax = 1;   // the largest k of its queries (result columns to copy)
};

// What the dispatcher sleeps for (wsr_server::sleeping): a waker clears it
// with one compare-exchange, so one thread makes the futex call.
constexpr int kAwake = 0, kWantWork = 1, kWantFull = 2, kWantSlot = 3;

}  // namespace

struct wsr_server {
  // batches in flight at once: the dispatcher fills and launches, a completer
  // thread retires them in launch order, so launching never waits for a
  // result hand-off
  static constexpr int kSlots = 4;
  static constexpr uint64_t kRing = 1u << 16;   // submitted, not yet batched queries
  wsr_handle* h = nullptr;
  int max_batch = 4096;
  int depth = 2;                     // batches in flight below which one launches at once
  int64_t window_ns = 200000;
  // submission ring (multi-producer, one consumer): a caller claims index
  // tail++, fills entry index % kRing and publishes it; the dispatcher takes
  // published entries in index order and advances `consumed`.  No lock on the
  // submit path: one fetch-add, and a futex wake only when the dispatcher
  // sleeps waiting for exactly what this submit brings.
  std::unique_ptr<Entry[]> ring;
  alignas(64) std::atomic<uint64_t> tail{0};
  alignas(64) std::atomic<uint64_t> consumed{0};
  alignas(64) std::atomic<uint32_t> wake_word{0};   // futex word: bumped to wake the dispatcher
  std::atomic<int> sleeping{kAwake};
  alignas(64) std::atomic<int> n_busy{0};
  std::atomic<bool> stop{false};
  // Close sets kStopBit in `tail` with one atomic OR: a submit whose claim
  // (its fetch-add on tail) returns the bit fails; every claim before it is
  // counted in the low bits, and the dispatcher ends only once it has taken
  // all of them (waiting for any still being written), so no request is left
  // in the ring at close.  The submit path keeps a single read-modify-write
  // (round 4's separate in-flight counter cost two more on a line that every
  // client thread writes: serving fell from ~5 to ~3 M q/s).
  static constexpr uint64_t kStopBit = 1ull << 62;
  std::atomic<uint64_t> stop_at{0};   // the claims before the bit (set with stop)
  std::thread worker, completer;
  Slot slots[kSlots];
  std::mutex fmu;                    // the launched batches, oldest first
  std::condition_variable cv_done;
  std::deque<Slot*> inflight;
  bool fstop = false;
  // fetch buffers of one batch (completer only), page-locked so the result
  // copies are DMA'd
  wsr_hit* hits = nullptr;
  int32_t* nh = nullptr;
  std::vector<wsr_query> qbuf;       // dispatcher only
  std::atomic<uint64_t> batches{0}, queries{0};
  // latency breakdown (ns): submit -> launch summed over queries; launch ->
  // end event seen and end event -> last signal summed over batches
  std::atomic<uint64_t> queue_ns{0}, gpu_ns{0}, handoff_ns{0};

  void wake(int reason_mask) {
    int s = sleeping.load(std::memory_order_seq_cst);
    if (s != kAwake && ((1 << s) & reason_mask) && sleeping.compare_exchange_strong(s, kAwake)) {
      wake_word.fetch_add(1, std::memory_order_seq_cst);
      syscall(SYS_futex, reinterpret_cast<uint32_t*>(&wake_word), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    }
  }

  // Sleep for `why` unless the state the decision was made on (ww: the wake
  // word read before it, tail_seen / busy_seen) changed meanwhile.  With the
  // flag set first (seq_cst) a submitter / the completer either sees it and
  // wakes us, or made its change before our re-check below.
  void doze(int why, uint32_t ww, uint64_t tail_seen, int busy_seen, int64_t timeout_ns) {
    sleeping.store(why, std::memory_order_seq_cst);
    if ((tail.load(std::memory_order_seq_cst) & ~kStopBit) != tail_seen ||
        n_busy.load(std::memory_order_seq_cst) != busy_seen ||
        stop.load(std::memory_order_seq_cst)) {
      sleeping.store(kAwake);
      return;
    }
    timespec ts{}, *tp = nullptr;
    if (timeout_ns >= 0) {
      ts.tv_sec = timeout_ns / 1000000000;
      ts.tv_nsec = timeout_ns % 1000000000;
      tp = &ts;
    }
    syscall(SYS_futex, reinterpret_cast<uint32_t*>(&wake_word), FUTEX_WAIT_PRIVATE, ww, tp, nullptr, 0);
    sleeping.store(kAwake);
  }

  void complete(Slot& s) {
    // poll the batch's end event, so the fetch below finds it done (a blocking
    // wait inside the fetch can sleep through the batch's end and wake late);
    // a HIP error ends the poll too, and the fetch reports it.  Yield for the
    // first millisecond (batches take 0.1-1 ms: a timed sleep would add the
    // kernel's timer slack, ~50 us, to every hand-off), then back off to short
    // sleeps, so that a long batch does not keep a host core busy.
    const auto spin_until = Clock::now() + std::chrono::microseconds(1000);
    while (wsr_batch_ready(h, s.b) == 0) {
      if (Clock::now() < spin_until) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    const int64_t t_ready = now_ns();
    int rc = wsr_batch_fetch_cols(h, s.b, hits, nh, s.kmax);
    for (size_t i = 0; i < s.reqs.size(); ++i) {
      Req* r = s.reqs[i];
      r->fail_with(rc);
      if (rc == WSR_OK) {
        const int32_t n = nh[i];
        std::memcpy(r->out, &hits[i * static_cast<size_t>(s.kmax)], sizeof(wsr_hit) * static_cast<size_t>(n));
        *r->n_out = n;
      }
      r->signal();
    }
    s.reqs.clear();
    const int64_t t_done = now_ns();
    gpu_ns += static_cast<uint64_t>(t_ready - s.t_launch);
    handoff_ns += static_cast<uint64_t>(t_done - t_ready);
  }

  // a slot's batch is over: free it and wake a dispatcher that waits for one
  void release(Slot& s) {
    s.busy.store(false, std::memory_order_release);
    n_busy.fetch_sub(1, std::memory_order_seq_cst);
    wake((1 << kWantSlot) | (1 << kWantFull));
  }

  // Completer: retires launched batches in order and frees their slots.
  void retire() {
    for (;;) {
      Slot* s = nullptr;
      {
        std::unique_lock<std::mutex> lk(fmu);
        cv_done.wait(lk, [&] { return !inflight.empty() || fstop; });
        if (inflight.empty()) return;
        s = inflight.front();
        inflight.pop_front();
      }
      complete(*s);
      release(*s);
    }
  }

  // Dispatch policy: with fewer than `depth` batches in flight, whatever is
  // queued runs at once (a lone query waits for one batch; under load the GPU
  // always has the next batch queued behind the running one, and a batch
  // holds what arrived while the one before it ran, so its size follows the
  // load); with more in flight, the next one fills until max_batch or until
  // its oldest request has waited `window`; with every slot in flight, it
  // waits for the completer.
  void run() {
    uint64_t next = 0, seq = 0;
    const uint64_t mask = kRing - 1;
    std::vector<Req*> take;
    for (;;) {
      const uint32_t ww = wake_word.load(std::memory_order_seq_cst);
      const uint64_t t_raw = tail.load(std::memory_order_seq_cst);
      uint64_t t = t_raw & ~kStopBit;   // claims (the bit: closing, no more of them)
      if (t_raw & kStopBit) {   // (claims after the bit failed: only those before it count)
        if (!stop.load(std::memory_order_seq_cst)) {
          std::this_thread::yield();
          continue;
        }
        t = stop_at.load(std::memory_order_seq_cst);
      }
      const uint64_t queued = t - next;
      const int busy = n_busy.load(std::memory_order_seq_cst);
      if (queued == 0) {
        if (t_raw & kStopBit) break;   // every claim was taken and launched
        doze(kWantWork, ww, t, busy, -1);
        continue;
      }
      if (busy >= kSlots) {
        doze(kWantSlot, ww, t, busy, -1);
        continue;
      }
      Entry& head = ring[next & mask];
      if (head.seq.load(std::memory_order_acquire) != next + 1) {   // claimed, not yet written
        std::this_thread::yield();
        continue;
      }
      if (busy >= depth && !stop.load() && queued < static_cast<uint64_t>(max_batch)) {
        const int64_t left = head.t_enq + window_ns - now_ns();
        if (left > 0) {
          doze(kWantFull, ww, t, busy, left);
          continue;
        }
      }
      // the published prefix, at most max_batch
      const int64_t t_launch = now_ns();
      uint64_t wait_ns = 0;
      take.clear();
      qbuf.clear();
      const uint64_t lim = std::min<uint64_t>(queued, static_cast<uint64_t>(max_batch));
      for (uint64_t i = 0; i < lim; ++i) {
        Entry& e = ring[(next + i) & mask];
        if (e.seq.load(std::memory_order_acquire) != next + i + 1) break;
        qbuf.push_back(e.q);
        take.push_back(e.r);
        wait_ns += static_cast<uint64_t>(t_launch - e.t_enq);
      }
      next += take.size();
      consumed.store(next, std::memory_order_release);
      queue_ns += wait_ns;
      Slot* slot = nullptr;
      for (auto& sl : slots)
        if (!sl.busy.load(std::memory_order_acquire)) { slot = &sl; break; }
      slot->busy.store(true, std::memory_order_relaxed);
      n_busy.fetch_add(1, std::memory_order_seq_cst);
      Slot& s = *slot;
      s.t_launch = t_launch;
      s.kmax = 1;
      for (const wsr_query& q : qbuf) s.kmax = std::max(s.kmax, q.k);
      int rc = wsr_batch_upload(h, s.b, qbuf.data(), static_cast<int32_t>(qbuf.size()));
      if (rc == WSR_OK) rc = wsr_batch_run(h, s.b);
      if (rc != WSR_OK) {
        // every request was checked at submit, so this is not one caller's bad
        // query: the batch is retried one request at a time, and only the
        // requests that fail on their own get an error
        for (size_t i = 0; i < take.size(); ++i) {
          Req* r = take[i];
          r->fail_with(wsr_search_batch(h, &qbuf[i], 1, std::max(1, qbuf[i].k), r->out, r->n_out));
          r->signal();
        }
        release(s);
        continue;
      }
      s.reqs.swap(take);
      s.seq = ++seq;
      ++batches;
      queries += s.reqs.size();
      {
        std::lock_guard<std::mutex> g(fmu);
        inflight.push_back(&s);
      }
      cv_done.notify_one();
    }
    {
      std::lock_guard<std::mutex> g(fmu);
      fstop = true;   // the completer drains what is in flight, then ends
    }
    cv_done.notify_one();
  }

  int submit(const wsr_query& q, Req* r) {
    // a bad request fails alone, here, and never joins a batch
    // (wsr_batch_upload rejects a whole batch for one bad query)
    const int qrc = wsr_check_query(h, &q);
    if (qrc != WSR_OK) return qrc;
    if (q.k > WSR_SERVER_MAX_K) return WSR_E_LIMIT;   // the slots' result columns
    if (stop.load(std::memory_order_relaxed)) return WSR_E_INVALID;   // (fast path; the bit decides)
    const uint64_t i = tail.fetch_add(1, std::memory_order_seq_cst);
    if (i & kStopBit) return WSR_E_INVALID;
    while (i - consumed.load(std::memory_order_acquire) >= kRing) std::this_thread::yield();   // (ring full)
    Entry& e = ring[i & (kRing - 1)];
    e.q = q;
    e.r = r;
    e.t_enq = now_ns();
    e.seq.store(i + 1, std::memory_order_seq_cst);
    // wake a dispatcher asleep for work, or for a full batch when this one fills it
    const int s = sleeping.load(std::memory_order_seq_cst);
    if (s == kWantWork || (s == kWantFull && i + 1 - consumed.load(std::memory_order_relaxed) >=
                                                static_cast<uint64_t>(max_batch)))
      wake((1 << kWantWork) | (1 << kWantFull));
    return WSR_OK;
  }

  // a short spin (results of a batch arrive together), then sleep on the
  // request's own flag: spinning callers would take the dispatcher's cores
  int wait(Req* r) {
    r->wait();
    return r->rc;
  }
};

extern "C" {

int wsr_server_open(wsr_handle* h, int32_t max_batch, int32_t window_us, wsr_server** out) {
  if (!h || !out || max_batch < 1 || window_us < 0) return WSR_E_INVALID;
  std::unique_ptr<wsr_server> s(new wsr_server());
  s->h = h;
  s->max_batch = max_batch;
  s->window_ns = static_cast<int64_t>(window_us) * 1000;
  s->ring.reset(new Entry[wsr_server::kRing]);
  if (const char* e = std::getenv("WSR_SERVER_DEPTH")) s->depth = std::max(1, std::min(wsr_server::kSlots, std::atoi(e)));
  int item_blocks = 63;
  if (const char* e = std::getenv("WSR_SERVER_ITEM_BLOCKS")) item_blocks = std::max(1, std::min(63, std::atoi(e)));
  for (auto& sl : s->slots) {
    int rc = wsr_batch_create(h, max_batch, WSR_SERVER_MAX_K, &sl.b);
    // shorter work items: a batch's latency is its longest item's, and the
    // server's batches are latency-bound (WSR_SERVER_ITEM_BLOCKS)
    if (rc == WSR_OK) rc = wsr_batch_set_item_blocks(h, sl.b, item_blocks);
    if (rc != WSR_OK) {
      for (auto& x : s->slots)
        if (x.b) wsr_batch_destroy(h, x.b);
      return rc;
    }
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&s->hits),
                    sizeof(wsr_hit) * static_cast<size_t>(max_batch) * WSR_SERVER_MAX_K) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&s->nh), sizeof(int32_t) * static_cast<size_t>(max_batch)) !=
          hipSuccess) {
    for (auto& x : s->slots) wsr_batch_destroy(h, x.b);
    if (s->hits) (void)hipHostFree(s->hits);
    return WSR_E_HIP;
  }
  s->worker = std::thread([p = s.get()] { p->run(); });
  s->completer = std::thread([p = s.get()] { p->retire(); });
  *out = s.release();
  return WSR_OK;
}

void wsr_server_close(wsr_server* s) {
  if (!s) return;
  const uint64_t prev = s->tail.fetch_or(wsr_server::kStopBit, std::memory_order_seq_cst);
  s->stop_at.store(prev & ~wsr_server::kStopBit, std::memory_order_seq_cst);
  s->stop.store(true, std::memory_order_seq_cst);
  s->wake((1 << kWantWork) | (1 << kWantFull) | (1 << kWantSlot));
  if (s->worker.joinable()) s->worker.join();         // launches what is queued, then stops the completer
  if (s->completer.joinable()) s->completer.join();   // retires what is in flight
  for (auto& sl : s->slots)
    if (sl.b) wsr_batch_destroy(s->h, sl.b);
  if (s->hits) (void)hipHostFree(s->hits);
  if (s->nh) (void)hipHostFree(s->nh);
  delete s;
}

int wsr_server_search(wsr_server* s, const wsr_query* q, wsr_hit* hits, int32_t* n_hits) {
  if (!s || !q || !hits || !n_hits) return WSR_E_INVALID;
  Req r;
  r.out = hits;
  r.n_out = n_hits;
  int rc = s->submit(*q, &r);
  if (rc != WSR_OK) return rc;
  rc = s->wait(&r);
  if (rc != WSR_OK) wiser::set_last_error(r.err);   // (it failed on the dispatcher's or completer's thread)
  return rc;
}

int wsr_server_bench(wsr_server* s, const wsr_query* q, int32_t nq, int32_t n_clients,
                     int32_t depth, double seconds, wsr_serve_stats* st) {
  if (!s || !q || nq < 1 || n_clients < 1 || depth < 1 || !st) return WSR_E_INVALID;
  std::atomic<int> first_rc{WSR_OK};
  std::vector<std::vector<float>> lat(static_cast<size_t>(n_clients));
  std::vector<uint64_t> done_per(static_cast<size_t>(n_clients), 0);
  const uint64_t b0 = s->batches.load(), q0 = s->queries.load();
  const uint64_t w0 = s->queue_ns.load(), g0 = s->gpu_ns.load(), h0 = s->handoff_ns.load();
  const auto t_start = Clock::now();
  const auto t_end = t_start + std::chrono::duration_cast<Clock::duration>(
                                   std::chrono::duration<double>(seconds));
  auto client = [&](int c) {
    std::vector<Req> rq(static_cast<size_t>(depth));
    std::vector<std::vector<wsr_hit>> out(static_cast<size_t>(depth), std::vector<wsr_hit>(WSR_SERVER_MAX_K));
    std::vector<int32_t> nout(static_cast<size_t>(depth));
    std::vector<Clock::time_point> t0(static_cast<size_t>(depth));
    uint64_t next_q = static_cast<uint64_t>(c) * 7919u;
    uint64_t& done = done_per[static_cast<size_t>(c)];
    auto issue = [&](int i) {
      Req& r = rq[static_cast<size_t>(i)];
      r.reset();
      r.out = out[static_cast<size_t>(i)].data();
      r.n_out = &nout[static_cast<size_t>(i)];
      t0[static_cast<size_t>(i)] = Clock::now();
      const int rc = s->submit(q[next_q++ % static_cast<uint64_t>(nq)], &r);
      if (rc != WSR_OK) { r.rc = rc; r.done.store(kDone); }
    };
    for (int i = 0; i < depth; ++i) issue(i);
    for (uint64_t it = 0;; ++it) {
      const int i = static_cast<int>(it % static_cast<uint64_t>(depth));
      const int rc = s->wait(&rq[static_cast<size_t>(i)]);
      const auto now = Clock::now();
      if (rc != WSR_OK) { int z = WSR_OK; first_rc.compare_exchange_strong(z, rc); }
      lat[static_cast<size_t>(c)].push_back(
          std::chrono::duration<float, std::milli>(now - t0[static_cast<size_t>(i)]).count());
      ++done;
      if (now < t_end) issue(i);
      else {   // drain the rest of this client's window
        for (int j = 1; j < depth; ++j) {
          const int k = static_cast<int>((it + static_cast<uint64_t>(j)) % static_cast<uint64_t>(depth));
          s->wait(&rq[static_cast<size_t>(k)]);
          lat[static_cast<size_t>(c)].push_back(std::chrono::duration<float, std::milli>(
              Clock::now() - t0[static_cast<size_t>(k)]).count());
          ++done;
        }
        break;
      }
    }
  };
  std::vector<std::thread> ts;
  for (int c = 0; c < n_clients; ++c) ts.emplace_back(client, c);
  for (auto& t : ts) t.join();
  const double el = std::chrono::duration<double>(Clock::now() - t_start).count();
  uint64_t n_done = 0;
  for (uint64_t d : done_per) n_done += d;
  std::vector<float> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) {
    if (all.empty()) return 0.0;
    size_t i = static_cast<size_t>(p * static_cast<double>(all.size() - 1) + 0.5);
    return static_cast<double>(all[std::min(i, all.size() - 1)]);
  };
  st->queries = n_done;
  st->seconds = el;
  st->qps = static_cast<double>(n_done) / el;
  st->p50_ms = pct(0.50);
  st->p99_ms = pct(0.99);
  st->batches = s->batches.load() - b0;
  const uint64_t nq_run = s->queries.load() - q0;
  st->mean_batch = st->batches ? static_cast<double>(nq_run) / st->batches : 0.0;
  st->queue_ms = nq_run ? static_cast<double>(s->queue_ns.load() - w0) * 1e-6 / nq_run : 0.0;
  st->gpu_ms = st->batches ? static_cast<double>(s->gpu_ns.load() - g0) * 1e-6 / st->batches : 0.0;
  st->handoff_ms = st->batches ? static_cast<double>(s->handoff_ns.load() - h0) * 1e-6 / st->batches : 0.0;
  return first_rc.load();
}

}  // extern "C"
