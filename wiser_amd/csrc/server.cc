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
  wsr_query q;
  Clock::time_point t_enq;
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

struct Slot {
  wsr_batch* b = nullptr;
  std::vector<Req*> reqs;
  bool busy = false;
  uint64_t seq = 0;   // launch order
  Clock::time_point t_launch;
  int32_t kmax = 1;   // the largest k of its queries (result columns to copy)
};

}  // namespace

struct wsr_server {
  // batches in flight at once: the dispatcher fills and launches, a completer
  // thread retires them in launch order, so launching never waits for a
  // result hand-off
  static constexpr int kSlots = 4;
  wsr_handle* h = nullptr;
  int max_batch = 4096;
  int depth = 2;                     // batches in flight below which one launches at once
  std::chrono::microseconds window{200};
  std::mutex mu;                     // queue, slot states, stop, idle
  std::condition_variable cv_work;   // dispatcher: requests arrived / a slot freed / stop
  std::deque<Req*> queue;
  bool stop = false;
  bool idle = false;                 // dispatcher asleep on cv_work with nothing to launch
  int n_busy = 0;
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

  void complete(Slot& s) {
    // poll the batch's end event, so the fetch below finds it done (a blocking
    // wait inside the fetch can sleep through the batch's end and wake late);
    // a HIP error ends the poll too, and the fetch reports it.  Yield for the
    // first 100 us, then back off to short sleeps, so that a long batch does
    // not keep a host core busy beside the clients and the dispatcher.
    const auto spin_until = Clock::now() + std::chrono::microseconds(100);
    while (wsr_batch_ready(h, s.b) == 0) {
      if (Clock::now() < spin_until) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    const auto t_ready = Clock::now();
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
    const auto t_done = Clock::now();
    gpu_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(t_ready - s.t_launch).count());
    handoff_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(t_done - t_ready).count());
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
      bool wake;
      {
        std::lock_guard<std::mutex> g(mu);
        s->busy = false;
        --n_busy;
        wake = idle;
      }
      if (wake) cv_work.notify_one();
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
    uint64_t seq = 0;
    for (;;) {
      std::vector<Req*> take;
      Slot* slot = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          if (queue.empty() && stop) break;
          if (!queue.empty() && n_busy < kSlots) {
            if (n_busy >= depth && !stop && static_cast<int>(queue.size()) < max_batch) {
              const auto due = queue.front()->t_enq + window;
              if (Clock::now() < due) {   // (submit wakes us early when the batch fills)
                idle = true;
                cv_work.wait_until(lk, due);
                idle = false;
                continue;
              }
            }
            break;
          }
          idle = true;
          cv_work.wait(lk);
          idle = false;
        }
        if (queue.empty()) break;   // stop, and everything was launched
        const size_t n = std::min<size_t>(queue.size(), static_cast<size_t>(max_batch));
        take.assign(queue.begin(), queue.begin() + static_cast<long>(n));
        queue.erase(queue.begin(), queue.begin() + static_cast<long>(n));
        for (auto& sl : slots)
          if (!sl.busy) { slot = &sl; break; }
        slot->busy = true;
        ++n_busy;
      }
      Slot& s = *slot;
      s.t_launch = Clock::now();
      {
        uint64_t w = 0;
        for (Req* r : take)
          w += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(s.t_launch - r->t_enq).count());
        queue_ns += w;
      }
      qbuf.resize(take.size());
      s.kmax = 1;
      for (size_t i = 0; i < take.size(); ++i) {
        qbuf[i] = take[i]->q;
        s.kmax = std::max(s.kmax, qbuf[i].k);
      }
      int rc = wsr_batch_upload(h, s.b, qbuf.data(), static_cast<int32_t>(qbuf.size()));
      if (rc == WSR_OK) rc = wsr_batch_run(h, s.b);
      if (rc != WSR_OK) {
        // every request was checked at submit, so this is not one caller's bad
        // query: the batch is retried one request at a time, and only the
        // requests that fail on their own get an error
        for (Req* r : take) {
          r->fail_with(wsr_search_batch(h, &r->q, 1, std::max(1, r->q.k), r->out, r->n_out));
          r->signal();
        }
        std::lock_guard<std::mutex> g(mu);
        s.busy = false;
        --n_busy;
        continue;
      }
      s.reqs = std::move(take);
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

  int submit(Req* r) {
    // a bad request fails alone, here, and never joins a batch
    // (wsr_batch_upload rejects a whole batch for one bad query)
    const int qrc = wsr_check_query(h, &r->q);
    if (qrc != WSR_OK) return qrc;
    if (r->q.k > WSR_SERVER_MAX_K) return WSR_E_LIMIT;   // the slots' result columns
    r->t_enq = Clock::now();
    bool wake;
    {
      std::lock_guard<std::mutex> g(mu);
      if (stop) return WSR_E_INVALID;
      queue.push_back(r);
      // the dispatcher sleeps with nothing to launch, or until a window ends:
      // wake it for the first request, or when a batch is full
      wake = idle && (queue.size() == 1 || static_cast<int>(queue.size()) == max_batch);
    }
    if (wake) cv_work.notify_one();
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
  s->window = std::chrono::microseconds(window_us);
  if (const char* e = std::getenv("WSR_SERVER_DEPTH")) s->depth = std::max(1, std::min(wsr_server::kSlots, std::atoi(e)));
  for (auto& sl : s->slots) {
    int rc = wsr_batch_create(h, max_batch, WSR_SERVER_MAX_K, &sl.b);
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
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->stop = true;
  }
  s->cv_work.notify_all();
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
  r.q = *q;
  r.out = hits;
  r.n_out = n_hits;
  int rc = s->submit(&r);
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
  std::atomic<uint64_t> done{0};
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
    auto issue = [&](int i) {
      Req& r = rq[static_cast<size_t>(i)];
      r.reset();
      r.q = q[next_q++ % static_cast<uint64_t>(nq)];
      r.out = out[static_cast<size_t>(i)].data();
      r.n_out = &nout[static_cast<size_t>(i)];
      t0[static_cast<size_t>(i)] = Clock::now();
      const int rc = s->submit(&r);
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
  std::vector<float> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) {
    if (all.empty()) return 0.0;
    size_t i = static_cast<size_t>(p * static_cast<double>(all.size() - 1) + 0.5);
    return static_cast<double>(all[std::min(i, all.size() - 1)]);
  };
  st->queries = done.load();
  st->seconds = el;
  st->qps = static_cast<double>(done.load()) / el;
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
