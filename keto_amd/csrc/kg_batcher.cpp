// kg_batcher.cpp -- native request batcher in front of kg_check_batch.
//
// The reference answers every Check RPC on its own goroutine, one CheckIsMember each
// (internal/check/handler.go:248-275 -> internal/check/engine.go:54-60).  Behind cgo the natural
// binding is the same shape: each handler goroutine makes ONE blocking call, kg_batcher_check,
// with its tuple.  Inside, concurrent callers' queries are appended to the open batch; a batch
// closes when it holds max_batch queries or its oldest query has waited max_wait_us, and one of
// `dispatchers` threads runs it through kg_check_batch (split over the snapshot's replicas, each
// dispatcher with its own lanes, so consecutive batches overlap on the devices).  Every caller of
// the batch is woken once its answers are in: allowed = a loop of CheckIsMember.
//
// Latency accounting: each batch records (oldest submission -> answers delivered) in a ring of
// the last 64 Ki batches, and each caller's own wait (submit -> wake-up) in a second ring; the
// percentiles of both are what BASELINE.json's "p99 batch latency" names.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "kg_snapshot.h"

namespace kg {

using Clock = std::chrono::steady_clock;

// A batch's callers sleep on its `done` word (a futex): the dispatcher wakes all of them with one
// syscall and none of them has to re-take a mutex on the way out -- with a condition variable,
// ~130 woken callers per batch queued on its mutex, and on a server whose cgroup holds 16 CPUs the
// convoy's CPU time (256 callers) ran the quota out: throttled for the rest of the period, p99 ~70 ms.
struct BBatch {
  std::vector<kg_query> q;
  std::vector<uint8_t> out;
  std::vector<uint32_t> err;
  Clock::time_point first;
  std::atomic<int> done{0};
  int rc = 0;
  void wait_done() {
    for (int spin = 0; spin < 64; spin++)
      if (done.load(std::memory_order_acquire)) return;
    while (!done.load(std::memory_order_acquire))
      syscall(SYS_futex, reinterpret_cast<int*>(&done), FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
  }
  void set_done() {
    done.store(1, std::memory_order_release);
    syscall(SYS_futex, reinterpret_cast<int*>(&done), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
  }
};
static_assert(sizeof(std::atomic<int>) == sizeof(int), "futex word");

struct LatRing {  // last 64 Ki samples (ns); writers claim slots with one atomic, no lock
  std::vector<std::atomic<uint64_t>> v = std::vector<std::atomic<uint64_t>>(1 << 16);
  std::atomic<uint64_t> n{0};
  void add(uint64_t x) { v[n.fetch_add(1, std::memory_order_relaxed) & (v.size() - 1)].store(x, std::memory_order_relaxed); }
  void reset() {
    n.store(0);
    for (auto& e : v) e.store(0, std::memory_order_relaxed);
  }
  double pct(double p) const {
    const size_t k = (size_t)std::min<uint64_t>(n.load(), v.size());
    if (!k) return 0.0;
    std::vector<uint64_t> s(k);
    for (size_t i = 0; i < k; i++) s[i] = v[i].load(std::memory_order_relaxed);
    const size_t at = std::min(k - 1, (size_t)(p / 100.0 * (double)(k - 1) + 0.5));
    std::nth_element(s.begin(), s.begin() + at, s.end());
    return (double)s[at] * 1e-6;
  }
};

struct Batcher {
  Snapshot* s = nullptr;
  int32_t gdepth = 5;
  size_t max_batch = 1 << 16;
  Clock::duration max_wait{};
  std::mutex mu;
  std::condition_variable cv;  // dispatchers wait for work here
  std::shared_ptr<BBatch> open;
  std::deque<std::shared_ptr<BBatch>> full;  // closed by size, not yet taken
  bool closing = false;
  std::vector<std::thread> th;
  std::mutex st_mu;
  LatRing batch_lat, call_lat;
  uint64_t batches = 0, checks = 0;
  // callers inside kg_batcher_check: kg_batcher_destroy frees the batcher only once every caller it
  // woke has left (a woken caller still records its latency and may loop for its next chunk)
  std::atomic<int> callers{0};

  void run();
};

struct CallerGuard {
  std::atomic<int>& c;
  explicit CallerGuard(std::atomic<int>& x) : c(x) { c.fetch_add(1, std::memory_order_acq_rel); }
  ~CallerGuard() { c.fetch_sub(1, std::memory_order_acq_rel); }
};

void Batcher::run() {
  for (;;) {
    std::shared_ptr<BBatch> b;
    {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        if (!full.empty()) {
          b = full.front();
          full.pop_front();
          break;
        }
        if (open) {
          const auto deadline = open->first + max_wait;
          if (closing || Clock::now() >= deadline) {
            b = open;
            open.reset();
            break;
          }
          cv.wait_until(lk, deadline);
          continue;
        }
        if (closing) return;
        cv.wait(lk);
      }
    }
    const size_t n = b->q.size();
    b->out.resize(n);
    b->err.resize(n);
    int rc = kg_check_batch(reinterpret_cast<kg_snapshot*>(s), b->q.data(), n, gdepth, b->out.data(), b->err.data(),
                            nullptr);
    const auto now = Clock::now();
    {
      std::lock_guard<std::mutex> lk(st_mu);
      batch_lat.add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - b->first).count());
      batches++;
      checks += n;
    }
    b->rc = rc;
    b->set_done();  // release: rc, out and err are visible to the woken callers
  }
}

}  // namespace kg

using kg::Batcher;
using kg::set_error;

extern "C" {

int kg_batcher_create(kg_snapshot* sp, int32_t global_max_depth, size_t max_batch, uint32_t max_wait_us,
                      int dispatchers, kg_batcher** out) {
  if (!sp || !out) return set_error(-2, "NULL argument");
  if (max_batch < 1 || max_batch > (1u << 26) || dispatchers < 1 || dispatchers > 16)
    return set_error(-2, "max_batch in [1, 2^26], dispatchers in [1, 16]");
  Batcher* b = new (std::nothrow) Batcher();
  if (!b) return set_error(-4, "host allocation failed");
  b->s = reinterpret_cast<kg::Snapshot*>(sp);
  b->gdepth = global_max_depth;
  b->max_batch = max_batch;
  b->max_wait = std::chrono::microseconds(max_wait_us);
  for (int i = 0; i < dispatchers; i++) b->th.emplace_back([b] { b->run(); });
  *out = reinterpret_cast<kg_batcher*>(b);
  return 0;
}

// Blocks until the n queries (one caller's burst, usually 1) are answered.  The queries may be
// split over consecutive batches when they do not fit the open one.
int kg_batcher_check(kg_batcher* bp, const kg_query* q, size_t n, uint8_t* out, uint32_t* err_code) {
  if (!bp || (n && (!q || !out))) return set_error(-2, "NULL argument");
  Batcher* b = reinterpret_cast<Batcher*>(bp);
  kg::CallerGuard guard(b->callers);  // destroy waits for it (the last thing this call touches is `b`)
  const auto t0 = kg::Clock::now();
  size_t done = 0;
  int rc = 0;
  while (done < n && !rc) {
    std::shared_ptr<kg::BBatch> mine;
    size_t pos = 0, take = 0;
    {
      std::lock_guard<std::mutex> lk(b->mu);
      if (b->closing) return set_error(-2, "batcher is closed");
      if (!b->open) {
        b->open = std::make_shared<kg::BBatch>();
        b->open->first = t0;
        b->open->q.reserve(std::min<size_t>(b->max_batch, 4096));
        b->cv.notify_one();  // a dispatcher starts the max_wait clock of the new batch
      }
      mine = b->open;
      pos = mine->q.size();
      take = std::min(n - done, b->max_batch - pos);
      mine->q.insert(mine->q.end(), q + done, q + done + take);
      if (mine->q.size() >= b->max_batch) {  // full: hand it to a dispatcher now
        b->full.push_back(mine);
        b->open.reset();
        b->cv.notify_one();
      }
    }
    mine->wait_done();
    if (mine->rc) {
      rc = set_error(mine->rc, "batch failed (%d)", mine->rc);
      break;
    }
    memcpy(out + done, mine->out.data() + pos, take);
    if (err_code) memcpy(err_code + done, mine->err.data() + pos, take * 4);
    done += take;
  }
  const uint64_t ns =
      (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(kg::Clock::now() - t0).count();
  b->call_lat.add(ns);  // lock-free: a server's callers do not queue on a stats mutex
  return rc;
}

int kg_batcher_stats(kg_batcher* bp, kg_batcher_stats_t* st) {
  if (!bp || !st) return set_error(-2, "NULL argument");
  Batcher* b = reinterpret_cast<Batcher*>(bp);
  std::lock_guard<std::mutex> lk(b->st_mu);
  st->batches = b->batches;
  st->checks = b->checks;
  st->batch_p50_ms = b->batch_lat.pct(50);
  st->batch_p99_ms = b->batch_lat.pct(99);
  st->call_p50_ms = b->call_lat.pct(50);
  st->call_p99_ms = b->call_lat.pct(99);
  return 0;
}

void kg_batcher_reset_stats(kg_batcher* bp) {
  if (!bp) return;
  Batcher* b = reinterpret_cast<Batcher*>(bp);
  std::lock_guard<std::mutex> lk(b->st_mu);
  b->batch_lat.reset();
  b->call_lat.reset();
  b->batches = b->checks = 0;
}

// Stops accepting queries, answers what is pending, joins the dispatchers, waits for every caller
// still inside kg_batcher_check to leave (callers blocked at the time get their answers, or an error
// for chunks not yet queued), then frees the batcher.  A call that STARTS after destroy returned is
// a use of a freed handle (as with any destroy).
void kg_batcher_destroy(kg_batcher* bp) {
  if (!bp) return;
  Batcher* b = reinterpret_cast<Batcher*>(bp);
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->closing = true;
  }
  b->cv.notify_all();
  for (auto& t : b->th) t.join();
  while (b->callers.load(std::memory_order_acquire) != 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
  delete b;
}

}  // extern "C"
