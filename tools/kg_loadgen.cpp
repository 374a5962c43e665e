// kg_loadgen.cpp -- benchmark load generator for the request batcher (NOT part of libketogpu).
//
// Mimics `keto serve` handler goroutines behind the cgo binding: `threads`
// callers, each making blocking kg_batcher_check calls of `per_call` queries in a loop, for
// `seconds`.  Called by bench.py --mode host through ctypes (the GIL is released for the whole
// run), so the request path is measured without Python in it.  When `expect` is given, every
// answer is compared with it (mismatches are counted).
#include <atomic>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "../include/ketogpu.h"

extern "C" int kgl_batcher_load(kg_batcher* b, const kg_query* qs, size_t nq, const uint8_t* expect, int threads,
                                int per_call, double seconds, uint64_t* checks_out, double* elapsed_out,
                                uint64_t* mismatches_out) {
  if (!b || !qs || nq == 0 || threads < 1 || per_call < 1 || (size_t)per_call > nq) return -2;
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> checks{0}, bad{0};
  std::atomic<int> failed{0};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      std::vector<uint8_t> out(per_call);
      std::vector<uint32_t> err(per_call);
      size_t i = ((size_t)t * 7919) % (nq - per_call + 1);
      uint64_t mine = 0, wrong = 0;
      while (!stop.load(std::memory_order_relaxed)) {
        if (kg_batcher_check(b, qs + i, per_call, out.data(), err.data()) != 0) {
          failed = 1;
          break;
        }
        if (expect)
          for (int k = 0; k < per_call; k++) wrong += out[k] != expect[i + k];
        mine += per_call;
        i += (size_t)per_call * threads;
        if (i + per_call > nq) i = (i + 1) % (nq - per_call + 1);
      }
      checks += mine;
      bad += wrong;
    });
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop = true;
  for (auto& x : th) x.join();
  *elapsed_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *checks_out = checks;
  if (mismatches_out) *mismatches_out = bad;
  return failed ? -1 : 0;
}
