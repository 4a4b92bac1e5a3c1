// HostParallel.h — a fork/join loop for the host halves of the path whose items are
// independent: per-source SpfResult materialisation (LinkState::runSpfBatch) and per-node
// route builds (SpfSolver::buildRouteDbs). The reference does both on its one Decision
// thread (Decision.cpp:568 buildRouteDb per rebuild); results here are identical, only
// the wall clock changes.
//
// Threads: OPENR_HOST_THREADS (1 = sequential), default min(hardware threads, 16) — a GPU
// box's CPU share is 16 even where hardware_concurrency() reports the whole machine.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace openr {

inline unsigned hostThreads() {
  if (const char* s = std::getenv("OPENR_HOST_THREADS")) {
    const long v = std::strtol(s, nullptr, 10);
    if (v >= 1) return unsigned(std::min(v, 256L));
  }
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// f(worker, i) for i in [0, n), items handed out `grain` at a time; worker in
// [0, workers) identifies the calling thread (0 = the caller). An exception ends the
// loop early; the one thrown by the lowest item index is rethrown here, so a failing
// build reports what the sequential loop would have reported first.
template <class F>
void parallelFor(size_t n, size_t grain, unsigned workers, F&& f) {
  grain = std::max<size_t>(grain, 1);
  workers = unsigned(std::min<size_t>(std::max(workers, 1u), (n + grain - 1) / grain));
  if (workers <= 1) {
    for (size_t i = 0; i < n; ++i) f(0u, i);
    return;
  }
  std::atomic<size_t> next{0};
  std::atomic<bool> stop{false};
  std::mutex errLock;
  size_t errIndex = n;
  std::exception_ptr err;
  auto run = [&](unsigned w) {
    for (;;) {
      if (stop.load(std::memory_order_relaxed)) return;
      const size_t lo = next.fetch_add(grain);
      if (lo >= n) return;
      const size_t hi = std::min(n, lo + grain);
      for (size_t i = lo; i < hi; ++i) {
        try {
          f(w, i);
        } catch (...) {
          std::lock_guard<std::mutex> g(errLock);
          if (i < errIndex) {
            errIndex = i;
            err = std::current_exception();
          }
          stop.store(true);
          return;
        }
      }
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(workers - 1);
  for (unsigned w = 1; w < workers; ++w) pool.emplace_back(run, w);
  run(0);
  for (auto& t : pool) t.join();
  if (err) std::rethrow_exception(err);
}

// Tuning aid: OPENR_HOST_PROF=1 prints the wall time of the host phases of a route build
// (prefetch, D2H, row store, per-node builds) to stderr.
inline bool hostProf() {
  static const bool on = [] {
    const char* s = std::getenv("OPENR_HOST_PROF");
    return s && *s == '1';
  }();
  return on;
}
struct HostPhase {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit HostPhase(const char* n) : name(n) {}
  double ms() const { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
  ~HostPhase() {
    if (hostProf() && name && *name) std::fprintf(stderr, "[host] %s %.1f ms\n", name, ms());
  }
};

inline unsigned parallelWorkers(size_t n, size_t grain) {
  grain = std::max<size_t>(grain, 1);
  return unsigned(std::min<size_t>(hostThreads(), std::max<size_t>(1, (n + grain - 1) / grain)));
}

}  // namespace openr
