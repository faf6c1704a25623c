// Parallel.h — the host worker pool of one RouteDb build.
//
// The reference builds a RouteDb on the Decision thread, one prefix at a
// time (openr/decision/Decision.cpp:313-534).  Once the SPF rows a build
// reads are resident (one device batch per area, SpfSolverImpl::prefetch),
// the per-prefix / per-label / per-destination work only reads them, so it
// is spread over host threads here.  Results are merged by the caller in a
// fixed order; nothing observable depends on which thread ran which item.
#pragma once

#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace openr {

// Worker threads for `n` independent items: OPENR_SPF_HOST_THREADS, else
// min(hardware threads, 16); 1 (run inline) for small batches.
inline unsigned hostThreads(size_t n, size_t minPerThread = 64) {
  static const unsigned t = [] { // read once: called several times per build
    if (const char* env = std::getenv("OPENR_SPF_HOST_THREADS")) {
      return (unsigned)std::max(1, std::atoi(env));
    }
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  }();
  const size_t cap = std::max<size_t>(1, n / std::max<size_t>(1, minPerThread));
  return (unsigned)std::min<size_t>(t, cap);
}

// Persistent workers: a parallel section used to start and join fresh
// std::threads (~30-50 us each), which on a RouteDb build (three sections of
// up to 16 threads) and a graph rebuild (five) cost more than the work.  One
// section runs at a time; a section started while another runs (from another
// host thread) or from inside a worker falls back to fresh threads.  The pool
// is never destroyed (its detached workers park on a condition variable); a
// forked child starts a new, empty one.  OPENR_HOST_POOL=0: fresh threads.
// After a section the workers (and the caller, for the join) spin for up to
// kSpin before blocking, so back-to-back sections (a graph rebuild runs ~10)
// start without a futex wake-up each.
class HostPool {
 public:
  static HostPool& get() {
    static const bool init = [] {
      pthread_atfork(nullptr, nullptr, [] { instance() = new HostPool(); });
      instance() = new HostPool();
      return true;
    }();
    (void)init;
    return *instance();
  }

  // body(w) for w in [0, threads): w = 0 on the calling thread.  false: the
  // pool is busy (or this is a worker): the caller runs the section itself.
  bool run(unsigned threads, const std::function<void(unsigned)>& body) {
    static const bool enabled = [] {
      const char* e = std::getenv("OPENR_HOST_POOL");
      return !(e && std::atoi(e) == 0);
    }();
    if (!enabled || inWorker() || threads <= 1) {
      return false; // (inWorker: also the calling thread of a running section)
    }
    std::unique_lock<std::mutex> job(jobMu_, std::try_to_lock);
    if (!job.owns_lock()) {
      return false;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      while (nworkers_ + 1 < threads) {
        const unsigned id = ++nworkers_;
        std::thread([this, id] { loop(id); }).detach();
      }
      body_ = &body;
      want_ = threads - 1;
      pending_ = threads - 1;
      ++gen_;
      awant_.store(want_, std::memory_order_relaxed);
      apending_.store(pending_, std::memory_order_relaxed);
      agen_.store(gen_, std::memory_order_release);
    }
    cv_.notify_all();
    inWorker() = true; // a nested section on this thread starts fresh threads
    body(0);
    inWorker() = false;
    spinUntil([this] { return apending_.load(std::memory_order_acquire) == 0; });
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [this] { return pending_ == 0; });
    body_ = nullptr;
    return true;
  }

 private:
  static HostPool*& instance() {
    static HostPool* p = nullptr;
    return p;
  }
  static bool& inWorker() {
    static thread_local bool w = false;
    return w;
  }
  static constexpr auto kSpin = std::chrono::microseconds(200);
  template <class Pred>
  static void spinUntil(Pred&& done) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned i = 1; !done(); ++i) {
      if ((i & 127) == 0 && std::chrono::steady_clock::now() - t0 > kSpin) {
        return;
      }
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
  }
  void loop(unsigned id) {
    inWorker() = true;
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned)>* body;
      spinUntil([&] {
        return agen_.load(std::memory_order_acquire) != seen &&
            id <= awant_.load(std::memory_order_relaxed);
      });
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return gen_ != seen && id <= want_; });
        seen = gen_;
        body = body_;
      }
      (*body)(id);
      {
        std::lock_guard<std::mutex> l(mu_);
        apending_.fetch_sub(1, std::memory_order_release);
        if (--pending_ == 0) {
          done_.notify_one();
        }
      }
    }
  }

  std::mutex jobMu_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  unsigned nworkers_ = 0;
  const std::function<void(unsigned)>* body_ = nullptr;
  unsigned want_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  // lock-free mirrors of gen_ / want_ / pending_ for the spins
  std::atomic<uint64_t> agen_{0};
  std::atomic<unsigned> awant_{0}, apending_{0};
};

// fn(item, worker) for item in [0, n), chunks handed out dynamically.  The
// first exception (by worker index) is rethrown after every worker joined.
template <class Fn>
void parallelFor(size_t n, unsigned threads, Fn&& fn, size_t chunk = 16) {
  if (threads <= 1 || n <= chunk) {
    for (size_t i = 0; i < n; ++i) {
      fn(i, 0u);
    }
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> errors(threads);
  auto body = [&](unsigned w) {
    try {
      for (;;) {
        const size_t b = next.fetch_add(chunk);
        if (b >= n) {
          break;
        }
        const size_t e = std::min(n, b + chunk);
        for (size_t i = b; i < e; ++i) {
          fn(i, w);
        }
      }
    } catch (...) {
      errors[w] = std::current_exception();
      next.store(n); // stop handing out work
    }
  };
  const std::function<void(unsigned)> job(body);
  if (!HostPool::get().run(threads, job)) {
    std::vector<std::thread> pool;
    pool.reserve(threads - 1);
    for (unsigned w = 1; w < threads; ++w) {
      pool.emplace_back(body, w);
    }
    body(0);
    for (auto& t : pool) {
      t.join();
    }
  }
  for (auto& e : errors) {
    if (e) {
      std::rethrow_exception(e);
    }
  }
}

// Route shards of a RouteDb build.  A route is built, and later freed
// (releaseRouteDb), by the one worker that takes its shard, so the frees of
// a shard land in the malloc arena its builder allocated from instead of
// every releasing thread taking every arena's lock (fabric 2-0-0, ~20k routes
// x ~40 next hops: release 67 ms on dynamically scheduled buckets).  The
// build records its shard counts in the RouteDb and the release reuses them.
inline unsigned routeShards(size_t routes) { return hostThreads(routes, 64); }

// fn(shard) for every shard in [0, shards): shard s runs on pool worker s
// (s = 0: the calling thread) in every section, not on whichever worker
// claims it first, so releaseRouteDb frees each shard's routes on the very
// thread (and malloc arena / tcache) that built them (round 6; with dynamic
// claiming most frees crossed threads).  OPENR_SHARD_DYNAMIC=1: the old
// dynamic hand-out.  The first exception (by shard) is rethrown after every
// shard ran.
template <class Fn>
void parallelShards(unsigned shards, Fn&& fn) {
  static const bool dynamic = [] {
    const char* e = std::getenv("OPENR_SHARD_DYNAMIC");
    return e && std::atoi(e) != 0;
  }();
  if (dynamic) {
    parallelFor(shards, shards, [&](size_t s, unsigned) { fn((unsigned)s); }, 1);
    return;
  }
  if (shards <= 1) {
    for (unsigned s = 0; s < shards; ++s) {
      fn(s);
    }
    return;
  }
  std::vector<std::exception_ptr> errors(shards);
  auto body = [&](unsigned w) {
    try {
      fn(w);
    } catch (...) {
      errors[w] = std::current_exception();
    }
  };
  const std::function<void(unsigned)> job(body);
  if (!HostPool::get().run(shards, job)) {
    std::vector<std::thread> pool;
    pool.reserve(shards - 1);
    for (unsigned w = 1; w < shards; ++w) {
      pool.emplace_back(body, w);
    }
    body(0);
    for (auto& t : pool) {
      t.join();
    }
  }
  for (auto& e : errors) {
    if (e) {
      std::rethrow_exception(e);
    }
  }
}

} // namespace openr
