// spg — a small persistent host worker pool for the prover's sequential-protocol work.
// Between two Fiat-Shamir challenges the prover computes a handful of independent fixed-base
// commitments and point encodings (tens of microseconds each); running them on several host cores
// shortens every sumcheck round. Bursts come every few tens of microseconds inside a proof, so a worker
// spins on the burst generation for a while (SPG_POOL_SPIN_US, default 20 ms) before it parks on the
// condition variable: a futex wake-up costs 10-30 us per burst, a spinning worker picks the burst up at once.
//
// Task indices are claimed with a CAS on one 64-bit word next_ = (burst generation, next index). A worker
// snapshots (generation, function, count) without a lock, so the caller publishes a burst in this order
// (all seq_cst): next_ = (g, CLOSED) -> fn_, n_, remaining_ -> next_ = (g, 0) -> gen_pub_ = g. Then
//  * a worker whose snapshot mixes generation G with the function/count of a newer burst G' read fn_ after
//    next_ was tagged G' (closed), so every later load of next_ carries a tag >= G' and its claim fails;
//  * a worker that read gen_pub_ = g reads fn_ / n_ of burst g or newer (never older);
//  * a successful claim (CAS on a (g, i < n_g) value) means burst g is still open, so its function is alive
//    and remaining_ still counts it: the caller returns only after every claimed task has finished.
// tests/test_product_host.py::test_pool_bursts runs bursts of varying size with a worker delayed between its
// snapshot loads (spgh_pool_stress) and checks that every task runs exactly once before parallel_for returns.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

namespace spg {

// CPUs the pool should live on (set by spg_init from the GPU's NUMA-local CPU list when SPG_PIN=1): the caller
// thread and the workers then share one CCD's L3, so a burst's hand-offs stay on-die instead of crossing sockets.
inline std::vector<int>& pool_cpus() {
  static std::vector<int> v;
  return v;
}
inline void pin_thread(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

// Scoped placement of the calling thread on the pool's CPUs for the duration of one prover call; the caller's
// own mask is restored on return, so the library never changes the affinity that threads or processes a host
// application creates later inherit (only the pool workers stay pinned).
struct HostPin {
  cpu_set_t saved;
  bool on = false;
  HostPin() {
    const std::vector<int>& c = pool_cpus();
    if (c.empty() || pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) != 0) return;
    pin_thread(c);
    on = true;
  }
  ~HostPin() {
    if (on) pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
  }
  HostPin(const HostPin&) = delete;
  HostPin& operator=(const HostPin&) = delete;
};

// CPUs this process may use: its affinity mask, capped by the cgroup v2 CPU quota (cpu.max), divided among the
// LOCAL_WORLD_SIZE processes of a node that share them (torchrun sets it; one process per GPU)
inline int usable_cpus() {
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[64] = {0};
    long period = 0;
    if (fscanf(f, "%63s %ld", q, &period) == 2 && period > 0 && q[0] != 'm') {
      const long quota = atol(q);
      if (quota > 0) n = std::min(n, (int)std::max(1L, (quota + period - 1) / period));
    }
    fclose(f);
  }
  const char* lws = getenv("LOCAL_WORLD_SIZE");
  if (lws && atoi(lws) > 1) n = std::max(1, n / atoi(lws));
  return n < 1 ? 1 : n;
}

class Pool {
 public:
  // test hooks: a worker sleeps snapshot_delay_us between its generation and function loads, the caller
  // sleeps publish_delay_us between storing a burst's function/count and opening it
  explicit Pool(int nthreads, int snapshot_delay_us = 0, int publish_delay_us = 0)
      : delay_us_(snapshot_delay_us), pub_delay_us_(publish_delay_us) {
    const char* e = getenv("SPG_POOL_SPIN_US");
    spin_ = std::chrono::microseconds(e ? atoi(e) : 20000);
    const std::vector<int> cpus = pool_cpus();
    for (int i = 0; i < nthreads; i++)
      threads_.emplace_back([this, cpus, i] {
        if (!cpus.empty()) pin_thread({cpus[(size_t)(i + 1) % cpus.size()]});
        worker();
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      quit_pub_.store(true);
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int size() const { return (int)threads_.size(); }  // workers besides the calling thread
  uint64_t bursts() const { return bursts_; }         // bursts so far (SPG_TRACE=2 counter)
  // runs f(0) .. f(n-1) on the pool and the calling thread; returns when all are done
  void parallel_for(int n, const std::function<void(int)>& f) {
    if (n <= 1 || threads_.empty()) {
      for (int i = 0; i < n; i++) f(i);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);  // one burst at a time
    uint32_t g;
    bool wake;
    g = ++gen_;
    bursts_++;
    next_.store(((uint64_t)g << 32) | kClosed);  // tag first: stale snapshots can no longer claim
    fn_.store(&f);
    n_.store(n);
    remaining_.store(n);
    if (pub_delay_us_) std::this_thread::sleep_for(std::chrono::microseconds(pub_delay_us_));
    next_.store((uint64_t)g << 32);  // open
    gen_pub_.store(g);  // seq_cst: pairs with a parking worker's sleepers_ increment (no lost wake-up)
    wake = sleepers_.load() > 0;
    if (wake) {
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_all();
    }
    work(g, &f, n);
    // the workers finish within microseconds: spin (a yield is a system call that may still be running when the
    // last task ends), yielding only after ~50k polls
    for (unsigned k = 0; remaining_.load() > 0; k++) {
      if (k < 50000) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      } else {
        std::this_thread::yield();
      }
    }
  }

 private:
  // claims and runs tasks of burst g until none is left; the tasks this thread ran leave remaining_ in one step at the
  // end (one contended update per thread and burst, not per task)
  void work(uint32_t g, const std::function<void(int)>* f, int n) {
    int ran = 0;
    for (;;) {
      uint64_t v = next_.load();
      if ((uint32_t)(v >> 32) != g || (uint32_t)v >= (uint32_t)n) break;  // kClosed >= any n
      if (!next_.compare_exchange_weak(v, v + 1)) continue;
      (*f)((int)(uint32_t)v);
      ran++;
    }
    if (ran) remaining_.fetch_sub(ran);
  }
  void worker() {
    uint32_t seen = 0;
    for (;;) {
      uint32_t g;
      const std::function<void(int)>* f;
      int n;
      // spin phase: pick up the next burst without a futex wake-up
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned k = 0; gen_pub_.load(std::memory_order_acquire) == seen && !quit_pub_.load(); k++) {
        if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > spin_) break;
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
      if (gen_pub_.load() == seen) {  // park until the next burst
        std::unique_lock<std::mutex> lk(mu_);
        sleepers_++;
        cv_.wait(lk, [&] { return quit_pub_.load() || gen_pub_.load() != seen; });
        sleepers_--;
      }
      if (quit_pub_.load()) return;
      // lock-free snapshot: f and n are at least as new as g; if a newer burst already replaced them, next_
      // was tagged with that newer generation before fn_ changed, so work() returns at once (header comment)
      seen = g = gen_pub_.load();
      if (delay_us_) std::this_thread::sleep_for(std::chrono::microseconds(delay_us_));
      f = fn_.load();
      n = n_.load();
      work(g, f, n);
    }
  }
  static constexpr uint32_t kClosed = 0xffffffffu;
  int delay_us_ = 0, pub_delay_us_ = 0;
  std::vector<std::thread> threads_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_;
  // the words every burst moves between cores, one cache line each: spinning workers poll gen_pub_, and the claims
  // (next_) and completions (remaining_) of a burst would otherwise invalidate the line they poll on every task
  alignas(64) std::atomic<const std::function<void(int)>*> fn_{nullptr};
  std::atomic<int> n_{0};
  uint32_t gen_ = 0;  // written by the (serialised) caller only
  uint64_t bursts_ = 0;
  alignas(64) std::atomic<uint64_t> next_{0};
  alignas(64) std::atomic<int> remaining_{0};
  alignas(64) std::atomic<uint32_t> gen_pub_{0};
  std::atomic<bool> quit_pub_{false};
  alignas(64) bool quit_ = false;
  std::atomic<int> sleepers_{0};
  std::chrono::microseconds spin_{20000};
};

// workers besides the calling thread
inline int pool_threads() {
  const char* e = getenv("SPG_POOL_THREADS");
  if (e) return atoi(e);
  // at most 7 workers + the caller: measured best on the GPU box (16-CPU quota per process; 15 workers were
  // 2-5 ms slower per SNARK::prove, scripts/pool_sweep.sh), and it leaves room for HIP's own threads; fewer
  // when the process' share of CPUs (usable_cpus) is smaller, so co-located provers do not oversubscribe
  const int n = usable_cpus() - 1;
  return n < 0 ? 0 : (n > 7 ? 7 : n);
}
inline Pool& pool() {
  static Pool p(pool_threads());
  return p;
}

}  // namespace spg
