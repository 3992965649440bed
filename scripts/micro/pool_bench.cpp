// Burst latency of the host pool variants (scripts/micro/README.md):
//   g++ -O2 -march=x86-64-v3 -std=c++17 -pthread -I spartan-parallel_amd/csrc scripts/micro/pool_bench.cpp
//   ./a.out WORKERS VARIANT   (one pool per process: idle pools' spinning workers would share the CPUs)
// shared: hpool.hpp (one claim counter shared by all threads); static: hpool_static.inc (static shares with
// per-worker claim words, the caller stealing late shares). Bursts of n tasks of w microseconds each.
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "hpool.hpp"
#include "hpool_static.inc"

using clk = std::chrono::steady_clock;
static void busy_us(double us) {
  const auto t0 = clk::now();
  while (std::chrono::duration<double, std::micro>(clk::now() - t0).count() < us) {
  }
}
template <class P>
static double burst_us(P& p, int n, double w, int reps) {
  for (int i = 0; i < 200; i++) p.parallel_for(n, [&](int) { busy_us(w); });
  const auto t0 = clk::now();
  for (int i = 0; i < reps; i++) p.parallel_for(n, [&](int) { busy_us(w); });
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
}
template <class P>
static void run(const char* name, int workers) {
  P p(workers);
  const int cases[][2] = {{8, 0}, {16, 0}, {8, 1}, {8, 3}, {2, 2}, {4, 1}};
  for (auto& c : cases)
    printf("%-9s workers %d  burst %2d x %d us: %.2f us\n", name, workers, c[0], c[1], burst_us(p, c[0], c[1], 5000));
}
int main(int argc, char** argv) {
  const int workers = argc > 1 ? atoi(argv[1]) : 7;
  const int v = argc > 2 ? atoi(argv[2]) : 0;
  if (v == 0) run<spg::Pool>("shared", workers);
  if (v == 1) run<pool_static::Pool>("static", workers);
  return 0;
}
