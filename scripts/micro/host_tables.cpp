// Host fixed-base commitments at the shape of a host Bullet round (2 MSMs of n/2 + 2 terms over a working set
// of G generators' byte-window tables, ~1 MB each): does the table working set (L3 = 32 MB per 8-core domain on
// the GPU box) set the cost?
// g++ -O2 -std=c++17 -pthread -I spartan-parallel_amd/csrc scripts/micro/host_tables.cpp -o scripts/micro/host_tables
#include <stdio.h>

#include <chrono>
#include <random>

#include "host.hpp"

using namespace spg;
using clk = std::chrono::steady_clock;

int main() {
  uint8_t basepoint[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
                           0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  h::HExt P;
  if (!h::hext_decompress(basepoint, P)) return 1;
  std::vector<uint8_t> comp;
  h::HExt Q = P;
  const int NG = 64;
  for (int i = 0; i < NG; i++) {
    Pt c = compress(Q);
    comp.insert(comp.end(), c.b, c.b + 32);
    Q = h::hext_add(Q, P);
  }
  std::mt19937_64 rng(7);
  auto rnd = [&] {
    Fq k;
    for (int i = 0; i < 8; i++) k.l[i] = (uint32_t)rng();
    k.l[7] &= 0x0fffffffu;
    return fq_to_mont(k);
  };
  using Job = std::pair<std::vector<size_t>, FqV>;
  for (int G : {4, 8, 16, 24, 34, 48, 64}) {
    HostGens hg;
    hg.init(comp.data(), NG);
    const int terms = 18;  // n = 32: n/2 + 2
    std::vector<std::vector<Job>> calls(64);
    for (auto& c : calls) {
      c.resize(2);
      for (auto& j : c)
        for (int t = 0; t < terms; t++) {
          j.first.push_back((size_t)(rng() % G));
          j.second.push_back(rnd());
        }
    }
    for (auto& c : calls) hg.commit_many(c);  // tables
    volatile uint8_t sink = 0;
    // cycle through G's tables between calls, as a prove does between rounds (other data evicts them too)
    auto t0 = clk::now();
    const int reps = 400;
    for (int r = 0; r < reps; r++) sink ^= hg.commit_many(calls[r % calls.size()])[0].b[0];
    const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
    t0 = clk::now();
    for (int r = 0; r < reps; r++) {
      auto& c = calls[r % calls.size()];
      h::HExt a = hg.msm(c[0].first, c[0].second), b = hg.msm(c[1].first, c[1].second);
      sink ^= compress(a).b[0] ^ compress(b).b[0];
    }
    const double us1 = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
    printf("[1 thread: %.2f us] ", us1);
    printf("tables of %2d generators (%5.1f MB): 2 x %d-term commit_many %.2f us\n", G, G * 32 * 256 * 120.0 / 1e6,
           terms, us);
  }
  return 0;
}
