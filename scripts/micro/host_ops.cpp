// Host-side cost of the prover's sequential-protocol primitives (radix-2^51 curve, 64-bit Fq, merlin):
// g++ -O2 -std=c++17 -pthread -I spartan-parallel_amd/csrc scripts/micro/host_ops.cpp
#include <chrono>
#include <stdio.h>

#include "host.hpp"

using namespace spg;
using clk = std::chrono::steady_clock;

template <class F>
double us_per(int n, F f) {
  auto t0 = clk::now();
  for (int i = 0; i < n; i++) f(i);
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

int main() {
  uint8_t basepoint[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
                           0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
  h::HExt P;
  if (!h::hext_decompress(basepoint, P)) { printf("decompress failed\n"); return 1; }
  FixedBase fb;
  fb.build(P);
  Fq k;
  for (int i = 0; i < 8; i++) k.l[i] = 0x12345678u * (i + 1);
  k.l[7] &= 0x0fffffffu;
  h::HExt acc = h::hext_identity();
  volatile uint8_t sink = 0;
  printf("hext_add        %.3f us\n", us_per(20000, [&](int) { acc = h::hext_add(acc, P); }));
  printf("fixed-base k*P  %.3f us (32 byte windows)\n", us_per(2000, [&](int) { fb.mul_add(acc, k); }));
  printf("compress        %.3f us\n", us_per(2000, [&](int) { Pt c = compress(acc); sink ^= c.b[0]; }));
  Fq a = k, b = k;
  printf("fq_mul (host)   %.4f us\n", us_per(200000, [&](int) { a = fq_mul(a, b); }));
  printf("fq_inv (host)   %.3f us\n", us_per(2000, [&](int) { a = fq_inv(fq_add(a, b)); }));
  Tr t("bench");
  printf("transcript append point %.3f us\n", us_per(20000, [&](int) { t.point("comm", Pt{}); }));
  printf("transcript challenge    %.3f us\n", us_per(20000, [&](int) { a = fq_add(a, t.challenge("c")); }));
  printf("pool burst (16 x no-op) %.3f us\n", us_per(2000, [&](int) { pool().parallel_for(16, [](int) {}); }));
  // sigma-protocol commitment bursts as the ZK sumcheck rounds issue them (HostGens::commit_many)
  std::vector<uint8_t> comp;
  h::HExt Q = P;
  for (int i = 0; i < 8; i++) {
    Pt c = compress(Q);
    comp.insert(comp.end(), c.b, c.b + 32);
    Q = h::hext_add(Q, P);
  }
  HostGens hg;
  hg.init(comp.data(), 8);
  FqV x(5);
  for (int i = 0; i < 5; i++) x[i] = fq_add(k, fq_from_u64(i + 1));
  using Job = std::pair<std::vector<size_t>, FqV>;
  std::vector<Job> one5 = {{{0, 1, 2, 3, 7}, x}};
  std::vector<Job> one2 = {{{4, 7}, {x[0], x[1]}}};
  std::vector<Job> three = {{{4, 7}, {x[0], x[1]}}, {{0, 1, 2, 3, 7}, x}, {{4, 7}, {x[2], x[3]}}};
  hg.commit_many(three);  // tables
  printf("commit_many 1 x 5 terms  %.3f us\n", us_per(2000, [&](int) { sink ^= hg.commit_many(one5)[0].b[0]; }));
  printf("commit_many 1 x 2 terms  %.3f us\n", us_per(2000, [&](int) { sink ^= hg.commit_many(one2)[0].b[0]; }));
  printf("commit_many 3 jobs (2,5,2) %.3f us\n", us_per(2000, [&](int) { sink ^= hg.commit_many(three)[0].b[0]; }));
  printf("sum_many 1 x 5 terms (no encoding) %.3f us\n", us_per(2000, [&](int) { acc = hg.sum_many(one5)[0]; }));
  // host Bullet rounds (DotProductProofLog with n <= 32 on the host): two MSMs of n/2 + 2 terms per round over
  // generator sets whose tables (~1 MB per generator) do not fit the caches; 8 sets of 34 generators rotated
  {
    const int G = 8 * 34;
    std::vector<uint8_t> c2;
    h::HExt R = P;
    for (int i = 0; i < G; i++) {
      Pt c = compress(R);
      c2.insert(c2.end(), c.b, c.b + 32);
      R = h::hext_add(R, h::hext_dbl(P));
    }
    HostGens big;
    big.init(c2.data(), G);
    std::vector<std::vector<Job>> rounds(8);
    for (int set = 0; set < 8; set++) {
      for (int b = 0; b < 2; b++) {
        Job j;
        for (int i = 0; i < 18; i++) {
          j.first.push_back((size_t)(set * 34 + b * 16 + i));
          j.second.push_back(fq_add(k, fq_from_u64(1000 * set + 100 * b + i)));
        }
        rounds[set].push_back(j);
      }
      big.commit_many(rounds[set]);  // tables
    }
    printf("host Bullet round (2 x 18 terms, 8 rotating sets) %.3f us\n",
           us_per(400, [&](int i) { sink ^= big.commit_many(rounds[i % 8])[0].b[0]; }));
  }
  printf("(sink %d %u)\n", (int)sink, a.l[0]);
  return 0;
}
