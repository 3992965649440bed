// Microbenchmark (host only): one Ristretto encoding per point (hext_compress: an inverse square root) against the
// batched encodings of doubles (hcurve.hpp hext_double_and_compress_batch, one inversion per batch) and their 8-lane
// IFMA form (hvec.hpp double_and_compress_batch8), per point, at batch sizes 1024 / 128 / 32 / 8.
//   g++ -O2 -std=c++17 -I include scripts/micro/enc_batch.cpp -o scripts/micro/enc_batch
#include <chrono>
#include <cstdio>
#include <vector>
#include "../../spartan-parallel_amd/csrc/host.hpp"
using namespace spg;
int main() {
  std::vector<h::HExt> P(1024);
  h::HExt B = h::hext_identity();
  // points: i-th = some walk
  h::HExt G = h::hext_from_dev(ristretto_from_uniform_bytes((const uint8_t*)"0123456789012345678901234567890123456789012345678901234567890123"));
  h::HExt acc = G;
  for (int i = 0; i < 1024; i++) { acc = h::hext_add(acc, G); acc = h::hext_dbl(acc); P[i] = acc; }
  std::vector<uint8_t> o(32 * 1024);
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 128; i++) h::hext_compress(P[i], &o[32 * i]);
    auto t1 = std::chrono::steady_clock::now();
    h::hext_double_and_compress_batch(P.data(), 1024, (uint8_t(*)[32])o.data());
    auto t2 = std::chrono::steady_clock::now();
    h::double_and_compress_batch8(P.data(), 1024, (uint8_t(*)[32])o.data());
    auto t3 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    printf("lone %.3f us/pt, batch %.3f us/pt, batch8 %.3f us/pt\n", us(t0, t1) / 128, us(t1, t2) / 1024, us(t2, t3) / 1024);
  }
  for (int m : {128, 32, 8}) {
    auto t0 = std::chrono::steady_clock::now();
    for (int rep = 0; rep < 64; rep++) h::double_and_compress_batch8(P.data(), m, (uint8_t(*)[32])o.data());
    auto t1 = std::chrono::steady_clock::now();
    printf("batch8 of %4d: %.2f us per call\n", m, std::chrono::duration<double, std::micro>(t1 - t0).count() / 64);
  }
}
