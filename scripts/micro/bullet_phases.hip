// Microbenchmark: where the time of one device Bullet round (k_bullet_round_q, csrc/bullet.hpp) goes.
// Random field data (timing only), a 254 x 4098-entry generator table like gens_r1cs_sat's. Per launch
// size: HIP-event time, and from the kernel's own wall_clock64 probes (100 MHz) the per-block phases:
// start skew, fold + recode, bucket additions, LDS tree, tail (bucket store, ticket, mailbox).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "../../spartan-parallel_amd/csrc/bullet.hpp"

using namespace spg;

namespace spg {
int set_err(spg_ctx*, int code, const std::string&) { return code; }
}

__global__ void k_null(unsigned* c) {
  if (threadIdx.x == 0 && c == nullptr) c[0] = 1;
}

static void fill(std::vector<uint32_t>& v, uint32_t seed) {
  for (auto& x : v) {
    seed = seed * 1664525u + 1013904223u;
    x = seed;
  }
}

template <int BS>
static void run(int n, int k, Niels* tab, int n1, Fq* st, uint32_t* gidx, unsigned* ctr, uint32_t* mb, Ext* bk,
                unsigned long long* probe) {
  const int NB = 64;
  Fq u, ui;
  for (int i = 0; i < 8; i++) u.l[i] = ui.l[i] = 0x01234567u * (i + 1);
  u.l[7] = ui.l[7] = 0x01000000u;
  BulletArgs a{st, st + 2 * (size_t)n, st + (size_t)n, st + 3 * (size_t)n, gidx, u, ui, k, n, n >> k, n1, tab, bk,
               ctr, mb, 1u, nullptr};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; w++) hipLaunchKernelGGL((k_bullet_round_q<7, BS>), dim3(NB + 1, 2), dim3(BS), 0, 0, a);
  const int R = 20;
  hipEventRecord(e0, 0);
  for (int r = 0; r < R; r++) hipLaunchKernelGGL((k_bullet_round_q<7, BS>), dim3(NB + 1, 2), dim3(BS), 0, 0, a);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  a.probe = probe;
  hipLaunchKernelGGL((k_bullet_round_q<7, BS>), dim3(NB + 1, 2), dim3(BS), 0, 0, a);
  hipDeviceSynchronize();
  std::vector<unsigned long long> p(8 * 2 * (NB + 1));
  hipMemcpy(p.data(), probe, p.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, tend = 0;
  double ph[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0}, skew = 0;
  for (int b = 0; b < 2 * (NB + 1); b++) t0 = std::min(t0, p[8 * b]);
  for (int b = 0; b < 2 * (NB + 1); b++) {
    const unsigned long long* q = &p[8 * b];
    skew = std::max(skew, (q[0] - t0) * 0.01);
    for (int i = 0; i < 4; i++) {
      const double d = (q[i + 1] - q[i]) * 0.01;
      ph[i] += d / (2 * (NB + 1));
      mx[i] = std::max(mx[i], d);
    }
    tend = std::max(tend, q[4]);
  }
  printf("n=%5d k=%d BS=%3d event %.1f us/launch | probes (us, avg/max): start skew max %.2f, fold+recode %.2f/%.2f, "
         "madds %.2f/%.2f, tree %.2f/%.2f, tail %.2f/%.2f, first start -> last end %.2f\n",
         n, k, BS, ms * 1000 / R, skew, ph[0], mx[0], ph[1], mx[1], ph[2], mx[2], ph[3], mx[3], (tend - t0) * 0.01);
}

__global__ void k_clock(unsigned long long* out, int iters) {
  unsigned long long w0 = wall_clock64(), c0 = clock64();
  float x = threadIdx.x;
  for (int i = 0; i < iters; i++) x = x * 0.999f + 1.0f;
  unsigned long long w1 = wall_clock64(), c1 = clock64();
  if (threadIdx.x == 0) {
    out[0] = w1 - w0;
    out[1] = c1 - c0;
    out[2] = (unsigned long long)x;
  }
}

// per-launch time of one Bullet round when launches are separated by host idle gaps (the prover's pattern)
template <int BS>
static void run_gaps(int n, Niels* tab, int n1, Fq* st, uint32_t* gidx, unsigned* ctr, uint32_t* mb, Ext* bk,
                     int gap_us, unsigned long long* clk) {
  const int NB = 64;
  Fq u, ui;
  for (int i = 0; i < 8; i++) u.l[i] = ui.l[i] = 0x01234567u * (i + 1);
  u.l[7] = ui.l[7] = 0x01000000u;
  BulletArgs a{st, st + 2 * (size_t)n, st + (size_t)n, st + 3 * (size_t)n, gidx, u, ui, 1, n, n >> 1, n1, tab, bk,
               ctr, mb, 1u, nullptr};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double tot = 0;
  const int R = 30;
  for (int r = 0; r < R + 3; r++) {
    std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_bullet_round_q<7, BS>), dim3(NB + 1, 2), dim3(BS), 0, 0, a);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r >= 3) tot += ms;
  }
  // shader clock after the same gap
  std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, clk, 20000);
  unsigned long long h[3];
  hipMemcpy(h, clk, 24, hipMemcpyDeviceToHost);
  printf("gap %5d us: n=%d round %.1f us/launch; shader clock %.0f MHz (single-wave loop after the gap)\n", gap_us, n,
         tot * 1000 / R, h[1] * 100.0 / h[0]);
}

int main() {
  const int n1 = 4098, rows = 254;
  Niels* tab;
  hipMalloc(&tab, (size_t)rows * n1 * sizeof(Niels));
  {
    std::vector<uint32_t> h((size_t)rows * n1 * sizeof(Niels) / 4);
    fill(h, 7);
    for (size_t i = 0; i < h.size(); i++) h[i] &= 0x7fffffffu;
    hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  }
  const int NMAX = 4096;
  Fq* st;
  hipMalloc(&st, 4 * NMAX * sizeof(Fq));
  {
    std::vector<uint32_t> h(4 * NMAX * 8);
    fill(h, 11);
    for (size_t i = 7; i < h.size(); i += 8) h[i] &= 0x0fffffffu;
    hipMemcpy(st, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  }
  uint32_t* gidx;
  hipMalloc(&gidx, NMAX * 4);
  {
    std::vector<uint32_t> h(NMAX);
    for (int i = 0; i < NMAX; i++) h[i] = i;
    hipMemcpy(gidx, h.data(), NMAX * 4, hipMemcpyHostToDevice);
  }
  unsigned* ctr;
  uint32_t* mb;
  Ext* bk;
  unsigned long long* probe;
  hipMalloc(&ctr, 64);
  hipMemset(ctr, 0, 64);
  hipMalloc(&mb, 4096);
  hipMalloc(&bk, 2 * 65 * sizeof(Ext));
  hipMalloc(&probe, 8 * 2 * 65 * 8);
  {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_null, dim3(64, 2), dim3(256), 0, 0, ctr);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 20; r++) hipLaunchKernelGGL(k_null, dim3(64, 2), dim3(256), 0, 0, ctr);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("null kernel (64 x 2 blocks): %.1f us/launch\n", ms * 1000 / 20);
  }
  unsigned long long* clk;
  hipMalloc(&clk, 64);
  for (int gap : {0, 20, 100, 1000})
    run_gaps<256>(512, tab, n1, st, gidx, ctr, mb, bk, gap, clk);
  for (int k = 0; k < 2; k++) {
    run<64>(128, k, tab, n1, st, gidx, ctr, mb, bk, probe);
    run<128>(256, k, tab, n1, st, gidx, ctr, mb, bk, probe);
    run<256>(512, k, tab, n1, st, gidx, ctr, mb, bk, probe);
    run<256>(1024, k, tab, n1, st, gidx, ctr, mb, bk, probe);
  }
  return 0;
}
