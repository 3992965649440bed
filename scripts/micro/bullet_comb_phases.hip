// Microbenchmark: where the time of one comb-form Bullet round (k_bullet_comb, csrc/bullet.hpp) goes.
// Random data (timing only) in a 13-bit comb table of 64 generator slots + h at 128-byte entries (the product's
// layout, 681 MB); parts and mailbox in coherent mapped host memory as in the product. Per round size: HIP-event time
// back to back and after 20 us host gaps, and from the kernel's wall_clock64 probes (100 MHz) the per-workgroup
// phases: start skew, fold products, recode + entry loads, mixed additions, LDS tree, parts + fence, ticket + post.
// Both forms (k_bullet_comb, k_bullet_comb_roll) alternate per size.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/micro/bullet_comb_phases scripts/micro/bullet_comb_phases.hip
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

static void fill(std::vector<uint32_t>& v, uint32_t seed) {
  for (auto& x : v) {
    seed = seed * 1664525u + 1013904223u;
    x = seed;
  }
}

constexpr int C = 13, G = 10, NS = 65, ST = 4;

template <int BS, bool ROLL>
static void launch(dim3 grid, const BulletCombArgs& a) {
  if (ROLL)
    hipLaunchKernelGGL((k_bullet_comb_roll<C, G, BS>), grid, dim3(BS), 0, 0, a);
  else
    hipLaunchKernelGGL((k_bullet_comb<C, G, BS>), grid, dim3(BS), 0, 0, a);
}

template <int BS, bool ROLL = false>
static void run(int n, const Niels* tab, Fq* st, uint32_t* gidx, unsigned* ctr, uint32_t* mb, Ext* parts,
                unsigned long long* probe, int gap_us) {
  const int R = 8, S = BS / 4, P = n / 2, wgs = (P * G + S - 1) / S;
  Fq u, ui;
  for (int i = 0; i < 8; i++) u.l[i] = ui.l[i] = 0x01234567u * (i + 1);
  u.l[7] = ui.l[7] = 0x01000000u;
  const int nk = n;  // one block: k rounds in, nk = n
  BulletCombArgs a{st, st + 2 * (size_t)n, st + (size_t)n, st + 3 * (size_t)n, gidx, u, ui, 1, n, nk, tab, NS, R,
                   parts, ctr, mb, 1u, ST};
  const dim3 grid(wgs, 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 30;
  double tot = 0;
  for (int r = 0; r < reps + 3; r++) {
    if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
    hipEventRecord(e0, 0);
    launch<BS, ROLL>(grid, a);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r >= 3) tot += ms;
  }
  a.probe = probe;
  const int nb = 2 * wgs;
  hipMemset(probe, 0, (size_t)8 * nb * 8);
  if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
  launch<BS, ROLL>(grid, a);
  hipDeviceSynchronize();
  std::vector<unsigned long long> p((size_t)8 * nb);
  hipMemcpy(p.data(), probe, p.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, tend = 0;
  double ph[6] = {0, 0, 0, 0, 0, 0}, mx[6] = {0, 0, 0, 0, 0, 0}, skew = 0;
  int cnt = 0;
  for (int b = 0; b < nb; b++) t0 = std::min(t0, p[8 * b]);
  for (int b = 0; b < nb; b++) {
    const unsigned long long* q = &p[8 * b];
    if (!q[1] || !q[2] || !q[3]) continue;  // workgroups past the last scalar skip the probes in the quad body
    cnt++;
    skew = std::max(skew, (q[0] - t0) * 0.01);
    for (int i = 0; i < 6; i++) {
      const double d = (q[i + 1] - q[i]) * 0.01;
      ph[i] += d;
      mx[i] = std::max(mx[i], d);
    }
    tend = std::max(tend, q[6]);
  }
  for (int i = 0; i < 6; i++) ph[i] /= std::max(cnt, 1);
  printf("%s n=%5d BS=%3d wgs=%4d gap %3d us: event %.2f us/launch | probes avg/max us: skew %.2f, fold %.2f/%.2f, "
         "recode+loads %.2f/%.2f, madds %.2f/%.2f, tree %.2f/%.2f, parts+fence %.2f/%.2f, ticket+post %.2f/%.2f, "
         "first start -> last end %.2f\n",
         ROLL ? "roll  " : "unroll", n, BS, nb, gap_us, tot * 1000 / reps, skew, ph[0], mx[0], ph[1], mx[1], ph[2], mx[2], ph[3], mx[3], ph[4],
         mx[4], ph[5], mx[5], (tend - t0) * 0.01);
}

int main() {
  const int W = 253 / C + 1, NB = 1 << (C - 1);
  const size_t entries = (size_t)W * NS * NB, words = entries * ST * 8;
  Niels* tab;
  if (hipMalloc(&tab, words * 4) != hipSuccess) return 1;
  {
    // random coordinates below 2^255, written in 64 MB chunks
    std::vector<uint32_t> h(16u << 20);
    for (size_t off = 0; off < words; off += h.size()) {
      fill(h, (uint32_t)(off * 2654435761u + 7));
      for (size_t i = 7; i < h.size(); i += 8) h[i] &= 0x3fffffffu;
      hipMemcpy((uint32_t*)tab + off, h.data(), std::min(h.size(), words - off) * 4, hipMemcpyHostToDevice);
    }
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
    for (int i = 0; i < NMAX; i++) h[i] = i % (NS - 1);
    hipMemcpy(gidx, h.data(), NMAX * 4, hipMemcpyHostToDevice);
  }
  unsigned* ctr;
  hipMalloc(&ctr, 64);
  hipMemset(ctr, 0, 64);
  void *mbh = nullptr, *parts_h = nullptr;
  uint32_t* mb;
  Ext* parts;
  hipHostMalloc(&mbh, 1 << 16, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&mb, mbh, 0);
  hipHostMalloc(&parts_h, 4096 * sizeof(Ext), hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&parts, parts_h, 0);
  unsigned long long* probe;
  hipMalloc(&probe, (size_t)8 * 2048 * 8);
  // the unrolled (k_bullet_comb) and rolled (k_bullet_comb_roll) forms alternated, twice
  for (int rep = 0; rep < 2; rep++)
    for (int gap : {0, 20}) {
      run<64, false>(2, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<64, true>(2, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<64, false>(32, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<64, true>(32, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<64, false>(128, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<64, true>(128, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<128, false>(256, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<128, true>(256, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<256, false>(1024, tab, st, gidx, ctr, mb, parts, probe, gap);
      run<256, true>(1024, tab, st, gidx, ctr, mb, parts, probe, gap);
    }
  return 0;
}
