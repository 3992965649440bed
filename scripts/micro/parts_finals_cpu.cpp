// Host-side microbenchmark (no GPU): the Bullet round's part sums as proto.hip parts_finals runs them -- B = 2 MSMs of
// `per` device-format partial points (8 x u32 limbs per coordinate), chunked over the pool, the last chunk's thread
// adding the chunk sums and encoding -- split into its pieces: limb conversion, additions, encodings, pool dispatch.
// With a GPU present, the same finals also run on parts a kernel has just written into coherent mapped host memory
// (cold in the host caches, as in the prover), with and without the prefetch pass.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../spartan-parallel_amd/csrc -o parts_finals_cpu parts_finals_cpu.cpp -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <memory>

#include "hcurve.hpp"
#include "hvec.hpp"
#include "keccak.hpp"
#include "hpool.hpp"

using namespace spg;
using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

__global__ void k_write(const Ext* __restrict__ src, Ext* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

static void finals(const Ext* bk, size_t per, int K, bool prefetch, uint8_t outb[2][32]) {
  const int B = 2;
  std::vector<h::HExt> part(B * K);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[B]);
  for (int b = 0; b < B; b++) left[b].store(K);
  pool().parallel_for(B * K, [&](int task) {
    const size_t b = task / K, c = task % K;
    const size_t lo = per * c / K, hi = per * (c + 1) / K;
    if (prefetch)
      for (const uint8_t* q = (const uint8_t*)(bk + b * per + lo); q < (const uint8_t*)(bk + b * per + hi); q += 64)
        __builtin_prefetch(q, 0, 0);
    h::HExt acc = h::hext_from_dev(bk[b * per + lo]);
    for (size_t i = lo + 1; i < hi; i++) acc = h::hext_add(acc, h::hext_from_dev(bk[b * per + i]));
    part[task] = acc;
    if (left[b].fetch_sub(1, std::memory_order_acq_rel) == 1) {
      h::HExt sum = part[b * K];
      for (int k = 1; k < K; k++) sum = h::hext_add(sum, part[b * K + k]);
      h::hext_compress(sum, outb[b]);
    }
  });
}

int main(int argc, char** argv) {
  const size_t per = argc > 1 ? (size_t)atol(argv[1]) : 704;
  // argv[2] = "pin": the pool on the first 8 CPUs of this process' mask (the prover pins it to one L3 domain)
  if (argc > 2 && !strcmp(argv[2], "pin")) {
    cpu_set_t set;
    sched_getaffinity(0, sizeof(set), &set);
    std::vector<int> c;
    for (int i = 0; i < CPU_SETSIZE && c.size() < 8; i++)
      if (CPU_ISSET(i, &set)) c.push_back(i);
    pool_cpus() = c;
    (void)pool();  // workers start pinned (the pool is sized from this thread's mask, so before pinning it)
    pin_thread({c[0]});
    printf("pool pinned to cpus %d..%d\n", c.front(), c.back());
  }
  const int R = 2000;
  // device-format points: random multiples of a fixed point, Z scaled, as the device leaves them
  std::vector<Ext> bk(2 * per);
  h::HExt P = h::hext_identity();
  uint8_t seed[32] = {9};
  h::HExt G;
  {
    // a valid point: decode the ristretto basepoint encoding
    const uint8_t B[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
                           0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
    if (!h::hext_decompress(B, G)) { printf("decode failed\n"); return 1; }
  }
  (void)seed;
  for (size_t i = 0; i < 2 * per; i++) {
    P = h::hext_add(P, G);
    uint8_t b[32];
    Ext e;
    const h::Fe* c[4] = {&P.X, &P.Y, &P.Z, &P.T};
    Fp* o[4] = {&e.X, &e.Y, &e.Z, &e.T};
    for (int k = 0; k < 4; k++) {
      h::fe_to_bytes(*c[k], b);
      for (int w = 0; w < 8; w++) o[k]->l[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) | ((uint32_t)b[4 * w + 3] << 24);
    }
    bk[i] = e;
  }
  // pieces, single thread
  auto t0 = clk::now();
  volatile uint64_t sink = 0;
  for (int r = 0; r < R; r++)
    for (size_t i = 0; i < per; i++) sink += h::hext_from_dev(bk[i]).X.v[0];
  printf("per=%zu: hext_from_dev %.1f ns each\n", per, us_since(t0) * 1e3 / R / per);
  std::vector<h::HExt> hx(per);
  for (size_t i = 0; i < per; i++) hx[i] = h::hext_from_dev(bk[i]);
  t0 = clk::now();
  for (int r = 0; r < R; r++) {
    h::HExt acc = hx[0];
    for (size_t i = 1; i < per; i++) acc = h::hext_add(acc, hx[i]);
    sink += acc.X.v[0];
  }
  printf("hext_add %.1f ns each\n", us_since(t0) * 1e3 / R / (per - 1));
  if (h::ifma_on()) {
    t0 = clk::now();
    for (int r = 0; r < R; r++) sink += h::ext_sum8(hx.data(), per).X.v[0];
    printf("ext_sum8 (8-lane IFMA full additions): %.1f ns per point\n", us_since(t0) * 1e3 / R / per);
    std::vector<h::HNiels> nl;
    h::hext_batch_to_niels(hx, nl);
    std::vector<const h::HNiels*> np(per);
    for (size_t i = 0; i < per; i++) np[i] = &nl[(i * 7919) % per];
    t0 = clk::now();
    for (int r = 0; r < R; r++) {
      h::HExt acc = h::hext_identity();
      for (size_t i = 0; i < per; i++) acc = h::hext_madd(acc, *np[i]);
      sink += acc.X.v[0];
    }
    printf("hext_madd (scalar mixed additions): %.1f ns each\n", us_since(t0) * 1e3 / R / per);
    t0 = clk::now();
    for (int r = 0; r < R; r++) sink += h::niels_sum8(np.data(), per).X.v[0];
    printf("niels_sum8 (8-lane IFMA mixed additions): %.1f ns per entry\n", us_since(t0) * 1e3 / R / per);
    for (size_t m : {8, 16, 32, 64}) {
      t0 = clk::now();
      for (int r = 0; r < R; r++) sink += h::niels_sum8(np.data(), m).X.v[0];
      const double v = us_since(t0) / R;
      t0 = clk::now();
      for (int r = 0; r < R; r++) {
        h::HExt acc = h::hext_identity();
        for (size_t i = 0; i < m; i++) acc = h::hext_madd(acc, *np[i]);
        sink += acc.X.v[0];
      }
      printf("  %zu entries: niels_sum8 %.2f us, scalar %.2f us\n", m, v, us_since(t0) / R);
    }
  }
  t0 = clk::now();
  for (int r = 0; r < R; r++) {
    uint8_t out[32];
    h::hext_compress(hx[r % per], out);
    sink += out[0];
  }
  printf("hext_compress %.2f us each\n", us_since(t0) / R);
  // the whole finals as parts_finals runs them (B = 2)
  const int threads = pool().size() + 1;
  for (int K : {1, 2, 4, 8, threads / 2, threads}) {
    if (K < 1) continue;
    t0 = clk::now();
    for (int r = 0; r < R; r++) {
      uint8_t outb[2][32];
      finals(bk.data(), per, K, true, outb);
      sink += outb[0][0] + outb[1][0];
    }
    printf("parts_finals B=2 K=%2d (pool %d threads, warm host memory): %.2f us\n", K, threads, us_since(t0) / R);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    Ext *d_src, *h_map, *d_map;
    hipMalloc(&d_src, bk.size() * sizeof(Ext));
    hipMemcpy(d_src, bk.data(), bk.size() * sizeof(Ext), hipMemcpyHostToDevice);
    hipHostMalloc(&h_map, bk.size() * sizeof(Ext), hipHostMallocCoherent | hipHostMallocMapped);
    hipHostGetDevicePointer((void**)&d_map, h_map, 0);
    for (int K : {2, 4, 8, threads / 2})
      for (int pf = 0; pf < 2; pf++) {
        double tot = 0;
        const int RR = 300;
        for (int r = 0; r < RR; r++) {
          hipLaunchKernelGGL(k_write, dim3((unsigned)((bk.size() + 255) / 256)), dim3(256), 0, 0, d_src, d_map, (int)bk.size());
          hipDeviceSynchronize();
          uint8_t outb[2][32];
          const auto t1 = clk::now();
          finals(h_map, per, K, pf != 0, outb);
          tot += us_since(t1);
          sink += outb[0][0];
        }
        printf("parts_finals B=2 K=%2d on parts a kernel just wrote (mapped coherent)%s: %.2f us\n", K,
               pf ? ", prefetch" : "", tot / RR);
      }
  }
  {  // merlin transcript operations (keccak-f[1600] per 166 bytes absorbed and per challenge)
    Merlin m("bench");
    uint8_t b[64] = {1};
    t0 = clk::now();
    for (int r = 0; r < R; r++) {
      KeccakState st;
      memset(st.a, r, sizeof(st.a));
      st.permute();
      sink += st.a[0];
    }
    printf("keccak-f[1600] %.3f us\n", us_since(t0) / R);
    t0 = clk::now();
    for (int r = 0; r < R; r++) m.message("claim_prod_left", b, 32);
    printf("merlin append 32 B %.3f us\n", us_since(t0) / R);
    t0 = clk::now();
    for (int r = 0; r < R; r++) m.challenge("rand_coeffs_next_layer", b, 64);
    printf("merlin challenge 64 B %.3f us\n", us_since(t0) / R);
    sink += b[0];
  }
  {  // the host scalar-field inverse (binary GCD, field.hpp fq_inv_host): u^-1 of every Bullet round
    Fq x = fq_from_u64(123456789);
    t0 = clk::now();
    for (int r = 0; r < R; r++) {
      Fq y = fq_inv(x);
      x = fq_add(x, y);
    }
    printf("fq_inv (host) %.2f us each\n", us_since(t0) / R);
    sink += x.l[0];
  }
  t0 = clk::now();
  for (int r = 0; r < R; r++) pool().parallel_for(threads, [&](int) { sink += 1; });
  printf("empty parallel_for over %d tasks: %.2f us\n", threads, us_since(t0) / R);
  return 0;
}
