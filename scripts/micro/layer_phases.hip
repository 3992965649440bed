// Microbenchmark: one fused SPARK layer-sumcheck round (k_layer_round, csrc/layer.hpp) at the prover's sizes.
// Random field data (timing only). Per (triples, len, fold): HIP-event time per launch (back to back, and
// with a host mailbox wait per launch as the prover does), and the kernel's own wall_clock64 phases:
// elements (loads, fold, products), block reduction, mailbox post (host-mapped, system scope).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../spartan-parallel_amd/csrc/layer.hpp"

using namespace spg;

namespace spg {
int set_err(spg_ctx*, int code, const std::string&) { return code; }
}

// the "armed" hand-off: the kernel of round i is launched before the host knows round i's challenge and waits
// (thread 0, bounded) for a host-written doorbell carrying it; one workgroup (the K == 1 rounds of the prover)
template <int BS>
__global__ void __launch_bounds__(BS) k_armed(const uint32_t* __restrict__ db, uint32_t dseq, const Triple* __restrict__ tr,
                                              const Fq* __restrict__ coeff, int nt, int log_len, int do_fold,
                                              const Fq* __restrict__ cin, Fq* __restrict__ cout, uint32_t* __restrict__ mb,
                                              uint32_t seq) {
  __shared__ uint32_t rw[8];
  __shared__ int go;
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned long long t0 = wall_clock64();
    int ok = 1;
    while (__hip_atomic_load(db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != dseq) {
      if (wall_clock64() - t0 > 200000000ull) {
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    for (int j = 0; j < 8; j++) rw[j] = __hip_atomic_load(db + 8 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    go = ok;
  }
  __syncthreads();
  if (!go) return;
  Fq r;
  for (int j = 0; j < 8; j++) r.l[j] = rw[j];
  Fq e = layer_round_elems(tr, coeff, nt, log_len, do_fold, r, cin, cout, t >> 2, BS / 4, nullptr);
  quad_block_sum<BS>(e);
  if (t < 3) {
    for (int j = 0; j < 8; j++) __hip_atomic_store(mb + 8 + 8 * t + j, e.l[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  if (t == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int BS>
static void run_armed(int nt, int log_len, Fq* cin, Fq* cout, Triple* dtr, Fq* dcoef, uint32_t* mb_dev,
                      volatile uint32_t* mb_host, uint32_t* db_dev, volatile uint32_t* db_host) {
  const int R = 40;
  uint32_t seq = 50000, dseq = 0;
  db_host[0] = 0;
  for (int j = 0; j < 8; j++) db_host[8 + j] = 0x01234567u * (j + 3) & 0x0fffffffu;
  hipDeviceSynchronize();
  // launch round 1 armed; then per round: doorbell i, launch i + 1 armed, wait mailbox i, ~1 us of host work
  hipLaunchKernelGGL(k_armed<BS>, dim3(1), dim3(BS), 0, 0, db_dev, dseq + 1, dtr, dcoef, nt, log_len, 1, cin, cout, mb_dev,
                     seq + 1);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 1; i <= R; i++) {
    __atomic_store_n(db_host, dseq + i, __ATOMIC_RELEASE);
    if (i < R)
      hipLaunchKernelGGL(k_armed<BS>, dim3(1), dim3(BS), 0, 0, db_dev, dseq + i + 1, dtr, dcoef, nt, log_len, 1, cin, cout,
                         mb_dev, seq + i + 1);
    while (__atomic_load_n(mb_host, __ATOMIC_ACQUIRE) != seq + (uint32_t)i) {
    }
    const auto h = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - h < std::chrono::microseconds(1)) {
    }
  }
  const double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
  hipDeviceSynchronize();
  // the same rounds with one launch per round after the host work (the prover's pattern), for comparison
  t0 = std::chrono::steady_clock::now();
  Fq r;
  for (int j = 0; j < 8; j++) r.l[j] = 0x01234567u * (j + 3) & 0x0fffffffu;
  for (int i = 1; i <= R; i++) {
    const uint32_t s = seq + 1000 + i;
    hipLaunchKernelGGL(k_layer_round_q<BS>, dim3(1), dim3(BS), 0, 0, dtr, dcoef, nt, log_len, 1, r, cin, cout, nullptr,
                       nullptr, mb_dev, s, nullptr, 0);
    while (__atomic_load_n(mb_host, __ATOMIC_ACQUIRE) != s) {
    }
    const auto h = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - h < std::chrono::microseconds(1)) {
    }
  }
  const double rl = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
  hipDeviceSynchronize();
  printf("armed nt=%2d len=%4d BS=%3d: armed round %.1f us, launch-per-round %.1f us (1 us host work each)\n", nt,
         1 << log_len, BS, rt, rl);
}

template <int BS, bool Q = false>
static void run(int nt, int log_len, int fold, unsigned K, Fq* vec, Fq* cin, Fq* cout, Triple* dtr, Fq* dcoef, Fq* part,
                unsigned* ctr, uint32_t* mb_dev, volatile uint32_t* mb_host, unsigned long long* probe) {
  Fq r;
  for (int i = 0; i < 8; i++) r.l[i] = 0x01234567u * (i + 3);
  r.l[7] = 0x01000000u;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  uint32_t seq = 1000;
  for (int w = 0; w < 3; w++)
    hipLaunchKernelGGL((Q ? k_layer_round_q<BS> : k_layer_round<BS>), dim3(K), dim3(BS), 0, 0, dtr, dcoef, nt, log_len, fold, r, cin, cout, part,
                       ctr, mb_dev, ++seq, nullptr, 0);
  const int R = 20;
  hipEventRecord(e0, 0);
  for (int i = 0; i < R; i++)
    hipLaunchKernelGGL((Q ? k_layer_round_q<BS> : k_layer_round<BS>), dim3(K), dim3(BS), 0, 0, dtr, dcoef, nt, log_len, fold, r, cin, cout, part,
                       ctr, mb_dev, ++seq, nullptr, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // the prover's pattern: launch, spin on the mailbox, next launch
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < R; i++) {
    const uint32_t s = ++seq;
    hipLaunchKernelGGL((Q ? k_layer_round_q<BS> : k_layer_round<BS>), dim3(K), dim3(BS), 0, 0, dtr, dcoef, nt, log_len, fold, r, cin, cout, part,
                       ctr, mb_dev, s, nullptr, 0);
    while (__atomic_load_n(mb_host, __ATOMIC_ACQUIRE) != s) {
    }
  }
  const double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
  hipDeviceSynchronize();
  hipLaunchKernelGGL((Q ? k_layer_round_q<BS> : k_layer_round<BS>), dim3(K), dim3(BS), 0, 0, dtr, dcoef, nt, log_len, fold, r, cin, cout, part, ctr,
                     mb_dev, ++seq, probe, 0);
  hipDeviceSynchronize();
  unsigned long long p[8];
  hipMemcpy(p, probe, 64, hipMemcpyDeviceToHost);
  printf("%s nt=%2d len=%5d fold=%d K=%3u BS=%3d: event %.1f us/launch, launch+mailbox round trip %.1f us | block 0: "
         "elements %.2f, reduce %.2f, post %.2f us\n",
         Q ? "quad" : "lane", nt, 1 << log_len, fold, K, BS, ms * 1000 / R, rt, (p[1] - p[0]) * 0.01, (p[2] - p[1]) * 0.01,
         K == 1 ? (p[3] - p[2]) * 0.01 : 0.0);
}

// the paired launch (k_layer_pair) of rounds (len, len / 2) against the two single quad rounds it replaces
template <int BS>
static void run_pair(int nt, int log_len, int nf, Fq* cin, Fq* cout, Triple* dtr, Fq* dcoef, Fq* part, unsigned* ctr,
                     uint32_t* mb_dev, volatile uint32_t* mb_host, unsigned long long* probe) {
  PairArgs P;
  P.tr = dtr;
  P.coeff = dcoef;
  P.nt = nt;
  P.log_len = log_len;
  P.nf = nf;
  for (int i = 0; i < 8; i++) P.r1.l[i] = P.r2.l[i] = P.r12.l[i] = 0x01234567u * (i + 3);
  P.r1.l[7] = P.r2.l[7] = P.r12.l[7] = 0x01000000u;
  P.cin = cin;
  P.cout = cout;
  P.partials = part;
  P.counter = ctr;
  P.mb = mb_dev;
  P.ends = 0;
  P.probe = nullptr;
  const long lanes = 16L * nt * (1L << (log_len - 1));
  const unsigned K = (unsigned)((lanes + BS - 1) / BS);
  uint32_t seq = 70000;
  for (int w = 0; w < 3; w++) {
    P.seq = ++seq;
    hipLaunchKernelGGL(k_layer_pair<BS>, dim3(K), dim3(BS), 0, 0, P);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R = 20;
  hipEventRecord(e0, 0);
  for (int i = 0; i < R; i++) {
    P.seq = ++seq;
    hipLaunchKernelGGL(k_layer_pair<BS>, dim3(K), dim3(BS), 0, 0, P);
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < R; i++) {
    P.seq = ++seq;
    hipLaunchKernelGGL(k_layer_pair<BS>, dim3(K), dim3(BS), 0, 0, P);
    while (__atomic_load_n(mb_host, __ATOMIC_ACQUIRE) != P.seq) {
    }
  }
  const double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
  hipDeviceSynchronize();
  P.seq = ++seq;
  P.probe = probe;
  hipLaunchKernelGGL(k_layer_pair<BS>, dim3(K), dim3(BS), 0, 0, P);
  hipDeviceSynchronize();
  unsigned long long p[8];
  hipMemcpy(p, probe, 64, hipMemcpyDeviceToHost);
  printf("pair nt=%2d len=%5d nf=%d K=%4u BS=%3d: event %.1f us/launch, launch+mailbox round trip %.1f us | block 0: "
         "fold %.2f, points %.2f, reduce %.2f, post %.2f us\n",
         nt, 1 << log_len, nf, K, BS, ms * 1000 / R, rt, (p[1] - p[0]) * 0.01, (p[2] - p[1]) * 0.01,
         (p[3] - p[2]) * 0.01, K == 1 ? (p[4] - p[3]) * 0.01 : 0.0);
}

// the tripled launch (k_layer_triple) of rounds (len, len / 2, len / 4), the prover's workgroup choice
static void run_triple(int nt, int log_len, int nf, Fq* cin, Fq* cout, Triple* dtr, Fq* dcoef, Fq* part, unsigned* ctr,
                       uint32_t* mb_dev, volatile uint32_t* mb_host, unsigned long long* probe) {
  TripleArgs P;
  P.tr = dtr;
  P.coeff = dcoef;
  P.nt = nt;
  P.log_len = log_len;
  P.nf = nf;
  for (int i = 0; i < 8; i++) P.r1.l[i] = 0x01234567u * (i + 3);
  P.r1.l[7] = 0x01000000u;
  P.r2 = P.r3 = P.r12 = P.r13 = P.r23 = P.r123 = P.r1;
  P.cin = cin;
  P.cout = cout;
  P.partials = part;
  P.counter = ctr;
  P.mb = mb_dev;
  P.ends = 0;
  P.probe = nullptr;
  const long E = (long)nt << (log_len - 2);
  const int BS = E <= 1 ? 64 : 256;
  const unsigned K = (unsigned)((E + BS / 64 - 1) / (BS / 64));
  auto launch = [&]() {
    if (BS == 64)
      hipLaunchKernelGGL(k_layer_triple<64>, dim3(K), dim3(64), 0, 0, P);
    else
      hipLaunchKernelGGL(k_layer_triple<256>, dim3(K), dim3(256), 0, 0, P);
  };
  uint32_t seq = 90000;
  for (int w = 0; w < 3; w++) {
    P.seq = ++seq;
    launch();
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R = 20;
  hipEventRecord(e0, 0);
  for (int i = 0; i < R; i++) {
    P.seq = ++seq;
    launch();
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < R; i++) {
    P.seq = ++seq;
    launch();
    while (__atomic_load_n(mb_host, __ATOMIC_ACQUIRE) != P.seq) {
    }
  }
  const double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
  hipDeviceSynchronize();
  P.seq = ++seq;
  P.probe = probe;
  launch();
  hipDeviceSynchronize();
  unsigned long long p[8];
  hipMemcpy(p, probe, 64, hipMemcpyDeviceToHost);
  printf("triple nt=%2d len=%5d nf=%d K=%4u BS=%4d: event %.1f us/launch, launch+mailbox round trip %.1f us | block 0: "
         "fold %.2f, grid %.2f, products %.2f, post %.2f us\n",
         nt, 1 << log_len, nf, K, BS, ms * 1000 / R, rt, (p[1] - p[0]) * 0.01, (p[2] - p[1]) * 0.01,
         (p[3] - p[2]) * 0.01, K == 1 ? (p[4] - p[3]) * 0.01 : 0.0);
}

int main() {
  const int NT = 32, MAXL = 4096;
  Fq *vec, *cin, *cout, *dcoef, *part;
  Triple* dtr;
  hipMalloc(&vec, (size_t)NT * 2 * 4 * MAXL * sizeof(Fq));
  hipMalloc(&cin, 4 * MAXL * sizeof(Fq));
  hipMalloc(&cout, 4 * MAXL * sizeof(Fq));
  hipMalloc(&dcoef, NT * sizeof(Fq));
  hipMalloc(&part, 3 * 4096 * sizeof(Fq));
  hipMalloc(&dtr, NT * sizeof(Triple));
  hipMemset(vec, 0x11, (size_t)NT * 2 * 4 * MAXL * sizeof(Fq));
  hipMemset(cin, 0x05, 4 * MAXL * sizeof(Fq));
  hipMemset(dcoef, 0x03, NT * sizeof(Fq));
  std::vector<Triple> tr(NT);
  for (int c = 0; c < NT; c++) tr[c] = {vec + (size_t)c * 8 * MAXL, vec + (size_t)c * 8 * MAXL + 4 * MAXL, nullptr};
  hipMemcpy(dtr, tr.data(), NT * sizeof(Triple), hipMemcpyHostToDevice);
  unsigned* ctr;
  hipMalloc(&ctr, 64);
  hipMemset(ctr, 0, 64);
  void* mbh;
  uint32_t* mbd;
  hipHostMalloc(&mbh, 65536, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&mbd, mbh, 0);
  unsigned long long* probe;
  hipMalloc(&probe, 8 * 4096 * 8);
  void* dbh;
  uint32_t* dbd;
  hipHostMalloc(&dbh, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&dbd, dbh, 0);
  for (int rep = 0; rep < 2; rep++) {
    run_armed<64>(1, 0, cin, cout, dtr, dcoef, mbd, (volatile uint32_t*)mbh, dbd, (volatile uint32_t*)dbh);
    run_armed<256>(8, 3, cin, cout, dtr, dcoef, mbd, (volatile uint32_t*)mbh, dbd, (volatile uint32_t*)dbh);
    run_armed<256>(6, 5, cin, cout, dtr, dcoef, mbd, (volatile uint32_t*)mbh, dbd, (volatile uint32_t*)dbh);
  }
  if (getenv("ARMED_ONLY")) return 0;
  if (getenv("TRIPLE_ONLY")) {  // a triple against the pair at the same round j (len) and at len / 2
    const int shapes[][2] = {{24, 2}, {24, 3}, {24, 4}, {24, 5}, {24, 6}, {4, 2}, {4, 4}, {4, 6}, {4, 8}};
    for (auto& sh : shapes) {
      const int nt = sh[0], lg = sh[1];
      for (int nf = 1; nf <= 3; nf++)
        run_triple(nt, lg, nf, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
      for (int l = lg; l >= lg - 1 && l >= 1; l--) {
        if (16L * nt * (1L << (l - 1)) <= 64)
          run_pair<64>(nt, l, 2, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
        else
          run_pair<256>(nt, l, 2, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
      }
    }
    return 0;
  }
  if (getenv("PAIR_ONLY")) {
    const int shapes[][2] = {{24, 1}, {24, 2}, {24, 4}, {24, 6}, {24, 8}, {4, 1}, {4, 4}, {4, 8}, {4, 10}};
    for (auto& sh : shapes) {
      const int nt = sh[0], lg = sh[1];
      for (int nf = 1; nf <= 2; nf++) {
        if (16L * nt * (1L << (lg - 1)) <= 64)
          run_pair<64>(nt, lg, nf, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
        else
          run_pair<256>(nt, lg, nf, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
      }
      // the single quad rounds it replaces (fold = 1): len and len / 2, the prover's grid
      for (int l = lg; l >= lg - 1 && l >= 0; l--) {
        const long W = (long)nt << l;
        const unsigned K = (unsigned)std::min<long>((W * 4 + 255) / 256, 2048);
        if (W <= 16)
          run<64, true>(nt, l, 1, (unsigned)((W * 4 + 63) / 64), vec, cin, cout, dtr, dcoef, part, ctr, mbd,
                        (volatile uint32_t*)mbh, probe);
        else
          run<256, true>(nt, l, 1, K, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
      }
    }
    return 0;
  }
  for (int fold = 0; fold < 2; fold++) {
    run<64, true>(1, 0, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256, true>(8, 3, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256, true>(24, 4, fold, 6, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256, true>(24, 6, fold, 24, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256, true>(24, 8, fold, 96, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<64>(1, 0, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<64>(8, 3, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256>(24, 4, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256>(24, 6, fold, 1, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256>(24, 6, fold, 4, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256>(24, 8, fold, 12, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
    run<256>(24, 8, fold, 24, vec, cin, cout, dtr, dcoef, part, ctr, mbd, (volatile uint32_t*)mbh, probe);
  }
  return 0;
}
