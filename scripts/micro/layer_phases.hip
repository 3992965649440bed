// Microbenchmark: one fused SPARK layer-sumcheck round (k_layer_round, csrc/layer.hpp) at the prover's sizes.
// Random field data (timing only). Per (triples, len, fold): HIP-event time per launch (back to back, and
// with a host mailbox wait per launch as the prover does), and the kernel's own wall_clock64 phases:
// elements (loads, fold, products), block reduction, mailbox post (host-mapped, system scope).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../spartan-parallel_amd/csrc/layer.hpp"

using namespace spg;

namespace spg {
int set_err(spg_ctx*, int code, const std::string&) { return code; }
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
