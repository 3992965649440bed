// Device Fp / Fq arithmetic vs the host implementations of the same functions (bit-exact), random inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <random>

#include "../../spartan-parallel_amd/csrc/field.hpp"

using namespace spg;

__global__ void __launch_bounds__(256) k_ops(const Fp* a, const Fp* b, const Fq* qa, const Fq* qb, Fp* o, Fq* q, int n) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[4 * i] = fp_mul(a[i], b[i]);
  o[4 * i + 1] = fp_sqr(a[i]);
  o[4 * i + 2] = fp_add(a[i], b[i]);
  o[4 * i + 3] = fp_sub(a[i], b[i]);
  q[3 * i] = fq_mul(qa[i], qb[i]);
  q[3 * i + 1] = fq_add(qa[i], qb[i]);
  q[3 * i + 2] = fq_sub(qa[i], qb[i]);
}

int main() {
  const int n = 1 << 16;
  std::mt19937_64 rng(7);
  std::vector<Fp> a(n), b(n), o(4 * n);
  std::vector<Fq> qa(n), qb(n), q(3 * n);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 8; k++) {
      a[i].l[k] = (uint32_t)rng();
      b[i].l[k] = (uint32_t)rng();
      qa[i].l[k] = (uint32_t)rng();
      qb[i].l[k] = (uint32_t)rng();
    }
    if (i < 16) for (int k = 0; k < 8; k++) a[i].l[k] = b[i].l[k] = 0xffffffffu;  // carry extremes
    qa[i].l[7] &= 0x0fffffffu;  // canonical-ish (< q is not required for the identities below)
    qb[i].l[7] &= 0x0fffffffu;
  }
  Fp *da, *db, *dout;
  Fq *dqa, *dqb, *dq;
  hipMalloc(&da, n * sizeof(Fp)); hipMalloc(&db, n * sizeof(Fp)); hipMalloc(&dout, 4 * n * sizeof(Fp));
  hipMalloc(&dqa, n * sizeof(Fq)); hipMalloc(&dqb, n * sizeof(Fq)); hipMalloc(&dq, 3 * n * sizeof(Fq));
  hipMemcpy(da, a.data(), n * sizeof(Fp), hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * sizeof(Fp), hipMemcpyHostToDevice);
  hipMemcpy(dqa, qa.data(), n * sizeof(Fq), hipMemcpyHostToDevice);
  hipMemcpy(dqb, qb.data(), n * sizeof(Fq), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_ops, dim3(n / 256), dim3(256), 0, 0, da, db, dqa, dqb, dout, dq, n);
  hipMemcpy(o.data(), dout, 4 * n * sizeof(Fp), hipMemcpyDeviceToHost);
  hipMemcpy(q.data(), dq, 3 * n * sizeof(Fq), hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < n; i++) {
    Fp h[4] = {fp_mul(a[i], b[i]), fp_sqr(a[i]), fp_add(a[i], b[i]), fp_sub(a[i], b[i])};
    for (int k = 0; k < 4; k++)
      if (!fp_eq(h[k], o[4 * i + k])) { if (bad < 5) printf("fp op %d mismatch at %d\n", k, i); bad++; }
    Fq g[3] = {fq_mul(qa[i], qb[i]), fq_add(qa[i], qb[i]), fq_sub(qa[i], qb[i])};
    for (int k = 0; k < 3; k++)
      if (!fq_eq(g[k], q[3 * i + k])) { if (bad < 5) printf("fq op %d mismatch at %d\n", k, i); bad++; }
  }
  printf("%s: %ld mismatches over %d inputs\n", bad ? "FAIL" : "OK", bad, n);
  return bad ? 1 : 0;
}
