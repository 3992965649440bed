// Microbenchmark: dependent-chain latency (shader clock cycles) of the device field / curve primitives,
// one wave, one primitive per kernel instantiation.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../spartan-parallel_amd/csrc/curve.hpp"
#include "../../spartan-parallel_amd/csrc/quad.hpp"

using namespace spg;

template <int W>
__global__ void __launch_bounds__(64) k_lat(const Fp* in, Fp* out, long long* cyc, int iters) {
  Fp a = in[threadIdx.x], b = in[threadIdx.x + 64];
  Fq qa, qb;
  for (int i = 0; i < 8; i++) {
    qa.l[i] = a.l[i] & 0x0fffffffu;
    qb.l[i] = b.l[i] & 0x0fffffffu;
  }
  Ext P = niels_to_ext(Niels{a, b, a});
  Niels N{b, a, b};
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if (W == 0) a = fp_mul(a, b);
    if (W == 1) a = fp_sqr(a);
    if (W == 2) P = ext_add(P, P);
    if (W == 3) P = ext_madd(P, N, false);
    if (W == 4) qa = fq_mul(qa, qb);
    if (W == 5) a = fp_add(a, b);
    if (W == 6) qa = fq_add(qa, qb);
    if (W == 7) P = quad_add(P, P, threadIdx.x & 3);
    if (W == 8) P = quad_madd(P, b, (i & 1) != 0, threadIdx.x & 3);
    if (W == 9) P = quad_dbl(P, threadIdx.x & 3);
    if (W == 10) a = fp_sub(a, b);
  }
  long long t1 = clock64();
  Fp q{{qa.l[0], qa.l[1], qa.l[2], qa.l[3], qa.l[4], qa.l[5], qa.l[6], qa.l[7]}};
  out[threadIdx.x] = fp_add(fp_add(a, P.X), q);
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / iters;
}

template <int W>
long long run(Fp* in, Fp* out, long long* cyc) {
  long long c = 0;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lat<W>, dim3(1), dim3(64), 0, 0, in, out, cyc, 4000);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  }
  return c;
}

int main() {
  Fp *in, *out;
  long long* cyc;
  hipMalloc(&in, 128 * sizeof(Fp));
  hipMalloc(&out, 128 * sizeof(Fp));
  hipMalloc(&cyc, 8);
  hipMemset(in, 0x35, 128 * sizeof(Fp));
  printf("fp_mul   %lld\n", run<0>(in, out, cyc));
  printf("fp_sqr   %lld\n", run<1>(in, out, cyc));
  printf("ext_add  %lld\n", run<2>(in, out, cyc));
  printf("ext_madd %lld\n", run<3>(in, out, cyc));
  printf("fq_mul   %lld\n", run<4>(in, out, cyc));
  printf("fp_add   %lld\n", run<5>(in, out, cyc));
  printf("fq_add   %lld\n", run<6>(in, out, cyc));
  printf("quad_add %lld\n", run<7>(in, out, cyc));
  printf("quad_madd %lld\n", run<8>(in, out, cyc));
  printf("quad_dbl %lld\n", run<9>(in, out, cyc));
  printf("fp_sub   %lld\n", run<10>(in, out, cyc));
  printf("(cycles per dependent op, one wave)\n");
  return 0;
}
