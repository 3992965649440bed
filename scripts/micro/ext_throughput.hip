// Microbenchmark: whole-GPU throughput of the device curve additions (ext_add, ext_madd) and Fp multiply
// as a function of resident waves per SIMD. Each lane runs an independent dependent chain; blocks of 256
// threads (one wave per SIMD of a CU), `bpc` blocks per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../spartan-parallel_amd/csrc/curve.hpp"
#include "../../spartan-parallel_amd/csrc/quad.hpp"

using namespace spg;

template <int W>
__global__ void __launch_bounds__(256) k_thr(const Fp* in, Fp* out, int iters) {
  const int t = threadIdx.x & 63;
  Fp a = in[t], b = in[t + 64];
  Ext P = niels_to_ext(Niels{a, b, a});
  Niels N{b, a, b};
  for (int i = 0; i < iters; i++) {
    if (W == 0) a = fp_mul(a, b);
    if (W == 1) P = ext_add(P, P);
    if (W == 2) P = ext_madd(P, N, false);
    if (W == 3) P = quad_madd(P, b, false, t & 3);  // 4 lanes per point: ops counted per quad below
  }
  out[blockIdx.x * 256 + threadIdx.x] = fp_add(a, P.X);
}

template <int W>
void run(const char* name, Fp* in, Fp* out, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 200;
  for (int bpc : {1, 2, 3, 4, 8}) {
    const int blocks = ncu * bpc;
    hipLaunchKernelGGL(k_thr<W>, dim3(blocks), dim3(256), 0, 0, in, out, 4);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_thr<W>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * 256 * iters / (W == 3 ? 4 : 1);
    printf("%-8s blocks/CU=%d  %.3f ms  %.3e ops/s  %.2f us per dependent op\n", name, bpc, ms, ops / (ms * 1e-3),
           ms * 1e3 / iters);
  }
}

int main() {
  Fp *in, *out;
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipMalloc(&in, 128 * sizeof(Fp));
  hipMalloc(&out, (size_t)ncu * 8 * 256 * sizeof(Fp));
  hipMemset(in, 0x35, 128 * sizeof(Fp));
  printf("CUs: %d\n", ncu);
  run<0>("fp_mul", in, out, ncu);
  run<1>("ext_add", in, out, ncu);
  run<2>("ext_madd", in, out, ncu);
  run<3>("quad_madd", in, out, ncu);
  return 0;
}
