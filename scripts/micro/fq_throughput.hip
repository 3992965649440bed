// Microbenchmark: whole-GPU throughput of the device Fq (scalar field, Montgomery) product fq_mul (product scanning,
// csrc/field.hpp) -- the peak the Fq-product-bound kernels (R1CSProof sumcheck evaluations, SPARK layer rounds) are
// priced against (bench.py FQ_PEAK, `roofline_fq`). Each lane runs `ilp` independent dependent chains; 256-thread
// blocks, `bpc` blocks per CU. Also the multiply-accumulate form acc += a b (one fq_mul + one fq_add).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o fq_throughput fq_throughput.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../spartan-parallel_amd/csrc/field.hpp"

using namespace spg;

template <int ILP, bool MAC>
__global__ void __launch_bounds__(256) k_fq(const Fq* in, Fq* out, int iters) {
  const int t = threadIdx.x & 63;
  Fq a[ILP], acc[ILP];
  const Fq b = in[t + 64];
#pragma unroll
  for (int j = 0; j < ILP; j++) {
    a[j] = in[(t + j) & 63];
    acc[j] = fq_zero();
  }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < ILP; j++) {
      if (MAC) {
        acc[j] = fq_add(acc[j], fq_mul(a[j], b));
        a[j] = acc[j];
      } else {
        a[j] = fq_mul(a[j], b);
      }
    }
  }
  Fq r = fq_zero();
#pragma unroll
  for (int j = 0; j < ILP; j++) r = fq_add(r, a[j]);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int ILP, bool MAC>
void run(const char* name, Fq* in, Fq* out, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 400;
  for (int bpc : {1, 2, 4, 8}) {
    const int blocks = ncu * bpc;
    hipLaunchKernelGGL((k_fq<ILP, MAC>), dim3(blocks), dim3(256), 0, 0, in, out, 4);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_fq<ILP, MAC>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * 256 * iters * ILP;
    printf("%-10s ilp=%d blocks/CU=%d  %.3f ms  %.3e Fq products/s  %.0f ns per dependent product\n", name, ILP, bpc,
           ms, ops / (ms * 1e-3), ms * 1e6 / iters / ILP * (ILP > 1 ? ILP : 1));
  }
}

int main() {
  Fq *in, *out;
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipMalloc(&in, 128 * sizeof(Fq));
  hipMalloc(&out, (size_t)ncu * 8 * 256 * sizeof(Fq));
  hipMemset(in, 0x05, 128 * sizeof(Fq));
  printf("CUs: %d\n", ncu);
  run<1, false>("fq_mul", in, out, ncu);
  run<2, false>("fq_mul", in, out, ncu);
  run<4, false>("fq_mul", in, out, ncu);
  run<1, true>("fq_mul_add", in, out, ncu);
  run<2, true>("fq_mul_add", in, out, ncu);
  return 0;
}
