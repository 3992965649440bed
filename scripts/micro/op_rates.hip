// Microbenchmark: cycles per instruction of the candidate multiply primitives for field arithmetic on gfx950
// (one wave, 8 independent chains, so the figure is the issue cost, not the dependent latency).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int OP>
__global__ void __launch_bounds__(64) k_rate(const uint64_t* in, uint64_t* out, long long* cyc, int iters) {
  uint64_t a[8];
  double d[8];
  uint32_t u[8];
  for (int j = 0; j < 8; j++) {
    a[j] = in[threadIdx.x + j];
    d[j] = (double)(a[j] & 0xfffffffffffffull);
    u[j] = (uint32_t)a[j];
  }
  const uint32_t m = (uint32_t)in[100];
  const double dm = (double)(in[101] & 0xfffffffffffffull);
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) a[j] = (uint64_t)(uint32_t)a[j] * m + (a[j] >> 32);  // v_mad_u64_u32
      if (OP == 1) d[j] = __builtin_fma(d[j], dm, d[j]);                 // v_fma_f64
      if (OP == 2) u[j] = u[j] * m + u[j];                              // v_mul_lo_u32 + add
      if (OP == 3) u[j] = __umul24(u[j], m) + u[j];        // v_mad_u32_u24
      if (OP == 4) u[j] = __umulhi(u[j], m) + u[j];                     // v_mul_hi_u32 + add
      if (OP == 5) u[j] = (u[j] + m) ^ (u[j] >> 1);                     // plain 32-bit ALU (2 ops)
    }
  }
  long long t1 = clock64();
  uint64_t s = 0;
  for (int j = 0; j < 8; j++) s += a[j] + (uint64_t)d[j] + u[j];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = (t1 - t0);
}

template <int OP>
double run(uint64_t* in, uint64_t* out, long long* cyc) {
  long long c = 0;
  const int iters = 2000;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_rate<OP>, dim3(1), dim3(64), 0, 0, in, out, cyc, iters);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  }
  return (double)c / (iters * 8.0);
}

int main() {
  uint64_t *in, *out;
  long long* cyc;
  hipMalloc(&in, 256 * 8);
  hipMalloc(&out, 256 * 8);
  hipMalloc(&cyc, 8);
  hipMemset(in, 0x35, 256 * 8);
  printf("v_mad_u64_u32          %.2f cycles/op\n", run<0>(in, out, cyc));
  printf("v_fma_f64              %.2f cycles/op\n", run<1>(in, out, cyc));
  printf("v_mul_lo_u32 + add     %.2f cycles/op\n", run<2>(in, out, cyc));
  printf("v_mad_u32_u24          %.2f cycles/op\n", run<3>(in, out, cyc));
  printf("v_mul_hi_u32 + add     %.2f cycles/op\n", run<4>(in, out, cyc));
  printf("2 x 32-bit ALU         %.2f cycles/op\n", run<5>(in, out, cyc));
  return 0;
}
