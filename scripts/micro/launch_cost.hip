// Microbenchmark: host-side cost of one kernel launch (time spent inside the launch call, back to back, 2000 launches
// between synchronisations) by launch API and kernel-argument size, and the device's back-to-back rate:
//   ggl_small   hipLaunchKernelGGL, 16 bytes of arguments
//   ggl_big     hipLaunchKernelGGL, a 1.7 KB struct argument (the R1CSProof evaluations' PqxArgs)
//   module_big  hipModuleLaunchKernel on the function handle (hipGetFuncBySymbol), the same 1.7 KB packed in `extra`
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o launch_cost launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

struct Big {
  unsigned w[432];  // 1728 bytes
};
__global__ void k_small(unsigned* out, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += v;
}
__global__ void k_big(unsigned* out, Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += b.w[431];
}
using clk = std::chrono::steady_clock;
int main() {
  unsigned* d;
  hipMalloc(&d, 64);
  hipMemset(d, 0, 64);
  Big b{};
  b.w[431] = 1;
  hipFunction_t fbig = nullptr;
  const bool have_mod = hipGetFuncBySymbol(&fbig, (const void*)k_big) == hipSuccess && fbig;
  const int N = 2000;
  for (int rep = 0; rep < 3; rep++) {
    double t[3] = {0, 0, 0};
    for (int m = 0; m < 3; m++) {
      if (m == 2 && !have_mod) continue;
      hipDeviceSynchronize();
      const auto t0 = clk::now();
      for (int i = 0; i < N; i++) {
        if (m == 0) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, 0, d, 1u);
        } else if (m == 1) {
          hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, 0, d, b);
        } else {
          struct {
            unsigned* out;
            Big b;
          } args{d, b};
          size_t sz = sizeof(args);
          void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
          hipModuleLaunchKernel(fbig, 1, 1, 1, 64, 1, 1, 0, 0, nullptr, extra);
        }
      }
      const double host = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      hipDeviceSynchronize();
      const double all = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      t[m] = host / N;
      printf("rep %d %-10s host %.2f us per launch, %.2f us per kernel incl. the device drain\n", rep,
             m == 0 ? "ggl_small" : (m == 1 ? "ggl_big" : "module_big"), host / N, all / N);
    }
  }
  unsigned h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("sum %u (module path %s)\n", h, have_mod ? "on" : "unavailable");
  return 0;
}
