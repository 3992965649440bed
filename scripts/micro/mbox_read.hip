// Microbenchmark: how long the host takes to read n scalars a kernel posted into a mapped host page (the mailbox of
// every sumcheck round: the round's sums, and at a layer's end every vector's entries), by page type and read method.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o mbox_read mbox_read.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <chrono>

__global__ void k_post(uint32_t* mb, uint32_t seq, int n) {
  for (int i = threadIdx.x; i < 8 * n; i += blockDim.x)
    __hip_atomic_store(mb + 8 + i, (uint32_t)(i * 2654435761u + seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;

int main() {
  const unsigned flags[3] = {hipHostMallocCoherent | hipHostMallocMapped, hipHostMallocMapped,
                             hipHostMallocNonCoherent | hipHostMallocMapped};
  const char* fname[3] = {"coherent", "default", "noncoherent"};
  static uint32_t out[8 * 4096];
  for (int f = 0; f < 3; f++) {
    void* h;
    uint32_t* d;
    if (hipHostMalloc(&h, 1 << 20, flags[f]) != hipSuccess) {
      printf("%s: alloc failed\n", fname[f]);
      continue;
    }
    hipHostGetDevicePointer((void**)&d, h, 0);
    volatile uint32_t* mb = (volatile uint32_t*)h;
    memset(h, 0, 1 << 20);
    uint32_t seq = 1;
    for (int n : {3, 15, 147, 303, 1024}) {
      double t[3] = {0, 0, 0};
      const int R = 50;
      for (int r = 0; r < R; r++)
        for (int m = 0; m < 3; m++) {
          ++seq;
          hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, 0, d, seq, n);
          while (__atomic_load_n(mb, __ATOMIC_ACQUIRE) != seq) {
          }
          const auto t0 = clk::now();
          if (m == 0) {
            for (int i = 0; i < 8 * n; i++) out[i] = mb[8 + i];
          } else if (m == 1) {
            memcpy(out, (const void*)(mb + 8), 32 * (size_t)n);
          } else {
            const uint8_t* s = (const uint8_t*)(mb + 8);
            for (size_t o = 0; o < 32 * (size_t)n; o += 64) __builtin_prefetch(s + o, 0, 0);
            memcpy(out, s, 32 * (size_t)n);
          }
          t[m] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
          hipDeviceSynchronize();
        }
      printf("%-11s n=%4d scalars: volatile words %.2f us, memcpy %.2f us, prefetch+memcpy %.2f us\n", fname[f], n,
             t[0] / R, t[1] / R, t[2] / R);
    }
    hipHostFree(h);
  }
  return 0;
}
