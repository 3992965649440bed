// Microbenchmark: host <-> device hand-off latency of one sumcheck-style round, two ways.
//  launch:  the host launches a one-workgroup kernel that posts a sequence number to a coherent mapped host page;
//           the host spins on it (what every libspg round does today)
//  resident: one workgroup stays resident and loops: post a number, spin (bounded) on a host-written reply page,
//           repeat; the host spins on the number and replies
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o pingpong pingpong.hip ; optional argv[1] = CPU to pin the host to
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

__global__ void k_post(uint32_t* mb, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// posts 1..n, waits for the host's echo of each; leaves on a stop word or after ~1 s without a reply
__global__ void k_resident(uint32_t* mb, const uint32_t* db, int n, int sleep) {
  __shared__ int stop;
  for (int j = 1; j <= n; j++) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(mb, (uint32_t)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned long long t0 = wall_clock64();
      int st = 0;
      while (__hip_atomic_load(db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint32_t)j) {
        if (__hip_atomic_load(db + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || wall_clock64() - t0 > 100000000ull) {
          st = 1;
          break;
        }
        if (sleep) __builtin_amdgcn_s_sleep(1);
      }
      stop = st;
    }
    __syncthreads();
    if (stop) return;
  }
}

int main(int argc, char** argv) {
  if (argc > 1) {
    cpu_set_t s;
    CPU_ZERO(&s);
    CPU_SET(atoi(argv[1]), &s);
    pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
  }
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  void *mb, *db;
  uint32_t *dmb, *ddb;
  hipHostMalloc(&mb, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostMalloc(&db, 4096, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&dmb, mb, 0);
  hipHostGetDevicePointer((void**)&ddb, db, 0);
  volatile uint32_t* hm = (volatile uint32_t*)mb;
  volatile uint32_t* hd = (volatile uint32_t*)db;
  const int N = 2000;
  using clk = std::chrono::steady_clock;
  for (int rep = 0; rep < 2; rep++) {
    hm[0] = 0;
    hipLaunchKernelGGL(k_post, dim3(1), dim3(64), 0, st, dmb, 0u);
    hipStreamSynchronize(st);
    auto t0 = clk::now();
    for (int j = 1; j <= N; j++) {
      hipLaunchKernelGGL(k_post, dim3(1), dim3(64), 0, st, dmb, (uint32_t)j);
      while (__atomic_load_n(hm, __ATOMIC_ACQUIRE) != (uint32_t)j) {
      }
    }
    const double us_launch = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
    for (int sl = 0; sl < 2; sl++) {
      hm[0] = 0;
      hd[0] = 0;
      hd[1] = 0;
      hipLaunchKernelGGL(k_resident, dim3(1), dim3(256), 0, st, dmb, ddb, N, sl);
      t0 = clk::now();
      for (int j = 1; j <= N; j++) {
        auto tw = clk::now();
        while (__atomic_load_n(hm, __ATOMIC_ACQUIRE) != (uint32_t)j) {
          if (clk::now() - tw > std::chrono::seconds(2)) {
            hd[1] = 1;
            printf("resident loop timed out at %d\n", j);
            hipStreamSynchronize(st);
            return 1;
          }
        }
        __atomic_store_n(hd, (uint32_t)j, __ATOMIC_RELEASE);
      }
      const double us_res = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
      hipStreamSynchronize(st);
      printf("rep %d: launch + mailbox %.2f us/round; resident loop (s_sleep %d) %.2f us/round\n", rep, us_launch, sl,
             us_res);
    }
  }
  return 0;
}
