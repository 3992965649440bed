// Microbenchmark: launch -> host-visible round trip of a kernel that posts n scalars (32 B each) and then a sequence
// number into the coherent mapped mailbox page, by store pattern:
//   lane_words   lane s writes scalar s as 8 separate 4-byte system-scope stores (one lane per scalar: the prover's
//                mbox_post3 / corner posts)
//   coalesced    lane t writes 4-byte word t of the payload (consecutive lanes, consecutive words), staged through LDS
//   x4           lane t writes 16-byte chunk t (dwordx4) of the payload, staged through LDS
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o mbox_post mbox_post.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <chrono>

typedef __attribute__((address_space(1))) uint32_t gu32;

__global__ void __launch_bounds__(256) k_post(uint32_t* mb, uint32_t seq, int n, int mode) {
  __shared__ uint32_t st[8 * 1024];
  const int t = threadIdx.x;
  // every lane s < n holds scalar s
  uint32_t v[8];
  for (int i = 0; i < 8; i++) v[i] = (uint32_t)(t * 2654435761u + i + seq);
  if (mode == 0) {
    for (int s = t; s < n; s += 256)
      for (int i = 0; i < 8; i++) __hip_atomic_store(mb + 8 + 8 * s + i, v[i] + s - t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    for (int s = t; s < n; s += 256)
      for (int i = 0; i < 8; i++) st[8 * s + i] = v[i] + s - t;
    __syncthreads();
    if (mode == 1) {
      for (int w = t; w < 8 * n; w += 256) __hip_atomic_store(mb + 8 + w, st[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      for (int c = t; c < 2 * n; c += 256) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 x = {st[4 * c], st[4 * c + 1], st[4 * c + 2], st[4 * c + 3]};
        ((u32x4*)(mb + 8))[c] = x;  // plain 16-byte stores; the system-scope release below makes them visible
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (t == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bullet-parts pattern: n points of 128 B (extended coordinates), written by every 4th lane (a quad's lane 0) with a
// plain struct store (mode 0), or staged in LDS and written as consecutive 16-byte chunks (mode 1); then the system
// release and the sequence number, as k_bullet_comb's ticket does
struct P128 {
  uint32_t w[32];
};
__global__ void __launch_bounds__(256) k_parts(uint32_t* mb, P128* parts, uint32_t seq, int n, int mode) {
  __shared__ uint32_t st[32 * 256];
  const int t = threadIdx.x;
  P128 v;
  for (int i = 0; i < 32; i++) v.w[i] = (uint32_t)(t * 7 + i + seq);
  if (mode == 0) {
    for (int s = t; s < 4 * n; s += 256)
      if ((s & 3) == 0) parts[s >> 2] = v;
  } else {
    for (int s = t; s < 4 * n; s += 256)
      if ((s & 3) == 0)
        for (int i = 0; i < 32; i++) st[32 * (s >> 2) + i] = v.w[i];
    __syncthreads();
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    for (int c = t; c < 8 * n; c += 256) {
      u32x4 x = {st[4 * c], st[4 * c + 1], st[4 * c + 2], st[4 * c + 3]};
      ((u32x4*)parts)[c] = x;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (t == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;

int main() {
  void* h;
  uint32_t* d;
  hipHostMalloc(&h, 1 << 20, hipHostMallocCoherent | hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&d, h, 0);
  volatile uint32_t* mb = (volatile uint32_t*)h;
  memset(h, 0, 1 << 20);
  uint32_t seq = 1;
  const char* names[3] = {"lane_words", "coalesced", "x4"};
  for (int rep = 0; rep < 2; rep++)
    for (int n : {0, 3, 15, 147, 303}) {
      double t[3] = {0, 0, 0};
      const int R = 200;
      bool ok = true;
      for (int r = 0; r < R; r++)
        for (int m = 0; m < 3; m++) {
          ++seq;
          const auto t0 = clk::now();
          hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, 0, d, seq, n, m);
          while (__atomic_load_n(mb, __ATOMIC_ACQUIRE) != seq) {
          }
          t[m] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
          // check the payload
          const uint32_t* p = (const uint32_t*)h + 8;
          for (int s = 0; s < n && ok; s++)
            for (int i = 0; i < 8; i++)
              if (p[8 * s + i] != (uint32_t)(s * 2654435761u + i + seq)) ok = false;
          hipDeviceSynchronize();
        }
      printf("rep %d n=%4d scalars: launch->seen %s %.2f us, %s %.2f us, %s %.2f us%s\n", rep, n, names[0], t[0] / R,
             names[1], t[1] / R, names[2], t[2] / R, ok ? "" : "  PAYLOAD MISMATCH");
    }
  P128* parts = (P128*)((uint8_t*)h + 65536);
  P128* dparts = (P128*)((uint8_t*)d + 65536);
  for (int n : {8, 16, 64}) {
    double t[2] = {0, 0};
    const int R = 200;
    for (int r = 0; r < R; r++)
      for (int m = 0; m < 2; m++) {
        ++seq;
        const auto t0 = clk::now();
        hipLaunchKernelGGL(k_parts, dim3(1), dim3(256), 0, 0, d, dparts, seq, n, m);
        while (__atomic_load_n(mb, __ATOMIC_ACQUIRE) != seq) {
        }
        t[m] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        hipDeviceSynchronize();
      }
    printf("parts n=%3d points: launch->seen struct stores %.2f us, coalesced 16B chunks %.2f us\n", n, t[0] / R, t[1] / R);
  }
  (void)parts;
  return 0;
}
