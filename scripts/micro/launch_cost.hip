// Host-side cost of the HIP calls a prove issues ~900 times: an async kernel launch (small / 2 KB arguments), with
// hipGetLastError, hipMemcpyAsync of 64 B (pinned / pageable, H2D), hipEventRecord. Host microseconds per call,
// measured over back-to-back calls on one stream (the device runs empty kernels meanwhile).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -o launch_cost launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <vector>

struct Blob {
  unsigned w[512];
};
__global__ void k_small(unsigned* p, unsigned x) {
  if (threadIdx.x == 0 && x == 0xffffffffu) p[0] = x;
}
__global__ void k_blob(unsigned* p, Blob b) {
  if (threadIdx.x == 0 && b.w[7] == 0xffffffffu) p[0] = b.w[0];
}

using clk = std::chrono::steady_clock;
template <class F>
double us_per(int n, hipStream_t s, F f) {
  hipStreamSynchronize(s);
  auto t0 = clk::now();
  for (int i = 0; i < n; i++) f(i);
  const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
  hipStreamSynchronize(s);
  return us;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  unsigned* d;
  hipMalloc(&d, 1 << 20);
  void* pin;
  hipHostMalloc(&pin, 4096);
  std::vector<char> page(4096);
  hipEvent_t e;
  hipEventCreate(&e);
  Blob b{};
  for (int rep = 0; rep < 2; rep++) {
    const int N = 2000;
    printf("launch small args       %.2f us\n", us_per(N, s, [&](int i) { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d, (unsigned)i); }));
    printf("launch 2 KB args        %.2f us\n", us_per(N, s, [&](int i) { b.w[1] = i; hipLaunchKernelGGL(k_blob, dim3(1), dim3(64), 0, s, d, b); }));
    printf("launch small + lasterr  %.2f us\n", us_per(N, s, [&](int i) { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d, (unsigned)i); (void)hipGetLastError(); }));
    printf("launch 1024 blocks      %.2f us\n", us_per(N, s, [&](int i) { hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, s, d, (unsigned)i); }));
    printf("memcpyAsync 64B pinned  %.2f us\n", us_per(N, s, [&](int i) { (void)hipMemcpyAsync(d + 64, pin, 64, hipMemcpyHostToDevice, s); }));
    printf("memcpyAsync 64B pageable %.2f us\n", us_per(N, s, [&](int i) { (void)hipMemcpyAsync(d + 64, page.data(), 64, hipMemcpyHostToDevice, s); }));
    printf("memcpyAsync D2D 4KB     %.2f us\n", us_per(N, s, [&](int i) { (void)hipMemcpyAsync(d + 4096, d, 4096, hipMemcpyDeviceToDevice, s); }));
    printf("eventRecord             %.2f us\n", us_per(N, s, [&](int i) { (void)hipEventRecord(e, s); }));
    printf("launch + streamSync     %.2f us\n", us_per(500, s, [&](int i) { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d, (unsigned)i); (void)hipStreamSynchronize(s); }));
    printf("streamQuery (idle)      %.2f us\n", us_per(N, s, [&](int i) { (void)hipStreamQuery(s); }));
  }
  return 0;
}
