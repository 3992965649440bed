// Does a small host-to-device hipMemcpyAsync from pageable memory return before the stream reaches it?
// A ~2 ms spin kernel is queued, then a 1 KB copy from pageable (std::vector) or page-locked memory; the host
// times the copy call itself. hipcc -O3 -std=c++17 --offload-arch=gfx950 -o pageable_copy pageable_copy.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <vector>

__global__ void k_spin(unsigned long long cycles, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) out[0] = 1;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* d;
  hipMalloc(&d, 1 << 20);
  std::vector<char> pageable(1 << 20, 1);
  void* pinned;
  hipHostMalloc(&pinned, 1 << 20);
  using clk = std::chrono::steady_clock;
  // wall_clock64 runs at 100 MHz on MI300/MI355X: 200000 ticks = 2 ms
  for (int rep = 0; rep < 3; rep++) {
    for (size_t bytes : {1024ul, 65536ul, 262144ul}) {
      for (int pin = 0; pin < 2; pin++) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000ull, d);
        auto t0 = clk::now();
        hipMemcpyAsync(d + 1024, pin ? pinned : (void*)pageable.data(), bytes, hipMemcpyHostToDevice, s);
        const double us_call = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        hipStreamSynchronize(s);
        const double us_all = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        printf("rep %d %7zu B %-8s: copy call %8.1f us, call + drain %8.1f us\n", rep, bytes, pin ? "pinned" : "pageable",
               us_call, us_all);
      }
    }
  }
  return 0;
}
