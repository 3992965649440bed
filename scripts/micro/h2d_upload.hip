// Microbenchmark: host-to-device upload of a caller's pageable buffer (a 134 MB witness), every
// strategy against the same destination:
//   pageable   one hipMemcpyAsync from the pageable buffer (HIP stages it internally), stream synchronised
//   register   hipHostRegister + hipMemcpyAsync + hipHostUnregister (the registration is part of the time)
//   ring T     T host threads; thread k copies chunks k, k + T, .. of CH bytes into its own two page-locked slots
//              and DMAs each on its own stream (slot reuse waits on the slot's event)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/micro/h2d_upload scripts/micro/h2d_upload.hip -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Lane {
  hipStream_t s;
  void* slot[2];
  hipEvent_t ev[2];
  bool used[2] = {false, false};
};

static double ring(const uint8_t* src, uint8_t* dst, size_t bytes, std::vector<Lane>& lanes, size_t CH) {
  const int T = (int)lanes.size();
  const double t0 = now();
  std::vector<std::thread> th;
  for (int k = 0; k < T; k++)
    th.emplace_back([&, k] {
      Lane& L = lanes[k];
      int u = 0;
      for (size_t c = k; c * CH < bytes; c += T) {
        const size_t off = c * CH, len = std::min(CH, bytes - off);
        if (L.used[u]) hipEventSynchronize(L.ev[u]);
        memcpy(L.slot[u], src + off, len);
        hipMemcpyAsync(dst + off, L.slot[u], len, hipMemcpyHostToDevice, L.s);
        hipEventRecord(L.ev[u], L.s);
        L.used[u] = true;
        u ^= 1;
      }
      hipStreamSynchronize(L.s);
    });
  for (auto& t : th) t.join();
  return now() - t0;
}

int main() {
  const size_t bytes = (size_t)134217728;
  std::vector<uint8_t> host(bytes);
  for (size_t i = 0; i < bytes; i++) host[i] = (uint8_t)(i * 2654435761u >> 13);
  uint8_t* dst;
  hipMalloc(&dst, bytes);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int rep = 0; rep < 3; rep++) {
    {
      const double t0 = now();
      hipMemcpyAsync(dst, host.data(), bytes, hipMemcpyHostToDevice, s);
      hipStreamSynchronize(s);
      const double dt = now() - t0;
      printf("pageable           %.3f ms  %.1f GB/s\n", dt * 1e3, bytes / dt / 1e9);
    }
    {
      const double t0 = now();
      hipHostRegister(host.data(), bytes, hipHostRegisterDefault);
      const double t1 = now();
      hipMemcpyAsync(dst, host.data(), bytes, hipMemcpyHostToDevice, s);
      hipStreamSynchronize(s);
      const double t2 = now();
      hipHostUnregister(host.data());
      const double t3 = now();
      printf("register           %.3f ms (register %.3f, copy %.3f = %.1f GB/s, unregister %.3f)\n", (t3 - t0) * 1e3,
             (t1 - t0) * 1e3, (t2 - t1) * 1e3, bytes / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
    }
    for (size_t CH : {(size_t)2 << 20, (size_t)4 << 20, (size_t)8 << 20})
      for (int T : {1, 2, 4, 8, 12, 16}) {
        std::vector<Lane> lanes(T);
        for (auto& L : lanes) {
          hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking);
          for (int u = 0; u < 2; u++) {
            hipHostMalloc(&L.slot[u], CH);
            memset(L.slot[u], 0, CH);
            hipEventCreateWithFlags(&L.ev[u], hipEventDisableTiming);
          }
        }
        ring(host.data(), dst, bytes, lanes, CH);  // warm
        const double dt = ring(host.data(), dst, bytes, lanes, CH);
        printf("ring T=%2d CH=%zu MB  %.3f ms  %.1f GB/s\n", T, CH >> 20, dt * 1e3, bytes / dt / 1e9);
        for (auto& L : lanes) {
          for (int u = 0; u < 2; u++) {
            hipHostFree(L.slot[u]);
            hipEventDestroy(L.ev[u]);
          }
          hipStreamDestroy(L.s);
        }
      }
  }
  // verify the last upload
  std::vector<uint8_t> back(bytes);
  hipMemcpy(back.data(), dst, bytes, hipMemcpyDeviceToHost);
  printf("verify %s\n", memcmp(back.data(), host.data(), bytes) ? "MISMATCH" : "ok");
  return 0;
}
