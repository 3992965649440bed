// spg — context management for the C-ABI (include/spg.h).
#include <stdio.h>

#include "ctx.hpp"

namespace spg {

int set_err(spg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

void* ws_get(spg_ctx* c, size_t slot, size_t bytes) {
  if (c->ws.size() <= slot) c->ws.resize(slot + 1);
  spg_ctx::Slot& s = c->ws[slot];
  if (s.bytes >= bytes && s.p) return s.p;
  if (s.p) {
    hipStreamSynchronize(c->stream);
    hipFree(s.p);
    s.p = nullptr;
    s.bytes = 0;
  }
  size_t want = bytes < 256 ? 256 : bytes;
  want += want / 4;  // headroom so repeated slightly-larger calls do not reallocate
  if (hipMalloc(&s.p, want) != hipSuccess) {
    s.p = nullptr;
    return nullptr;
  }
  s.bytes = want;
  return s.p;
}

void timer_start(spg_ctx* c) { hipEventRecord(c->ev0, c->stream); }
void timer_stop(spg_ctx* c) { hipEventRecord(c->ev1, c->stream); }

}  // namespace spg

extern "C" int spg_init(int device, spg_ctx** out) {
  if (!out) return SPG_E_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return SPG_E_NODEVICE;
  if (device < 0 || device >= count) return SPG_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SPG_E_NODEVICE;
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) return SPG_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return SPG_E_HIP;
  spg_ctx* c = new spg_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    delete c;
    return SPG_E_HIP;
  }
  *out = c;
  return SPG_OK;
}

extern "C" int spg_free(spg_ctx* c) {
  if (!c) return SPG_OK;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto& s : c->ws)
    if (s.p) hipFree(s.p);
  hipEventDestroy(c->ev0);
  hipEventDestroy(c->ev1);
  hipStreamDestroy(c->stream);
  delete c;
  return SPG_OK;
}

extern "C" const char* spg_last_error(const spg_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" double spg_last_kernel_us(const spg_ctx* c) { return c ? c->last_us : 0.0; }
