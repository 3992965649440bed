// spg — bank-conflict-free LDS staging for block reductions and scans of multi-word values.
// A 128-byte Ext (or 32-byte Fq) stored as an array of structs puts lane t at bank (32 t) mod 64 (or 8 t), so
// every ds_write/ds_read of a wave serialises 16-32 ways. Stored component-major (word k of lane t at
// s[k * BS + t]) consecutive lanes hit consecutive banks.
#pragma once
#include <hip/hip_runtime.h>

namespace spg {

template <int BS, class T>
__device__ __forceinline__ void soa_put(uint32_t* s, int t, const T& v) {
  static_assert(sizeof(T) % 4 == 0, "word-sized components");
  const uint32_t* p = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) s[k * BS + t] = p[k];
}
template <int BS, class T>
__device__ __forceinline__ T soa_get(const uint32_t* s, int t) {
  T v;
  uint32_t* p = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) p[k] = s[k * BS + t];
  return v;
}
// words of one BS-lane SoA buffer of T
template <class T, int BS>
constexpr int soa_words() {
  return (int)(sizeof(T) / 4) * BS;
}

}  // namespace spg
