// Shared helpers for the libmanette_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>

#include "../../include/manette_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace mt {

void set_error(const char *fmt, ...);

#define MT_CHECK_ARG(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::mt::set_error(__VA_ARGS__);      \
      return MT_ERR_ARG;                 \
    }                                    \
  } while (0)

#define MT_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ::mt::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                      \
      return MT_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

// Check the launch that was just issued.
#define MT_LAUNCHED() MT_HIP(hipGetLastError())

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// Wave-wide (64 lanes) sum via butterfly shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace mt
