// Shared device/host helpers for libyanerf_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/yanerf_hip.h"

namespace yanerf {

// ------------------------------------------------------------------------------------------ errors
void set_error(const char* fmt, ...);
#define YN_CHECK(cond, ...)                \
  do {                                     \
    if (!(cond)) {                         \
      ::yanerf::set_error(__VA_ARGS__);    \
      return 1;                            \
    }                                      \
  } while (0)
#define YN_LAUNCH_CHECK(name)                                                          \
  do {                                                                                 \
    hipError_t _e = hipGetLastError();                                                 \
    YN_CHECK(_e == hipSuccess, "%s launch failed: %s", name, hipGetErrorString(_e));   \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------------------------------ types
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short us4 __attribute__((ext_vector_type(4)));
typedef unsigned short us8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short f2bf(float x) {
  // round-to-nearest-even (NaN stays NaN via the hardware cast)
  __bf16 b = (__bf16)x;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __builtin_bit_cast(float, ((unsigned int)h) << 16);
}

// ------------------------------------------------------------------------------------------ Philox
// Philox4x32-10 (Salmon et al., SC'11). Counter-based: stream element (seed, offset, idx) -> 4 uint32.
struct u4 { uint32_t x, y, z, w; };
__device__ __forceinline__ u4 philox(uint64_t seed, uint64_t ctr_hi, uint64_t ctr_lo) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32), c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }  // [0,1)
__device__ __forceinline__ float normal_from(uint32_t a, uint32_t b) {
  float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0,1]
  float u2 = u01(b);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// ------------------------------------------------------------------------------------------ torch CPU
// torch.linspace (float32) scalar formula: start + step*i (first half), end - step*(n-1-i) (second half).
// torch.linspace on CPU for float32 (aten RangeFactoriesKernel linspace_kernel): start + step * i on the first half,
// end - step * (n - 1 - i) on the second, each as ONE fused multiply-add (the compiled kernel contracts them: checked
// bit for bit against torch.linspace on 449,515 values of random (start, end, n), tools/linspace_model.py)
__device__ __forceinline__ float torch_linspace_at(float start, float end, int64_t n, int64_t i) {
  if (n == 1) return start;
  float step = (end - start) / (float)(n - 1);
  return (i < n / 2) ? __fmaf_rn(step, (float)i, start) : __fmaf_rn(-step, (float)(n - 1 - i), end);
}

// Wave-level helpers (wave64).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace yanerf
