// Probe of the scale operand of gfx950's v_cvt_scalef32_pk_fp8_bf16 / v_cvt_scalef32_pk_bf16_fp8: encode 1.0 and 3.0
// with scale 4.0 and 0.25, decode the byte with scale 1.0, 4.0 and 0.25; prints the decoded values.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bh2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));
__global__ void k(float* out) {
  const float scales[3] = {1.0f, 4.0f, 0.25f};
  bh2 v = {(__bf16)1.0f, (__bf16)3.0f};
  int o = 0;
  for (int a = 0; a < 3; ++a) {
    s2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s2{0, 0}, v, scales[a], false);
    unsigned packed = __builtin_bit_cast(unsigned, r) & 0xffff;
    out[o++] = (float)(packed & 0xff);
    for (int b = 0; b < 3; ++b) {
      bh2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(packed, scales[b], false);
      out[o++] = (float)d.x;
      out[o++] = (float)d.y;
    }
  }
}
int main() {
  float* d;
  hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d);
  float h[64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[3] = {"1", "4", "0.25"};
  int o = 0;
  for (int a = 0; a < 3; ++a) {
    printf("encode scale %s: byte0 0x%02x;", nm[a], (unsigned)h[o++]);
    for (int b = 0; b < 3; ++b) { printf(" decode scale %s -> (%g, %g);", nm[b], h[o], h[o + 1]); o += 2; }
    printf("\n");
  }
  return 0;
}
