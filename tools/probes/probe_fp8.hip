// Probe of gfx950's bf16 <-> fp8 (e4m3) conversions with scale 1.0: every non-negative bf16 bit pattern is encoded with
// v_cvt_scalef32_pk_fp8_bf16 and decoded with v_cvt_scalef32_pk_bf16_fp8; the table (bf16 in, fp8 byte, bf16 out) is
// written to the file named by argv[1] for comparison with the OCP e4m3fn definition.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __bf16 bh2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));

__global__ void roundtrip(unsigned short* enc, unsigned short* dec, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * t + 1 >= n) return;
  unsigned in = (unsigned)(2 * t) | ((unsigned)(2 * t + 1) << 16);
  s2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s2{0, 0}, __builtin_bit_cast(bh2, in), 1.0f, false);
  unsigned packed = __builtin_bit_cast(unsigned, r) & 0xffff;
  bh2 back = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(packed, 1.0f, false);
  unsigned b = __builtin_bit_cast(unsigned, back);
  enc[2 * t] = packed & 0xff;
  enc[2 * t + 1] = (packed >> 8) & 0xff;
  dec[2 * t] = b & 0xffff;
  dec[2 * t + 1] = b >> 16;
}

int main(int argc, char** argv) {
  const int n = 65536;
  unsigned short *e, *d;
  hipMalloc(&e, n * 2);
  hipMalloc(&d, n * 2);
  hipLaunchKernelGGL(roundtrip, dim3(n / 512), dim3(256), 0, 0, e, d, n);
  std::vector<unsigned short> he(n), hd(n);
  hipMemcpy(he.data(), e, n * 2, hipMemcpyDeviceToHost);
  hipMemcpy(hd.data(), d, n * 2, hipMemcpyDeviceToHost);
  FILE* f = fopen(argc > 1 ? argv[1] : "fp8_table.bin", "wb");
  fwrite(he.data(), 2, n, f);
  fwrite(hd.data(), 2, n, f);
  fclose(f);
  printf("ok\n");
  hipFree(e);
  hipFree(d);
  return 0;
}
