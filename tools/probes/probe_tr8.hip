// Probe of ds_read_b64_tr_b8 semantics on gfx950: LDS byte (row r, col c) of a [16 rows][16 B] image holds 16 r + c;
// lane i of each 16-lane group supplies the address of row i / 2, bytes 8 (i % 2) .. + 7; every lane prints the 8
// bytes it receives (decoded as row:col).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void probe(unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char img[64 * 16];
  const int t = threadIdx.x;
  for (int i = t; i < 64 * 16; i += 64) img[i] = (unsigned char)(i & 0xff);
  __syncthreads();
  const int grp = t >> 4, i = t & 15;
  const int addr = grp * 256 + (i >> 1) * 16 + 8 * (i & 1);
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(img + addr));
  out[2 * t] = (unsigned)v.x;
  out[2 * t + 1] = (unsigned)v.y;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 2 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int t = 0; t < 32; ++t) {
    printf("lane %2d:", t);
    for (int b = 0; b < 8; ++b) {
      unsigned byte = (h[2 * t + b / 4] >> (8 * (b % 4))) & 0xff;
      printf(" %d:%d", (byte >> 4), byte & 15);
    }
    printf("\n");
  }
  hipFree(d);
  return 0;
}
