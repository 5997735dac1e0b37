// Probe: the exact accumulation order / rounding of the two MFMAs the fp32 and fp32x3 MLP GEMMs issue, so the reference
// can be re-run in the HIP kernels' own summation order (tests/golden/make_golden.py gen_sensitivity, trial (e)).
//   f32 : v_mfma_f32_16x16x4_f32   (lane l: A[l % 16][l / 16], B[l / 16][l % 16], C/D rows 4 (l / 16) + r, column l % 16)
//   bf16: v_mfma_f32_16x16x32_bf16 (lane l: A[l % 16][8 (l / 16) + j], B[8 (l / 16) + j][l % 16], j = 0..7)
// Input file (written by tools/mfma_order_model.py): int32 mode (0 f32, 1 bf16), int32 n, then per trial the 64 lanes'
// A operand (f32: 1 float, bf16: 8 u16), B operand (same) and C (4 floats). Output file: per trial the 64 lanes' D.
//   hipcc --offload-arch=gfx950 -O3 -o probe_mfma_order probe_mfma_order.hip && ./probe_mfma_order in.bin out.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short us8 __attribute__((ext_vector_type(8)));

__global__ void k_f32(const float* a, const float* b, const f4* c, f4* d, int n) {
  const int t = blockIdx.x, l = threadIdx.x;
  if (t >= n) return;
  d[t * 64 + l] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t * 64 + l], b[t * 64 + l], c[t * 64 + l], 0, 0, 0);
}

__global__ void k_bf16(const us8* a, const us8* b, const f4* c, f4* d, int n) {
  const int t = blockIdx.x, l = threadIdx.x;
  if (t >= n) return;
  d[t * 64 + l] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a[t * 64 + l]),
                                                          __builtin_bit_cast(bf8, b[t * 64 + l]), c[t * 64 + l], 0, 0, 0);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int hdr[2];
  if (fread(hdr, 4, 2, f) != 2) return 2;
  const int mode = hdr[0], n = hdr[1];
  if (n <= 0 || n > (1 << 20) || (mode != 0 && mode != 1)) return 2;
  const size_t opb = mode == 0 ? 4 : 16;  // bytes of one lane's A / B operand
  std::vector<char> ha((size_t)n * 64 * opb), hb((size_t)n * 64 * opb);
  std::vector<f4> hc((size_t)n * 64), hd((size_t)n * 64);
  if (fread(ha.data(), 1, ha.size(), f) != ha.size() || fread(hb.data(), 1, hb.size(), f) != hb.size() ||
      fread(hc.data(), sizeof(f4), hc.size(), f) != hc.size())
    return 2;
  fclose(f);
  void *da, *db;
  f4 *dc, *dd;
  hipMalloc(&da, ha.size());
  hipMalloc(&db, hb.size());
  hipMalloc(&dc, hc.size() * sizeof(f4));
  hipMalloc(&dd, hd.size() * sizeof(f4));
  hipMemcpy(da, ha.data(), ha.size(), hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), hb.size(), hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), hc.size() * sizeof(f4), hipMemcpyHostToDevice);
  if (mode == 0)
    hipLaunchKernelGGL(k_f32, dim3(n), dim3(64), 0, 0, (const float*)da, (const float*)db, dc, dd, n);
  else
    hipLaunchKernelGGL(k_bf16, dim3(n), dim3(64), 0, 0, (const us8*)da, (const us8*)db, dc, dd, n);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipMemcpy(hd.data(), dd, hd.size() * sizeof(f4), hipMemcpyDeviceToHost);
  FILE* o = fopen(argv[2], "wb");
  fwrite(hd.data(), sizeof(f4), hd.size(), o);
  fclose(o);
  printf("probe_mfma_order: mode %d, %d trials\n", mode, n);
  return 0;
}
