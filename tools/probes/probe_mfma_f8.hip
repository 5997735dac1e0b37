// Probe of gfx950's block-scaled fp8 MFMAs (v_mfma_scale_f32_32x32x64_f8f6f4, _16x16x128_) with e4m3 operands.
// Hypothesis checked (exact small-integer data): lane l holds A[row l % M][k = 32 (l / M) + j] and
// B[k = 32 (l / M) + j][col l % M] in byte j of its 8 operand dwords (M = 32 or 16), C/D in the standard maps, and the
// e8m0 scale operand of a lane (opsel 0: byte 0) multiplies the 32 products it supplies by 2^(E - 127).
// Because the MFMA sums over k, the test only needs A and B to share one k map; it checks that and the row/column maps.
// Prints the mismatch count per case (0 = hypothesis holds).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

// fp8 e4m3fn encoding of small integers -8..8 (exact)
static unsigned char e4m3(int v) {
  if (v == 0) return 0;
  unsigned s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v;
  int e = 0;
  while ((a >> e) > 1) ++e;              // a in [2^e, 2^(e+1))
  int mant = (a << 3 >> e) & 7;          // 3 mantissa bits (exact for |v| <= 16)
  return (unsigned char)(s | ((e + 7) << 3) | mant);
}

__global__ void k32(const v8i* a, const v8i* b, const int* sa, const int* sb, float* out) {
  const int l = threadIdx.x;
  v16f c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}
__global__ void k16(const v8i* a, const v8i* b, const int* sa, const int* sb, float* out) {
  const int l = threadIdx.x;
  v4f c = {};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

static int run(int M, bool lane_scales) {
  const int K = M == 32 ? 64 : 128;
  static unsigned char ab[64][32], bb[64][32];
  static int av[64][32], bv[64][32];
  int sa[64], sb[64];
  for (int l = 0; l < 64; ++l) {
    for (int j = 0; j < 32; ++j) {
      av[l][j] = rand() % 17 - 8;
      bv[l][j] = rand() % 17 - 8;
      ab[l][j] = e4m3(av[l][j]);
      bb[l][j] = e4m3(bv[l][j]);
    }
    sa[l] = 127 + (lane_scales ? (l % 5) - 2 : -3);
    sb[l] = 127 + (lane_scales ? (l % 3) - 1 : 1);
  }
  v8i *da, *db; int *dsa, *dsb; float* dout;
  hipMalloc(&da, sizeof(ab)); hipMalloc(&db, sizeof(bb));
  hipMalloc(&dsa, sizeof(sa)); hipMalloc(&dsb, sizeof(sb)); hipMalloc(&dout, 64 * 16 * 4);
  hipMemcpy(da, ab, sizeof(ab), hipMemcpyHostToDevice);
  hipMemcpy(db, bb, sizeof(bb), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa, sizeof(sa), hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb, sizeof(sb), hipMemcpyHostToDevice);
  if (M == 32) hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dout);
  else hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dout);
  float h[64 * 16];
  hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
  // expected D[i][c] = sum_k A[i][k] B[k][c] 2^(sa + sb) under the hypothesis
  double D[32][32] = {};
  for (int i = 0; i < M; ++i)
    for (int c = 0; c < M; ++c)
      for (int k = 0; k < K; ++k) {
        const int la = i + M * (k / 32), lb = c + M * (k / 32), j = k % 32;
        D[i][c] += (double)av[la][j] * bv[lb][j] * std::ldexp(1.0, (sa[la] - 127) + (sb[lb] - 127));
      }
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < (M == 32 ? 16 : 4); ++r) {
      int row, col = l % M;
      if (M == 32) row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      else row = 4 * (l >> 4) + r;
      const float got = h[l * (M == 32 ? 16 : 4) + r];
      if (got != (float)D[row][col]) {
        if (bad < 4) printf("  M=%d lane %d reg %d (row %d col %d): got %g want %g\n", M, l, r, row, col, got, D[row][col]);
        ++bad;
      }
    }
  hipFree(da); hipFree(db); hipFree(dsa); hipFree(dsb); hipFree(dout);
  return bad;
}

int main() {
  srand(1);
  printf("32x32x64 uniform scales: %d mismatches\n", run(32, false));
  printf("32x32x64 per-lane scales: %d mismatches\n", run(32, true));
  printf("16x16x128 uniform scales: %d mismatches\n", run(16, false));
  printf("16x16x128 per-lane scales: %d mismatches\n", run(16, true));
  return 0;
}
