/* A Linear layer evaluated in the summation order of the fp32 HIP GEMMs (csrc/mlp.hip gemm_run / mma_blk<float>), for
 * the reference trial in that order (make_golden.gen_sensitivity, trial (e)). Test infrastructure only: built and
 * loaded by the golden generator in the build container, never by the product.
 *
 * The fp32 kernels compute out[n][m] = bias[n] + sum_k W[n][k] x[m][k] as a chain of v_mfma_f32_16x16x4_f32 over
 * 64-byte K-blocks (16 values): per K-block, MFMA s = 0..3 takes k = 16 kb + 4 g + s from lane group g = 0..3 (each lane
 * holds one 16-byte chunk of the row, 4 consecutive k). The accumulator starts from the bias (trunk, intermediate and
 * colour layers) or from zero with the bias added afterwards (the density and colour-output heads, 16-row tiles). What
 * one MFMA does with its four products was measured on the MI355X (tools/probes/probe_mfma_order.hip,
 * tools/mfma_order_model.py, profiles/r5_mfma_order.txt); `inner` selects that model:
 *   0  a fused fma chain over g = 0..3
 *   1  the four products and the accumulator summed exactly, rounded once (round to nearest even)
 * gcc -O2 -fopenmp -shared -fPIC -o mfma_order.so mfma_order.c -lm   (no -ffast-math: every fmaf / add rounds as written) */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* exact sum of the accumulator and four fp32 products, rounded once to fp32: the products are exact in double (48-bit
 * significands) and a double-double (two-sum) accumulation of five terms holds the sum exactly unless the terms span
 * more than ~100 binary orders, far outside this data; the final round-to-fp32 of hi + lo is then correctly rounded
 * except for double-rounding ties resolved through lo. */
static float sum5_round(float acc, const double p[4]) {
  double hi = (double)acc, lo = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double s = hi + p[i];
    const double bp = s - hi;
    const double err = (hi - (s - bp)) + (p[i] - bp);
    hi = s;
    lo += err;
  }
  const double s = hi + lo;
  const double e = lo - (s - hi);
  float r = (float)s;
  /* round-to-nearest-even of s + e to fp32: if s sits exactly on a tie of fp32 rounding, e decides */
  const double back = (double)r;
  if (back != s) {
    const double half = fabs((double)nextafterf(r, (float)(s > back ? INFINITY : -INFINITY)) - back) * 0.5;
    if (fabs(s - back) == half && e != 0.0) {
      const float other = nextafterf(r, (float)(s > back ? INFINITY : -INFINITY));
      if ((s > back) == (e > 0.0)) r = other;
    }
  }
  return r;
}

/* X [M][K] row-major, W [N][K] row-major, bias [N] or NULL, Y [M][N].
 * bias_first 1: the chain starts from the bias; 0: it starts from +0 and the bias is added after (fp32 add). */
void hip_order_linear(const float* X, int64_t M, int K, const float* W, int N, const float* bias, int bias_first,
                      int inner, float* Y) {
  const int nkb = (K + 15) / 16;
#pragma omp parallel for schedule(static)
  for (int64_t m = 0; m < M; ++m) {
    const float* x = X + m * (int64_t)K;
    for (int n = 0; n < N; ++n) {
      const float* w = W + (int64_t)n * K;
      float acc = (bias && bias_first) ? bias[n] : 0.0f;
      for (int kb = 0; kb < nkb; ++kb) {
        for (int s = 0; s < 4; ++s) {
          if (inner == 0) {
            for (int g = 0; g < 4; ++g) {
              const int k = 16 * kb + 4 * g + s;
              if (k < K) acc = fmaf(w[k], x[k], acc);
            }
          } else {
            double p[4];
            for (int g = 0; g < 4; ++g) {
              const int k = 16 * kb + 4 * g + s;
              p[g] = k < K ? (double)w[k] * (double)x[k] : 0.0;
            }
            acc = sum5_round(acc, p);
          }
        }
      }
      if (bias && !bias_first) acc = acc + bias[n];
      Y[m * (int64_t)N + n] = acc;
    }
  }
}
