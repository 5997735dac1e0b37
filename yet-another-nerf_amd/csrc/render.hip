// Ray generation, emission-absorption compositing (fwd/bwd), inverse-CDF importance sampling + merge,
// photometric loss and Adam for the yet-another-nerf hot path on gfx950.
//
// Layout: one thread per ray for ray generation / loss; one wave64 per ray for every per-ray scan
// (compositing cumsum, CDF, merge), lanes owning contiguous sample chunks so HBM rows [R][P] are read
// coalesced. Built with -ffp-contract=off so the float op sequence matches the reference's aten ops.
#include <cmath>

#include "common.hpp"

namespace yanerf {

thread_local std::string g_last_error;
void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// ============================================================================================ raygen
// Keyed pseudo-random permutation of [0, n) (balanced Feistel network + cycle walking): the first R
// images of 0..R-1 are R distinct pixels, uniformly spread. Replaces torch.multinomial(ones, R,
// replacement=False) (ray_sampler.py:317-358) for the uniform-weight case.
__device__ uint64_t feistel_perm(uint64_t i, uint64_t n, uint64_t seed, uint64_t offset) {
  int bits = 2;
  while ((1ull << bits) < n) ++bits;
  if (bits & 1) ++bits;
  const int h = bits / 2;
  const uint64_t mask = (1ull << h) - 1;
  uint64_t x = i;
  do {
    uint64_t L = x >> h, Rr = x & mask;
#pragma unroll
    for (int round = 0; round < 4; ++round) {
      u4 r = philox(seed, offset ^ (0x5bd1e995ull * (round + 1)), Rr);
      uint64_t F = r.x & mask;
      uint64_t nl = Rr, nr = (L ^ F) & mask;
      L = nl; Rr = nr;
    }
    x = (L << h) | Rr;
  } while (x >= n);
  return x;
}

// One thread per (ray, group of RG_J consecutive depths): the ray-level work (pixel id, xys, origin, direction) by the
// group-0 thread of each ray, every depth by the thread of its group, one Philox call per 4 consecutive draws (the
// counter is idx >> 2, so a group aligned to 4 needs one). The per-element arithmetic is unchanged. (One thread per
// ray with a serial loop over the depths -- 4096 threads for the Lego batch, 64 Philox calls each -- took 39 us.)
constexpr int RG_J = 4;
__global__ void raygen_kernel(const float* __restrict__ poses, const float* __restrict__ focal,
                              const float* __restrict__ xy, const int64_t* __restrict__ pixel_ids, int64_t B,
                              int64_t R, int64_t grid_w, int64_t grid_h, float cfg_w, float cfg_h, float near,
                              float far, int64_t P, int jitter_mode, const float* __restrict__ jitter_u,
                              uint64_t seed, uint64_t offset, float* __restrict__ origins,
                              float* __restrict__ directions, float* __restrict__ lengths,
                              float* __restrict__ xys, int64_t* __restrict__ ids_out,
                              const float* __restrict__ bounds, const uint64_t* __restrict__ rng_base) {
  if (bounds) {  // device-resident depth range (no host read of LLFF's per-image bounds)
    near = bounds[0];
    far = bounds[1];
  }
  if (rng_base) offset += *rng_base;  // graph replay: the step's Philox base lives on the device
  const int64_t G = (P + RG_J - 1) / RG_J;  // depth groups per ray (>= 1: the ray-level work needs group 0)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * R * (G > 0 ? G : 1)) return;
  const int64_t gid = t / (G > 0 ? G : 1), jg = t % (G > 0 ? G : 1);
  const int64_t b = gid / R;
  if (jg == 0) {
    float x, y;
    if (xy) {
      x = xy[gid * 2 + 0];
      y = xy[gid * 2 + 1];
    } else {
      int64_t id;
      if (pixel_ids) {
        id = pixel_ids[gid];
      } else {
        id = (int64_t)feistel_perm((uint64_t)(gid - b * R), (uint64_t)(grid_w * grid_h), seed, offset + 7919ull * b);
      }
      if (ids_out) ids_out[gid] = id;
      x = (float)(id % grid_w);
      y = (float)(id / grid_w);
    }
    xys[gid * 2 + 0] = x;
    xys[gid * 2 + 1] = y;
    const float* p = poses + b * 12;
    const float f = focal[b];
    // ray_sampler.py:300-312: v = [(x - W/2)/f, (y - H/2)/f, 1]; d_i = sum_j R_ij v_j
    const float vx = (x - cfg_w * 0.5f) / f;
    const float vy = (y - cfg_h * 0.5f) / f;
    const float vz = 1.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      directions[gid * 3 + i] = (p[i * 4 + 0] * vx + p[i * 4 + 1] * vy) + p[i * 4 + 2] * vz;
      origins[gid * 3 + i] = p[i * 4 + 3];
    }
  }
  float* z = lengths + gid * P;
  u4 r = u4{0u, 0u, 0u, 0u};
  int64_t rc = -1;  // Philox counter held in r
#pragma unroll
  for (int jj = 0; jj < RG_J; ++jj) {
    const int64_t j = jg * RG_J + jj;
    if (j >= P) break;
    float zj = torch_linspace_at(near, far, P, j);
    if (jitter_mode) {
      // _jiggle_within_stratas (ray_sampler.py:381-385)
      float lower = (j == 0) ? zj : 0.5f * (zj + torch_linspace_at(near, far, P, j - 1));
      float upper = (j == P - 1) ? zj : 0.5f * (torch_linspace_at(near, far, P, j + 1) + zj);
      float u;
      if (jitter_mode == 1) {
        u = jitter_u[gid * P + j];
      } else {
        const int64_t idx = gid * P + j;
        if ((idx >> 2) != rc) {
          rc = idx >> 2;
          r = philox(seed, offset, (uint64_t)rc);
        }
        uint32_t w = (idx & 3) == 0 ? r.x : (idx & 3) == 1 ? r.y : (idx & 3) == 2 ? r.z : r.w;
        u = u01(w);
      }
      zj = lower + (upper - lower) * u;
    }
    z[j] = zj;
  }
}

// ============================================================================================ composite
// One wave per ray. Lane l owns samples [l*S, l*S + S), S = ceil(P / 64) <= 8.
constexpr int kMaxS = 8;  // P <= 512

struct RayCtx {
  int S;
  int i0;
};

__device__ __forceinline__ double wave_incl_scan_d(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ float noise_at(const yanerf_raymarch_opts& o, const float* noise, int64_t idx) {
  if (o.noise_mode == 0 || !(o.noise_std > 0.0f)) return 0.0f;
  float n;
  if (o.noise_mode == 1) {
    n = noise[idx];
  } else {
    u4 r = philox(o.seed, o.offset + (o.rng_base ? *o.rng_base : 0ull), (uint64_t)(idx >> 1));
    n = (idx & 1) ? normal_from(r.z, r.w) : normal_from(r.x, r.y);
  }
  return n * o.noise_std;
}

// the capping function 1 - exp(-x) (renderer.py capping_function "exponential") with a correctly rounded exp (double,
// rounded once): a pure function of its fp32 argument that a CPU reproduces bit for bit (make_golden's trial in the
// HIP kernels' arithmetic); torch's vectorised expf is within an ulp of it
__device__ __forceinline__ float exp_cr(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float cap_fn(int kind, float x) { return kind == 0 ? 1.0f - exp_cr(-x) : fminf(x, 1.0f); }
__device__ __forceinline__ float cap_grad(int kind, float x) { return kind == 0 ? exp_cr(-x) : (x <= 1.0f ? 1.0f : 0.0f); }

// the photometric loss of the fused training composite (MODE 2): rgb_loss_kernel's arithmetic on the ray's features
struct CompositeLoss {
  const float* image;  // [B][H][W][C]
  const float* xys;    // [B * rays_per_image][2]
  int64_t rays_per_image, H, W;
  float scale;
  float* sq;      // [R] per-ray squared error (may be null)
  float* g_feat;  // [R][C] dL/dfeatures (may be null)
};

// MODE 0: forward (features, depths, alpha, weights); 1: backward from g_features / g_depths / g_alpha; 2: the training
// pass of the fused trainer in one launch -- the forward outputs, the loss of the features against the image
// (rgb_loss_kernel's arithmetic, on lane 0's features as the separate kernels see them) and the backward from that
// gradient (g_depths = g_alpha = 0), bit-identical to the three launches it replaces
template <int MODE>
__global__ void __launch_bounds__(256) composite_kernel(
    yanerf_raymarch_opts o, const float* __restrict__ sigma_raw, const float* __restrict__ rgb,
    const float* __restrict__ lengths, const float* __restrict__ dirs, const float* __restrict__ bg,
    const float* __restrict__ noise, int64_t R, int64_t P, int64_t C, float* __restrict__ features,
    float* __restrict__ depths, float* __restrict__ alpha_out, float* __restrict__ weights_out,
    const float* __restrict__ g_features, const float* __restrict__ g_depths, const float* __restrict__ g_alpha,
    float* __restrict__ g_sigma, float* __restrict__ g_rgb, CompositeLoss loss) {
  constexpr bool BACKWARD = MODE == 1;
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (ray >= R) return;
  const int S = (int)((P + 63) / 64);
  const int i0 = lane * S;
  const float* zr = lengths + ray * P;
  const float dx = dirs[ray * 3 + 0], dy = dirs[ray * 3 + 1], dz = dirs[ray * 3 + 2];
  const float dn = sqrtf(dx * dx + dy * dy + dz * dz);

  float z[kMaxS], delta[kMaxS], pre[kMaxS], wd[kMaxS], capped[kMaxS], cs[kMaxS], op[kMaxS], w[kMaxS];
  // -------- forward (also recomputed by the backward)
  double local = 0.0;
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    z[s] = (i < P) ? zr[i] : 0.0f;
  }
  // next-z for the last owned sample comes from the next lane's first sample
  float znext_lane = __shfl_down(z[0], 1, 64);
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    float d = 0.0f, p = 0.0f, v = 0.0f;
    if (i < P) {
      float zn = (s + 1 < S) ? z[s + 1] : znext_lane;
      d = (i < P - 1) ? (zn - z[s]) : o.background_opacity;
      d = d * dn;
      float sr = sigma_raw[ray * P + i];
      float nz = noise_at(o, noise, ray * P + i);
      p = (nz != 0.0f) ? sr + nz : sr;
      v = o.density_relu ? fmaxf(p, 0.0f) + o.background_density_bias : p;
      v = d * v;
    }
    delta[s] = d;
    pre[s] = p;
    wd[s] = v;
    capped[s] = cap_fn(o.capping, v);
    local += (double)v;
  }
  // inclusive scan of wd in double (torch CPU cumsum accumulates float in double)
  double incl = wave_incl_scan_d(local, lane);
  double run = incl - local;
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    run += (double)wd[s];
    cs[s] = (float)run;
    op[s] = cap_fn(o.capping, cs[s]);
  }
  float op_own_last = 0.0f;
#pragma unroll
  for (int s = 0; s < kMaxS; ++s)
    if (s == S - 1) op_own_last = op[s];
  float op_prev_lane = __shfl_up(op_own_last, 1, 64);
  // last valid op (alpha)
  const int last_lane = (int)((P - 1) / S), last_s = (int)((P - 1) % S);
  float op_last_mine = 0.0f;
#pragma unroll
  for (int s = 0; s < kMaxS; ++s)
    if (s == last_s) op_last_mine = op[s];
  const float alpha = __shfl(op_last_mine, last_lane, 64);
  float absorb[kMaxS];
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    float prev = (s > 0) ? op[s - 1] : op_prev_lane;
    absorb[s] = (i == 0) ? 1.0f : 1.0f - prev;
    float ww = (o.weight_fn == 0) ? capped[s] * absorb[s] : fminf(capped[s], absorb[s]);
    w[s] = (i < P) ? ww : 0.0f;
  }
  // background colour for this ray
  float bgc[4];
  for (int c = 0; c < C && c < 4; ++c)
    bgc[c] = bg ? bg[ray * C + c] : (o.bg_default_n == 1 ? o.bg_default[0] : o.bg_default[c]);

  float gL[4] = {0, 0, 0, 0};  // MODE 2: dL/dfeatures
  if (!BACKWARD) {
    float dep = 0.0f, F[4] = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) {
      if (s >= S) break;
      int i = i0 + s;
      if (i >= P) break;
      weights_out[ray * P + i] = w[s];
      dep += w[s] * z[s];
      for (int c = 0; c < C && c < 4; ++c) {
        float col = rgb[(ray * P + i) * C + c];
        if (o.hard_background && i == P - 1) col = bgc[c];
        F[c] += w[s] * col;
      }
    }
    dep = wave_sum(dep);
    for (int c = 0; c < C && c < 4; ++c) F[c] = wave_sum(F[c]);
    if (lane == 0) {
      depths[ray] = dep;
      alpha_out[ray] = alpha;
      for (int c = 0; c < C && c < 4; ++c) {
        float f = F[c];
        if (!o.hard_background) {
          float A = o.blend_output ? alpha : 1.0f;
          f = A * F[c] + (1.0f - alpha) * bgc[c];
        }
        features[ray * C + c] = f;
      }
    }
    if constexpr (MODE == 0) return;
    // loss (rgb_loss_kernel): lane 0's features, as the separate kernels read them back
    const int64_t b = ray / loss.rays_per_image;
    const int64_t x = (int64_t)loss.xys[ray * 2 + 0], y = (int64_t)loss.xys[ray * 2 + 1];
    const float* px = loss.image + ((b * loss.H + y) * loss.W + x) * C;
    float sq = 0.0f;
    for (int c = 0; c < C && c < 4; ++c) {
      float f = F[c];
      if (!o.hard_background) {
        float A = o.blend_output ? alpha : 1.0f;
        f = A * F[c] + (1.0f - alpha) * bgc[c];
      }
      f = __shfl(f, 0, 64);
      const float d = f - px[c];
      sq += d * d;
      gL[c] = loss.scale * 2.0f * d;
      if (lane == 0 && loss.g_feat) loss.g_feat[ray * C + c] = gL[c];
    }
    if (lane == 0 && loss.sq) loss.sq[ray] = sq;
  }

  // -------- backward
  float gF[4] = {0, 0, 0, 0};
  float gD = (MODE == 1 && g_depths) ? g_depths[ray] : 0.0f;
  float gA = (MODE == 1 && g_alpha) ? g_alpha[ray] : 0.0f;
  float g_op_last = gA;
  float Fsum[4] = {0, 0, 0, 0};
  if (!o.hard_background && o.blend_output) {
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) {
      if (s >= S) break;
      int i = i0 + s;
      if (i >= P) break;
      for (int c = 0; c < C && c < 4; ++c) Fsum[c] += w[s] * rgb[(ray * P + i) * C + c];
    }
    for (int c = 0; c < C && c < 4; ++c) Fsum[c] = wave_sum(Fsum[c]);
  }
  for (int c = 0; c < C && c < 4; ++c) {
    float g = MODE == 2 ? gL[c] : g_features[ray * C + c];
    if (!o.hard_background) {
      float A = o.blend_output ? alpha : 1.0f;
      gF[c] = g * A;
      g_op_last += -g * bgc[c];
      if (o.blend_output) g_op_last += g * Fsum[c];
    } else {
      gF[c] = g;
    }
  }
  float gw[kMaxS];
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    float acc = 0.0f;
    if (i < P) {
      for (int c = 0; c < C && c < 4; ++c) {
        float col = rgb[(ray * P + i) * C + c];
        bool is_bg = o.hard_background && i == P - 1;
        if (is_bg) col = bgc[c];
        acc += gF[c] * col;
        g_rgb[(ray * P + i) * C + c] = is_bg ? 0.0f : w[s] * gF[c];
      }
      acc += gD * z[s];
    }
    gw[s] = acc;
  }
  // w = f(capped, absorb)
  float g_capped[kMaxS], g_abs[kMaxS];
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    if (o.weight_fn == 0) {
      g_capped[s] = gw[s] * absorb[s];
      g_abs[s] = gw[s] * capped[s];
    } else {
      bool eq = capped[s] == absorb[s];
      g_capped[s] = eq ? gw[s] * 0.5f : (capped[s] < absorb[s] ? gw[s] : 0.0f);
      g_abs[s] = eq ? gw[s] * 0.5f : (absorb[s] < capped[s] ? gw[s] : 0.0f);
    }
  }
  // g_op[i] = -g_abs[i+1] (i < P-1) + [i == P-1] g_op_last; g_cs = g_op * cap'(cs)
  float gabs_next_lane = __shfl_down(g_abs[0], 1, 64);
  double gcs_local = 0.0;
  float g_cs[kMaxS];
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    float gop = 0.0f;
    if (i < P - 1) gop = -((s + 1 < S) ? g_abs[s + 1] : gabs_next_lane);
    if (i == P - 1) gop += g_op_last;
    g_cs[s] = (i < P) ? gop * cap_grad(o.capping, cs[s]) : 0.0f;
    gcs_local += (double)g_cs[s];
  }
  // suffix sums of g_cs (cumsum backward: flip-cumsum-flip, double accumulation)
  double total = gcs_local;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off, 64);
  double incl_pref = wave_incl_scan_d(gcs_local, lane);
  double suffix = total - (incl_pref - gcs_local);  // sum over samples >= my first sample
#pragma unroll
  for (int s = 0; s < kMaxS; ++s) {
    if (s >= S) break;
    int i = i0 + s;
    float gwd = (float)suffix + g_capped[s] * cap_grad(o.capping, wd[s]);
    suffix -= (double)g_cs[s];
    float gs = gwd * delta[s];
    float gsig = o.density_relu ? (pre[s] > 0.0f ? gs : 0.0f) : gs;
    if (i < P) g_sigma[ray * P + i] = gsig;
  }
}

// ============================================================================================ sample_pdf
// torch CPU float32 row-sum order (aten vectorized_inner_sum, 8-wide vectors, 4-way ILP row_sum) so that
// pdf = w / sum rounds exactly like the reference; that rounding decides `denom < eps`
// (renderers/utils.py:128-129). Run by one lane over an LDS row, n < 512.
__device__ float torch_row_sum(const float* x, int n) {
  const int V = 8;
  int nv = n / V;
  int size_ilp = nv / 4;
  float ps[4][8];
  for (int k = 0; k < 4; ++k)
    for (int l = 0; l < V; ++l) ps[k][l] = (size_ilp >= 1) ? x[k * V + l] : 0.0f;
  for (int i = 1; i < size_ilp; ++i)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < V; ++l) ps[k][l] += x[(4 * i + k) * V + l];
  for (int i = size_ilp * 4; i < nv; ++i)
    for (int l = 0; l < V; ++l) ps[0][l] += x[i * V + l];
  for (int k = 1; k < 4; ++k)
    for (int l = 0; l < V; ++l) ps[0][l] += ps[k][l];
  float acc = 0.0f;
  for (int k = nv * V; k < n; ++k) acc += x[k];
  if (nv > 0)
    for (int l = 0; l < V; ++l) acc += ps[0][l];
  return acc;
}

// torch_row_sum with its 32 partial-sum chains ps[k][l] on lanes 8k + l (each chain's adds in torch's order, so every
// rounding is the same), combined as torch combines them: ps[0][l] += ps[1][l], ps[2][l], ps[3][l], then the tail
// elements and ps[0][0..7] into one accumulator. Result on every lane. (One lane over the whole row: ~100 dependent
// LDS reads per ray.)
__device__ float torch_row_sum_wave(const float* x, int n, int lane) {
  const int V = 8, nv = n / V, size_ilp = nv / 4;
  const int k = (lane >> 3) & 3, l = lane & 7;
  float v = 0.0f;
  if (lane < 32) {
    v = (size_ilp >= 1) ? x[k * V + l] : 0.0f;
    for (int i = 1; i < size_ilp; ++i) v += x[(4 * i + k) * V + l];
    if (k == 0)
      for (int i = size_ilp * 4; i < nv; ++i) v += x[i * V + l];
  }
  const float p1 = __shfl(v, 8 + l, 64), p2 = __shfl(v, 16 + l, 64), p3 = __shfl(v, 24 + l, 64);
  v = ((v + p1) + p2) + p3;  // ps[0][l] on lanes 0..7
  float acc = 0.0f;
  for (int kk = nv * V; kk < n; ++kk) acc += x[kk];
  if (nv > 0) {
#pragma unroll
    for (int ll = 0; ll < 8; ++ll) acc += __shfl(v, ll, 64);
  }
  return acc;
}

constexpr int kPdfMaxBins = 512;
constexpr int kMergeMax = 1024;  // P + n_fine, power-of-two padded

// One wave per ray. bins [nb+1], w [nb] (row pointers), writes N samples to out (row pointer, stride 1).
__device__ void sample_pdf_wave(const float* __restrict__ bins, const float* __restrict__ wrow, int nb, int N, int det,
                                const float* __restrict__ urow, uint64_t seed, uint64_t offset, int64_t ray,
                                float* __restrict__ out, float* s_w, float* s_cdf, float* s_bins, int lane) {
  const float eps = 1e-5f;
  for (int i = lane; i < nb; i += 64) s_w[i] = wrow[i] + eps;
  for (int i = lane; i < nb + 1; i += 64) s_bins[i] = bins[i];
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  const float sum = torch_row_sum_wave(s_w, nb, lane);
  // cdf = [0, cumsum(pdf)] with double accumulation
  const int S = (nb + 63) / 64;
  double local = 0.0;
  for (int s = 0; s < S; ++s) {
    int i = lane * S + s;
    if (i < nb) local += (double)(s_w[i] / sum);
  }
  double run = wave_incl_scan_d(local, lane) - local;
  for (int s = 0; s < S; ++s) {
    int i = lane * S + s;
    if (i < nb) {
      run += (double)(s_w[i] / sum);
      s_cdf[i + 1] = (float)run;
    }
  }
  if (lane == 0) s_cdf[0] = 0.0f;
  __syncthreads();
  const int ncdf = nb + 1;
  for (int k = lane; k < N; k += 64) {
    float u;
    if (det) {
      u = torch_linspace_at(0.0f, 1.0f, N, k);
    } else if (urow) {
      u = urow[k];
    } else {
      int64_t idx = ray * N + k;
      u4 r = philox(seed, offset, (uint64_t)(idx >> 2));
      uint32_t ww = (idx & 3) == 0 ? r.x : (idx & 3) == 1 ? r.y : (idx & 3) == 2 ? r.z : r.w;
      u = u01(ww);
    }
    // searchsorted(cdf, u, right=True): number of cdf entries <= u
    int lo = 0, hi = ncdf;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (s_cdf[mid] <= u) lo = mid + 1; else hi = mid;
    }
    int inds = lo;
    int below = inds - 1 < 0 ? 0 : inds - 1;
    int above = inds > ncdf - 1 ? ncdf - 1 : inds;
    float cb = s_cdf[below], ca = s_cdf[above];
    float bb = s_bins[below], ba = s_bins[above];
    float denom = ca - cb;
    if (denom < eps) denom = 1.0f;
    float t = (u - cb) / denom;
    out[k] = bb + t * (ba - bb);
  }
}

__global__ void __launch_bounds__(64) sample_pdf_kernel(const float* __restrict__ bins, const float* __restrict__ w,
                                                        int64_t R, int nb, int N, int det, const float* __restrict__ u,
                                                        uint64_t seed, uint64_t offset, float* __restrict__ out) {
  __shared__ float s_w[kPdfMaxBins], s_cdf[kPdfMaxBins + 1], s_bins[kPdfMaxBins + 1];
  int64_t ray = blockIdx.x;
  if (ray >= R) return;
  sample_pdf_wave(bins + ray * (nb + 1), w + ray * nb, nb, N, det, u ? u + ray * N : nullptr, seed, offset, ray,
                  out + ray * N, s_w, s_cdf, s_bins, threadIdx.x);
}

// Ascending bitonic sort of 64 * EPL floats held EPL per lane (element e = EPL * lane + r): partners at distance
// j < EPL inside the lane, else across lanes (lane ^ j / EPL) through shuffles; the compare-exchange of the LDS version
template <int EPL>
__device__ __forceinline__ void wave_bitonic(float (&v)[EPL], int lane) {
  constexpr int N = 64 * EPL;
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j < EPL) {
#pragma unroll
        for (int r = 0; r < EPL; ++r) {
          const int rp = r ^ j;
          if (rp > r) {
            const bool up = ((EPL * lane + r) & k) == 0;
            const float a = v[r], b = v[rp];
            if ((a > b) == up) {
              v[r] = b;
              v[rp] = a;
            }
          }
        }
      } else {
        const int lj = j / EPL;
        const bool lower = (lane & lj) == 0;
#pragma unroll
        for (int r = 0; r < EPL; ++r) {
          const float o = __shfl_xor(v[r], lj, 64);
          const bool up = ((EPL * lane + r) & k) == 0;
          // the pair (lower, upper) = (v[r] here, o) or (o, v[r]); swap iff (lower > upper) == up
          const float lo_v = lower ? v[r] : o, hi_v = lower ? o : v[r];
          const bool sw = (lo_v > hi_v) == up;
          v[r] = sw ? o : v[r];
        }
      }
    }
  }
}
// sort row[0..n) in LDS (n <= 512) with the register bitonic of the smallest lane width that holds it
template <int EPL>
__device__ __forceinline__ void sort_lds_row_t(float* row, int n, int lane) {
  float v[EPL];
#pragma unroll
  for (int r = 0; r < EPL; ++r) {
    const int e = EPL * lane + r;
    v[r] = e < n ? row[e] : __builtin_inff();
  }
  wave_bitonic<EPL>(v, lane);
#pragma unroll
  for (int r = 0; r < EPL; ++r) {
    const int e = EPL * lane + r;
    if (e < n) row[e] = v[r];
  }
}
__device__ __forceinline__ void sort_lds_row(float* row, int n, int lane) {
  __syncthreads();
  if (n <= 64) sort_lds_row_t<1>(row, n, lane);
  else if (n <= 128) sort_lds_row_t<2>(row, n, lane);
  else if (n <= 256) sort_lds_row_t<4>(row, n, lane);
  else sort_lds_row_t<8>(row, n, lane);
  __syncthreads();
}

// RayPointRefiner: mids = lerp(z[1:], z[:-1], 0.5) = z[:-1] - (z[:-1] - z[1:]) * 0.5 (aten lerp, w >= 0.5
// branch); samples from w[1:-1]; cat + sort (bitonic, LDS) .
__global__ void __launch_bounds__(64) refine_kernel(const float* __restrict__ z, const float* __restrict__ w, int64_t R,
                                                    int P, int NF, int det, const float* __restrict__ u,
                                                    uint64_t seed, uint64_t offset, int add_input,
                                                    float* __restrict__ out, const uint64_t* __restrict__ rng_base) {
  if (rng_base) offset += *rng_base;
  __shared__ float s_w[kPdfMaxBins], s_cdf[kPdfMaxBins + 1], s_bins[kPdfMaxBins + 1];
  __shared__ float s_mid[kPdfMaxBins + 1];
  __shared__ float s_all[kMergeMax];
  const int lane = threadIdx.x;
  int64_t ray = blockIdx.x;
  if (ray >= R) return;
  const float* zr = z + ray * P;
  for (int i = lane; i < P - 1; i += 64) {
    float a = zr[i], b = zr[i + 1];
    s_mid[i] = a - (a - b) * 0.5f;
  }
  __syncthreads();
  const int total = add_input ? P + NF : NF;
  int npow = 1;
  while (npow < total) npow <<= 1;
  // samples go to s_all[off..off+NF)
  const int off = add_input ? P : 0;
  sample_pdf_wave(s_mid, w + ray * P + 1, P - 2, NF, det, u ? u + ray * NF : nullptr, seed, offset, ray, s_all + off,
                  s_w, s_cdf, s_bins, lane);
  if (NF <= 64 * 8 && P <= 64 * 8) {
    // the fine samples (and the coarse depths) sorted in registers, then merged by rank: values only, so any correct
    // sort of the union gives torch.sort's output bit for bit
    float* s_fine = s_all + off;
    float* s_coarse = s_mid;  // free once sample_pdf_wave copied the bins
    if (add_input)
      for (int i = lane; i < P; i += 64) s_coarse[i] = zr[i];
    __syncthreads();
    sort_lds_row(s_fine, NF, lane);
    if (add_input) sort_lds_row(s_coarse, P, lane);
    __syncthreads();
    float* orow = out + ray * total;
    if (!add_input) {
      for (int i = lane; i < NF; i += 64) orow[i] = s_fine[i];
      return;
    }
    // merge: coarse i goes to i + #{fine < a}, fine j to j + #{coarse <= b} (ties: coarse first)
    for (int i = lane; i < P; i += 64) {
      const float a = s_coarse[i];
      int lo = 0, hi = NF;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_fine[mid] < a) lo = mid + 1; else hi = mid;
      }
      orow[i + lo] = a;
    }
    for (int j = lane; j < NF; j += 64) {
      const float b = s_fine[j];
      int lo = 0, hi = P;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_coarse[mid] <= b) lo = mid + 1; else hi = mid;
      }
      orow[j + lo] = b;
    }
    return;
  }
  if (add_input)
    for (int i = lane; i < P; i += 64) s_all[i] = zr[i];
  for (int i = total + lane; i < npow; i += 64) s_all[i] = __builtin_inff();
  __syncthreads();
  // bitonic sort ascending (sizes past the register sort)
  for (int k = 2; k <= npow; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < npow; i += 64) {
        int ixj = i ^ j;
        if (ixj > i) {
          float a = s_all[i], b = s_all[ixj];
          bool up = (i & k) == 0;
          if ((a > b) == up) {
            s_all[i] = b;
            s_all[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  float* orow = out + ray * total;
  for (int i = lane; i < total; i += 64) orow[i] = s_all[i];
}

// ============================================================================================ loss, adam
__global__ void rgb_loss_kernel(const float* __restrict__ pred, const float* __restrict__ image,
                                const float* __restrict__ xys, int64_t B, int64_t R, int64_t H, int64_t W, int64_t C,
                                float scale, float* __restrict__ sq, float* __restrict__ g) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * R) return;
  int64_t b = gid / R;
  int64_t x = (int64_t)xys[gid * 2 + 0], y = (int64_t)xys[gid * 2 + 1];
  const float* px = image + ((b * H + y) * W + x) * C;
  float acc = 0.0f;
  for (int c = 0; c < C; ++c) {
    float d = pred[gid * C + c] - px[c];
    acc += d * d;
    if (g) g[gid * C + c] = scale * 2.0f * d;
  }
  if (sq) sq[gid] = acc;
}

// ---- scatter_rays_to_image (pipelines/utils.py:299-323; nerf_pipeline.py:307-324 _rasterize_mc_samples): the
// Monte-Carlo rays' outputs splatted onto full-size images. Fill with the background (0 + bg, as the reference's
// new_zeros + bg_color), then one thread per (ray, channel) writes its value at the pixel x + W * y -- the index
// computed in float from the float xys and truncated, as the reference's `.long()` of the float expression.
__global__ void scatter_fill_kernel(float* __restrict__ out, int64_t n, int64_t C, const float* __restrict__ bg) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= n) return;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = bg ? 0.0f + bg[(i0 + k) % C] : 0.0f;
  if (i0 + 4 <= n && ((reinterpret_cast<uintptr_t>(out + i0) & 15) == 0)) {
    *(f4*)(out + i0) = f4{v[0], v[1], v[2], v[3]};
  } else {
    for (int k = 0; k < 4 && i0 + k < n; ++k) out[i0 + k] = v[k];
  }
}
__global__ void scatter_rays_kernel(const float* __restrict__ values, const float* __restrict__ xys, int64_t B,
                                    int64_t R, int64_t C, int64_t H, int64_t W, float* __restrict__ out,
                                    int* __restrict__ oob) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * R * C) return;
  const int64_t c = gid % C, br = gid / C, b = br / R;
  const float fi = xys[br * 2 + 0] + (float)W * xys[br * 2 + 1];
  const int64_t pix = (int64_t)fi;
  if (pix < 0 || pix >= H * W) {  // the reference's scatter_ raises on this index: flag it for the caller
    if (oob) *oob = 1;            // (a plain store of the same value from every such lane)
    return;
  }
  out[(b * H * W + pix) * C + c] = values[gid];
}

// torch.optim.Adam's per-element arithmetic (torch/optim/adam.py _multi_tensor_adam, the default on the GPU), op for
// op: the scalars arrive already rounded to float from the host's double arithmetic, exactly as torch casts its
// Python-float scalars, and the multiply-adds are fused where torch's foreach kernels fuse them. Pinned bit for bit by
// tools/adam_emulation_check.py against torch on the MI355X (foreach: weight decay `grad + wd * p`, lerp
// `m + w1 * (g - m)`, addcmul `v * b2 + w2 * (g * g)` and addcdiv `p + (-step_size) * (m / denom)` all fused; the
// denominator a true division) and by tests/test_gpu_trainer.py::test_adam_matches_torch_adam.
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float w1, float b2, float w2, float eps, float wd,
                            float neg_step_size, float bc2_sqrt) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float pi = p[i];
  float gi = g[i];
  if (wd != 0.0f) gi = __fmaf_rn(wd, pi, gi);             // torch._foreach_add(grads, params, alpha=weight_decay)
  const float mi = __fmaf_rn(w1, gi - m[i], m[i]);       // _foreach_lerp_(exp_avgs, grads, 1 - beta1)
  const float vi = __fmaf_rn(w2, gi * gi, v[i] * b2);    // _foreach_mul_(beta2); _foreach_addcmul_(g, g, 1 - beta2)
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;        // _foreach_sqrt; _foreach_div_(bc2_sqrt); _foreach_add_(eps)
  p[i] = __fmaf_rn(neg_step_size, mi / denom, pi);        // _foreach_addcdiv_(params, exp_avgs, denom, -step_size)
}
// the same update with the step's two scalars read on the device from a per-step table (row *index): a graph-captured
// step replays with the schedule's values of the step it runs as. grad_div != 1: the gradients are the sum over the
// data-parallel ranks and are first averaged in place, g = g / world (the true division DDP's `div_` does,
// run.py:162-166), so the exchange's divide costs no launch of its own
__global__ void adam_table_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                  float* __restrict__ v, int64_t n, float w1, float b2, float w2, float eps, float wd,
                                  const float* __restrict__ table, const int64_t* __restrict__ index, float grad_div) {
  const int64_t k = *index;
  const float neg_step_size = table[2 * k], bc2_sqrt = table[2 * k + 1];
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float pi = p[i];
  float gi = g[i];
  if (grad_div != 1.0f) {
    gi = gi / grad_div;
    g[i] = gi;
  }
  if (wd != 0.0f) gi = __fmaf_rn(wd, pi, gi);
  const float mi = __fmaf_rn(w1, gi - m[i], m[i]);
  const float vi = __fmaf_rn(w2, gi * gi, v[i] * b2);
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = __fmaf_rn(neg_step_size, mi / denom, pi);
}
// end of a step: the Philox base moves past the step's draws and the Adam table index to the next step (one thread;
// stream-ordered after every kernel of the step that reads them)
__global__ void step_advance_kernel(uint64_t* state, uint64_t rng_delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    state[0] += rng_delta;
    state[1] += 1;
  }
}

}  // namespace yanerf

using namespace yanerf;

extern "C" {

const char* yanerf_last_error(void) { return g_last_error.c_str(); }
int yanerf_version(void) { return 1; }
#ifndef YANERF_SRC_SHA
#define YANERF_SRC_SHA "unknown"
#endif
const char* yanerf_build_id(void) { return YANERF_SRC_SHA; }

int yanerf_raygen(const float* poses, const float* focal, const float* xy, const int64_t* pixel_ids, int64_t B,
                  int64_t R, int64_t grid_w, int64_t grid_h, float cfg_w, float cfg_h, float near, float far,
                  int64_t P, int jitter_mode, const float* jitter_u, uint64_t seed, uint64_t offset, float* origins,
                  float* directions, float* lengths, float* xys, int64_t* ids_out, const float* bounds,
                  const uint64_t* rng_base, void* stream) {
  YN_CHECK(B >= 0 && R >= 0 && P >= 0, "yanerf_raygen: negative size");
  if (B * R == 0) return 0;  // empty bundles: nothing to read or write (their buffers may be NULL)
  YN_CHECK(poses && focal && origins && directions && xys && (lengths || P == 0), "yanerf_raygen: null pointer");
  YN_CHECK(jitter_mode >= 0 && jitter_mode <= 2, "yanerf_raygen: bad jitter_mode %d", jitter_mode);
  YN_CHECK(jitter_mode != 1 || jitter_u, "yanerf_raygen: jitter_mode 1 needs jitter_u");
  if (!xy && !pixel_ids) YN_CHECK(R <= grid_w * grid_h, "yanerf_raygen: %lld rays > %lld pixels", (long long)R, (long long)(grid_w * grid_h));
  if (!xy) YN_CHECK(grid_w > 0 && grid_h > 0, "yanerf_raygen: grid size needed for pixel ids");
  if (B * R == 0) return 0;
  int64_t n = B * R;
  const int64_t nt = n * ((P + RG_J - 1) / RG_J > 0 ? (P + RG_J - 1) / RG_J : 1);
  hipLaunchKernelGGL(raygen_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, as_stream(stream), poses, focal, xy,
                     pixel_ids, B, R, grid_w, grid_h, cfg_w, cfg_h, near, far, P, jitter_mode, jitter_u, seed, offset,
                     origins, directions, lengths, xys, ids_out, bounds, rng_base);
  YN_LAUNCH_CHECK("raygen");
  return 0;
}

static int composite_common(const yanerf_raymarch_opts* o, int64_t R, int64_t P, int64_t C) {
  YN_CHECK(o, "composite: null opts");
  YN_CHECK(P >= 1 && P <= 64 * kMaxS, "composite: P=%lld out of range [1, %d]", (long long)P, 64 * kMaxS);
  YN_CHECK(C >= 1 && C <= 4, "composite: feature dim %lld out of range [1,4]", (long long)C);
  YN_CHECK(o->capping == 0 || o->capping == 1, "composite: bad capping function");
  YN_CHECK(o->weight_fn == 0 || o->weight_fn == 1, "composite: bad weight function");
  YN_CHECK(o->bg_default_n == 1 || o->bg_default_n == C, "composite: bg colour has %d channels vs %lld features",
           o->bg_default_n, (long long)C);
  return 0;
}

int yanerf_composite_forward(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                             const float* lengths, const float* directions, const float* bg, const float* noise,
                             int64_t R, int64_t P, int64_t C, float* features, float* depths, float* alpha,
                             float* weights, void* stream) {
  if (composite_common(o, R, P, C)) return 1;
  YN_CHECK(R >= 0, "composite_forward: negative size");
  if (R == 0) return 0;
  YN_CHECK(sigma_raw && rgb && lengths && directions && features && depths && alpha && weights,
           "composite_forward: null pointer");
  YN_CHECK(o->noise_mode != 1 || noise, "composite_forward: noise_mode 1 needs noise");
  hipLaunchKernelGGL(composite_kernel<0>, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, as_stream(stream), *o,
                     sigma_raw, rgb, lengths, directions, bg, noise, R, P, C, features, depths, alpha, weights, nullptr,
                     nullptr, nullptr, nullptr, nullptr, CompositeLoss{});
  YN_LAUNCH_CHECK("composite_forward");
  return 0;
}

int yanerf_composite_backward(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                              const float* lengths, const float* directions, const float* bg, const float* noise,
                              const float* g_features, const float* g_depths, const float* g_alpha, int64_t R,
                              int64_t P, int64_t C, float* g_sigma, float* g_rgb, void* stream) {
  if (composite_common(o, R, P, C)) return 1;
  YN_CHECK(R >= 0, "composite_backward: negative size");
  if (R == 0) return 0;
  YN_CHECK(g_features && g_sigma && g_rgb, "composite_backward: null gradient pointer");
  YN_CHECK(o->noise_mode != 1 || noise, "composite_backward: noise_mode 1 needs noise");
  hipLaunchKernelGGL(composite_kernel<1>, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, as_stream(stream), *o,
                     sigma_raw, rgb, lengths, directions, bg, noise, R, P, C, nullptr, nullptr, nullptr, nullptr,
                     g_features, g_depths, g_alpha, g_sigma, g_rgb, CompositeLoss{});
  YN_LAUNCH_CHECK("composite_backward");
  return 0;
}
int yanerf_composite_train(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                           const float* lengths, const float* directions, const float* bg, const float* noise,
                           const float* image, const float* xys, int64_t B, int64_t R, int64_t P, int64_t C,
                           int64_t H, int64_t W, float scale, float* features, float* depths, float* alpha,
                           float* weights, float* sq_err_per_ray, float* g_features, float* g_sigma, float* g_rgb,
                           void* stream) {
  YN_CHECK(B >= 1 && R % B == 0, "composite_train: %lld rays do not split over %lld images", (long long)R,
           (long long)B);
  if (composite_common(o, R, P, C)) return 1;
  YN_CHECK(H > 0 && W > 0, "composite_train: image size %lld x %lld", (long long)H, (long long)W);
  if (R == 0) return 0;
  YN_CHECK(features && depths && alpha && weights && g_sigma && g_rgb && image && xys,
           "composite_train: null pointer");
  YN_CHECK(o->noise_mode != 1 || noise, "composite_train: noise_mode 1 needs noise");
  const CompositeLoss loss{image, xys, R / B, H, W, scale, sq_err_per_ray, g_features};
  hipLaunchKernelGGL(composite_kernel<2>, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, as_stream(stream), *o,
                     sigma_raw, rgb, lengths, directions, bg, noise, R, P, C, features, depths, alpha, weights,
                     nullptr, nullptr, nullptr, g_sigma, g_rgb, loss);
  YN_LAUNCH_CHECK("composite_train");
  return 0;
}

int yanerf_sample_pdf(const float* bins, const float* weights, int64_t R, int64_t nb, int64_t N, int det,
                      const float* u, uint64_t seed, uint64_t offset, float* samples, void* stream) {
  YN_CHECK(nb >= 1 && nb <= kPdfMaxBins, "sample_pdf: n_bins %lld out of range", (long long)nb);
  YN_CHECK(N >= 1, "sample_pdf: N must be >= 1");
  if (R == 0) return 0;
  hipLaunchKernelGGL(sample_pdf_kernel, dim3((unsigned)R), dim3(64), 0, as_stream(stream), bins, weights, R, (int)nb,
                     (int)N, det, u, seed, offset, samples);
  YN_LAUNCH_CHECK("sample_pdf");
  return 0;
}

int yanerf_refine(const float* lengths, const float* ray_weights, int64_t R, int64_t P, int64_t n_fine, int det,
                  const float* u, uint64_t seed, uint64_t offset, int add_input, float* lengths_out,
                  const uint64_t* rng_base, void* stream) {
  YN_CHECK(P >= 3 && P - 2 <= kPdfMaxBins, "refine: P=%lld out of range", (long long)P);
  YN_CHECK(n_fine >= 1, "refine: n_fine must be >= 1");
  YN_CHECK((add_input ? P + n_fine : n_fine) <= kMergeMax, "refine: P + n_fine > %d", kMergeMax);
  if (R == 0) return 0;
  hipLaunchKernelGGL(refine_kernel, dim3((unsigned)R), dim3(64), 0, as_stream(stream), lengths, ray_weights, R, (int)P,
                     (int)n_fine, det, u, seed, offset, add_input, lengths_out, rng_base);
  YN_LAUNCH_CHECK("refine");
  return 0;
}

int yanerf_rgb_loss(const float* pred, const float* image, const float* xys, int64_t B, int64_t R, int64_t H,
                    int64_t W, int64_t C, float scale, float* sq_err_per_ray, float* g_pred, void* stream) {
  YN_CHECK(B >= 0 && R >= 0, "rgb_loss: negative size");
  if (B * R == 0) return 0;
  YN_CHECK(pred && image && xys && sq_err_per_ray, "rgb_loss: null pointer");
  int64_t n = B * R;
  hipLaunchKernelGGL(rgb_loss_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), pred, image,
                     xys, B, R, H, W, C, scale, sq_err_per_ray, g_pred);
  YN_LAUNCH_CHECK("rgb_loss");
  return 0;
}

int yanerf_scatter_rays(const float* values, const float* xys, int64_t B, int64_t R, int64_t C, int64_t H, int64_t W,
                        const float* bg, float* out, int* oob, void* stream) {
  YN_CHECK(B >= 0 && R >= 0 && C >= 1 && H >= 1 && W >= 1, "scatter_rays: bad sizes");
  YN_CHECK(out || B == 0, "scatter_rays: null output");
  YN_CHECK((values && xys) || B * R == 0, "scatter_rays: null pointer");
  const int64_t n = B * H * W * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scatter_fill_kernel, dim3((unsigned)(((n + 3) / 4 + 255) / 256)), dim3(256), 0,
                     as_stream(stream), out, n, C, bg);
  YN_LAUNCH_CHECK("scatter_fill");
  if (B * R == 0) return 0;
  hipLaunchKernelGGL(scatter_rays_kernel, dim3((unsigned)((B * R * C + 255) / 256)), dim3(256), 0, as_stream(stream),
                     values, xys, B, R, C, H, W, out, oob);
  YN_LAUNCH_CHECK("scatter_rays");
  return 0;
}

int yanerf_adam_scalars(double lr, double beta1, double beta2, int64_t step, float* out2) {
  YN_CHECK(step >= 1, "adam: step must be >= 1");
  YN_CHECK(out2, "adam_scalars: null pointer");
  // the host-side scalars in double, as torch computes them in Python (adam.py: bias corrections, step size)
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const double step_size = lr / bc1;
  out2[0] = (float)(-step_size);
  out2[1] = (float)std::sqrt(bc2);
  return 0;
}

int yanerf_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream) {
  YN_CHECK(n >= 0, "adam: negative size");
  float sc[2];
  if (yanerf_adam_scalars(lr, beta1, beta2, step, sc)) return 1;
  if (n == 0) return 0;
  YN_CHECK(params && grads && exp_avg && exp_avg_sq, "adam: null pointer");
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), params, grads,
                     exp_avg, exp_avg_sq, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     (float)weight_decay, sc[0], sc[1]);
  YN_LAUNCH_CHECK("adam");
  return 0;
}

int yanerf_adam_table(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const float* table, const int64_t* index, double beta1, double beta2, double eps,
                      double weight_decay, int64_t avg_over, void* stream) {
  YN_CHECK(n >= 0, "adam_table: negative size");
  YN_CHECK(avg_over >= 1 && avg_over <= (1 << 24), "adam_table: avg_over %lld", (long long)avg_over);
  if (n == 0) return 0;
  YN_CHECK(params && grads && exp_avg && exp_avg_sq && table && index, "adam_table: null pointer");
  hipLaunchKernelGGL(adam_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), params,
                     grads, exp_avg, exp_avg_sq, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                     (float)eps, (float)weight_decay, table, index, (float)avg_over);
  YN_LAUNCH_CHECK("adam_table");
  return 0;
}

int yanerf_step_advance(uint64_t* state, uint64_t rng_delta, void* stream) {
  YN_CHECK(state, "step_advance: null pointer");
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, as_stream(stream), state, rng_delta);
  YN_LAUNCH_CHECK("step_advance");
  return 0;
}

}  // extern "C"
