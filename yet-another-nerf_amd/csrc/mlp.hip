// NeRF MLP on gfx950: fused harmonic embedding + 8x256 trunk (skip) + heads, forward and backward.
//
// Reference: NeRFMLP (yanerf/pipelines/models/nerf_mlp.py:12-183), MLPWithInputSkips (:186-289),
// HarmonicEmbedding / LinearWithRepeat (yanerf/pipelines/models/utils.py:17-211).
//
// Formulation: every layer is computed TRANSPOSED, out[feature n][point m] = sum_k W[n][k] act[m][k], so
//   * A operand = weights, read straight from L2 in PyTorch's [out][in] layout (16 B per lane),
//   * B operand = the point tile's activations, resident in LDS as point-major rows act[m][k],
//   * the 16x16 accumulator holds 4 consecutive features of one point per lane, which is exactly one
//     16-byte (fp32) / 8-byte (bf16) row segment of the next layer's LDS tile.
// One workgroup owns a tile of M points for the whole network (PE -> 8 layers -> heads), so activations
// never leave the CU between layers. Weights (1.19 MB bf16 / 2.4 MB fp32 per model) stream from the
// XCD's L2. Both precisions use the same byte geometry: a K-block is 64 B of a row (16 fp32 = 4 x
// v_mfma_f32_16x16x4_f32 with k permuted consistently on both operands, or 32 bf16 = 1 x
// v_mfma_f32_16x16x32_bf16).
//
// LDS image: act[M][320] (cols 0..255 hidden, 256..319 xyz-PE / dir-PE), 16-byte chunks XOR-swizzled by
// row so the 16 rows a ds_read_b128 lane group touches land on distinct bank slots.
//
// Backward: (1) a fused dX kernel walks the heads and trunk in reverse for a point tile, writing every
// layer's pre-activation gradient dZ_l (feature-major, [row][point]); (2) a split-K dW kernel computes
// dW_l = sum_points dZ_l x input_l (+ a virtual ones-row giving the bias gradient) into fp32 partial slabs,
// (3) a deterministic reduce sums the slabs straight into the reference-layout parameter gradients.
#include <type_traits>

#include "common.hpp"

// The measured alternatives of rounds 1-3 (build macros selecting A/B variants and timing ablations) were removed in
// round 4; every variant below is the measured default. DESIGN.md §9 lists them with the commits that measured them.

namespace yanerf {

typedef unsigned short bf16_t;

// fp32 emulated on bf16 MFMAs: every operand is split into three bf16 planes (x = x0 + x1 + x2 exactly) and a
// product is the six terms x_i y_j with i + j <= 2 (the dropped ones are below 2^-24 relative)
struct x3_t {};

// per precision: point tile M, waves per workgroup, elements per 16-byte chunk (EPC) and per 64-byte K-block (KB),
// weight-ring depth, occupancy target (waves per SIMD), operand planes, and the element types of the LDS tile,
// of the saved activations / gradients in HBM and of the packed weights
//
// fp32: 64-point tiles, 4 waves, two workgroups per CU (WPE); 32-point tiles at 3-4 workgroups per CU, two tiles per
// workgroup and 5-wave store-wave workgroups all measured slower.
// bf16: 4 waves x (64 features x 128 points) for the forward and the dX kernel -- half the LDS operand reads per MFMA of
// an 8-wave (32 x 128) tiling: training forward 1.47 -> 1.26 ms, dX 1.40 -> 1.26 ms (round 1). PM: saved activations /
// backward gradients stored point-major in per-section arrays ([Npad][width], written from the LDS tile with 16-byte
// stores, read by the dW kernel with transposed LDS reads) instead of feature-major rows.
template <typename T> struct Cfg;
template <> struct Cfg<float> {
  static constexpr int M = 64, WAVES = 4, DXWAVES = 4, EPC = 4, KB = 16, APREF = 1, WPE = 2, PLANES = 1;
  static constexpr bool PM = false;
  typedef float lds_t;
  typedef float st_t;
  typedef float w_t;
};
template <> struct Cfg<bf16_t> {
  static constexpr int M = 128, WAVES = 4, DXWAVES = 4, EPC = 8, KB = 32, APREF = 2, WPE = 2, PLANES = 1;
  static constexpr bool PM = true;
  typedef bf16_t lds_t;
  typedef bf16_t st_t;
  typedef bf16_t w_t;
};
template <> struct Cfg<x3_t> {
  static constexpr int M = 64, WAVES = 8, DXWAVES = 8, EPC = 8, KB = 32, APREF = 2, WPE = 2, PLANES = 3;
  static constexpr bool PM = false;
  typedef bf16_t lds_t;
  typedef float st_t;
  typedef bf16_t w_t;
};
template <typename T> constexpr bool is_x3 = false;
template <> constexpr bool is_x3<x3_t> = true;

constexpr int ROW = 320;    // LDS row length (elements)
constexpr int PE_COL = 256; // xyz-PE / dir-PE column base
constexpr int KPE = 64;     // padded xyz PE width
constexpr int KDIR = 32;    // padded dir PE width
constexpr int KC = 288;     // color layer K (256 + 32)
constexpr int HC = 128;     // padded color hidden width
constexpr int CMAX = 4;
constexpr int MAXL = 16;

struct MlpLayout {
  int L;
  uint32_t skip;
  int fx, fd, ax, ad, xyz_dim, dir_dim, hid, hdir, cdim;
  int64_t w_off[MAXL];
  int kpad[MAXL];
  int64_t wt_off[MAXL];
  int64_t wint_off, wintT_off, wc_off, wcT_off;
  int64_t wdh_off, woh_off;  // density / colour-output heads as 16-row GEMM operands (rows past 1 / cdim are 0)
  int64_t t_elems;
  int64_t t_plane;  // elements between the bf16 planes of an x3 operand (0 otherwise)
  int64_t f_base;  // byte offset of the fp32 section
  int64_t b_off[MAXL];
  int64_t bint_off, bc_off, wd_off, bd_off, wo_off, bo_off;
  int64_t f_elems;
  int64_t bytes;
  int s16;  // YANERF_PREC_BF16S: point-major sections and gradient rows in bf16 (no fp8)
};

// saved activation rows (each row_ld(Npad) elements of T)
struct SavedRows {
  int64_t pe, h0, y, dpe, c, rows;
};
__host__ __device__ inline SavedRows saved_rows(int L) {
  SavedRows s;
  s.pe = 0;
  s.h0 = KPE;
  s.y = s.h0 + 256LL * L;
  s.dpe = s.y + 256;
  s.c = s.dpe + KDIR;
  s.rows = s.c + HC;
  return s;
}
// backward gradient rows
struct GradRows {
  int64_t dz0, dyx, dzc, du, rows;
};
__host__ __device__ inline GradRows grad_rows(int L, bool pm = false) {
  GradRows g;
  g.dz0 = 0;
  g.dyx = 256LL * L;  // feature-major: 256 rows dY + 1 row dsigma; point-major: dY [Npad][256] (dsigma in dU)
  g.dzc = g.dyx + (pm ? 256 : 257);
  g.du = g.dzc + HC;  // point-major dU [Npad][16]: du_j at column j, dsigma at column PM_DSIG
  g.rows = g.du + 16;
  return g;
}
constexpr int PM_DSIG = 8;
// Point-major (Cfg::PM) storage: the section that starts at feature-row r0 (saved_rows / grad_rows offsets) with width
// w is an [Npad][w] array at element r0 * Npad; element (point p, column c) at r0 * Npad + p * w + c.

// ReLU masks, kept for the dX kernel instead of re-reading the saved activations:
//  * trunk layers: the forward and dX kernels share one wave->tile decomposition (Cfg<T>), so every lane packs
//    ITS OWN 4 bits of each of its NT*MT (16; 8 for x3) accumulator tiles into one u64 per layer
//    (index ((layer * n_wg + wg) * WAVES + wave) * 64 + lane, trunk_mask_words per layer): one coalesced 8-byte
//    load per lane in dX;
//  * colour hidden layer: the __ballot of each 16x16 tile (4 u64 words; bit `lane` = feature 4*(lane>>4)+r of
//    point lane&15), read per point by the VALU colour-head backward.
// Both are 256 bits per point per layer (trunk: 512 in x3, whose 8-wave tiles hold 64 points).
__host__ __device__ inline int64_t mask_words_per_slot(int64_t Npad) { return Npad / 16 * 16 * 4; }
// u64 mask words per lane per trunk layer: 4 bits for each of the lane's NT x MT accumulator tiles, 16 tiles a word
template <typename T> __host__ __device__ constexpr int mask_w() {
  return ((256 / 16 / Cfg<T>::WAVES) * (Cfg<T>::M / 16) + 15) / 16;
}
// u64 words of one trunk layer's per-lane masks, indexed ((wg * WAVES + wave) * MW + w) * 64 + lane
template <typename T> __host__ __device__ inline int64_t trunk_mask_words(int64_t Npad) {
  return Npad / Cfg<T>::M * Cfg<T>::WAVES * 64 * mask_w<T>();
}
static bool prec_bf16(int prec);
static int64_t trunk_mask_words_prec(int prec, int64_t Npad) {
  return prec == YANERF_PREC_F32 ? trunk_mask_words<float>(Npad)
         : prec_bf16(prec)       ? trunk_mask_words<bf16_t>(Npad)
                                 : trunk_mask_words<x3_t>(Npad);
}
__device__ __forceinline__ int64_t mask_index(int64_t Npad, int slot, int64_t pt16, int ft) {
  return (((int64_t)slot * (Npad / 16) + pt16) * 16 + ft) * 4;
}
// Row stride of the feature-major saved / gradient buffers: Npad padded so a row is an ODD multiple of 256 B.
// With Npad a multiple of large powers of two, equal points of consecutive rows would otherwise sit on the
// same HBM channel, and a dW stage reading 384 rows at one point offset would hit that one channel.
__host__ __device__ inline int64_t row_ld(int64_t Npad, size_t es) {
  int64_t units = (Npad * (int64_t)es + 255) / 256;
  if ((units & 1) == 0) ++units;
  return units * 256 / (int64_t)es;
}
// bf16 point-major saves (Cfg<bf16_t>::PM): the non-negative (post-ReLU) sections -- H_0..H_{L-1} and the colour hidden
// C, 2,176 of the 2,528 values a point saves -- are stored as fp8 e4m3 (OCP e4m3fn, 1 byte; values clamped to its 448
// maximum, round to nearest even by v_cvt_scalef32_pk_fp8_bf16; exact-RNE against the e4m3fn definition on the MI355X:
// tools/probes/probe_fp8.hip), the signed ones (PE, Y, dir-PE) stay bf16. They are the weight gradients' X operands
// only (the dX kernel uses the ReLU mask words, never the activations), and the dW tile widens them back to bf16 (exact)
// for the bf16 MFMA. Measured on a trained model (procedural scene, 3k steps): dW relative L2 error 0.6-0.9 % from the
// fp8 rounding, against 0.03 % from bf16 storage and >10 % from the bf16 forward chain itself. Layout: byte offsets of
// [Npad][width] sections (round-2 A/B: bf16 backward 2.85 -> 2.16 ms against bf16 sections).
constexpr int PM_HB = 1;  // bytes per saved H / C element
// Y (intermediate_linear's output, signed, the X operand of color_layer.0's weight gradient only) as fp8 e4m3 with a
// power-of-two scale per 128-point tile, like the backward's gradient rows
constexpr int PM_YB = 1;
// YANERF_PREC_BF16S (s16): the same point-major sections, all bf16 (H, Y, C, and the gradient rows: 2 bytes)
__host__ __device__ constexpr int pm_hb(bool s16) { return s16 ? 2 : PM_HB; }
__host__ __device__ constexpr int pm_yb(bool s16) { return s16 ? 2 : PM_YB; }
struct PmSave {
  int64_t pe, h0, y, dpe, c, ysc, total;
};
__host__ __device__ inline PmSave pm_save(int L, int64_t Npad, bool s16 = false) {
  PmSave s;
  int64_t o = 0;
  s.pe = o; o += 2LL * KPE * Npad;
  s.h0 = o; o += (int64_t)pm_hb(s16) * 256 * L * Npad;
  s.y = o; o += (int64_t)pm_yb(s16) * 256 * Npad;
  s.dpe = o; o += 2LL * KDIR * Npad;
  s.c = o; o += (int64_t)pm_hb(s16) * HC * Npad;
  s.ysc = o; o += 4LL * (Npad / 128);
  s.total = (o + 255) / 256 * 256;
  return s;
}
// byte offset and element bytes of the saved section that starts at SavedRows row r0 (point-major bf16 layout)
static int64_t pm_sec_bytes(int L, int64_t Npad, int64_t r0, int* es, int64_t* scale_off = nullptr, bool s16 = false) {
  const SavedRows SR = saved_rows(L);
  const PmSave PS = pm_save(L, Npad, s16);
  *es = 2;
  if (r0 == SR.pe) return PS.pe;
  if (r0 >= SR.h0 && r0 < SR.y) {
    *es = pm_hb(s16);
    return PS.h0 + (r0 - SR.h0) / 256 * (int64_t)pm_hb(s16) * 256 * Npad;
  }
  if (r0 == SR.y) {
    *es = pm_yb(s16);
    if (scale_off && !s16) *scale_off = PS.ysc;
    return PS.y;
  }
  if (r0 == SR.dpe) return PS.dpe;
  *es = pm_hb(s16);
  return PS.c;  // r0 == SR.c
}
constexpr int PM_GB = 1;  // bytes per dZ / dY / dZc element in the bf16 backward workspace (fp8 e4m3, scaled)
__host__ __device__ constexpr int pm_gb(bool s16) { return s16 ? 2 : PM_GB; }
// bf16 backward workspace (point-major): byte offsets of the gradient sections, the dU section (bf16: du_j at column j,
// dsigma at PM_DSIG) and the per-(section, 128-point tile) fp8 scales (float; sections dZ_0..dZ_{L-1}, dY, dZc)
struct PmGrad {
  int64_t dz0, dy, dzc, du, scale, total;
};
__host__ __device__ inline PmGrad pm_grad(int L, int64_t Npad, bool s16 = false) {
  PmGrad g;
  int64_t o = 0;
  g.dz0 = o; o += (int64_t)pm_gb(s16) * 256 * L * Npad;
  g.dy = o; o += (int64_t)pm_gb(s16) * 256 * Npad;
  g.dzc = o; o += (int64_t)pm_gb(s16) * HC * Npad;
  g.du = o; o += 2LL * 16 * Npad;
  g.scale = o; o += 4LL * (L + 2) * (Npad / 128);
  g.total = (o + 255) / 256 * 256;
  return g;
}
// byte offset, element bytes and scale array (or null) of the gradient section starting at GradRows row r0
static int64_t pm_grad_sec(int L, int64_t Npad, int64_t r0, int* es, int64_t* scale_off, bool s16 = false) {
  const GradRows GR = grad_rows(L, true);
  const PmGrad PG = pm_grad(L, Npad, s16);
  *es = pm_gb(s16);
  *scale_off = -1;
  int sec;
  int64_t off;
  if (r0 >= GR.dz0 && r0 < GR.dyx) {
    sec = (int)((r0 - GR.dz0) / 256);
    off = PG.dz0 + (int64_t)sec * pm_gb(s16) * 256 * Npad;
  } else if (r0 == GR.dyx) {
    sec = L;
    off = PG.dy;
  } else if (r0 == GR.dzc) {
    sec = L + 1;
    off = PG.dzc;
  } else {  // dU (bf16, unscaled)
    *es = 2;
    return PG.du;
  }
  if (!s16) *scale_off = PG.scale + 4LL * sec * (Npad / 128);
  return off;
}
// backward workspace bytes before the dW slabs
static int64_t grad_t_bytes(int L, int64_t Npad, size_t es, bool pm, bool s16 = false) {
  if (pm) return pm_grad(L, Npad, s16).total;
  return grad_rows(L).rows * row_ld(Npad, es) * (int64_t)es;
}
static int64_t saved_t_bytes(int L, int64_t Npad, size_t es, bool pm, bool s16 = false) {
  if (pm) return pm_save(L, Npad, s16).total;
  return saved_rows(L).rows * row_ld(Npad, es) * (int64_t)es;
}

// the bf16 kernels serve both bf16 precisions (YANERF_PREC_BF16S only changes the storage of the saved sections)
static bool prec_bf16(int prec) { return prec == YANERF_PREC_BF16 || prec == YANERF_PREC_BF16S; }
static int64_t tile_m(int prec) {
  return prec == YANERF_PREC_F32 ? Cfg<float>::M : prec_bf16(prec) ? Cfg<bf16_t>::M : Cfg<x3_t>::M;
}
// Npad: a multiple of the point tile, so every workgroup holds a whole tile
static int64_t npad_of(int prec, int64_t n) {
  const int64_t M = tile_m(prec);
  return (n + M - 1) / M * M;
}
// element size of the saved activations / gradient rows (fp32 for both fp32 modes)
static size_t elem_size(int prec) { return prec_bf16(prec) ? 2 : 4; }
// element size and plane count of the packed GEMM operands
static size_t w_size(int prec) { return prec == YANERF_PREC_F32 ? 4 : 2; }
static int w_planes(int prec) { return prec == YANERF_PREC_F32X3 ? 3 : 1; }
static bool prec_pm(int prec) {
  return prec == YANERF_PREC_F32 ? Cfg<float>::PM : prec_bf16(prec) ? Cfg<bf16_t>::PM : Cfg<x3_t>::PM;
}

static int check_desc(const yanerf_mlp_desc* d) {
  YN_CHECK(d, "mlp: null desc");
  YN_CHECK(d->n_layers >= 1 && d->n_layers <= MAXL, "mlp: n_layers %d out of [1,%d]", d->n_layers, MAXL);
  YN_CHECK((d->skip_mask & 1u) == 0, "mlp: a skip at layer 0 is not defined by the reference");
  int xyz_dim = 3 * (2 * d->n_freq_xyz + (d->append_xyz ? 1 : 0));
  int dir_dim = 3 * (2 * d->n_freq_dir + (d->append_dir ? 1 : 0));
  YN_CHECK(d->n_freq_xyz >= 0 && xyz_dim <= KPE && xyz_dim > 0, "mlp: xyz embedding dim %d unsupported (<= %d)",
           xyz_dim, KPE);
  YN_CHECK(d->n_freq_dir >= 0 && dir_dim <= KDIR, "mlp: dir embedding dim %d unsupported (<= %d)", dir_dim, KDIR);
  YN_CHECK(d->hidden_xyz >= 1 && d->hidden_xyz <= 256, "mlp: n_hidden_neurons_xyz %d unsupported", d->hidden_xyz);
  YN_CHECK(d->hidden_dir >= 1 && d->hidden_dir <= HC, "mlp: n_hidden_neurons_dir %d unsupported", d->hidden_dir);
  YN_CHECK(d->color_dim >= 1 && d->color_dim <= CMAX, "mlp: color_dim %d unsupported", d->color_dim);
  return 0;
}

static MlpLayout make_layout(const yanerf_mlp_desc* d, int prec) {
  MlpLayout L{};
  L.L = d->n_layers;
  L.skip = d->skip_mask;
  L.fx = d->n_freq_xyz;
  L.fd = d->n_freq_dir;
  L.ax = d->append_xyz;
  L.ad = d->append_dir;
  L.xyz_dim = 3 * (2 * d->n_freq_xyz + (d->append_xyz ? 1 : 0));
  L.dir_dim = 3 * (2 * d->n_freq_dir + (d->append_dir ? 1 : 0));
  L.hid = d->hidden_xyz;
  L.hdir = d->hidden_dir;
  L.cdim = d->color_dim;
  int64_t t = 0;
  for (int l = 0; l < L.L; ++l) {
    L.kpad[l] = (l == 0) ? KPE : ((L.skip >> l) & 1u) ? 320 : 256;
    L.w_off[l] = t;
    t += 256LL * L.kpad[l];
  }
  for (int l = 1; l < L.L; ++l) {
    L.wt_off[l] = t;
    t += 256LL * 256;
  }
  L.wint_off = t; t += 256LL * 256;
  L.wintT_off = t; t += 256LL * 256;
  L.wc_off = t; t += (int64_t)HC * KC;
  L.wcT_off = t; t += 256LL * HC;
  L.wdh_off = t; t += 16LL * 256;
  L.woh_off = t; t += 16LL * HC;
  L.t_elems = t;
  L.t_plane = w_planes(prec) > 1 ? t : 0;
  int64_t tb = t * (int64_t)w_size(prec) * w_planes(prec);
  L.f_base = (tb + 255) / 256 * 256;
  int64_t f = 0;
  for (int l = 0; l < L.L; ++l) { L.b_off[l] = f; f += 256; }
  L.bint_off = f; f += 256;
  L.bc_off = f; f += HC;
  L.wd_off = f; f += 256;
  L.bd_off = f; f += 4;
  L.wo_off = f; f += CMAX * HC;
  L.bo_off = f; f += CMAX;
  L.f_elems = f;
  L.bytes = L.f_base + f * 4;
  L.s16 = prec == YANERF_PREC_BF16S;
  return L;
}

// ============================================================================================ pack
struct PackJob {
  const float* src;
  void* dst;            // the job's first output: the model's T section + dst_off elements, or its fp32 section + dst_off
  int32_t elem_base;    // the job's first element in the launch's element space (4-column groups, jobs back to back)
  int32_t t_plane;      // x3: elements per bf16 plane of the job's model
  int16_t src_rows, src_ld, rows, cols;
  int16_t seg0, seg1_start, seg1_len;
  uint8_t transpose, is_f32;
};
// one launch packs up to this many jobs (two default-size MLPs: 2 x 35); 40 B each keeps the kernel arguments < 4 KB
constexpr int kMaxPackJobs = 96;
struct PackJobs {
  PackJob j[kMaxPackJobs];
  int n;
  int32_t total;
};

// One thread per 4 consecutive columns of one row of a job (every job's cols is a multiple of 4, so a group never
// straddles jobs or rows, and in fragment order its 4 outputs are contiguous: c % EPC runs over an aligned 4 of EPC).
// The jobs of several MLPs (the trainer's coarse and fine models) go in one launch.
template <typename T>
__global__ void pack_kernel(PackJobs jobs) {
  const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e0 >= jobs.total) return;
  int lo = 0, hi = jobs.n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (jobs.j[mid].elem_base <= e0) lo = mid; else hi = mid - 1;
  }
  const PackJob& J = jobs.j[lo];
  const int64_t local0 = e0 - J.elem_base;
  const int cols = J.cols;
  const int r = (int)(local0 / cols), c0 = (int)(local0 % cols);
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + i;
    const int n = J.transpose ? c : r;  // output-feature index
    const int k = J.transpose ? r : c;  // input-feature index (packed column)
    int sk = -1;
    if (k < J.seg0) sk = k;
    else if (k >= J.seg1_start && k < J.seg1_start + J.seg1_len) sk = J.seg0 + (k - J.seg1_start);
    v[i] = (sk >= 0 && n < J.src_rows) ? J.src[(int64_t)n * J.src_ld + sk] : 0.0f;
  }
  if (J.is_f32) {
    *(f4*)((float*)J.dst + local0) = f4{v[0], v[1], v[2], v[3]};
    return;
  }
  // GEMM operands are stored in MFMA A-fragment order: for each 16-row tile and 64-byte K-block, 64 lanes x 16 B,
  // lane = 16 * (k-chunk) + (row within the tile), so one wave-wide 16-byte load reads 1 KiB contiguously
  constexpr int KB = Cfg<T>::KB, EPC = Cfg<T>::EPC;
  const int64_t fi = (((int64_t)(r >> 4) * (cols / KB) + c0 / KB) * 64 + ((c0 % KB) / EPC) * 16 + (r & 15)) * EPC +
                     c0 % EPC;
  if constexpr (is_x3<T>) {
    // three bf16 planes, x = x0 + x1 + x2 exactly (each residual is exact in fp32)
    bf16_t x[3][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[0][i] = f2bf(v[i]);
      const float r1 = v[i] - bf2f(x[0][i]);
      x[1][i] = f2bf(r1);
      x[2][i] = f2bf(r1 - bf2f(x[1][i]));
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const uint2 w = {(uint32_t)x[pl][0] | ((uint32_t)x[pl][1] << 16), (uint32_t)x[pl][2] | ((uint32_t)x[pl][3] << 16)};
      *(uint2*)((bf16_t*)J.dst + (int64_t)pl * J.t_plane + fi) = w;
    }
  } else if constexpr (sizeof(T) == 4) {
    *(f4*)((float*)J.dst + fi) = f4{v[0], v[1], v[2], v[3]};
  } else {
    const uint2 w = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                     (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
    *(uint2*)((bf16_t*)J.dst + fi) = w;
  }
}

// ============================================================================================ device core
template <typename T> __device__ __forceinline__ int swz(int m, int c);
template <> __device__ __forceinline__ int swz<float>(int m, int c) { return c ^ (m & 15); }
template <> __device__ __forceinline__ int swz<bf16_t>(int m, int c) { return c ^ ((m >> 1) & 7); }
template <> __device__ __forceinline__ int swz<x3_t>(int m, int c) { return c ^ ((m >> 1) & 7); }

template <typename T> __device__ __forceinline__ int lds_idx(int m, int col) {
  constexpr int EPC = Cfg<T>::EPC;
  return m * ROW + swz<T>(m, col / EPC) * EPC + (col % EPC);
}
template <typename T> __device__ __forceinline__ f4 lds_chunk(const typename Cfg<T>::lds_t* act, int m, int c) {
  return *(const f4*)(act + m * ROW + swz<T>(m, c) * Cfg<T>::EPC);
}
// x3: split an fp32 value into three bf16 terms, v = t0 + t1 + t2 exactly (each residual is exact in fp32)
__device__ __forceinline__ void split3(float v, bf16_t& t0, bf16_t& t1, bf16_t& t2) {
  t0 = f2bf(v);
  const float r1 = v - bf2f(t0);
  t1 = f2bf(r1);
  t2 = f2bf(r1 - bf2f(t1));
}
// write one value into LDS element (m, col) in T's representation (x3: three planes, plane stride M * ROW)
template <typename T> __device__ __forceinline__ void lds_put1(typename Cfg<T>::lds_t* act, int m, int col, float v) {
  const int i = m * ROW + swz<T>(m, col / Cfg<T>::EPC) * Cfg<T>::EPC + (col % Cfg<T>::EPC);
  if constexpr (is_x3<T>) {
    constexpr int PL = Cfg<T>::M * ROW;
    bf16_t t0, t1, t2;
    split3(v, t0, t1, t2);
    act[i] = t0;
    act[PL + i] = t1;
    act[2 * PL + i] = t2;
  } else if constexpr (sizeof(typename Cfg<T>::lds_t) == 4) {
    act[i] = v;
  } else {
    act[i] = f2bf(v);
  }
}
// write EPC consecutive values (one 16-byte chunk c of row m) into LDS in T's representation
template <typename T>
__device__ __forceinline__ void lds_put_chunk(typename Cfg<T>::lds_t* act, int m, int c, const float (&v)[Cfg<T>::EPC]) {
  const int i = m * ROW + swz<T>(m, c) * Cfg<T>::EPC;
  if constexpr (sizeof(typename Cfg<T>::lds_t) == 4) {
    *(f4*)(act + i) = f4{v[0], v[1], v[2], v[3]};
  } else {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef float f2_ __attribute__((ext_vector_type(2)));
    typedef __bf16 bh2_ __attribute__((ext_vector_type(2)));
    auto pk2 = [](float a, float b) {
      return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_{a, b}, bh2_));
    };
    if constexpr (is_x3<T>) {
      constexpr int PL = Cfg<T>::M * ROW;
      float r1[8], r2[8];
      u32x4 w0, w1, w2;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t h = pk2(v[e], v[e + 1]);
        w0[e / 2] = h;
        r1[e] = v[e] - __uint_as_float(h << 16);
        r1[e + 1] = v[e + 1] - __uint_as_float(h & 0xffff0000u);
        const uint32_t h1 = pk2(r1[e], r1[e + 1]);
        w1[e / 2] = h1;
        r2[e] = r1[e] - __uint_as_float(h1 << 16);
        r2[e + 1] = r1[e + 1] - __uint_as_float(h1 & 0xffff0000u);
        w2[e / 2] = pk2(r2[e], r2[e + 1]);
      }
      *(u32x4*)(act + i) = w0;
      *(u32x4*)(act + PL + i) = w1;
      *(u32x4*)(act + 2 * PL + i) = w2;
    } else {
      *(u32x4*)(act + i) = u32x4{pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7])};
    }
  }
}
// one value in T's saved / gradient row representation
template <typename T> __device__ __forceinline__ typename Cfg<T>::st_t to_st(float v) {
  if constexpr (sizeof(typename Cfg<T>::st_t) == 4) return v;
  else return f2bf(v);
}
template <typename T> __device__ __forceinline__ T to_t(float v);
template <> __device__ __forceinline__ float to_t<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t to_t<bf16_t>(float v) { return f2bf(v); }
template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }

template <typename T> __device__ __forceinline__ f4 mma_blk(f4 a, f4 b, f4 c);
template <> __device__ __forceinline__ f4 mma_blk<float>(f4 a, f4 b, f4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}
template <> __device__ __forceinline__ f4 mma_blk<bf16_t>(f4 a, f4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}
// (x3 operands are single bf16 planes at this level; gemm_lds combines the six plane products)
template <> __device__ __forceinline__ f4 mma_blk<x3_t>(f4 a, f4 b, f4 c) { return mma_blk<bf16_t>(a, b, c); }

// acc[i][j] += A_i x B_j over one 64-byte K-block for a grid of independent accumulators. fp32: the four
// 16x16x4 k-steps are the OUTER loop so consecutive MFMAs never depend on each other (dependent-accumulator
// latency 40 cycles > 32-cycle issue); bf16: one 16x16x32 per pair.
// SWAP: multiply b x a instead (the C tile comes out transposed: lane (g, li) holds column li of rows 4g..4g+3 of
// the b side)
template <typename T, int NI, int NJ, bool SWAP = false>
__device__ __forceinline__ void mma_grid(const f4 (&a)[NI], const f4 (&b)[NJ], f4 (&acc)[NI][NJ]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][s], a[i][s], acc[i][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = SWAP ? mma_blk<T>(b[j], a[i], acc[i][j]) : mma_blk<T>(a[i], b[j], acc[i][j]);
  }
}

// acc[nt][mt] (rows nrow0 + 16nt.., points 16mt..) = W[rows][kblocks] x act[points][kblocks]^T
//
// bf16: a K-block is only 16 MFMAs per wave (256 cycles), shorter than an L2 round trip, so the weight fragments
// stream through a register ring APREF K-blocks deep and the LDS fragments of block kb+1 are read while block kb
// multiplies (the loop is unrolled by the ring depth so every ring slot is a static register set). Loads past the
// last K-block re-read the last block (uniform, in-bounds, a few redundant L2 hits per layer).
// bf16 weight-fragment ring (see gemm_lds). A caller may fill it for the NEXT GEMM before running the current
// layer's epilogue, so that GEMM starts on weights already in registers instead of an L2 round trip.
template <typename T, int NT> struct ARing { f4 a[Cfg<T>::APREF][Cfg<T>::PLANES][NT]; };
template <typename T, int NT, bool OPQ = false>
__device__ __forceinline__ void ring_fill(ARing<T, NT>& R, const typename Cfg<T>::w_t* __restrict__ W, int64_t wplane,
                                          int ldw, int nrow0, int nkb, int lane) {
  if constexpr (sizeof(typename Cfg<T>::w_t) == 2) {
    constexpr int D = Cfg<T>::APREF, EPC = Cfg<T>::EPC, KB = Cfg<T>::KB, FRAG = 64 * EPC, NP = Cfg<T>::PLANES;
    // OPQ (the dX layer loop): an opaque lane id, as in gemm_run, so the per-lane weight base is recomputed per fill
    // instead of being hoisted out of the loop and spilled -- the bf16 dX reloaded it every layer, and the scratch
    // reload waited (shared in-order vmcnt) for all of the wave's gradient-row stores: dX 1.01 -> 0.935 ms. (The
    // forward keeps the hoisted base: opaque there it measured 0.94 -> 0.96 ms.)
    if constexpr (OPQ) asm volatile("" : "+v"(lane));
#pragma unroll
    for (int r = 0; r < D; ++r) {
      const int k = r < nkb ? r : nkb - 1;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          R.a[r][pl][nt] = *(const f4*)(W + pl * wplane +
                                        ((size_t)((nrow0 >> 4) + nt) * (ldw / KB) * 64 + lane) * EPC + k * FRAG);
    }
  }
}

// Accumulator layout: acc[nt][mt] lane (g, li) holds features nrow0 + 16nt + 4g .. +3 of point 16mt + li. The
// accumulators start from the bias when one is given (the reference's addmm also accumulates onto the bias).
// fp32 forward: the saved rows of the GEMM's input (post-ReLU H of the previous layer, as the LDS tile holds it) are
// written from the B fragments during the GEMM instead of from the accumulators in the previous epilogue. Wave w stores
// K-blocks kb = w, w + 4, ... (all of the tile's points), after that K-block's MFMAs: each weight wait then covers the
// stores of one earlier K-block rather than the whole epilogue's burst (training forward 7.78 -> 7.61 ms). The fp32 dX
// does the same for dY and dZ_l, with a K-block's stores BEFORE its MFMAs (6.88 ms, against 7.29 ms after them).
// RSV (gemm_run / gemm_lds template argument): 0 no row stores, 1 a K-block's stores after its MFMAs (the forward),
// 2 before them (the dX kernel).
constexpr int RSV_FWD = 1, RSV_DX = 2;
// fp32 saved / gradient rows with non-temporal stores (the rows are read back by the dW kernel milliseconds and
// gigabytes later, never from L2; the weight fragments the GEMMs stream share that L2): training forward 7.59 -> 7.53
// ms, bitwise equal. x3 keeps plain stores (its dX measured 4.43 -> 4.56 ms with them).
template <bool NT = true>
__device__ __forceinline__ void st_row_f32(const char* p, float v) {
  if constexpr (NT) __builtin_nontemporal_store(v, (float*)p);
  else *(float*)p = v;
}
struct RowSave {
  float* base;    // saved row of the GEMM's feature 0 at the tile's first point
  uint32_t voff;  // this lane's byte offset in a 16x16 row tile (4g rows + li points)
  int ldb;        // row stride, bytes
  int nkb;        // K-blocks to store (the H columns; a skip layer's PE columns are saved elsewhere)
  int wave, waves;
};

template <typename T, int NT, int MT, int RSV = 0>
__device__ __forceinline__ void gemm_run(const typename Cfg<T>::w_t* __restrict__ W, int64_t wplane, int ldw, int nrow0,
                                         const typename Cfg<T>::lds_t* act, int kc0, int nkb, f4 (&acc)[NT][MT],
                                         int lane, const float* __restrict__ bias, ARing<T, NT>& R,
                                         const RowSave& rs = RowSave{}) {
  constexpr int EPC = Cfg<T>::EPC, KB = Cfg<T>::KB;
  // an opaque copy of the lane id: the per-K-block LDS fragment addresses (the row swizzle makes each one distinct)
  // and weight pointers are then recomputed at every call instead of being hoisted out of the caller's layer loop,
  // where they would hold ~16 VGPRs across every GEMM (spilled and reloaded in the 4-wave dX and the x3 dX)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int g = ln >> 4, li = ln & 15;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const f4 b0 = bias ? *(const f4*)(bias + nrow0 + 16 * nt + 4 * g) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = b0;
  }
  // W is in A-fragment order (pack_kernel): row tile rt, K-block kb at ((rt * ldw / KB + kb) * 64 + lane) * EPC
  const typename Cfg<T>::w_t* wp[NT];
  constexpr int FRAG = 64 * EPC;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wp[nt] = W + ((size_t)((nrow0 >> 4) + nt) * (ldw / KB) * 64 + ln) * EPC;
  if constexpr (is_x3<T>) {
    // x3: per K-block and (nt, mt) the six bf16 products w_i x a_j (i + j <= 2), smallest first, each term issued
    // across all accumulators before the next so consecutive MFMAs never share one
    constexpr int D = Cfg<T>::APREF, PL = Cfg<T>::M * ROW;
    f4(&a)[D][3][NT] = R.a;
    f4 b[3][MT];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[pl][mt] = lds_chunk<T>(act + pl * PL, 16 * mt + li, kc0 + g);
    auto step = [&](int kb, f4(&ar)[3][NT], bool refill) {
      const int kn = kb + 1 < nkb ? kb + 1 : kb;
      f4 bn[3][MT];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) bn[pl][mt] = lds_chunk<T>(act + pl * PL, 16 * mt + li, kc0 + kn * 4 + g);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int TI[6] = {2, 1, 0, 1, 0, 0}, TJ[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = mma_blk<bf16_t>(ar[TI[t]][nt], b[TJ[t]][mt], acc[nt][mt]);
      __builtin_amdgcn_sched_barrier(0);
      if (refill) {
        const int ka = kb + D < nkb ? kb + D : nkb - 1;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) ar[pl][nt] = *(const f4*)(wp[nt] + pl * wplane + ka * FRAG);
      }
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) b[pl][mt] = bn[pl][mt];
    };
    int kb = 0;
    for (; kb + D <= nkb; kb += D) {
#pragma unroll
      for (int r = 0; r < D; ++r) step(kb + r, a[r], true);
    }
#pragma unroll
    for (int r = 0; r < D - 1; ++r)
      if (kb + r < nkb) step(kb + r, a[r], false);
    return;
  }
  if constexpr (sizeof(T) == 2 && MT == 8 && NT >= 4) {
    // bf16 with 64-feature x 128-point wave tiles: 128 accumulator VGPRs leave room for one K-block of LDS fragments
    // only, so the K-block is split into two 4-tile point halves and each half's fragments are read while the other
    // half multiplies (two 16-VGPR half buffers instead of a 64-VGPR double buffer)
    constexpr int D = Cfg<T>::APREF, MH = MT / 2;
    f4(&a)[D][1][NT] = R.a;
    f4 b0[MH], b1[MH];
#pragma unroll
    for (int mt = 0; mt < MH; ++mt) b0[mt] = lds_chunk<T>(act, 16 * mt + li, kc0 + g);
    auto step = [&](int kb, f4(&ar)[NT], bool refill) {
      const int kn = kb + 1 < nkb ? kb + 1 : kb;
#pragma unroll
      for (int mt = 0; mt < MH; ++mt) b1[mt] = lds_chunk<T>(act, 16 * (mt + MH) + li, kc0 + kb * 4 + g);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MH; ++mt) acc[nt][mt] = mma_blk<T>(ar[nt], b0[mt], acc[nt][mt]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < MH; ++mt) b0[mt] = lds_chunk<T>(act, 16 * mt + li, kc0 + kn * 4 + g);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MH; ++mt) acc[nt][mt + MH] = mma_blk<T>(ar[nt], b1[mt], acc[nt][mt + MH]);
      __builtin_amdgcn_sched_barrier(0);
      if (refill) {
        const int ka = kb + D < nkb ? kb + D : nkb - 1;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) ar[nt] = *(const f4*)(wp[nt] + ka * FRAG);
      }
    };
    int kb = 0;
    for (; kb + D <= nkb; kb += D) {
#pragma unroll
      for (int r = 0; r < D; ++r) step(kb + r, a[r][0], true);
    }
#pragma unroll
    for (int r = 0; r < D - 1; ++r)
      if (kb + r < nkb) step(kb + r, a[r][0], false);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    constexpr int D = Cfg<T>::APREF;
    f4(&a)[D][1][NT] = R.a;
    f4 b[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) b[mt] = lds_chunk<T>(act, 16 * mt + li, kc0 + g);
    // one K-block: read block kb+1's LDS fragments, multiply block kb, refill the ring slot with block kb+D
    auto step = [&](int kb, f4(&ar)[NT], bool refill) {
      const int kn = kb + 1 < nkb ? kb + 1 : kb;
      f4 bn[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) bn[mt] = lds_chunk<T>(act, 16 * mt + li, kc0 + kn * 4 + g);
      __builtin_amdgcn_sched_barrier(0);
      mma_grid<T, NT, MT>(ar, b, acc);
      __builtin_amdgcn_sched_barrier(0);
      if (refill) {
        const int ka = kb + D < nkb ? kb + D : nkb - 1;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) ar[nt] = *(const f4*)(wp[nt] + ka * FRAG);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt] = bn[mt];
    };
    int kb = 0;
    for (; kb + D <= nkb; kb += D) {
#pragma unroll
      for (int r = 0; r < D; ++r) step(kb + r, a[r][0], true);
    }
    // tail of nkb % D blocks, straight-line (ring slot r holds block kb + r)
#pragma unroll
    for (int r = 0; r < D - 1; ++r)
      if (kb + r < nkb) step(kb + r, a[r][0], false);
    return;
  }
  // fp32: one weight-fragment set plus the next block's prefetch (two static register sets and a 2-block lookahead
  // measured slower)
  f4 a[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) a[nt] = *(const f4*)(wp[nt]);
  // this K-block's in-GEMM row stores (wave w stores K-blocks w, w + waves, ...): a uniform 64-bit base of the K-block's
  // 16 rows and 32-bit lane offsets (an opaque copy, so the compiler does not hoist 64-bit addresses for every K-block
  // out of the caller's layer loop)
  auto row_stores = [&](int kb, const f4(&b)[MT]) {
    if (kb < rs.nkb && kb % rs.waves == rs.wave) {
      const char* rb = (const char*)rs.base + (int64_t)(16 * kb) * rs.ldb;
      uint32_t vo = rs.voff;
      asm volatile("" : "+v"(vo));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint32_t o = vo + 16 * mt * 4;
        st_row_f32(rb + o, b[mt].x);
        st_row_f32(rb + o + (uint32_t)rs.ldb, b[mt].y);
        st_row_f32(rb + o + 2u * (uint32_t)rs.ldb, b[mt].z);
        st_row_f32(rb + o + 3u * (uint32_t)rs.ldb, b[mt].w);
      }
    }
  };
  for (int kb = 0; kb < nkb; ++kb) {
    f4 an[NT];
    const int kn = (kb + 1 < nkb) ? kb + 1 : kb;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) an[nt] = *(const f4*)(wp[nt] + kn * FRAG);
    f4 b[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) b[mt] = lds_chunk<T>(act, 16 * mt + li, kc0 + kb * 4 + g);
    if constexpr (RSV == RSV_DX) {
      __builtin_amdgcn_sched_barrier(0);
      row_stores(kb, b);
      __builtin_amdgcn_sched_barrier(0);
    }
    mma_grid<T, NT, MT>(a, b, acc);
    if constexpr (RSV == RSV_FWD) {
      __builtin_amdgcn_sched_barrier(0);
      row_stores(kb, b);
      __builtin_amdgcn_sched_barrier(0);
    }
    // GEMMs without row stores: the copy of the prefetched fragments pinned after the K-block's MFMAs (left free, the
    // compiler interleaves the copies with the MFMAs and waits for the next block's loads a quarter of the way into
    // this one): inference forward 7.04 -> 6.93 ms; with row stores (already between the MFMAs and the copies) the dX
    // measured slower pinned (6.90 -> 7.19 ms)
    if constexpr (RSV == 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) a[nt] = an[nt];
  }
}

// gemm_run with a weight ring: `pre` was filled by the caller (ring_fill before the previous epilogue), else a local
// one is filled here. (Two call paths, no pointer select, so the ring stays in registers.)
template <typename T, int NT, int MT, int RSV = 0>
__device__ __forceinline__ void gemm_lds(const typename Cfg<T>::w_t* __restrict__ W, int64_t wplane, int ldw, int nrow0,
                                         const typename Cfg<T>::lds_t* act, int kc0, int nkb, f4 (&acc)[NT][MT],
                                         int lane, const float* __restrict__ bias = nullptr,
                                         ARing<T, NT>* pre = nullptr, const RowSave& rs = RowSave{}) {
  if (pre) {
    gemm_run<T, NT, MT, RSV>(W, wplane, ldw, nrow0, act, kc0, nkb, acc, lane, bias, *pre, rs);
  } else {
    ARing<T, NT> own;
    ring_fill<T, NT>(own, W, wplane, ldw, nrow0, nkb, lane);
    gemm_run<T, NT, MT, RSV>(W, wplane, ldw, nrow0, act, kc0, nkb, acc, lane, bias, own, rs);
  }
}

// ---- epilogue helpers on a "packed tile": features n..n+3 of one point (one accumulator lane) in storage form.
// fp32: the f4 itself; bf16: two u32 words (x | y << 16, z | w << 16) from two v_cvt_pk_bf16_f32.
// ReLU is an integer max with 0 on the stored bits (negative floats / bf16 are negative integers, +0 stays 0),
// which avoids the IEEE canonicalisation a float max needs, and for bf16 runs on both halves at once.
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bh2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
template <typename T> struct Pk;
template <> struct Pk<float> { f4 v; };
template <> struct Pk<bf16_t> { uint32_t w0, w1; };
template <> struct Pk<x3_t> { f4 v; };  // kept in fp32; split into the three LDS planes when written

template <typename T> __device__ __forceinline__ Pk<T> pk_make(f4 v);
template <> __device__ __forceinline__ Pk<float> pk_make<float>(f4 v) { return Pk<float>{v}; }
template <> __device__ __forceinline__ Pk<bf16_t> pk_make<bf16_t>(f4 v) {
  const bh2 lo = __builtin_convertvector(f2{v.x, v.y}, bh2), hi = __builtin_convertvector(f2{v.z, v.w}, bh2);
  return Pk<bf16_t>{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}
template <> __device__ __forceinline__ Pk<x3_t> pk_make<x3_t>(f4 v) { return Pk<x3_t>{v}; }
template <typename T> __device__ __forceinline__ Pk<T> pk_relu(Pk<T> p);
template <> __device__ __forceinline__ Pk<float> pk_relu<float>(Pk<float> p) {
  f4 r;
  r.x = __int_as_float(max(__float_as_int(p.v.x), 0));
  r.y = __int_as_float(max(__float_as_int(p.v.y), 0));
  r.z = __int_as_float(max(__float_as_int(p.v.z), 0));
  r.w = __int_as_float(max(__float_as_int(p.v.w), 0));
  return Pk<float>{r};
}
template <> __device__ __forceinline__ Pk<x3_t> pk_relu<x3_t>(Pk<x3_t> p) {
  return Pk<x3_t>{pk_relu<float>(Pk<float>{p.v}).v};
}
template <> __device__ __forceinline__ Pk<bf16_t> pk_relu<bf16_t>(Pk<bf16_t> p) {
  const s2 z = {0, 0};
  return Pk<bf16_t>{__builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, p.w0), z)),
                    __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, p.w1), z))};
}
// 4-bit ReLU mask of a relu'd packed tile: bit r = element r > 0
template <typename T> __device__ __forceinline__ uint32_t pk_bits(Pk<T> p);
template <> __device__ __forceinline__ uint32_t pk_bits<float>(Pk<float> p) {
  const uint32_t b0 = min(__float_as_uint(p.v.x), 1u), b1 = min(__float_as_uint(p.v.y), 1u),
                 b2 = min(__float_as_uint(p.v.z), 1u), b3 = min(__float_as_uint(p.v.w), 1u);
  return b0 | (b1 << 1) | (b2 << 2) | (b3 << 3);
}
template <> __device__ __forceinline__ uint32_t pk_bits<x3_t>(Pk<x3_t> p) { return pk_bits<float>(Pk<float>{p.v}); }
template <> __device__ __forceinline__ uint32_t pk_bits<bf16_t>(Pk<bf16_t> p) {
  const u2 one = {1, 1};
  const uint32_t m0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u2, p.w0), one));
  const uint32_t m1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u2, p.w1), one));
  const uint32_t t = m0 | (m1 << 2);  // x@0 z@2 y@16 w@18
  return (t & 5u) | ((t >> 15) & 10u);
}
// write the packed tile to LDS row m, features n..n+3
template <typename T> __device__ __forceinline__ void pk_lds(typename Cfg<T>::lds_t* act, int m, int n, Pk<T> p);
template <> __device__ __forceinline__ void pk_lds<float>(float* act, int m, int n, Pk<float> p) {
  *(f4*)(act + m * ROW + swz<float>(m, n / 4) * 4) = p.v;
}
template <> __device__ __forceinline__ void pk_lds<bf16_t>(bf16_t* act, int m, int n, Pk<bf16_t> p) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  *(u32x2*)(act + m * ROW + swz<bf16_t>(m, n / 8) * 8 + (n & 7)) = u32x2{p.w0, p.w1};
}
template <> __device__ __forceinline__ void pk_lds<x3_t>(bf16_t* act, int m, int n, Pk<x3_t> p) {
  // v = t0 + t1 + t2 per element, each plane packed pairwise (v_cvt_pk_bf16_f32) like the bf16 tile
  constexpr int PL = Cfg<x3_t>::M * ROW;
  const f4 v0 = p.v;
  const Pk<bf16_t> h0 = pk_make<bf16_t>(v0);
  const f4 r1 = v0 - f4{__uint_as_float(h0.w0 << 16), __uint_as_float(h0.w0 & 0xffff0000u),
                        __uint_as_float(h0.w1 << 16), __uint_as_float(h0.w1 & 0xffff0000u)};
  const Pk<bf16_t> h1 = pk_make<bf16_t>(r1);
  const f4 r2 = r1 - f4{__uint_as_float(h1.w0 << 16), __uint_as_float(h1.w0 & 0xffff0000u),
                        __uint_as_float(h1.w1 << 16), __uint_as_float(h1.w1 & 0xffff0000u)};
  const Pk<bf16_t> h2 = pk_make<bf16_t>(r2);
  pk_lds<bf16_t>(act, m, n, h0);
  pk_lds<bf16_t>(act + PL, m, n, h1);
  pk_lds<bf16_t>(act + 2 * PL, m, n, h2);
}
// Store a packed tile into 4 feature-major rows (fp32 / x3; bf16 stores point-major sections, copy_tile_pm) given the
// tile's uniform base (layer, row tile, point tile: SGPRs), this lane's byte offset `voff` (4g rows + li points, one VGPR
// for every tile), the row stride `ldb` and the byte offset `so` of the 16-point group. Plain global stores (buffer
// stores measured slower here: fp32 training forward 7.7 -> 8.4 ms); fp32 non-temporal, x3 temporal (st_row_f32).
template <typename T>
__device__ __forceinline__ void pk_store_rows_b(typename Cfg<T>::st_t* base, uint32_t voff, int ldb, int so, Pk<T> p);
template <>
__device__ __forceinline__ void pk_store_rows_b<float>(float* base, uint32_t voff, int ldb, int so, Pk<float> p) {
  char* b = (char*)base + so + voff;
  st_row_f32(b, p.v.x);
  st_row_f32(b + ldb, p.v.y);
  st_row_f32(b + 2 * (int64_t)ldb, p.v.z);
  st_row_f32(b + 3 * (int64_t)ldb, p.v.w);
}
template <>
__device__ __forceinline__ void pk_store_rows_b<x3_t>(float* base, uint32_t voff, int ldb, int so, Pk<x3_t> p) {
  char* b = (char*)base + so + voff;
  st_row_f32<false>(b, p.v.x);
  st_row_f32<false>(b + ldb, p.v.y);
  st_row_f32<false>(b + 2 * (int64_t)ldb, p.v.z);
  st_row_f32<false>(b + 3 * (int64_t)ldb, p.v.w);
}

// Per-lane trunk ReLU mask words of one layer: 4 bits for each of the lane's NT*MT accumulator tiles, tile t in
// word t >> 4; within the word (u = t & 15):
//  fp32 / x3: element r at bit 4u + r (pk_bits);
//  bf16: element r at bit 32 (u >> 3) + 8 r + (u & 7): the relu'd halves h in [0, 0x7fff] are nonzero iff
//        bit 15 of h + 0x7fff is set (both halves of a packed pair in one add, no carry between them), one v_perm
//        gathers the four flag bytes and a shift + and-or places them.
// (Called without explicit template arguments so the bf16 overload is picked by partial ordering.)
template <typename T, int W> __device__ __forceinline__ void mask_acc(uint64_t (&bits)[W], Pk<T> h, int t) {
  bits[t >> 4] |= (uint64_t)pk_bits<T>(h) << (4 * (t & 15));
}
template <int W> __device__ __forceinline__ void mask_acc(uint64_t (&bits)[W], Pk<bf16_t> h, int t) {
  const uint32_t f = __builtin_amdgcn_perm(h.w1 + 0x7fff7fffu, h.w0 + 0x7fff7fffu, 0x07050301u);  // flags at 8r + 7
  const int j = t & 7;
  const uint32_t w = (f >> (7 - j)) & (0x01010101u << j);
  bits[t >> 4] |= (uint64_t)w << (32 * ((t >> 3) & 1));
}
__device__ __forceinline__ f4 apply_mask4(f4 v, uint64_t bits, int sh);
// zero the elements of tile t of a value whose mask bit (mask_acc layout) is clear
template <typename T, int W> __device__ __forceinline__ f4 apply_mask_tile(f4 v, const uint64_t (&bits)[W], int t) {
  if constexpr (sizeof(T) == 2 && !is_x3<T>) {
    const uint32_t w = (uint32_t)(bits[t >> 4] >> (32 * ((t >> 3) & 1)));
    const int j = t & 7;
    f4 r;
    r.x = __int_as_float(__float_as_int(v.x) & __builtin_amdgcn_sbfe(w, j, 1));
    r.y = __int_as_float(__float_as_int(v.y) & __builtin_amdgcn_sbfe(w, 8 + j, 1));
    r.z = __int_as_float(__float_as_int(v.z) & __builtin_amdgcn_sbfe(w, 16 + j, 1));
    r.w = __int_as_float(__float_as_int(v.w) & __builtin_amdgcn_sbfe(w, 24 + j, 1));
    return r;
  } else {
    return apply_mask4(v, bits[t >> 4], 4 * (t & 15));
  }
}
__device__ __forceinline__ f4 apply_mask4(f4 v, uint64_t bits, int sh) {
  const uint32_t w = (uint32_t)(bits >> sh);
  f4 r;
  r.x = __int_as_float(__float_as_int(v.x) & __builtin_amdgcn_sbfe(w, 0, 1));
  r.y = __int_as_float(__float_as_int(v.y) & __builtin_amdgcn_sbfe(w, 1, 1));
  r.z = __int_as_float(__float_as_int(v.z) & __builtin_amdgcn_sbfe(w, 2, 1));
  r.w = __int_as_float(__float_as_int(v.w) & __builtin_amdgcn_sbfe(w, 3, 1));
  return r;
}

// Harmonic embedding (models/utils.py:98-102) of 3-vector x: columns [sin(x_i 2^f) i-major f-minor | cos(...) | x],
// zero-padded to `width`, written into LDS row m at column col0 (and, when `sv` is set, into feature-major saved
// rows sv[k * ld]). The TPP threads of a point share the work: thread q takes the (i, f) pairs j = q, q+TPP, ...
// and one sincosf per pair yields both the sin column j and the cos column 3F + j.
template <typename T>
__device__ __forceinline__ void harmonic_to_lds(typename Cfg<T>::lds_t* act, int m, int col0, int width,
                                                const float x[3], int F, int append, int q,
                                                typename Cfg<T>::st_t* sv, int64_t ld) {
  constexpr int TPP = Cfg<T>::WAVES * 64 / Cfg<T>::M;
  if constexpr (!is_x3<T> && sizeof(T) == 2) {
    // bf16 mode: the hardware sin/cos of the angle reduced to revolutions (|error| ~1e-4 rad at the top frequency,
    // far below the bf16 rounding of the value). TPP == 4: thread q < 3 takes coordinate q at every frequency,
    // thread 3 writes [x, zero padding]; TPP == 2: thread 0 takes coordinates 0 and 2, thread 1 coordinate 1 and
    // [x, padding].
    static_assert(TPP == 4 || TPP == 2, "bf16 harmonic split");
    auto coord = [&](int c) {
      const float xi = c == 0 ? x[0] : (c == 1 ? x[1] : x[2]);
      const float r0 = xi * 0.15915494309189535f;
      for (int f = 0; f < F; ++f) {
        const float r = __builtin_amdgcn_fractf(r0 * (float)(1 << f));
        const float sn = __builtin_amdgcn_sinf(r), cs = __builtin_amdgcn_cosf(r);
        const int j = c * F + f;
        lds_put1<T>(act, m, col0 + j, sn);
        lds_put1<T>(act, m, col0 + 3 * F + j, cs);
        if (sv) {
          sv[(int64_t)j * ld] = to_st<T>(sn);
          sv[(int64_t)(3 * F + j) * ld] = to_st<T>(cs);
        }
      }
    };
    auto tail = [&]() {
      for (int k = 6 * F; k < width; ++k) {
        const int a = k - 6 * F;
        float v = a == 0 ? x[0] : 0.0f;
        v = a == 1 ? x[1] : v;
        v = a == 2 ? x[2] : v;
        v = append ? v : 0.0f;
        lds_put1<T>(act, m, col0 + k, v);
        if (sv) sv[(int64_t)k * ld] = to_st<T>(v);
      }
    };
    if constexpr (TPP == 4) {
      if (q < 3) coord(q);
      else tail();
    } else {
      coord(q);
      if (q == 0) coord(2);
      else tail();
    }
    return;
  }
  for (int j = q; j < 3 * F; j += TPP) {
    const int i = j / F, f = j - i * F;
    float xi = x[0];
    xi = i == 1 ? x[1] : xi;
    xi = i == 2 ? x[2] : xi;
    // the fp32 modes: correctly rounded sin / cos (evaluated in double, rounded once), so the embedding is a pure
    // function of its fp32 argument that a CPU reproduces bit for bit (make_golden.hip_order_model); the device libm's
    // sincosf differs from it in ~19 % of the Lego embedding values by an ulp. Its cost is < 1 % of the forward.
    double sd, cd;
    sincos((double)(xi * (float)(1 << f)), &sd, &cd);
    const float sn = (float)sd, cs = (float)cd;
    lds_put1<T>(act, m, col0 + j, sn);
    lds_put1<T>(act, m, col0 + 3 * F + j, cs);
    if (sv) {
      sv[(int64_t)j * ld] = to_st<T>(sn);
      sv[(int64_t)(3 * F + j) * ld] = to_st<T>(cs);
    }
  }
  for (int k = 6 * F + q; k < width; k += TPP) {
    const int a = k - 6 * F;
    float v = a == 0 ? x[0] : 0.0f;
    v = a == 1 ? x[1] : v;
    v = a == 2 ? x[2] : v;
    v = append ? v : 0.0f;
    lds_put1<T>(act, m, col0 + k, v);
    if (sv) sv[(int64_t)k * ld] = to_st<T>(v);
  }
}

__device__ __forceinline__ void store_mask_tile(uint64_t* masks, int64_t Npad, int slot, int64_t pt16, int ft, f4 v,
                                                int lane) {
  const uint64_t b0 = __ballot(v.x > 0.f), b1 = __ballot(v.y > 0.f), b2 = __ballot(v.z > 0.f),
                 b3 = __ballot(v.w > 0.f);
  if (lane < 4) masks[mask_index(Npad, slot, pt16, ft) + lane] = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
}

// cache-policy bits of the point-major saves' buffer stores (gfx950: 1 sc0, 2 nt, 16 sc1): nt measured bf16 backward
// -2.5 %, forward unchanged (sc0 / sc1: no gain)
constexpr int PM_STORE_AUX = 2;
// Point-major (Cfg::PM) save: columns [col0, col0 + W) of the LDS tile's M points -> the [Npad][W] section at
// dst = section + p0 * W. A lane moves one 16-byte chunk: a 16-lane group reads 256 contiguous bytes of one LDS row
// (the row swizzle permutes chunks within aligned groups of 8) and a wave-instruction writes 1 KiB contiguously.
template <typename T, int NTHR, int W>
__device__ __forceinline__ void copy_tile_pm(const typename Cfg<T>::lds_t* act, int col0, typename Cfg<T>::st_t* dst,
                                             int tid) {
  static_assert(sizeof(typename Cfg<T>::st_t) == 2 && !is_x3<T>, "point-major save: bf16 tiles");
  constexpr int M = Cfg<T>::M, CPR = W / 8, TOT = M * CPR, IT = TOT / NTHR;
  static_assert(TOT % NTHR == 0, "copy_tile_pm: whole chunks per thread");
  constexpr int GRP = IT < 4 ? IT : 4;  // chunks in flight per lane (bounds the live registers)
  // an opaque copy of tid: the address arithmetic below is redone at every call instead of being hoisted out of the
  // caller's layer loop (where its 2 x IT address registers would be live across every GEMM)
  int t = tid;
  asm volatile("" : "+v"(t));
  // global side: a buffer resource on the section (uniform) + one 32-bit lane offset; chunk i is NTHR * 16 bytes on
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
  const int m0 = t / CPR, c = t % CPR;
  const uint32_t goff = (uint32_t)(t * 16);
  static_assert(NTHR % CPR == 0, "copy_tile_pm: whole rows per pass");
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += GRP) {
    f4 v[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) v[i] = lds_chunk<T>(act, m0 + (NTHR / CPR) * (i0 + i), col0 / 8 + c);
    // The chunk offset goes into the VGPR offset with soffset = 0, NOT into soffset: gfx950 has a write-after-read
    // hazard between a 128-bit buffer store's data VGPRs and a following VALU write of them, which LLVM's hazard
    // recognizer only covers when soffset is not a register (GCNHazardRecognizer::createsVALUHazard). With an SGPR
    // soffset the compiler reused a data VGPR in the next instruction and, under load (another kernel on the
    // chip), the store took the new value for some lanes: tools/debug_bf16_overlap.py, dZc rows 32..47 of a tile.
#pragma unroll
    for (int i = 0; i < GRP; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint32_t __attribute__((ext_vector_type(4))), v[i]), rs,
                                             goff + (uint32_t)((i0 + i) * NTHR * 16), 0, PM_STORE_AUX);
  }
}

// The fp8 save of a point-major section: like copy_tile_pm, but a lane reads two 16-byte LDS chunks
// (16 bf16 features of one point), converts them to 16 fp8 e4m3 (clamped to 448: the tile holds post-ReLU values, so
// an integer min on the bf16 bits is the clamp) and writes one 16-byte chunk; a wave-instruction writes 1 KiB
// contiguously.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
// four bf16 (two packed words) -> four fp8 e4m3 of value / scale (v_cvt_scalef32_pk_fp8_bf16 divides by its scale
// operand and v_cvt_scalef32_pk_bf16_fp8 multiplies: tools/probes/probe_fp8_scale.hip). CLAMP: the inputs are
// non-negative and may exceed 448 (integer min on the bf16 bits); otherwise the caller's scale keeps |value| < 448.
template <bool CLAMP>
__device__ __forceinline__ uint32_t fp8x4_from_bf16(uint32_t w0, uint32_t w1, float scale) {
  if constexpr (CLAMP) {
    const u16x2 cap = {0x43E0, 0x43E0};  // 448.0 in bf16
    w0 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, w0), cap));
    w1 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, w1), cap));
  }
  i16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(i16x2{0, 0}, __builtin_bit_cast(bf16x2, w0), scale, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2, w1), scale, true);
  return __builtin_bit_cast(uint32_t, r);
}
template <typename T, int NTHR, int W, bool CLAMP = true, int GMAX = 4>
__device__ __forceinline__ void copy_tile_pm_fp8(const typename Cfg<T>::lds_t* act, int col0, uint8_t* dst, int tid,
                                                 float scale = 1.0f) {
  static_assert(sizeof(typename Cfg<T>::lds_t) == 2 && !is_x3<T>, "fp8 save: bf16 tiles");
  constexpr int M = Cfg<T>::M, OPR = W / 16, TOT = M * OPR, IT = TOT / NTHR;
  static_assert(TOT % NTHR == 0 && NTHR % OPR == 0, "copy_tile_pm_fp8: whole chunks / rows per pass");
  constexpr int GRP = IT < GMAX ? IT : GMAX;  // output chunks in flight per lane (8 + 4 VGPRs each)
  int t = tid;
  asm volatile("" : "+v"(t));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
  const int m0 = t / OPR, j = t % OPR;
  const uint32_t goff = (uint32_t)(t * 16);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += GRP) {
    f4 lo[GRP], hi[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      const int m = m0 + (NTHR / OPR) * (i0 + i);
      lo[i] = lds_chunk<T>(act, m, col0 / 8 + 2 * j);
      hi[i] = lds_chunk<T>(act, m, col0 / 8 + 2 * j + 1);
    }
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      const u32x4 out = {fp8x4_from_bf16<CLAMP>(__float_as_uint(lo[i].x), __float_as_uint(lo[i].y), scale),
                         fp8x4_from_bf16<CLAMP>(__float_as_uint(lo[i].z), __float_as_uint(lo[i].w), scale),
                         fp8x4_from_bf16<CLAMP>(__float_as_uint(hi[i].x), __float_as_uint(hi[i].y), scale),
                         fp8x4_from_bf16<CLAMP>(__float_as_uint(hi[i].z), __float_as_uint(hi[i].w), scale)};
      // offset in the VGPR offset, soffset = 0 (the wide-store hazard note at copy_tile_pm); the nop keeps the next
      // group's LDS reads (which reuse these VGPRs) one instruction away from the store
      __builtin_amdgcn_raw_buffer_store_b128(out, rs, goff + (uint32_t)((i0 + i) * NTHR * 16), 0, PM_STORE_AUX);
      asm volatile("s_nop 0" ::: "memory");
    }
  }
}
// save of a post-ReLU section as fp8
template <typename T, int NTHR, int W>
__device__ __forceinline__ void save_relu_pm(const typename Cfg<T>::lds_t* act, int col0, char* dst, int tid) {
  copy_tile_pm_fp8<T, NTHR, W>(act, col0, (uint8_t*)dst, tid);
}

// fp8 gradient rows: the dX kernel's pre-activation gradients dZ_l, dY and dZc are the dW kernel's A
// operands only. Each leaves a tile as fp8 e4m3 of value / s with one power-of-two s per (section, 128-point tile),
// chosen so the tile's largest |value| lands in [128, 256) (below e4m3's 448 after the bf16 rounding of the LDS copy);
// s goes to a small scale array beside the rows and the dW tile widens the fragments with it (exact).
// max over the wave without address registers: DPP within each 16-lane row (quad xor 1, xor 2, half-row mirror,
// row mirror), then the four rows through readlane (the result is wave-uniform). A __shfl_xor form needs six
// ds_bpermute address VGPRs, which the compiler hoisted out of the dX layer loop and spilled: every reload then
// waited (shared in-order vmcnt) for all of the wave's outstanding gradient-row stores.
template <int CTRL>
__device__ __forceinline__ float dpp_fmax(float v) {
  const int o = __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xf, 0xf, false);
  return fmaxf(v, __int_as_float(o));
}
__device__ __forceinline__ float wave_max(float v) {
  v = dpp_fmax<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v = dpp_fmax<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v = dpp_fmax<0x141>(v);  // row_half_mirror
  v = dpp_fmax<0x140>(v);  // row_mirror
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
// running |max| of packed bf16 tile values as two u16 maxima of the magnitude bits (one VGPR, two VALU per chunk)
struct G8Max {
  u16x2 m = {0, 0};
  template <typename T> __device__ __forceinline__ void add(const Pk<T>& h) {
    if constexpr (std::is_same<T, bf16_t>::value) {
      m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2, h.w0 & 0x7fff7fffu));
      m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2, h.w1 & 0x7fff7fffu));
    }
  }
  __device__ __forceinline__ float value() const {
    const uint32_t b = m.x > m.y ? m.x : m.y;
    return __uint_as_float(b << 16);
  }
};
__device__ __forceinline__ float g8_scale(float amax) {
  const uint32_t e = (__float_as_uint(amax) >> 23) & 0xffu;
  return e <= 7u ? 1.0f : __uint_as_float((e - 7u) << 23);
}
// the gradient tile's save: `red` holds each wave's |max| of the section (written before the last barrier)
template <typename T, int NTHR, int W>
__device__ __forceinline__ void save_grad_pm(const typename Cfg<T>::lds_t* act, char* dst, float* scale_out,
                                             const float* red, int waves, int tid) {
  float amax = red[0];
  for (int w = 1; w < waves; ++w) amax = fmaxf(amax, red[w]);
  const float sc = g8_scale(amax);
  if (tid == 0) *scale_out = sc;
  // two chunks in flight: the dX trunk step copies while the next layer's weight ring is live
  copy_tile_pm_fp8<T, NTHR, W, false, 2>(act, 0, (uint8_t*)dst, tid, sc);
}

// YANERF_PREC_BF16S: the same sections stay bf16 -- the LDS tile copied as it is (copy_tile_pm), no fp8 scales
template <typename T, int NTHR, int W, bool S16>
__device__ __forceinline__ void save_act_pm(const typename Cfg<T>::lds_t* act, char* dst, int tid) {
  if constexpr (S16) copy_tile_pm<T, NTHR, W>(act, 0, (typename Cfg<T>::st_t*)dst, tid);
  else save_relu_pm<T, NTHR, W>(act, 0, dst, tid);
}
template <typename T, int NTHR, int W, bool S16>
__device__ __forceinline__ void save_grad_rows_pm(const typename Cfg<T>::lds_t* act, char* dst, float* scale_out,
                                                  const float* red, int waves, int tid) {
  if constexpr (S16) copy_tile_pm<T, NTHR, W>(act, 0, (typename Cfg<T>::st_t*)dst, tid);
  else save_grad_pm<T, NTHR, W>(act, dst, scale_out, red, waves, tid);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global stores (the
// saved rows / gradients / masks written between barriers are read by later kernels only). __syncthreads() is a
// workgroup fence as well and waits for every outstanding store (vmcnt(0)) at each of the ~24 barriers per tile.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ============================================================================================ forward
// SAVE: training forward (saved activation rows + ReLU masks for the backward); else inference, outputs only. The two
// are separate instantiations, so the saves' presence is known at compile time: with a run-time saved-pointer test the
// compiler waited vmcnt(0) at the next GEMM's first weight use, i.e. for the epilogue's stores too (x3 training forward
// 4.97 -> 4.86 ms, fp32 7.57 -> 7.52 ms, bitwise equal).
template <typename T, bool SAVE, bool S16 = false>
__global__ void __launch_bounds__(Cfg<T>::WAVES * 64)
    __attribute__((amdgpu_waves_per_eu(Cfg<T>::WPE))) mlp_fwd_kernel(
    MlpLayout lay, const typename Cfg<T>::w_t* __restrict__ Wt, const float* __restrict__ Wf,
    const float* __restrict__ origins, const float* __restrict__ dirs, const float* __restrict__ lengths, int64_t R,
    int64_t P, float* __restrict__ sigma, float* __restrict__ rgb, typename Cfg<T>::st_t* __restrict__ saved,
    uint64_t* __restrict__ masks, int64_t Npad) {
  constexpr int M = Cfg<T>::M, WAVES = Cfg<T>::WAVES, MT = M / 16;
  constexpr int NT = 256 / 16 / WAVES, NTC = HC / 16 / WAVES;
  constexpr int EPC = Cfg<T>::EPC, KB = Cfg<T>::KB, TPP = WAVES * 64 / M;  // threads per point
  constexpr int MW = mask_w<T>();  // u64 ReLU-mask words per lane per layer
  typedef typename Cfg<T>::lds_t LT;
  __shared__ __attribute__((aligned(16))) LT act[Cfg<T>::PLANES * M * ROW];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t N = R * P;
  const int64_t tile = (int64_t)blockIdx.x, ntiles = (int64_t)gridDim.x;
  const int64_t p0 = tile * M;
  typedef typename Cfg<T>::st_t ST;
  const int64_t ld = row_ld(Npad, sizeof(ST)), ldb = ld * (int64_t)sizeof(ST);
  const uint32_t soff = (uint32_t)(4 * g * ldb + li * (int64_t)sizeof(ST));  // this lane's offset in a 16x16 row tile
  if constexpr (!SAVE) saved = nullptr;
  constexpr bool sv = SAVE;
  const int64_t wpl = lay.t_plane;
  const SavedRows SR = saved_rows(lay.L);
  const PmSave PS = pm_save(lay.L, Npad, S16);  // byte offsets of the point-major sections (bf16)
  constexpr int HB = pm_hb(S16), YB = pm_yb(S16);
  const int mt_ = tid / TPP, q = tid % TPP;
  const int64_t p = p0 + mt_;
  const int64_t pc = p < N ? p : N - 1;
  const int64_t ray = pc / P;
  float o3[3], d3[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    o3[i] = origins[ray * 3 + i];
    d3[i] = dirs[ray * 3 + i];
  }
  const float t = lengths[pc];
  float x3[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) x3[i] = o3[i] + t * d3[i];  // models/utils.py:244
  constexpr bool PM = Cfg<T>::PM;
  constexpr int NTHR = WAVES * 64;
  harmonic_to_lds<T>(act, mt_, PE_COL, KPE, x3, lay.fx, lay.ax, q, (saved && !PM) ? saved + SR.pe * ld + p : nullptr,
                     ld);
  lds_barrier();

  f4 acc[NT][MT];
  const int nrow0 = wave * NT * 16;
  // weight ring of the next GEMM, filled before the current layer's epilogue (bf16; no-op for fp32)
  ARing<T, NT> ring;
  ring_fill<T, NT>(ring, Wt + lay.w_off[0], wpl, lay.kpad[0], nrow0, KPE / KB, lane);
  // point-major saves are issued AFTER the following GEMM (and its next-ring loads): loads and stores share vmcnt
  // and complete in order, so a store issued before a GEMM's weight loads makes every wait on those loads wait for
  // the store's write acknowledgement too. The GEMM of layer l + 1 still reads H_l from the LDS tile, so H_l (and the
  // mask words of layer l) leave during iteration l + 1, between its GEMM and its epilogue barrier.
  uint64_t pbits[MW] = {};
  // fp32: H_l's saved rows leave from the B fragments of the GEMM that reads H_l (gemm_run RSV_FWD)
  constexpr bool GS = std::is_same<T, float>::value && SAVE;
  auto hsave = [&](int hl) {
    return RowSave{(sv && hl >= 0) ? (float*)(void*)(saved + (SR.h0 + 256LL * hl) * ld + p0) : nullptr, soff,
                   (int)ldb, (sv && hl >= 0) ? 256 / KB : 0, wave, WAVES};
  };
  for (int l = 0; l < lay.L; ++l) {
    const bool sk = (lay.skip >> l) & 1u;
    const int kc0 = (l == 0) ? PE_COL / EPC : 0;
    const int nkb = (l == 0) ? KPE / KB : (sk ? 320 / KB : 256 / KB);
    gemm_lds<T, NT, MT, GS ? RSV_FWD : 0>(Wt + lay.w_off[l], wpl, lay.kpad[l], nrow0, act, kc0, nkb, acc, lane,
                                          Wf + lay.b_off[l], &ring, hsave(l - 1));
    if (l + 1 < lay.L)
      ring_fill<T, NT>(ring, Wt + lay.w_off[l + 1], wpl, lay.kpad[l + 1], nrow0, lay.kpad[l + 1] / KB, lane);
    else ring_fill<T, NT>(ring, Wt + lay.wint_off, wpl, 256, nrow0, 256 / KB, lane);
    if constexpr (PM && sv) {
      if (l == 0) {
        copy_tile_pm<T, NTHR, KPE>(act, PE_COL, (ST*)((char*)saved + PS.pe) + p0 * KPE, tid);
      } else {
        save_act_pm<T, NTHR, 256, S16>(act, (char*)saved + PS.h0 + ((l - 1) * Npad + p0) * 256LL * HB, tid);
#pragma unroll
        for (int w = 0; w < MW; ++w)
          masks[((((int64_t)(l - 1) * ntiles + tile) * WAVES + wave) * MW + w) * 64 + lane] = pbits[w];
      }
    }
    lds_barrier();
    uint64_t bits[MW] = {};
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nrow0 + 16 * nt + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const Pk<T> h = pk_relu<T>(pk_make<T>(acc[nt][mt]));
        const int m = 16 * mt + li;
        pk_lds<T>(act, m, n, h);
        if constexpr (sv) {
          if constexpr (!PM && !GS)  // x3: feature-major rows from the epilogue
            pk_store_rows_b<T>((saved + (SR.h0 + 256LL * l + nrow0 + 16 * nt) * ld + p0), soff, (int)ldb,
                               16 * mt * (int)sizeof(ST), h);
          mask_acc(bits, h, nt * MT + mt);
        }
      }
    }
    if constexpr (PM) {
#pragma unroll
      for (int w = 0; w < MW; ++w) pbits[w] = bits[w];
    } else if constexpr (sv) {
#pragma unroll
      for (int w = 0; w < MW; ++w)
        masks[((((int64_t)l * ntiles + tile) * WAVES + wave) * MW + w) * 64 + lane] = bits[w];
    }
    lds_barrier();
  }
  // ---- density head: sigma = w_d . h + b_d (nerf_mlp.py:173; density_layer 256->1) as one 16-row MFMA tile per
  // 16-point group (rows past 0 are zero weights); wave w takes groups w, w + WAVES, ...; lanes g == 0 hold sigma of
  // point 16 * group + li. Shifting the LDS base by 16 * group rows keeps the row swizzle (it depends on row mod 16).
  constexpr int HG = (MT + WAVES - 1) / WAVES;  // head groups per wave
  float sig[HG];
#pragma unroll
  for (int hg = 0; hg < HG; ++hg) {
    const int grp = wave + hg * WAVES;
    sig[hg] = 0.f;
    if (grp < MT) {
      f4 hacc[1][1];
      gemm_lds<T, 1, 1>(Wt + lay.wdh_off, wpl, 256, 0, act + 16 * grp * ROW, 0, 256 / KB, hacc, lane);
      sig[hg] = hacc[0][0].x + Wf[lay.bd_off];
    }
  }
  // ---- intermediate_linear (no activation)
  gemm_lds<T, NT, MT, GS ? RSV_FWD : 0>(Wt + lay.wint_off, wpl, 256, nrow0, act, 0, 256 / KB, acc, lane,
                                        Wf + lay.bint_off, &ring, hsave(lay.L - 1));
  const int crow0 = wave * NTC * 16;
  ARing<T, NTC> ringc;
  ring_fill<T, NTC>(ringc, Wt + lay.wc_off, wpl, KC, crow0, KC / KB, lane);
  if constexpr (PM && sv) {
    save_act_pm<T, NTHR, 256, S16>(act, (char*)saved + PS.h0 + ((lay.L - 1) * Npad + p0) * 256LL * HB, tid);
#pragma unroll
    for (int w = 0; w < MW; ++w)
      masks[((((int64_t)(lay.L - 1) * ntiles + tile) * WAVES + wave) * MW + w) * 64 + lane] = pbits[w];
  }
  lds_barrier();
  // fp8 Y: each wave's |max| of Y in the PE columns 32.. of row 16 (free once the trunk is done: the direction
  // embedding takes columns 0..31), read by the Y save after the colour GEMM
  [[maybe_unused]] float* const yred = (float*)(act + 16 * ROW + PE_COL + 32);
  {
    G8Max gmax;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nrow0 + 16 * nt + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f4 v = acc[nt][mt];
        const int m = 16 * mt + li;
        const Pk<T> h = pk_make<T>(v);
        pk_lds<T>(act, m, n, h);
        if constexpr (PM && !S16) gmax.add(h);
        if constexpr (sv && !PM)
          pk_store_rows_b<T>((saved + (SR.y + nrow0 + 16 * nt) * ld + p0), soff, (int)ldb, 16 * mt * (int)sizeof(ST), h);
      }
    }
    if constexpr (PM && !S16) {
      static_assert(PE_COL + 32 + 2 * WAVES <= ROW, "Y scale slots");
      const float am = wave_max(gmax.value());
      if (sv && lane == 0) yred[wave] = am;
    }
  }
  // ---- direction embedding of normalize(d) (nerf_mlp.py:105-108) into cols 256..287
  {
    const float nrm = fmaxf(sqrtf(d3[0] * d3[0] + d3[1] * d3[1] + d3[2] * d3[2]), 1e-12f);
    float dn[3] = {d3[0] / nrm, d3[1] / nrm, d3[2] / nrm};
    harmonic_to_lds<T>(act, mt_, PE_COL, KDIR, dn, lay.fd, lay.ad, q, (saved && !PM) ? saved + SR.dpe * ld + p : nullptr,
                       ld);
  }
  lds_barrier();
  // ---- color layer: LinearWithRepeat(256 + 27 -> 128) + ReLU as one K = 288 GEMM over [Y, dirPE]
  {
    f4 accc[NTC][MT];
    gemm_lds<T, NTC, MT>(Wt + lay.wc_off, wpl, KC, crow0, act, 0, KC / KB, accc, lane, Wf + lay.bc_off, &ringc);
    if constexpr (PM && sv) {
      save_grad_rows_pm<T, NTHR, 256, S16>(act, (char*)saved + PS.y + p0 * 256 * YB,
                                           (float*)((char*)saved + PS.ysc) + tile, yred, WAVES, tid);
      copy_tile_pm<T, NTHR, KDIR>(act, PE_COL, (ST*)((char*)saved + PS.dpe) + p0 * KDIR, tid);
    }
    lds_barrier();
#pragma unroll
    for (int nt = 0; nt < NTC; ++nt) {
      const int n = crow0 + 16 * nt + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f4 v = accc[nt][mt];
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        const int m = 16 * mt + li;
        const Pk<T> h = pk_make<T>(v);
        pk_lds<T>(act, m, n, h);
        if constexpr (sv) {
          if constexpr (!PM)
            pk_store_rows_b<T>((saved + (SR.c + crow0 + 16 * nt) * ld + p0), soff, (int)ldb,
                               16 * mt * (int)sizeof(ST), h);
          store_mask_tile(masks + (int64_t)lay.L * trunk_mask_words<T>(Npad), Npad, 0, p0 / 16 + mt,
                          (crow0 + 16 * nt) / 16, v, lane);
        }
      }
    }
  }
  lds_barrier();
  // ---- output layer 128 -> color_dim + sigmoid, as for the density head (nerf_mlp.py:169-171)
#pragma unroll
  for (int hg = 0; hg < HG; ++hg) {
    const int grp = wave + hg * WAVES;
    f4 hacc[1][1] = {{f4{0.f, 0.f, 0.f, 0.f}}};
    if (grp < MT) gemm_lds<T, 1, 1>(Wt + lay.woh_off, wpl, HC, 0, act + 16 * grp * ROW, 0, HC / KB, hacc, lane);
    const int64_t pw = p0 + 16 * grp + li;
    if (grp < MT && g == 0 && pw < N) {
      sigma[pw] = sig[hg];
      const float u[CMAX] = {hacc[0][0].x, hacc[0][0].y, hacc[0][0].z, hacc[0][0].w};
#pragma unroll
      for (int j = 0; j < CMAX; ++j) {
        if (j < lay.cdim) {
          float z = u[j] + Wf[lay.bo_off + j];
          rgb[pw * lay.cdim + j] = 1.0f / (1.0f + expf(-z));
        }
      }
    }
  }
  if constexpr (PM && sv) save_act_pm<T, NTHR, HC, S16>(act, (char*)saved + PS.c + p0 * (int64_t)HC * HB, tid);
}

// ---- the colour layer's direction columns by rays (fp32). LinearWithRepeat (nerf_mlp.py) feeds every
// point of a ray the same direction embedding, so dW_dir[c][k] = sum_p dZc[p][c] dirPE[ray(p)][k]
// = sum_r dirPE[r][k] (sum_{p in r} dZc[p][c]). The dX kernel sums dZc per ray over each thread-chunk of its tile
// (dzc_chunk points, ascending), the block kernel adds a ray's chunk partials (ascending) and accumulates the products
// over blocks of DIRB rays (ascending), the final kernel adds the blocks (ascending): deterministic, and a 128 x 27
// product over R rays replaces a 128 x 64 dW tile over every point. Used when P >= dzc_chunk (a ray then touches at
// most two partials per chunk slot). fp32 only: its fine backward measured 15.2 -> 15.0 ms; bf16 and x3 gained less in
// dW than the per-ray sums cost in their dX (bf16 1.76 -> 1.79 ms, x3 10.11 -> 10.15 ms).
template <typename T> __host__ __device__ constexpr int dzc_chunk() { return Cfg<T>::M / (Cfg<T>::DXWAVES * 64 / HC); }
constexpr int DIRB = 16;  // rays per block of the dirPE product
template <typename T> __device__ __forceinline__ float lds_val(const typename Cfg<T>::lds_t* act, int m, int col);
template <> __device__ __forceinline__ float lds_val<float>(const float* act, int m, int col) {
  return act[lds_idx<float>(m, col)];
}
template <> __device__ __forceinline__ float lds_val<bf16_t>(const bf16_t* act, int m, int col) {
  return bf2f(act[lds_idx<bf16_t>(m, col)]);
}
template <> __device__ __forceinline__ float lds_val<x3_t>(const bf16_t* act, int m, int col) {
  constexpr int PL = Cfg<x3_t>::M * ROW;  // exact: the three planes hold disjoint bits of the fp32 value
  const int i = lds_idx<x3_t>(m, col);
  return (bf2f(act[i]) + bf2f(act[PL + i])) + bf2f(act[2 * PL + i]);
}

// ============================================================================================ backward dX
template <typename T, bool S16 = false>
__global__ void __launch_bounds__(Cfg<T>::DXWAVES * 64)
    __attribute__((amdgpu_waves_per_eu(Cfg<T>::WPE))) mlp_bwd_dx_kernel(
    MlpLayout lay, const typename Cfg<T>::w_t* __restrict__ Wt, const float* __restrict__ Wf,
    const uint64_t* __restrict__ masks, const float* __restrict__ rgb, const float* __restrict__ g_sigma,
    const float* __restrict__ g_rgb, int64_t N, int64_t Npad, typename Cfg<T>::st_t* __restrict__ grad, int64_t P,
    float* __restrict__ dzc_part) {
  constexpr int M = Cfg<T>::M, WAVES = Cfg<T>::DXWAVES, MT = M / 16;
  // ReLU-mask words: the forward (Cfg::WAVES waves) wrote mask_w<T>() words per lane per layer; a dX wave whose
  // NT x MT tiles are exactly one 16-tile word of a forward wave reads that word at the same index
  // ((layer * grid + wg) * DXWAVES + wave) * 64 + lane, with the same bit positions
  constexpr int NT = 256 / 16 / WAVES, MW = (NT * MT + 15) / 16;
  static_assert(Cfg<T>::WAVES * mask_w<T>() == WAVES * MW &&
                    (Cfg<T>::WAVES == WAVES || (NT * MT == 16 && (256 / 16 / Cfg<T>::WAVES) % NT == 0)),
                "dX wave tiles must map onto the forward's mask words");
  constexpr int KB = Cfg<T>::KB, TPP = WAVES * 64 / M, CPT = HC / TPP;  // colour columns per thread
  static_assert(CPT % 16 == 0, "colour-head backward: whole 16-feature tiles per thread");
  typedef typename Cfg<T>::lds_t LT;
  __shared__ __attribute__((aligned(16))) LT act[Cfg<T>::PLANES * M * ROW];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t tile = (int64_t)blockIdx.x, ntiles = (int64_t)gridDim.x;
  const int64_t p0 = tile * M;
  typedef typename Cfg<T>::st_t ST;
  const int64_t ld = row_ld(Npad, sizeof(ST)), ldb = ld * (int64_t)sizeof(ST);
  const uint32_t soff = (uint32_t)(4 * g * ldb + li * (int64_t)sizeof(ST));  // this lane's offset in a row tile
  const int64_t wpl = lay.t_plane;
  constexpr bool PM = Cfg<T>::PM;
  constexpr int NTHR = WAVES * 64;
  const GradRows GR = grad_rows(lay.L, PM);
  // point-major: byte sections (pm_grad); per-wave |max| of each gradient section for its fp8 scale in LDS slots past
  // the colour-output weights (PE columns of row 16), two sets used alternately: a set is rewritten only after the
  // barrier that follows the copy reading it
  [[maybe_unused]] char* const gb = (char*)grad;
  [[maybe_unused]] const PmGrad PG = pm_grad(lay.L, Npad, S16);
  constexpr int GB = pm_gb(S16);
  [[maybe_unused]] float* const g8red = (float*)(act + 16 * ROW + PE_COL);
  [[maybe_unused]] float* const g8scl = (float*)(gb + PG.scale) + tile;
  [[maybe_unused]] const int64_t ntile = Npad / M;
  auto g8_note = [&](int set, float amax) {  // this wave's |max| of the section being formed
    if constexpr (PM && !S16) {
      amax = wave_max(amax);
      if (lane == 0) g8red[8 * set + wave] = amax;
    }
  };
  const int mt_ = tid / TPP, q = tid % TPP;
  const int64_t p = p0 + mt_;
  const bool valid = p < N;
  const int cd = lay.cdim;
  // fp32 slot i of the heads-step staging (w_d at 0..255, dsigma at 256 + point) in the PE columns of rows 20.. (the
  // dX kernel's GEMMs never read the PE columns; rows 0..15 hold the colour-output weights, row 16 the fp8 scale slots)
  constexpr int HFPR = KPE * (int)sizeof(LT) / 4;  // fp32 slots per row
  static_assert(20 + (256 + M) / HFPR <= M, "heads-step staging rows");
  auto hd_lds = [&](int i) -> float* { return (float*)(act + (20 + i / HFPR) * ROW + PE_COL) + (i % HFPR); };
  // ---- sigmoid backward (grad * (1 - y) * y) and output layer backward
  float du[CMAX] = {0.f, 0.f, 0.f, 0.f};
  const float gs = valid ? g_sigma[p] : 0.0f;
  for (int j = 0; j < cd; ++j) {
    if (valid) {
      float y = rgb[p * cd + j];
      du[j] = (g_rgb[p * cd + j] * (1.0f - y)) * y;
    }
  }
  // dU / dsigma rows: stored after the colour head (below), whose mask-word loads would otherwise wait for them
  auto store_du = [&]() {
    if (q == 0) {
      if constexpr (PM) {
        ST* gdu = (ST*)(gb + PG.du) + p * 16;
        for (int j = 0; j < cd; ++j) gdu[j] = to_st<T>(du[j]);
        gdu[PM_DSIG] = to_st<T>(gs);
      } else {
        for (int j = 0; j < cd; ++j) grad[(GR.du + j) * ld + p] = to_st<T>(du[j]);
        grad[(GR.dyx + 256) * ld + p] = to_st<T>(gs);
      }
    }
  };
  {
    // the colour-output weights (cd x HC fp32, <= 2 KB) are staged once in the LDS tile's PE columns, which the dX
    // kernel never uses: the colour-head backward then reads them as 16-byte LDS broadcasts (the lanes of one point
    // group read the same address) instead of CMAX * CPT per-lane global loads (measured: the colour head cost
    // 0.16 ms of the 1.28 ms bf16 dX with those loads)
    constexpr int WFPR = KPE * (int)sizeof(LT) / 4;  // fp32 slots per row in the PE columns
    static_assert(WFPR % 8 == 0 && (CMAX * HC) / WFPR <= M, "colour-output weights in the PE columns");
    auto wo_row = [&](int i) -> float* { return (float*)(act + (i / WFPR) * ROW + PE_COL) + (i % WFPR); };
    for (int i = tid; i < CMAX * HC; i += NTHR) *wo_row(i) = i < cd * HC ? Wf[lay.wo_off + i] : 0.0f;
    // the density-head weights w_d and this tile's dsigma, for the heads step's w_d (x) dsigma term (read there from
    // LDS: as global loads after the dY stores, each waited on the in-order vmcnt for those stores)
    for (int i = tid; i < 256; i += NTHR) hd_lds(i)[0] = Wf[lay.wd_off + i];
    if (q == 0) hd_lds(256 + mt_)[0] = gs;
    // colour-hidden ReLU masks for this point: feature tiles CPT/16 * q .. (slot L)
    constexpr int TT = CPT / 16;
    uint64_t cw[TT][4];
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cw[t][r] = masks[lay.L * trunk_mask_words<T>(Npad) + mask_index(Npad, 0, p / 16, TT * q + t) + r];
    // statically indexed (tile t, feature cl) loops keep the mask words in registers (a runtime index into cw
    // would put it in scratch); the colour-output sum runs over j < cd with the reference's order, unrolled to CMAX
    // with a predicate, and every 16-byte chunk of the row goes to LDS in one store
    constexpr int EPC = Cfg<T>::EPC;
    static_assert(16 * ROW + PE_COL + 16 * (int)sizeof(float) / (int)sizeof(LT) <= M * ROW &&
                      (CMAX * HC) / WFPR <= 16, "fp8 scale slots after the colour-output weights");
    float amax = 0.0f;
    lds_barrier();
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int c0 = 0; c0 < 16; c0 += EPC) {
        // dc[e] = sum_j du_j * Wo[j][c0 + e] over this chunk's EPC columns, j ascending (the reference's order);
        // Wo's chunk row j is EPC consecutive slots of one LDS row
        float dc[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) dc[e] = 0.0f;
#pragma unroll
        for (int j = 0; j < CMAX; ++j)
          if (j < cd) {
#pragma unroll
            for (int e = 0; e < EPC; e += 4) {
              const f4 v = *(const f4*)wo_row(j * HC + CPT * q + 16 * t + c0 + e);
              dc[e] += du[j] * v.x;
              dc[e + 1] += du[j] * v.y;
              dc[e + 2] += du[j] * v.z;
              dc[e + 3] += du[j] * v.w;
            }
          }
        float dz[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const int cl = c0 + e, c = CPT * q + 16 * t + cl;
          // feature cl within its 16-feature tile: ballot word cl & 3, bit 16 * (cl >> 2) + point
          const bool on = (cw[t][cl & 3] >> (16 * (cl >> 2) + (mt_ & 15))) & 1ull;
          dz[e] = on ? dc[e] : 0.0f;
          if constexpr (!PM) grad[(GR.dzc + c) * ld + p] = to_st<T>(dz[e]);
          amax = fmaxf(amax, fabsf(dz[e]));
        }
        lds_put_chunk<T>(act, mt_, (CPT * q + 16 * t + c0) / EPC, dz);
      }
    g8_note(0, amax);  // dZc: set 0
  }
  store_du();
  lds_barrier();
  f4 acc[NT][MT];
  const int nrow0 = wave * NT * 16;
  // ---- dY = Wc[:, :256]^T dZc   (K = 128)
  gemm_lds<T, NT, MT>(Wt + lay.wcT_off, wpl, HC, nrow0, act, 0, HC / KB, acc, lane);
  ARing<T, NT> ring;  // next GEMM's weights, fetched during the epilogue (bf16)
  ring_fill<T, NT, true>(ring, Wt + lay.wintT_off, wpl, 256, nrow0, 256 / KB, lane);
  // point-major gradients leave the LDS tile after the GEMM that reads them (and its next-ring loads): see the
  // forward's trunk loop on the shared, in-order vmcnt
  if constexpr (PM)
    save_grad_rows_pm<T, NTHR, HC, S16>(act, gb + PG.dzc + p0 * HC * GB, g8scl + (lay.L + 1) * ntile, g8red, WAVES,
                                        tid);
  if (dzc_part) {
    // per-ray sums of dZc over this thread's chunk of the tile (column c), for the dirPE weight gradient by rays
    constexpr int CH = dzc_chunk<T>();
    static_assert(NTHR % HC == 0 && CH * (NTHR / HC) == M, "dZc chunks");
    const int c = tid % HC, ul = tid / HC;
    const int64_t pc0 = p0 + (int64_t)ul * CH, u = pc0 / CH;
    // P >= CH: the chunk holds the tail of its first ray [0, nb) and at most the head of the next [nb, n)
    const int n = (int)(N - pc0 < CH ? (N - pc0 > 0 ? N - pc0 : 0) : CH);
    const int nb = (int)(P - pc0 % P) < n ? (int)(P - pc0 % P) : n;
    const int m0 = ul * CH;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
    for (int i = 0; i < nb; ++i) s0 += lds_val<T>(act, m0 + i, c);
#pragma unroll 8
    for (int i = nb; i < n; ++i) s1 += lds_val<T>(act, m0 + i, c);
    if (n > 0) dzc_part[(u * 2) * HC + c] = s0;
    if (n > nb) dzc_part[(u * 2 + 1) * HC + c] = s1;
  }
  lds_barrier();
  // fp32: dY and dZ_l (l >= 1) leave from the B fragments of the GEMM that reads them, each K-block's stores BEFORE its
  // MFMAs (RSV_DX; after them, as the forward does, measured slower here); dZ_0 from the last epilogue
  constexpr bool GSX = std::is_same<T, float>::value;
  G8Max gmax;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nrow0 + 16 * nt + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      f4 v = acc[nt][mt];
      const Pk<T> h = pk_make<T>(v);
      if constexpr (PM && !S16) gmax.add(h);
      pk_lds<T>(act, m, n, h);
      if constexpr (!PM && !GSX)  // else stored by the first trunk step's GEMM
        pk_store_rows_b<T>((grad + (GR.dyx + nrow0 + 16 * nt) * ld + p0),
                             soff, (int)ldb, 16 * mt * (int)sizeof(ST), h);
    }
  }
  g8_note(1, gmax.value());  // dY: set 1
  lds_barrier();
  // ---- dH_{L-1} = Wint^T dY + w_d (x) dsigma ; dZ_{L-1} = dH * [H_{L-1} > 0], then trunk layer l -> l-1.
  // One step: the GEMM with the transposed weights (Wint^T from the heads, else layer l's), then the masked epilogue
  // into dZ_{l-1}. The step from the heads (HEAD: adds the density-head term w_d * dsigma) is peeled off the loop, so
  // the loop body keeps no per-point dsigma values live.
  auto trunk_step = [&](auto head, int l) {
    constexpr bool HEAD = decltype(head)::value;
    const typename Cfg<T>::w_t* A = HEAD ? Wt + lay.wintT_off : Wt + lay.wt_off[l];
    const int hl = l - 1;  // layer whose output gradient we form
    uint64_t bits[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w)
      bits[w] = masks[((((int64_t)hl * ntiles + tile) * WAVES + wave) * MW + w) * 64 + lane];
    gemm_lds<T, NT, MT, GSX ? RSV_DX : 0>(A, wpl, 256, nrow0, act, 0, 256 / KB, acc, lane, nullptr, &ring,
                                          RowSave{(float*)(void*)(grad + (HEAD ? GR.dyx : GR.dz0 + 256LL * l) * ld + p0),
                                                  soff, (int)ldb, 256 / KB, wave, WAVES});
    if (l - 1 >= 1) ring_fill<T, NT, true>(ring, Wt + lay.wt_off[l - 1], wpl, 256, nrow0, 256 / KB, lane);
    // fp8 scale sets: dZc 0, dY 1, then dZ_{L-1}, dZ_{L-2}, ... alternate from set 0
    if constexpr (PM) {  // the GEMM's input: dY (from the heads) or dZ_l
      if constexpr (HEAD)
        save_grad_rows_pm<T, NTHR, 256, S16>(act, gb + PG.dy + p0 * 256 * GB, g8scl + lay.L * ntile, g8red + 8, WAVES,
                                             tid);
      else
        save_grad_rows_pm<T, NTHR, 256, S16>(act, gb + PG.dz0 + ((int64_t)l * Npad + p0) * 256 * GB, g8scl + l * ntile,
                                             g8red + 8 * ((lay.L + 1 - l) & 1), WAVES, tid);
    }
    lds_barrier();
    G8Max gmax;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nrow0 + 16 * nt + 4 * g;
      f4 wdv = f4{0.f, 0.f, 0.f, 0.f};
      if constexpr (HEAD) wdv = *(const f4*)hd_lds(n);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + li;
        f4 v = acc[nt][mt];
        if constexpr (HEAD) {
          const float gsm = *hd_lds(256 + m);  // 0 past N (gs of an invalid point)
          v = v + wdv * gsm;
        }
        // ReLU mask of H_{hl}: this lane's own bits of this tile (packed by the forward)
        const Pk<T> h = pk_make<T>(apply_mask_tile<T, MW>(v, bits, nt * MT + mt));
        if constexpr (PM && !S16) gmax.add(h);
        pk_lds<T>(act, m, n, h);
        if constexpr (!PM)
          if (!GSX || hl == 0)
            pk_store_rows_b<T>((grad + (GR.dz0 + 256LL * hl + nrow0 + 16 * nt) * ld + p0), soff, (int)ldb,
                               16 * mt * (int)sizeof(ST), h);
      }
    }
    g8_note((lay.L + 1 - hl) & 1, gmax.value());  // dZ_hl
    lds_barrier();
  };
  trunk_step(std::integral_constant<bool, true>{}, lay.L);
  for (int l = lay.L - 1; l >= 1; --l) trunk_step(std::integral_constant<bool, false>{}, l);
  if constexpr (PM)
    save_grad_rows_pm<T, NTHR, 256, S16>(act, gb + PG.dz0 + p0 * 256 * GB, g8scl, g8red + 8 * ((lay.L + 1) & 1), WAVES,
                                         tid);
}

// ============================================================================================ backward dW
// dW_l[n][k] = sum_points dZ_l[n][p] * X_l[k][p] (+ bias column: sum_points dZ_l[n][p]). One workgroup owns a
// [BN x BK] tile of one layer's dW for a contiguous split of the points; partial tiles go to per-split fp32 slabs and
// dw_reduce sums them in split order (deterministic, no atomics) straight into the reference-layout gradient tensors.
// Three tile kinds: fp32 (dw_tile: feature-major rows staged by LDS-DMA, fp32 MFMA), bf16 (dw_tile_pm: point-major fp8 /
// bf16 sections, transposed LDS reads, fp8 block-scaled or bf16 MFMA) and x3 (dw_tile_x3: fp32 rows split into three
// bf16 planes on the way into LDS).
struct DwJob {
  // (column / row counts are int16: the whole DwJobs block is a kernel argument and must stay within 4 KB)
  const void* A;  // dZ rows [a_rows][ld] (points contiguous)
  const void* X0;  // layer input rows: segment 0 then segment 1
  const void* X1;
  int64_t slab_off;
  float* W;  // grad of weight [a_rows][ktot] (reference layout)
  float* b;  // grad of bias [a_rows]
  const float* a_scale;  // A's decode scale per 128-point tile
  const float* x_scale;  // X0's decode scale per 128-point tile (fp8 Y), or null
  // fp32: this job also forms a head's weight gradient in its tiles, into that head job's slab region at ext_slab_off
  // (the head job then has no tiles of its own):
  //  ext 1 (intermediate_linear): density -- the dsigma row (the gradient row right after the job's 256 A rows)
  //        against the job's own X = H_{L-1};
  //  ext 2 (color_layer.0, its first k-tile): color_layer.2 -- ext_rows dU rows (ext_a) against the 128 rows of C
  //        (ext_x), both staged beside the tile's own operands
  int64_t ext_slab_off;
  const void* ext_a;
  const void* ext_x;
  int wg_base;  // first workgroup of the job in the 1-D grid (k_tiles * S workgroups per job)
  int16_t a_rows;
  int16_t x0_rows;
  int16_t x1_rows;
  int16_t ktot;  // x0 + x1 ; slab row length = ktot + 1 (bias column)
  int16_t bn;    // 256 | 128 | 64 rows per tile
  int16_t k_full;   // tiles of dw_bkmax(prec) columns, then (if k_tiles > k_full) one tail tile of bk_tail columns
  int16_t bk_tail;  // 64 | 128 | 256
  int16_t k_tiles;
  // point-major operands (Cfg::PM): A / X0 / X1 are [Npad][ld] sections (A already offset to its first column);
  // a_chunks = 16-byte chunks of A per point that hold data; the tile's column space is "virtual": X0's columns
  // padded to x0p (a multiple of 8), then X1's (ktot_v = x0p + x1_rows); k-tiles are laid over ktot_v
  int16_t a_ld, a_chunks, x0_ld, x1_ld, x0p, ktot_v;
  int16_t w_ld;  // row stride of W: ktot, or more when trailing columns come from elsewhere (the per-ray dirPE term)
  int16_t x0_u8, x1_u8;  // X0 / X1 stored as fp8 e4m3 (the post-ReLU sections, Y); a k-tile is one format
  int16_t a_u8;          // A stored as fp8 e4m3 of value / scale (dZ_l, dY, dZc; not dU)
  int16_t ext, ext_rows, ext_ktot;
  int16_t gi;  // index of the job's weight gradient in the parameter list (2 * layer, ...)
};
constexpr int kMaxDwJobs = MAXL + 4;
struct DwJobs {
  DwJob j[kMaxDwJobs];
  int n;
  int total_tiles;
  int total_wg;  // workgroups of the dW launch (total_tiles * S)
  int S;         // point splits of every k-tile
  int64_t slab_elems;
  int64_t slab_stride;  // elements between two splits' slabs: slab_elems padded to a multiple of 4 (dw_slab_pad)
};
constexpr int DW_THREADS = 512;
// widest dW column tile: bf16 is HBM/L2-bound (a 256-wide tile reads each dZ row once), fp32 is MFMA-bound and
// runs faster with 128-wide tiles (measured: fp32 dW 8.3 ms vs 11.0 ms at 256; bf16 1.66 vs 2.0 ms at 128)
__host__ __device__ constexpr int dw_bkmax(int prec) {
  return (prec == YANERF_PREC_BF16 || prec == YANERF_PREC_BF16S) ? 256 : 128;
}
template <typename T> constexpr int prec_of = YANERF_PREC_BF16;
template <> constexpr int prec_of<float> = YANERF_PREC_F32;
template <> constexpr int prec_of<x3_t> = YANERF_PREC_F32X3;

__device__ __forceinline__ float hsum4(f4 v) { return (v.x + v.y) + (v.z + v.w); }

// fp32 stage ring: DW32_STAGES buffers of up to 392 rows x 128 B (two K-blocks = 32 points per row), filled by LDS-DMA
// (global_load_lds_dwordx4; one wave-instruction = 8 whole rows) DW32_STAGES - 1 stages ahead of the one being
// multiplied. The DMA destination is lane-linear, so the bank swizzle (16-byte chunk c of row r stored at
// c ^ ((r >> 1) & 7), conflict-free for the 16x16 fragment reads) goes on the SOURCE chunk. One raw barrier per stage:
// after it every wave's DMA for this stage has landed (each wave waited for its own with a counted vmcnt) and every wave
// is done reading the buffer the next DMA overwrites. Two K-blocks per stage halve the stage barriers of one K-block
// per stage (round 2, with the stagger below: 7.98 -> 7.86 ms). A stage holds at most 256 + 128 rows (dw_bkmax 128) +
// DW_EXT_ROWS: 3 stages of 49 KB. (Smaller rings so two workgroups share a CU measured slower: the fp32 dW's idle MFMA
// cycles are not stage-barrier bubbles another workgroup could fill.)
constexpr int DW_CPR = 8;           // 16-byte chunks per staged row
constexpr int DW_RB = 16 * DW_CPR;  // staged row bytes
constexpr int DW_RPI = 64 / DW_CPR; // rows per DMA wave-instruction
constexpr int DW32_STAGES = 3;
// + DW_EXT_ROWS rows per stage for a fused head (one DMA wave-instruction of A rows: the dsigma row or the dU rows,
// then spare rows); the colour tile (128 + 128 rows) stages C's 128 rows beside them in the same 392-row stage. The
// heads' weight gradients inside the bigger tiles: the density and colour-output jobs, as 64-row tiles with one / three
// useful rows, took 0.42 ms of the 7.6 ms fine fp32 dW (fused: 7.65 -> 7.39 ms, bitwise equal).
constexpr int DW_EXT_ROWS = 8;
constexpr int DW32_STAGE_BYTES = (256 + 128 + DW_EXT_ROWS) * DW_RB;
// points per dW stage
constexpr int X3_SPTS = 32;   // x3: one bf16 K-block, register staged
constexpr int PM_SPTS = 64;   // bf16: two stacked 32-point K-blocks per LDS-DMA stage (half the stage barriers)
static int64_t dw_stage_pts(int prec) {
  if (prec == YANERF_PREC_F32X3) return X3_SPTS;
  if (prec == YANERF_PREC_BF16) return PM_SPTS;
  if (prec == YANERF_PREC_BF16S) return 32;  // bf16 images: a 256 x 256 tile's 32-point stage fills PM_STAGE_BYTES
  return Cfg<float>::KB * (DW_CPR / 4);
}
__device__ __forceinline__ int dw_swz4(int row, int c) { return c ^ (((row >> 3) & 1) << 1); }  // 64-byte rows (x3)
__device__ __forceinline__ int dw_swz(int row, int c) { return c ^ ((row >> 1) & 7); }          // 128-byte rows

// fp32 dW tile. Staggered SIMD partners: a 512-thread workgroup puts waves w and w + 4 on one SIMD; waves 4-7 multiply
// the previous stage's second K-block (kept in registers) and then this stage's first, waves 0-3 both K-blocks of this
// stage, so while one partner waits on its LDS reads after the stage barrier the other has MFMAs ready (round 2:
// 8.15 -> 7.95 ms). Per accumulator the points still arrive in order: bitwise equal to the unstaggered loop.
template <int BN, int BK, int EXT = 0>
__device__ __forceinline__ void dw_tile(const DwJob& J, int k0, int s, int S, int64_t Npad, float* __restrict__ slab,
                                        int64_t slab_elems, char* smem) {
  typedef float T;
  constexpr int EPC = Cfg<T>::EPC, KB = Cfg<T>::KB;
  constexpr int RSTG = DW32_STAGES, RSB = DW32_STAGE_BYTES;  // ring depth, bytes per stage
  constexpr int WN = BN / 64, WK0 = 8 / WN, WK = (BK / 16 < WK0) ? BK / 16 : WK0, KTW = BK / WK / 16;
  static_assert(KTW >= 1 && WN * WK <= 8, "dW wave tiling");
  // EXT: DW_EXT_ROWS head A rows after the X rows (rows XE ..), then (EXT 2) the head's 128 X rows (rows XX ..)
  constexpr int XE = BN + BK, XX = XE + DW_EXT_ROWS, XH = EXT == 2 ? 128 : 0;
  constexpr int ROWS = BN + BK + (EXT ? DW_EXT_ROWS + XH : 0), PW = (ROWS + 8 * DW_RPI - 1) / (8 * DW_RPI);
  static_assert((ROWS + DW_RPI - 1) / DW_RPI * DW_RPI * DW_RB <= RSB, "dW stage buffer");
  static_assert(EXT == 0 || (BK == 128 && ((EXT == 1 && BN == 256) || (EXT == 2 && BN == 128))),
                "fused heads: fp32 256 x 128 (density) / 128 x 128 (colour output) tiles");
  constexpr int KBS = DW_CPR / 4;  // K-blocks per stage
  static_assert(KBS == 2, "the staggered loop below takes two K-blocks per stage");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int wn = wave / WK, wk = wave % WK;
  const bool mma_wave = wave < WN * WK;
  const int64_t nst = Npad / (KB * KBS), ld = row_ld(Npad, sizeof(T));
  const int64_t st_lo = nst * s / S, st_hi = nst * (s + 1) / S;
  // this lane's DMA source rows: wave-instruction i covers rows DW_RPI * (8 i + wave) .. + DW_RPI, lane -> (row, slot);
  // rows past ROWS (padding of the last instruction) re-read a valid row into unused LDS
  const T* src[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int row = DW_RPI * (8 * i + wave) + lane / DW_CPR;
    const int ch = dw_swz(row, lane % DW_CPR);
    const T* p;
    if (row < BN) {
      p = (const T*)J.A + (int64_t)(row < J.a_rows ? row : 0) * ld;  // rows past a_rows: any valid row (unused)
    } else if (EXT == 1 && row >= XE) {
      p = (const T*)J.A + (int64_t)(row < ROWS ? BN + (row - XE) : 0) * ld;  // dsigma (+ following rows)
    } else if (EXT == 2 && row >= XX) {
      p = (const T*)J.ext_x + (int64_t)(row < ROWS ? row - XX : 0) * ld;  // C
    } else if (EXT == 2 && row >= XE) {
      p = (const T*)J.ext_a + (int64_t)(row - XE) * ld;  // dU rows 0 .. 7
    } else {
      const int k = k0 + row - BN;
      if (k < J.x0_rows) p = (const T*)J.X0 + (int64_t)k * ld;
      else if (k < J.ktot) p = (const T*)J.X1 + (int64_t)(k - J.x0_rows) * ld;
      else p = (const T*)J.X0;  // columns past ktot / padding rows are never stored
    }
    src[i] = p + ch * EPC;
  }
  auto issue = [&](int64_t st) {
    char* dst = smem + (int)(st % RSTG) * RSB;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      // a wave-instruction whose 1 KB would reach past the stage (EXT's last one, waves >= 1) goes to the spare KB after
      // the ring, so every wave issues PW loads per stage and the counted vmcnt waits stay uniform
      char* d = ((8 * i + wave) * 1024 + 1024 <= RSB) ? dst + (8 * i + wave) * 1024 : smem + RSTG * RSB;
      __builtin_amdgcn_global_load_lds(src[i] + st * (KB * KBS), (__attribute__((address_space(3))) void*)d, 16, 0, 0);
    }
  };
  const f4 zero = f4{0.f, 0.f, 0.f, 0.f};
  constexpr int BPT = BN * DW_CPR / DW_THREADS > 0 ? BN * DW_CPR / DW_THREADS : 1;  // bias chunks per thread
  float rsum[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) rsum[i] = 0.f;
  const bool do_bias = (k0 == 0);
  f4 acc[4][KTW];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int q = 0; q < KTW; ++q) acc[nt][q] = zero;
  [[maybe_unused]] f4 acc_e = zero;     // EXT: the head rows' accumulator (this wave's 16 columns)
  [[maybe_unused]] float rsum_e = 0.f;  // EXT: the head biases (thread DW_CPR j + c sums chunk c of head row j)
  auto bias_rows = [&](const char* buf) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + DW_THREADS * i, row = idx / DW_CPR, ch = idx % DW_CPR;
      if (row < BN) rsum[i] += hsum4(*(const f4*)(buf + row * DW_RB + (ch << 4)));
    }
    if constexpr (EXT != 0) {
      if (tid < DW_CPR * J.ext_rows)
        rsum_e += hsum4(*(const f4*)(buf + (XE + tid / DW_CPR) * DW_RB + ((tid % DW_CPR) << 4)));
    }
  };
  {
    const bool late = wave >= 4;
    f4 a0[4], b0[KTW], a1[2][4], b1[2][KTW];
    // EXT: the extra 16-row A fragment (the head rows first; rows past the staged 8 read whatever LDS holds there --
    // their products are never stored) and its accumulator. EXT 1: wave w multiplies it with its own column fragment
    // QE = w / 2, so the 8 waves cover the tile's 8 column fragments once (wave w owns fragments 4 (w % 2) .. + 3);
    // EXT 2: with column fragment w of C (rows XX + 16 w ..)
    [[maybe_unused]] f4 e0 = zero, e1[2] = {zero, zero}, x0 = zero, x1[2] = {zero, zero};
    const int QE = wave >> 1;
    auto rf = [&](const char* buf, int kb, f4 (&fa)[4], f4 (&fb)[KTW], f4& fe, f4& fx) {
#pragma unroll
      for (int q = 0; q < KTW; ++q) {
        const int row = BN + (wk * KTW + q) * 16 + li;
        fb[q] = *(const f4*)(buf + row * DW_RB + (dw_swz(row, kb * 4 + g) << 4));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int row = wn * 64 + 16 * nt + li;
        fa[nt] = *(const f4*)(buf + row * DW_RB + (dw_swz(row, kb * 4 + g) << 4));
      }
      if constexpr (EXT != 0) {
        const int row = XE + li;
        fe = *(const f4*)(buf + row * DW_RB + (dw_swz(row, kb * 4 + g) << 4));
      }
      if constexpr (EXT == 2) {
        const int row = XX + 16 * wave + li;
        fx = *(const f4*)(buf + row * DW_RB + (dw_swz(row, kb * 4 + g) << 4));
      }
    };
    auto kblock = [&](const f4 (&fa)[4], const f4 (&fb)[KTW], const f4& fe, const f4& fx) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int q = 0; q < KTW; ++q)
            acc[nt][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[nt][ks], fb[q][ks], acc[nt][q], 0, 0, 0);
      if constexpr (EXT == 1) {
        static_assert(EXT != 1 || KTW == 4, "fused density row: four column fragments per wave");
        const f4 bq = QE == 0 ? fb[0] : QE == 1 ? fb[1] : QE == 2 ? fb[KTW > 2 ? 2 : 0] : fb[KTW > 3 ? 3 : 0];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc_e = __builtin_amdgcn_mfma_f32_16x16x4f32(fe[ks], bq[ks], acc_e, 0, 0, 0);
      } else if constexpr (EXT == 2) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc_e = __builtin_amdgcn_mfma_f32_16x16x4f32(fe[ks], fx[ks], acc_e, 0, 0, 0);
      }
    };
#pragma unroll
    for (int i = 0; i < RSTG - 1; ++i)
      if (st_lo + i < st_hi) issue(st_lo + i);
    auto begin_stage = [&](int64_t sc) {
      const int64_t ahead = st_hi - 1 - sc;
      static_assert(RSTG >= 2 && RSTG <= 5, "wait ladder below");
      if (ahead >= RSTG - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * (RSTG - 2)) : "memory");
      else if (RSTG == 5 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * 2) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (sc + RSTG - 1 < st_hi) issue(sc + RSTG - 1);
      return (const char*)(smem + (int)(sc % RSTG) * RSB);
    };
    if (late && mma_wave) {
      if (st_lo < st_hi) {
        const char* buf = begin_stage(st_lo);
        rf(buf, 0, a0, b0, e0, x0);
        rf(buf, 1, a1[0], b1[0], e1[0], x1[0]);
        kblock(a0, b0, e0, x0);
        if (do_bias) bias_rows(buf);
      }
      for (int64_t st = st_lo + 1; st < st_hi; st += 2) {
#pragma unroll
        for (int h = 1; h >= 0; --h) {
          const int64_t sc = st + (1 - h);
          if (sc < st_hi) {
            const char* buf = begin_stage(sc);
            rf(buf, 0, a0, b0, e0, x0);
            rf(buf, 1, a1[h], b1[h], e1[h], x1[h]);
            kblock(a1[h ^ 1], b1[h ^ 1], e1[h ^ 1], x1[h ^ 1]);
            kblock(a0, b0, e0, x0);
            if (do_bias) bias_rows(buf);
          }
        }
      }
      if (st_hi > st_lo) {
        if (((st_hi - 1 - st_lo) & 1) == 0) kblock(a1[0], b1[0], e1[0], x1[0]);
        else kblock(a1[1], b1[1], e1[1], x1[1]);
      }
    } else {
      for (int64_t sc = st_lo; sc < st_hi; ++sc) {
        const char* buf = begin_stage(sc);
        if (mma_wave) {
          rf(buf, 0, a0, b0, e0, x0);
          rf(buf, 1, a1[0], b1[0], e1[0], x1[0]);
          kblock(a0, b0, e0, x0);
          kblock(a1[0], b1[0], e1[0], x1[0]);
        }
        if (do_bias) bias_rows(buf);
      }
    }
  }
  float* out = slab + (int64_t)s * slab_elems + J.slab_off;
  const int kv = J.ktot + 1;
  if (mma_wave) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int q = 0; q < KTW; ++q) {
        const int k = k0 + (wk * KTW + q) * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = wn * 64 + 16 * nt + 4 * g + r;
          if (n < J.a_rows && k < J.ktot) out[(int64_t)n * kv + k] = acc[nt][q][r];
        }
      }
  }
  if constexpr (EXT != 0) {
    // the head rows: rows 0 .. ext_rows - 1 of the extra tile (lanes g == 0, elements 0 .. 3), this wave's column
    // fragment (EXT 1: QE of the tile's columns; EXT 2: column fragment w of C); the head job's slab rows hold
    // ext_ktot weights then the bias
    float* oute = slab + (int64_t)s * slab_elems + J.ext_slab_off;
    const int kve = J.ext_ktot + 1;
    const int k = EXT == 1 ? k0 + (wk * KTW + (wave >> 1)) * 16 + li : 16 * wave + li;
    if (g == 0 && k < J.ext_ktot) {
      const float v[4] = {acc_e.x, acc_e.y, acc_e.z, acc_e.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < J.ext_rows) oute[(int64_t)r * kve + k] = v[r];
    }
    if (do_bias) {
      float v = rsum_e;
#pragma unroll
      for (int o = 1; o < DW_CPR; o <<= 1) v += __shfl_xor(v, o, 64);
      if (tid % DW_CPR == 0 && tid < DW_CPR * J.ext_rows) oute[(int64_t)(tid / DW_CPR) * kve + J.ext_ktot] = v;
    }
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int idx = tid + DW_THREADS * i, row = idx / DW_CPR;
      float v = rsum[i];
#pragma unroll
      for (int o = 1; o < DW_CPR; o <<= 1) v += __shfl_xor(v, o, 64);
      if (idx % DW_CPR == 0 && row < BN && row < J.a_rows) out[(int64_t)row * kv + J.ktot] = v;
    }
  }
}

// Point-major bf16 dW (Cfg::PM). A stage is 32 points (one 16x16x32 K-block): the A image [32 points][BN features]
// and the X image [32 points][BK features], 2*BN / 2*BK bytes per point row, each filled by LDS-DMA from BN / BK
// contiguous features of the point's row in its section (512-byte runs for 256-wide tiles). MFMA operands come
// from the images with ds_read_b64_tr_b16: for lane group g (points 8g..8g+7) two transposed reads of 4 points x 16
// features give the 8-point fragment of 16 features, for dZ^T (A, rows = output features) and X (B, columns).
// 16-byte chunk c of image row r sits at chunk c ^ pm_swz(r): every transposed read is conflict-free (a 32-lane half
// touches rows {r0..r0+3, r0+8..r0+11} x 2 chunks -> 16 distinct bank slots). Bias gradients ride along as an extra
// MFMA against a ones fragment in the k-tile-0 workgroups (column sums over the points).
template <int ROWB>
__device__ __forceinline__ int pm_swz(int r) {
  static_assert(ROWB == 128 || ROWB == 256 || ROWB == 512, "pm image row width");
  if constexpr (ROWB == 128) return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
}

// stage buffer: the widest image pair (A + X, 64 points) of any instantiation (256-row fp8 A + 256-column fp8 X)
constexpr int PM_STAGE_BYTES = 32 * 1024;
// LDS-DMA ring depth of the point-major (bf16) dW tile: as many stages as fit 128 KB (2 / 3 stages so that two
// workgroups could share a CU measured flat)
constexpr int PM_STAGES = 4;
// wait until this wave's DMA of the stage about to be read has landed, given how many stages it issued after that
// one: vmcnt(PW * min(ahead, MAXA)) (the count must be an immediate)
template <int PW, int MAXA>
__device__ __forceinline__ void wait_dma_ahead(int64_t ahead) {
  static_assert(PW * MAXA <= 63, "vmcnt range");
  if (ahead >= MAXA) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * MAXA) : "memory");
    return;
  }
  if constexpr (MAXA > 1) wait_dma_ahead<PW, MAXA - 1>(ahead);
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// fp8 gradient scales of one split (one per 128-point tile), staged in LDS after the ring at the tile's start: a load
// per stage would be a vector load (the DMA intrinsics keep the compiler from proving the scales read-only for a
// scalar load), and waiting for it would drain the in-order DMA counter
constexpr int PM_SCALES = 512;
typedef short s4v __attribute__((ext_vector_type(4)));
// fragment of 16 features x 8 points (points 8g..8g+7 of the stage for lane group g) from an image with ROWB-byte rows
template <int ROWB>
__device__ __forceinline__ f4 pm_frag(const char* img, int f0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c = f0 / 8 + (p >> 1);
  f4 out;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int r = 8 * g + 4 * hh + q;
    const char* a = img + r * ROWB + 16 * (c ^ pm_swz<ROWB>(r)) + 8 * (p & 1);
    const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a));
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v w = __builtin_bit_cast(f2v, v);
    if (hh == 0) { out.x = w.x; out.y = w.y; } else { out.z = w.x; out.w = w.y; }
  }
  return out;
}

// fp8 X images ([32 points][RB bytes], RB = BK): chunk c of row r at c ^ pm_swz8(r), so that the transposed reads of a
// 32-lane half (16 rows x one chunk, two 8-byte halves) hit 64 distinct banks for RB = 64 / 128 / 256
template <int RB>
__device__ __forceinline__ int pm_swz8(int r) {
  static_assert(RB == 64 || RB == 128 || RB == 256, "fp8 pm image row width");
  return (r / (256 / RB)) & (RB / 16 - 1);
}
// fragment of 16 features x 8 points from an fp8 image: ds_read_b64_tr_b8 (per 16-lane group, lane 2q+p supplies row q,
// bytes 8p..8p+7 of a 16-byte chunk; lane i receives column i of the 8 rows, row q in byte q: tools/probes/probe_tr8.hip)
// gives lane (g, i) points 8g..8g+7 of feature f0 + i, widened to bf16 exactly (e4m3 fits bf16) for the bf16 MFMA
template <int RB>
__device__ __forceinline__ f4 pm_frag8(const char* img, int f0, int lane, float scale = 1.0f) {
  const int g = lane >> 4, i = lane & 15, q = i >> 1, p = i & 1;
  const int r = 8 * g + q;
  const char* a = img + r * RB + 16 * ((f0 / 16) ^ pm_swz8<RB>(r)) + 8 * p;
  typedef int i32x2 __attribute__((ext_vector_type(2)));
  const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(a));
  f4 out;
  out.x = __builtin_bit_cast(float, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, scale, false));
  out.y = __builtin_bit_cast(float, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, scale, true));
  out.z = __builtin_bit_cast(float, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, scale, false));
  out.w = __builtin_bit_cast(float, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, scale, true));
  return out;
}

// fp8 x fp8 tiles on the block-scaled fp8 MFMA: a 64-point stage is ONE
// v_mfma_scale_f32_32x32x64_f8f6f4 per 32 x 32 output tile (e4m3 operands, 64 cycles: twice the bf16 rate, and no
// widening), with the stage's power-of-two tile scales as the operands' e8m0 scales (exact, like the widening they
// replace). Operand map (tools/probes/probe_mfma_f8.hip, exact on the MI355X): lane l holds A[row l % 32][k = 32 (l / 32)
// + j] and B[k = 32 (l / 32) + j][col l % 32] in byte j of its 8 dwords. With points as k, lane (g, i) of a 16-lane group
// needs points 32 (g >> 1) + 0..31 of feature 16 (g & 1) + i: four ds_read_b64_tr_b8 (8 points each). Fine dW
// 1.06 -> 0.87 ms against the bf16 MFMA on widened operands (round 2).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
// image swizzle for those reads: a 32-lane half touches 8 consecutive rows x the chunk pair (c0, c0 ^ 1), c0 even, so
// s(r) >> 1 must differ over the 8 rows (RB = 256) or over the 4 rows of one parity (RB = 128, two rows per bank sweep)
template <int RB>
__device__ __forceinline__ int f8m_swz(int r) {
  static_assert(RB == 128 || RB == 256, "fp8 MFMA image row width");
  if constexpr (RB == 256) return 2 * (r & 7);
  else return 2 * ((r >> 1) & 3);
}
template <int RB>
__device__ __forceinline__ i32x8 f8m_frag(const char* img, int f0, int lane) {
  typedef int i32x2 __attribute__((ext_vector_type(2)));
  const int g = lane >> 4, i = lane & 15, q = i >> 1, p = i & 1;
  const int c = f0 / 16 + (g & 1);
  i32x8 out;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int r = 32 * (g >> 1) + 8 * t + q;
    const char* a = img + r * RB + 16 * (c ^ f8m_swz<RB>(r)) + 8 * p;
    const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(a));
    out[2 * t] = v.x;
    out[2 * t + 1] = v.y;
  }
  return out;
}
// e8m0 exponent of a power-of-two float scale
__device__ __forceinline__ int e8m0_of(float s) { return (int)((__float_as_uint(s) >> 23) & 0xffu); }
template <int BN, int BK, bool X8, bool A8, int SP = PM_SPTS>
constexpr bool use_f8mma() {
  return X8 && A8 && BK == 256 && (BN == 256 || BN == 128) && SP == 64;
}

// SP: points per stage -- PM_SPTS (64) for the fp8 tiles, 32 for YANERF_PREC_BF16S, whose bf16 256 x 256 tile images
// (16 KB + 16 KB per 32 points) would not fit a 32 KB stage at 64 points
template <int BN, int BK, bool X8, bool A8, int SP = PM_SPTS>
__device__ __forceinline__ void dw_tile_pm(const DwJob& J, int k0, int s, int S, int64_t Npad, float* __restrict__ slab,
                                           int64_t slab_elems, char* smem) {
  constexpr int WN = BN / 64, WK0 = 8 / WN, WK = (BK / 16 < WK0) ? BK / 16 : WK0, KTW = BK / WK / 16;
  static_assert(KTW >= 1 && WN * WK <= 8, "dW wave tiling");
  constexpr bool F8M = use_f8mma<BN, BK, X8, A8, SP>();
  constexpr int XEB = X8 ? 1 : 2, RBX = BK * XEB;             // X element bytes, X image row bytes
  constexpr int AEB = A8 ? 1 : 2, RBA = BN * AEB;
  constexpr int SPT = Cfg<bf16_t>::M / SP;  // stages per fp8 scale tile
  static_assert(SPT * SP == Cfg<bf16_t>::M, "an fp8 scale covers whole dW stages");
  constexpr int AB = SP * RBA, XB = SP * RBX;       // image bytes
  constexpr int NI = (AB + XB + 1023) / 1024, PW = (NI + 7) / 8;  // DMA wave-instructions per stage / per wave
  static_assert((AB + XB) % 1024 == 0, "pm dW images: whole DMA wave-instructions");
  static_assert(PW * 8 * 1024 <= PM_STAGE_BYTES, "pm dW stage");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int wn = wave / WK, wk = wave % WK;
  const bool mma_wave = wave < WN * WK;
  const int64_t nst = Npad / SP;
  const int64_t st_lo = nst * s / S, st_hi = nst * (s + 1) / S;
  // this lane's DMA source per wave-instruction and its per-stage advance (32 points of its section), in bytes
  const char* src[PW];
  int64_t adv[PW];
  const int x0b = J.x0_u8 ? 1 : 2, x1b = J.x1_u8 ? 1 : 2;  // == XEB for the section(s) this tile reads
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int ii = 8 * i + wave;
    const int b = (ii < NI ? ii : 0) * 1024 + lane * 16;
    if (b < AB) {
      const int r = b / RBA;
      int c;
      if constexpr (F8M) c = ((b % RBA) / 16) ^ f8m_swz<RBA>(r);
      else if constexpr (A8) c = ((b % RBA) / 16) ^ pm_swz8<RBA>(r);
      else c = ((b % RBA) / 16) ^ pm_swz<RBA>(r);
      src[i] = (const char*)J.A + (int64_t)r * J.a_ld * AEB + 16 * (c < J.a_chunks ? c : 0);
      adv[i] = (int64_t)SP * J.a_ld * AEB;
    } else if (b < AB + XB) {
      const int bx = b - AB, r = bx / RBX;
      int c;
      if constexpr (F8M) c = ((bx % RBX) / 16) ^ f8m_swz<RBX>(r);
      else if constexpr (X8) c = ((bx % RBX) / 16) ^ pm_swz8<RBX>(r);
      else c = ((bx % RBX) / 16) ^ pm_swz<RBX>(r);
      const int j = k0 + (16 / XEB) * c;  // virtual column
      if (j < J.x0p) {
        src[i] = (const char*)J.X0 + ((int64_t)r * J.x0_ld + j) * x0b;
        adv[i] = (int64_t)SP * J.x0_ld * x0b;
      } else if (j - J.x0p < J.x1_ld && J.X1) {
        src[i] = (const char*)J.X1 + ((int64_t)r * J.x1_ld + (j - J.x0p)) * x1b;
        adv[i] = (int64_t)SP * J.x1_ld * x1b;
      } else {  // past the virtual width: any valid address (never stored)
        src[i] = (const char*)J.X0 + (int64_t)r * J.x0_ld * x0b;
        adv[i] = (int64_t)SP * J.x0_ld * x0b;
      }
    } else {  // padding of the last wave-instruction: a valid source into unused LDS
      src[i] = (const char*)J.A;
      adv[i] = 0;
    }
  }
  // the operand stream is read once per launch (every split its own points, BK = 256: each gradient row in one
  // k-tile), so the LDS-DMA loads go non-temporal (aux 2: MI355X_MICROARCH.md nt-weights): bf16 fine dW 0.79 -> 0.755 ms
  // (microbench, two interleaved rounds, gradients bitwise equal: profiles/r5_ab_bf16_dw_nt.jsonl)
  auto issue = [&](int64_t st) {
    char* dst = smem + ((int)st % PM_STAGES) * PM_STAGE_BYTES;  // 32-bit modulo (the ring depth need not be 2^k)
#pragma unroll
    for (int i = 0; i < PW; ++i)
      __builtin_amdgcn_global_load_lds(src[i] + st * adv[i],
                                       (__attribute__((address_space(3))) void*)(dst + (8 * i + wave) * 1024), 16, 0, 2);
  };
  float* const scl = (float*)(smem + PM_STAGES * PM_STAGE_BYTES);
  const int64_t t0 = st_lo / SPT;
  // X0's scales (fp8 Y) in the next PM_SCALES slots, for the k-tiles over X0
  const bool xs = X8 && J.x_scale && k0 < J.x0p;
  float* const sclx = scl + PM_SCALES;
  {  // visible to every wave after the first stage's barrier (lgkmcnt(0) before it)
    const int ntl = st_lo < st_hi ? (int)((st_hi - 1) / SPT - t0 + 1) : 0;
    if constexpr (A8)
      for (int i = tid; i < ntl; i += DW_THREADS) scl[i] = J.a_scale[t0 + i];
    if (xs)
      for (int i = tid; i < ntl; i += DW_THREADS) sclx[i] = J.x_scale[t0 + i];
  }
  if constexpr (F8M) {
    // wave tile: 64 rows (two 32-row MFMA tiles) x BK / WK columns (NQ 32-column tiles)
    constexpr int WKF = 8 / WN, NQ = BK / WKF / 32;
    static_assert(NQ >= 1 && WN * WKF == 8, "fp8 MFMA dW wave tiling");
    const int wnf = wave / WKF, wkf = wave % WKF;
    const bool do_bias = (k0 == 0) && wkf == 0;
    const i32x8 ones = i32x8{0x38383838, 0x38383838, 0x38383838, 0x38383838,
                             0x38383838, 0x38383838, 0x38383838, 0x38383838};  // e4m3 1.0
    f16v acc[2][NQ], accb[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) accb[mt][e] = 0.f;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mt][q][e] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < PM_STAGES - 1; ++i)
      if (st_lo + i < st_hi) issue(st_lo + i);
    for (int64_t st = st_lo; st < st_hi; ++st) {
      const int64_t ahead = st_hi - 1 - st;
      wait_dma_ahead<PW, PM_STAGES - 2>(ahead);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (st + PM_STAGES - 1 < st_hi) issue(st + PM_STAGES - 1);
      const char* buf = smem + ((int)st % PM_STAGES) * PM_STAGE_BYTES;
      const int sa = e8m0_of(scl[st / SPT - t0]);
      const int sx = xs ? e8m0_of(sclx[st / SPT - t0]) : 127;
      i32x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) a[mt] = f8m_frag<RBA>(buf, wnf * 64 + 32 * mt, lane);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const i32x8 b = f8m_frag<RBX>(buf + AB, (wkf * NQ + q) * 32, lane);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt][q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[mt], b, acc[mt][q], 0, 0, 0, sa, 0, sx);
      }
      if (do_bias) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          accb[mt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[mt], ones, accb[mt], 0, 0, 0, sa, 0, 127);
      }
    }
    // C/D: column lane & 31, row (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
    float* out = slab + (int64_t)s * slab_elems + J.slab_off;
    const int kv = J.ktot + 1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = k0 + (wkf * NQ + q) * 32 + (lane & 31);  // virtual column -> weight column
      const int k = j < J.x0p ? (j < J.x0_rows ? j : -1) : (j - J.x0p < J.x1_rows ? J.x0_rows + j - J.x0p : -1);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = wnf * 64 + 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          if (n < J.a_rows && k >= 0) out[(int64_t)n * kv + k] = acc[mt][q][e];
        }
    }
    if (do_bias && (lane & 31) == 0) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = wnf * 64 + 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          if (n < J.a_rows) out[(int64_t)n * kv + J.ktot] = accb[mt][e];
        }
    }
  } else {
  const f4 zero = f4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = (k0 == 0) && wk == 0;
  const float one2 = __uint_as_float(0x3f803f80u);  // two bf16 1.0 halves
  const f4 ones = f4{one2, one2, one2, one2};
  f4 acc[4][KTW], accb[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    accb[nt] = zero;
#pragma unroll
    for (int q = 0; q < KTW; ++q) acc[nt][q] = zero;
  }
#pragma unroll
  for (int i = 0; i < PM_STAGES - 1; ++i)
    if (st_lo + i < st_hi) issue(st_lo + i);
  for (int64_t st = st_lo; st < st_hi; ++st) {
    const int64_t ahead = st_hi - 1 - st;
    static_assert(PM_STAGES >= 2, "pm dW ring");
    wait_dma_ahead<PW, PM_STAGES - 2>(ahead);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + PM_STAGES - 1 < st_hi) issue(st + PM_STAGES - 1);
    const char* buf = smem + ((int)st % PM_STAGES) * PM_STAGE_BYTES;
#pragma unroll
    for (int kb = 0; kb < SP / 32; ++kb)
    if (mma_wave) {
      // K-block kb of the stage: 32-point images at kb * 32 rows (the row swizzles repeat every 16 rows)
      const char* bufa = buf + kb * 32 * RBA;
      const char* bufx = buf + AB + kb * 32 * RBX;
      f4 a[4];
      const float sx = xs ? sclx[st / SPT - t0] : 1.0f;
      if constexpr (A8) {
        const float sa = scl[st / SPT - t0];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) a[nt] = pm_frag8<RBA>(bufa, wn * 64 + 16 * nt, lane, sa);
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) a[nt] = pm_frag<RBA>(bufa, wn * 64 + 16 * nt, lane);
      }
      constexpr int QG = KTW < 4 ? KTW : 4;
#pragma unroll
      for (int q0 = 0; q0 < KTW; q0 += QG) {
        f4 b[QG];
#pragma unroll
        for (int q = 0; q < QG; ++q) {
          if constexpr (X8) b[q] = pm_frag8<RBX>(bufx, (wk * KTW + q0 + q) * 16, lane, sx);
          else b[q] = pm_frag<RBX>(bufx, (wk * KTW + q0 + q) * 16, lane);
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int q = 0; q < QG; ++q) acc[nt][q0 + q] = mma_blk<bf16_t>(a[nt], b[q], acc[nt][q0 + q]);
      }
      if (do_bias) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) accb[nt] = mma_blk<bf16_t>(a[nt], ones, accb[nt]);
      }
    }
  }
  float* out = slab + (int64_t)s * slab_elems + J.slab_off;
  const int kv = J.ktot + 1;
  if (mma_wave) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int q = 0; q < KTW; ++q) {
        const int j = k0 + (wk * KTW + q) * 16 + li;  // virtual column -> weight column
        const int k = j < J.x0p ? (j < J.x0_rows ? j : -1) : (j - J.x0p < J.x1_rows ? J.x0_rows + j - J.x0p : -1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = wn * 64 + 16 * nt + 4 * g + r;
          if (n < J.a_rows && k >= 0) out[(int64_t)n * kv + k] = acc[nt][q][r];
        }
      }
    if (do_bias && li == 0) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = wn * 64 + 16 * nt + 4 * g + r;
          if (n < J.a_rows) out[(int64_t)n * kv + J.ktot] = accb[nt][r];
        }
    }
  }
  }
}

// x3 dW: dZ and the layer inputs are fp32 rows in HBM (the x3 forward / dX save fp32). Each stage of 32 points is
// loaded with 16-byte register loads (4 points of one row per thread-load), split into three bf16 planes on the way
// into LDS (same 64-byte rows and swizzle as the bf16 dW tile) and multiplied with the six plane products per 16x16x32
// step. Software pipelined over two LDS buffers with one barrier per stage: while a wave multiplies stage st from one
// buffer it splits stage st + 1 (loaded during stage st - 1) into the other, one staged segment after each of the six
// product terms, and reloads that segment's registers with stage st + 2 right away. The loop body is one basic block
// (no per-segment branches: every staging slot is a real row, the last stage's split and reloads are harmless repeats),
// so the split's VALU and LDS writes interleave with the MFMAs instead of running between two barriers with the
// SIMD's matrix pipe idle (round 3's pipelined variant kept the per-segment branches and measured equal). Per
// accumulator the stages and the six terms arrive in the same order: gradients bitwise equal to the unpipelined loop
// (Lego fine dW 5.44-5.63 -> 4.95-5.15 ms; the alternatives measured in round 6 are in profiles/r6_x3_dw_ab.md).
// Bias gradients are fp32 row sums of the loaded dZ segments.
template <int BN, int BK>
__device__ __forceinline__ void dw_tile_x3(const DwJob& J, int k0, int s, int S, int64_t Npad,
                                           float* __restrict__ slab, int64_t slab_elems, char* smem) {
  constexpr int WN = BN / 64, WK0 = 8 / WN, WK = (BK / 16 < WK0) ? BK / 16 : WK0, KTW = BK / WK / 16;
  static_assert(KTW >= 1 && KTW <= 4 && WN * WK == 8, "dW wave tiling: eight multiplying waves, one column group");
  constexpr int ROWS = BN + BK;
  static_assert(ROWS * 8 % DW_THREADS == 0, "x3 dW staging: whole 16-byte segments per thread");
  constexpr int LPT = ROWS * 8 / DW_THREADS;  // 16-B loads per thread per stage; slot i holds row tid / 8 + 64 i
  constexpr int LA = BN * 8 / DW_THREADS;     // slots 0 .. LA - 1 hold dZ rows (bias sums)
  static_assert(LPT <= 6, "x3 dW pipeline: one staged segment per product term");
  constexpr int PLB = 384 * 64, BUFB = 3 * PLB;  // plane / buffer bytes
  static_assert(ROWS <= 384, "x3 dW staging: at most 384 rows");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int wn = wave / WK, wk = wave % WK;
  const int64_t nst = Npad / X3_SPTS, ld = row_ld(Npad, sizeof(float));
  const int64_t st_lo = nst * s / S, st_hi = nst * (s + 1) / S;
  const float* src[LPT];
  int dst[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int flat = tid + DW_THREADS * i, row = flat >> 3, seg = flat & 7;
    const float* p;
    if (row < BN) {
      p = (const float*)J.A + (int64_t)(row < J.a_rows ? row : 0) * ld;
    } else {
      const int k = k0 + row - BN;
      if (k < J.x0_rows) p = (const float*)J.X0 + (int64_t)k * ld;
      else if (k < J.ktot) p = (const float*)J.X1 + (int64_t)(k - J.x0_rows) * ld;
      else p = (const float*)J.X0;
    }
    src[i] = p + seg * 4;
    dst[i] = row * 64 + (dw_swz4(row, seg >> 1) << 4) + (seg & 1) * 8;
  }
  f4 regs[LPT];
  float rsum[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) rsum[i] = 0.f;
  const f4 zero = f4{0.f, 0.f, 0.f, 0.f};
  f4 acc[4][KTW];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int q = 0; q < KTW; ++q) acc[nt][q] = zero;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  // split staged segment i (fp32) into the three bf16 planes of buffer `buf` (+ the dZ row sums)
  auto split_one = [&](int i, char* buf, bool sum) {
    const f4 v0 = regs[i];
    if (i < LA) {
      const float r = rsum[i] + ((v0.x + v0.y) + (v0.z + v0.w));
      rsum[i] = sum ? r : rsum[i];  // a select: the loop body stays one basic block
    }
    const Pk<bf16_t> h0 = pk_make<bf16_t>(v0);
    const f4 r1 = v0 - f4{__uint_as_float(h0.w0 << 16), __uint_as_float(h0.w0 & 0xffff0000u),
                          __uint_as_float(h0.w1 << 16), __uint_as_float(h0.w1 & 0xffff0000u)};
    const Pk<bf16_t> h1 = pk_make<bf16_t>(r1);
    const f4 r2 = r1 - f4{__uint_as_float(h1.w0 << 16), __uint_as_float(h1.w0 & 0xffff0000u),
                          __uint_as_float(h1.w1 << 16), __uint_as_float(h1.w1 & 0xffff0000u)};
    const Pk<bf16_t> h2 = pk_make<bf16_t>(r2);
    *(u32x2*)(buf + dst[i]) = u32x2{h0.w0, h0.w1};
    *(u32x2*)(buf + PLB + dst[i]) = u32x2{h1.w0, h1.w1};
    *(u32x2*)(buf + 2 * PLB + dst[i]) = u32x2{h2.w0, h2.w1};
  };
  if (st_lo < st_hi) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) regs[i] = *(const f4*)(src[i] + st_lo * X3_SPTS);
#pragma unroll
    for (int i = 0; i < LPT; ++i) split_one(i, smem + (int)(st_lo & 1) * BUFB, true);
    const int64_t st1 = st_lo + 1 < st_hi ? st_lo + 1 : st_lo;
#pragma unroll
    for (int i = 0; i < LPT; ++i) regs[i] = *(const f4*)(src[i] + st1 * X3_SPTS);
  }
  lds_barrier();
  // static priority for the second-dispatched half, the arbitration loser of each stage's start (5.12 -> 5.10 ms)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  constexpr int TI[6] = {2, 1, 0, 1, 0, 0}, TJ[6] = {0, 1, 2, 0, 1, 0};
  for (int64_t st = st_lo; st < st_hi; ++st) {
    const char* buf = smem + (int)(st & 1) * BUFB;
    char* nbuf = smem + (int)((st + 1) & 1) * BUFB;
    const int64_t st2 = st + 2 < st_hi ? st + 2 : st_hi - 1;  // the last stages reload a valid stage (unused)
    const bool nxt = st + 1 < st_hi;                           // the split of stage st + 1 is real
    f4 a[3][4], b[3][KTW];
    // the first term's operands (A plane 2, B plane 0) first
#pragma unroll
    for (int pl = 2; pl >= 0; --pl) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int row = wn * 64 + 16 * nt + li;
        a[pl][nt] = *(const f4*)(buf + pl * PLB + row * 64 + (dw_swz4(row, g) << 4));
      }
#pragma unroll
      for (int q = 0; q < KTW; ++q) {
        const int row = BN + (wk * KTW + q) * 16 + li;
        b[2 - pl][q] = *(const f4*)(buf + (2 - pl) * PLB + row * 64 + (dw_swz4(row, g) << 4));
      }
    }
    // one scheduling region per product term: its MFMAs, two VALU of the split after each, then the segment's three
    // plane writes and its reload (the first region also carries the operand reads not needed by the first term)
    constexpr int MT = 4 * KTW;  // MFMAs per term
#pragma unroll
    for (int t = 0; t < 6; ++t) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < KTW; ++q) acc[nt][q] = mma_blk<bf16_t>(a[TI[t]][nt], b[TJ[t]][q], acc[nt][q]);
      if (t < LPT) {
        split_one(t, nbuf, nxt);
        regs[t] = *(const f4*)(src[t] + st2 * X3_SPTS);
      }
      if (t == 0) __builtin_amdgcn_sched_group_barrier(0x100, 4 + KTW, 0);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (t == 0 && j < 2 * (4 + KTW)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 32 / MT, 0);
      }
      if (t < LPT) {
        __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
  }
  float* out = slab + (int64_t)s * slab_elems + J.slab_off;
  const int kv = J.ktot + 1;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int q = 0; q < KTW; ++q) {
      const int k = k0 + (wk * KTW + q) * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wn * 64 + 16 * nt + 4 * g + r;
        if (n < J.a_rows && k < J.ktot) out[(int64_t)n * kv + k] = acc[nt][q][r];
      }
    }
  if (k0 == 0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int flat = tid + DW_THREADS * i, row = flat >> 3;
      float v = rsum[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if ((flat & 7) == 0 && row < J.a_rows) out[(int64_t)row * kv + J.ktot] = v;
    }
  }
}

// stage bytes of a point-major dW tile; the dispatch below only instantiates the tiles that fit PM_STAGE_BYTES (the
// host checks every job's tiles against the same function before the launch)
__host__ __device__ constexpr int pm_tile_bytes(int bn, int bk, bool x8, bool a8, int sp = PM_SPTS) {
  return sp * (bn * (a8 ? 1 : 2) + bk * (x8 ? 1 : 2));
}
template <int BN, int BK, bool X8, bool A8, int SP = PM_SPTS>
__device__ __forceinline__ void run_pm(const DwJob& J, int k0, int s, int S, int64_t Npad, float* __restrict__ slab,
                                       int64_t slab_elems, char* smem) {
  if constexpr (pm_tile_bytes(BN, BK, X8, A8, SP) <= PM_STAGE_BYTES)
    dw_tile_pm<BN, BK, X8, A8, SP>(J, k0, s, S, Npad, slab, slab_elems, smem);
  // else: not instantiated; launch_bwd refuses a job with such a tile before the launch
}

template <typename T, bool S16 = false>
__global__ void __launch_bounds__(DW_THREADS) mlp_dw_kernel(DwJobs jobs, int64_t Npad, float* __restrict__ slab) {
  // x3: two buffers of three 384-row bf16 planes (144 KB); otherwise the LDS-DMA ring
  __shared__ __attribute__((aligned(16))) char smem[is_x3<T>      ? 2 * 3 * 384 * 64
                                                    : Cfg<T>::PM ? PM_STAGES * PM_STAGE_BYTES + 2 * PM_SCALES * 4
                                                                 : DW32_STAGES * DW32_STAGE_BYTES + 1024];
  // 1-D grid in job order (heaviest first: the light jobs fill the last round); jobs own consecutive workgroup ranges
  // (wg_base), k_tiles * S each, split-major inside a job so the k-tiles sharing a dZ slab run together. (An XCD-aware
  // order -- the tiles of jobs that share a section as consecutive blocks of one XCD -- measured slower: bf16 dW 1.175
  // -> 1.21 ms, fp32 8.23 -> 9.10 ms; per-k-tile split counts balancing the grid measured slower too, round 3: the bf16
  // dW streams its operands at the HBM rate, so the lighter last round is not idle time.)
  const int b = blockIdx.x;
  int ji = 0;
  while (ji + 1 < jobs.n && jobs.j[ji + 1].wg_base <= b) ++ji;
  const DwJob& J = jobs.j[ji];
  const int local = b - J.wg_base;
  const int S = jobs.S;
  int s = local / J.k_tiles, kt = local % J.k_tiles;
  if (is_x3<T> && (S & 7) == 0 && (J.wg_base & 7) == 0 && J.k_tiles > 1) {
    // x3: the k-tiles of one split 8 blocks apart: blocks go to the 8 XCDs round robin, so every k-tile that stages
    // the split's dZ rows runs on the same XCD (one L2) at about the same time (block b's XCD is b % 8). x3 dW 5.69 ->
    // 5.55 ms; fp32 measured 7.62 -> 7.68 ms although its HBM reads drop 24.2 -> 21.5 GB per fine launch, so fp32 keeps
    // the plain order
    const int grp = local / (8 * J.k_tiles), r = local % (8 * J.k_tiles);
    kt = r >> 3;
    s = grp * 8 + (r & 7);
  }
  constexpr int BKMAX = dw_bkmax(prec_of<T>);
  const int k0 = kt * BKMAX;
  const int bk = kt < J.k_full ? BKMAX : J.bk_tail;
  const int64_t se = jobs.slab_stride;
  if constexpr (Cfg<T>::PM && S16) {
    // YANERF_PREC_BF16S: every operand bf16, 32-point stages, the bf16 MFMA (the dU rows' 64-row tiles as in the fp8 mode)
    constexpr int SP = 32;
    if (J.bn == 256) {
      if (bk == 256) run_pm<256, 256, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
      else if (bk == 128) run_pm<256, 128, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
      else run_pm<256, 64, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
    } else if (J.bn == 128) {
      if (bk == 256) run_pm<128, 256, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
      else if (bk == 128) run_pm<128, 128, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
      else run_pm<128, 64, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
    } else {
      if (bk == 256) run_pm<64, 256, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
      else run_pm<64, 128, false, false, SP>(J, k0, s, S, Npad, slab, se, smem);
    }
  } else if constexpr (Cfg<T>::PM) {
    // the tile's X format: fp8 if its columns come from an fp8 section (a k-tile never mixes formats: host check)
    const bool x8 = (k0 < J.x0p) ? J.x0_u8 : J.x1_u8;
    // and its A format: the 128 / 256-row tiles are fp8 gradient sections, a 64-row tile is a narrow fp8 gradient
    // section or the bf16 dU rows (host check in launch_bwd)
    auto run = [&](auto xc) {
      constexpr bool X8 = decltype(xc)::value;
      if (J.bn == 256) {
        if (bk == 256) run_pm<256, 256, X8, true>(J, k0, s, S, Npad, slab, se, smem);
        else if (bk == 128) run_pm<256, 128, X8, true>(J, k0, s, S, Npad, slab, se, smem);
        else run_pm<256, 64, X8, true>(J, k0, s, S, Npad, slab, se, smem);
      } else if (J.bn == 128) {
        if (bk == 256) run_pm<128, 256, X8, true>(J, k0, s, S, Npad, slab, se, smem);
        else if (bk == 128) run_pm<128, 128, X8, true>(J, k0, s, S, Npad, slab, se, smem);
        else run_pm<128, 64, X8, true>(J, k0, s, S, Npad, slab, se, smem);
      } else if (J.a_u8) {
        if (bk == 256) run_pm<64, 256, X8, true>(J, k0, s, S, Npad, slab, se, smem);
        else run_pm<64, 128, X8, true>(J, k0, s, S, Npad, slab, se, smem);
      } else {
        if (bk == 256) run_pm<64, 256, X8, false>(J, k0, s, S, Npad, slab, se, smem);
        else run_pm<64, 128, X8, false>(J, k0, s, S, Npad, slab, se, smem);
      }
    };
    if (x8) run(std::integral_constant<bool, true>{});
    else run(std::integral_constant<bool, false>{});
  } else if constexpr (is_x3<T>) {
    if (J.bn == 256) {
      if (bk == 128) dw_tile_x3<256, 128>(J, k0, s, S, Npad, slab, se, smem);
      else dw_tile_x3<256, 64>(J, k0, s, S, Npad, slab, se, smem);
    } else if (J.bn == 128) {
      if (bk == 128) dw_tile_x3<128, 128>(J, k0, s, S, Npad, slab, se, smem);
      else dw_tile_x3<128, 64>(J, k0, s, S, Npad, slab, se, smem);
    } else {
      dw_tile_x3<64, 128>(J, k0, s, S, Npad, slab, se, smem);
    }
  } else {
    // (fp32 tiles are at most dw_bkmax = 128 wide: no 256-column instantiations, whose 128 accumulators per wave would
    // set the whole kernel's VGPR count)
    static_assert(BKMAX == 128, "fp32 dW tiles");
    if (J.bn == 256) {
      if (bk == 128 && J.ext == 1) dw_tile<256, 128, 1>(J, k0, s, S, Npad, slab, se, smem);
      else if (bk == 128) dw_tile<256, 128>(J, k0, s, S, Npad, slab, se, smem);
      else dw_tile<256, 64>(J, k0, s, S, Npad, slab, se, smem);
    } else if (J.bn == 128) {
      if (bk == 128 && J.ext == 2 && k0 == 0) dw_tile<128, 128, 2>(J, k0, s, S, Npad, slab, se, smem);
      else if (bk == 128) dw_tile<128, 128>(J, k0, s, S, Npad, slab, se, smem);
      else dw_tile<128, 64>(J, k0, s, S, Npad, slab, se, smem);
    } else {
      dw_tile<64, 128>(J, k0, s, S, Npad, slab, se, smem);
    }
  }
}

// dirPE of ray r, column k: kind 0 = fp32 feature-major saved rows (ld floats apart), 1 = bf16 point-major [Npad][KDIR]
__device__ __forceinline__ float dirpe_at(const void* dpe, int kind, int64_t ld, int64_t p, int k) {
  if (kind == 0) return ((const float*)dpe)[(int64_t)k * ld + p];
  return bf2f(((const bf16_t*)dpe)[p * KDIR + k]);
}
// One block per DIRB rays: the rays' dirPE rows and dZc sums staged in LDS, then thread (c, k-half) accumulates its
// 16 products over the block's rays in ray order. Point indices fit 32 bits (the host checks).
__global__ void __launch_bounds__(256) dirpe_dw_block_kernel(const float* __restrict__ part, int R, int P, int CH,
                                                             const void* __restrict__ dpe, int kind, int64_t ld,
                                                             int kd, float* __restrict__ blockp) {
  __shared__ float Dl[DIRB][KDIR + 1];
  __shared__ float Sl[DIRB][HC];
  const int tid = threadIdx.x, r0 = blockIdx.x * DIRB;
#pragma unroll 8
  for (int i = tid; i < DIRB * KDIR; i += 256) {
    const int r = i % DIRB, k = i / DIRB;
    Dl[r][k] = (r0 + r < R && k < kd) ? dirpe_at(dpe, kind, ld, (int64_t)(r0 + r) * P, k) : 0.f;
  }
  {
    const int c = tid % HC;
#pragma unroll
    for (int r = tid / HC; r < DIRB; r += 256 / HC) {
      const int rr = r0 + r;
      float sr = 0.f;
      if (rr < R) {
        const unsigned pa = (unsigned)rr * (unsigned)P, u0 = pa / CH, u1 = (pa + P - 1) / CH;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // predicated, so a ray's (<= 4 for P <= 3 CH) partials load together
          const unsigned u = u0 + j;
          v[j] = u <= u1 ? part[((int64_t)u * 2 + (rr - u * CH / P)) * HC + c] : 0.f;
        }
        sr = ((v[0] + v[1]) + v[2]) + v[3];
        for (unsigned u = u0 + 4; u <= u1; ++u) sr += part[((int64_t)u * 2 + (rr - u * CH / P)) * HC + c];
      }
      Sl[r][c] = sr;
    }
  }
  __syncthreads();
  const int c = tid % HC, k0 = (tid / HC) * (KDIR / 2);
  float acc[KDIR / 2];
#pragma unroll
  for (int k = 0; k < KDIR / 2; ++k) acc[k] = 0.f;
  for (int r = 0; r < DIRB; ++r) {
    const float sv = Sl[r][c];
#pragma unroll
    for (int k = 0; k < KDIR / 2; ++k) acc[k] += sv * Dl[r][k0 + k];
  }
  float* out = blockp + ((int64_t)blockIdx.x * HC + c) * KDIR + k0;
#pragma unroll
  for (int k = 0; k < KDIR / 2; k += 4) *(f4*)(out + k) = f4{acc[k], acc[k + 1], acc[k + 2], acc[k + 3]};
}
__global__ void __launch_bounds__(256) dirpe_dw_final_kernel(const float* __restrict__ blockp, int nblk, int kd,
                                                             float* __restrict__ W, int w_ld, int col0) {
  __shared__ float red[8][KDIR];
  const int c = blockIdx.x, k = threadIdx.x % KDIR, g = threadIdx.x / KDIR;
  float s = 0.f;
#pragma unroll 8
  for (int b = g; b < nblk; b += 8) s += blockp[((int64_t)b * HC + c) * KDIR + k];
  red[g][k] = s;
  __syncthreads();
  if (g == 0 && k < kd) {
    float t = red[0][k];
#pragma unroll
    for (int i = 1; i < 8; ++i) t += red[i][k];
    W[(int64_t)c * w_ld + col0 + k] = t;
  }
}

// Sums the S split slabs in split order (deterministic): a thread owns 4 consecutive slab elements and reads them as
// one 16-byte load per split, 8 splits' loads in flight before their adds (the slab stride is padded to a multiple of
// 4 elements, dw_slab_pad, so past-the-end elements of the last group read in-bounds padding); the sum order per
// element is s = 0, 1, ..., S - 1.
__global__ void dw_reduce_kernel(DwJobs jobs, const float* __restrict__ slab) {
  const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e0 >= jobs.slab_elems) return;
  const int64_t stride = jobs.slab_stride;
  int jix[4];
  int ji = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t e = e0 + i;
    jix[i] = -1;
    if (e >= jobs.slab_elems) continue;
    while (ji + 1 < jobs.n && jobs.j[ji + 1].slab_off <= e) ++ji;
    jix[i] = ji;
  }
  const int S = jobs.S;
  f4 sum = f4{0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *(const f4*)(slab + (int64_t)(s + u) * stride + e0);
#pragma unroll
    for (int u = 0; u < 8; ++u) sum += v[u];
  }
  for (; s < S; ++s) sum += *(const f4*)(slab + (int64_t)s * stride + e0);
  const float vals[4] = {sum.x, sum.y, sum.z, sum.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (jix[i] < 0) break;
    const DwJob& J = jobs.j[jix[i]];
    const int64_t local = e0 + i - J.slab_off;
    const int kv = J.ktot + 1;
    const int n = (int)(local / kv), k = (int)(local % kv);
    if (k < J.ktot) J.W[(int64_t)n * J.w_ld + k] = vals[i];
    else J.b[n] = vals[i];
  }
}

// ============================================================================================ host helpers
static int num_params(const yanerf_mlp_desc* d) { return 2 * d->n_layers + 8; }
// element count of parameter i in the reference's state_dict order (the shapes build_pack_jobs reads)
static int64_t param_numel(const MlpLayout& L, int i) {
  if (i < 2 * L.L) {
    const int l = i / 2, nout = (l + 1 < L.L) ? 256 : L.hid;
    const bool sk = (L.skip >> l) & 1u;
    const int din = (l == 0) ? L.xyz_dim : (sk ? 256 + L.xyz_dim : 256);
    return (i % 2 == 0) ? (int64_t)nout * din : nout;
  }
  switch (i - 2 * L.L) {
    case 0: return (int64_t)L.hid * L.hid;                 // intermediate_linear.weight
    case 1: return L.hid;                                   // intermediate_linear.bias
    case 2: return L.hid;                                   // density_layer.weight [1][hid]
    case 3: return 1;                                       // density_layer.bias
    case 4: return (int64_t)L.hdir * (L.hid + L.dir_dim);   // color_layer.0.weight
    case 5: return L.hdir;                                  // color_layer.0.bias
    case 6: return (int64_t)L.cdim * L.hdir;                // color_layer.2.weight
    default: return L.cdim;                                 // color_layer.2.bias
  }
}

// appends one model's jobs to J (which may already hold another model's); nonzero when they do not fit one launch
static int build_pack_jobs(const yanerf_mlp_desc* d, const MlpLayout& L, int precision, const float* const* prm,
                           void* packed, PackJobs& J) {
  (void)d;
  char* tsec = (char*)packed;
  float* fsec = (float*)(tsec + L.f_base);
  const int64_t tsize = precision == YANERF_PREC_F32 ? 4 : 2;
  int fail = 0;
  auto add = [&](const float* src, int src_rows, int src_ld, int64_t dst_off, int rows, int cols, int seg0,
                 int seg1_start, int seg1_len, int transpose, int is_f32) {
    if (J.n >= kMaxPackJobs || (int64_t)J.total + (int64_t)rows * cols > INT32_MAX) {
      fail = 1;
      return;
    }
    PackJob& j = J.j[J.n++];
    j.src = src;
    j.dst = is_f32 ? (void*)(fsec + dst_off) : (void*)(tsec + dst_off * tsize);
    j.elem_base = J.total;
    j.t_plane = (int32_t)L.t_plane;
    j.src_rows = (int16_t)src_rows; j.src_ld = (int16_t)src_ld; j.rows = (int16_t)rows; j.cols = (int16_t)cols;
    j.seg0 = (int16_t)seg0; j.seg1_start = (int16_t)seg1_start; j.seg1_len = (int16_t)seg1_len;
    j.transpose = (uint8_t)transpose; j.is_f32 = (uint8_t)is_f32;
    J.total += rows * cols;  // cols % 4 == 0 for every job (pack_kernel's 4-column groups)
  };
  const int nl = L.L;
  for (int l = 0; l < nl; ++l) {
    const float* W = prm[2 * l];
    const float* b = prm[2 * l + 1];
    const int nout = (l + 1 < nl) ? 256 : L.hid;
    const bool sk = (L.skip >> l) & 1u;
    const int src_ld = (l == 0) ? L.xyz_dim : (sk ? 256 + L.xyz_dim : 256);
    if (l == 0) add(W, nout, src_ld, L.w_off[0], 256, KPE, L.xyz_dim, 0, 0, 0, 0);
    else if (sk) add(W, nout, src_ld, L.w_off[l], 256, 320, 256, 256, L.xyz_dim, 0, 0);
    else add(W, nout, src_ld, L.w_off[l], 256, 256, 256, 0, 0, 0, 0);
    if (l >= 1) add(W, nout, src_ld, L.wt_off[l], 256, 256, 256, 0, 0, 1, 0);
    add(b, 1, nout, L.b_off[l], 1, 256, nout, 0, 0, 0, 1);
  }
  const float** h = (const float**)prm + 2 * nl;
  // intermediate_linear [hid][hid], density [1][hid], color0 [hd][hid + dir], color2 [cd][hd]
  add(h[0], L.hid, L.hid, L.wint_off, 256, 256, L.hid, 0, 0, 0, 0);
  add(h[0], L.hid, L.hid, L.wintT_off, 256, 256, L.hid, 0, 0, 1, 0);
  add(h[1], 1, L.hid, L.bint_off, 1, 256, L.hid, 0, 0, 0, 1);
  add(h[2], 1, L.hid, L.wd_off, 1, 256, L.hid, 0, 0, 0, 1);
  add(h[2], 1, L.hid, L.wdh_off, 16, 256, L.hid, 0, 0, 0, 0);
  add(h[3], 1, 1, L.bd_off, 1, 4, 1, 0, 0, 0, 1);
  add(h[4], L.hdir, L.hid + L.dir_dim, L.wc_off, HC, KC, L.hid, 256, L.dir_dim, 0, 0);
  add(h[4], L.hdir, L.hid + L.dir_dim, L.wcT_off, 256, HC, L.hid, 0, 0, 1, 0);
  add(h[5], 1, L.hdir, L.bc_off, 1, HC, L.hdir, 0, 0, 0, 1);
  add(h[6], L.cdim, L.hdir, L.wo_off, CMAX, HC, L.hdir, 0, 0, 0, 1);
  add(h[6], L.cdim, L.hdir, L.woh_off, 16, HC, L.hdir, 0, 0, 0, 0);
  add(h[7], 1, L.cdim, L.bo_off, 1, CMAX, L.cdim, 0, 0, 0, 1);
  return fail;
}

// point splits per dW tile. fp32 / x3 (at most 64): enough workgroups that the light jobs dispatched last fill the
// tail of the heavy ones (their grids are whole rounds of the 256 CUs: fp32 20 tiles x 64, x3 24 x 64).
// bf16 (point-major, one 132 KB-LDS workgroup per CU, bound by its operand stream): whole rounds of one workgroup per
// CU -- floor(256 / tiles) splits per round, as few rounds as the fp8 gradient scales allow (one split's scales must
// fit the tile's PM_SCALES LDS slots). Lego fine pass (14 tiles): 18 splits = one round of 252 workgroups, dW 0.88-0.89
// -> 0.79-0.81 ms and reduce 0.021 -> 0.016 ms against the former 32 splits (448 workgroups, 1.75 rounds); 36 (two
// rounds) 0.84-0.86, 16 0.82-0.83, 24 / 28 0.90-0.98 (profiles/r4_ab_bf16_dw_splits.jsonl)
constexpr int DW_SMAX = 64;
constexpr int DW_CUS = 256;  // MI355X compute units
static int dw_splits(int total_tiles, int64_t n_stages, bool pm, bool s16 = false) {
  int64_t S;
  if (pm && s16) {  // no fp8 scales to fit: one round of one workgroup per CU
    S = DW_CUS / total_tiles > 0 ? DW_CUS / total_tiles : 1;
    if (S > n_stages) S = n_stages;
  } else if (pm) {
    const int64_t cap = (int64_t)(Cfg<bf16_t>::M / PM_SPTS) * (PM_SCALES - 2);  // stages per split whose scales fit
    const int64_t need = (n_stages + cap - 1) / cap;
    const int64_t per_round = DW_CUS / total_tiles > 0 ? DW_CUS / total_tiles : 1;
    S = per_round * (((need > 1 ? need : 1) + per_round - 1) / per_round);
    if (S > n_stages) S = n_stages;  // (>= need)
  } else {
    S = (DW_SMAX * 64 + total_tiles - 1) / total_tiles;
    if (S > n_stages) S = n_stages;
    if (S > DW_SMAX) S = DW_SMAX;
  }
  if (S < 1) S = 1;
  return (int)S;
}

static int dw_bn(int a_rows) { return a_rows > 128 ? 256 : (a_rows > 64 ? 128 : 64); }
// column tiling of one dW job: full dw_bkmax tiles, then one tail tile rounded up to 64 / 128 / 256 (>= 128 when
// BN = 64, whose 8 waves need 16 columns each)
static void dw_ktiles(int ktot, int bn, int prec, int* k_full, int* bk_tail, int* k_tiles) {
  const int bkmax = dw_bkmax(prec);
  *k_full = ktot / bkmax;
  const int rem = ktot - *k_full * bkmax;
  int bt = rem <= 64 ? 64 : (rem <= 128 ? 128 : 256);
  if (bn == 64 && bt < 128) bt = 128;
  *bk_tail = bt;
  *k_tiles = *k_full + (rem > 0 ? 1 : 0);
}

// enumerate the dW jobs (shared by the size query and the launch): A = the gradient rows / section (first row,
// rows, section width, first column), X0 / X1 = the layer-input rows / sections (first row, rows, section width)
struct DwSpec {
  int64_t arow;
  int a_rows, a_w, a_col;
  int64_t x0;
  int x0_rows, x0_w;
  int64_t x1;
  int x1_rows, x1_w;
  int gi;
};
template <typename F>
static void for_each_dw_job(const MlpLayout& L, bool pm, F&& f, bool dir_by_ray = false) {
  const SavedRows SR = saved_rows(L.L);
  const GradRows GR = grad_rows(L.L, pm);
  for (int l = 0; l < L.L; ++l) {
    const int nout = (l + 1 < L.L) ? 256 : L.hid;
    const bool sk = (L.skip >> l) & 1u;
    if (l == 0) f(DwSpec{GR.dz0, nout, 256, 0, SR.pe, L.xyz_dim, KPE, -1, 0, 0, 2 * l});
    else if (sk)
      f(DwSpec{GR.dz0 + 256LL * l, nout, 256, 0, SR.h0 + 256LL * (l - 1), 256, 256, SR.pe, L.xyz_dim, KPE, 2 * l});
    else f(DwSpec{GR.dz0 + 256LL * l, nout, 256, 0, SR.h0 + 256LL * (l - 1), 256, 256, -1, 0, 0, 2 * l});
  }
  // heaviest jobs first: the grid is dispatched in job order, so the light ones fill the last round
  const int h = 2 * L.L;
  const int64_t hl = SR.h0 + 256LL * (L.L - 1);
  f(DwSpec{GR.dyx, L.hid, 256, 0, hl, L.hid, 256, -1, 0, 0, h + 0});                      // intermediate_linear
  if (dir_by_ray)  // the dirPE columns come from the per-ray reduction (dirpe_dw_*_kernel), not from a k-tile
    f(DwSpec{GR.dzc, L.hdir, HC, 0, SR.y, L.hid, 256, -1, 0, 0, h + 4});
  else f(DwSpec{GR.dzc, L.hdir, HC, 0, SR.y, L.hid, 256, SR.dpe, L.dir_dim, KDIR, h + 4});     // color_layer.0
  if (pm) f(DwSpec{GR.du, 1, 16, PM_DSIG, hl, L.hid, 256, -1, 0, 0, h + 2});             // density_layer
  else f(DwSpec{GR.dyx + 256, 1, 256, 0, hl, L.hid, 256, -1, 0, 0, h + 2});
  f(DwSpec{GR.du, L.cdim, 16, 0, SR.c, L.hdir, HC, -1, 0, 0, h + 6});                    // color_layer.2
}

// X0's padded width in a point-major tile: whole 16-byte chunks (8 bf16 / 16 fp8 columns)
// (a whole number of k-tiles when X1 has the other element format: a k-tile reads one format)
static int dw_x0p(const MlpLayout& L, bool pm, const DwSpec& sp) {
  if (!pm) return sp.x0_rows;
  int es = 2, es1 = 2;
  pm_sec_bytes(L.L, 128, sp.x0, &es, nullptr, L.s16);
  if (sp.x1 >= 0) pm_sec_bytes(L.L, 128, sp.x1, &es1, nullptr, L.s16);
  const int q = (sp.x1 >= 0 && es1 != es) ? dw_bkmax(YANERF_PREC_BF16) : (es == 1 ? 16 : 8);
  return (sp.x0_rows + q - 1) / q * q;
}

// a split's slab stride: whole 16-byte groups, so the reduce reads every split with aligned 16-byte loads
static int64_t dw_slab_pad(int64_t e) { return (e + 3) / 4 * 4; }
static void build_dw_jobs(const MlpLayout& L, int prec, const void* saved, void* gradbuf, int64_t Npad,
                          float* const* grads, DwJobs& D, bool dir_by_ray = false) {
  const size_t es = elem_size(prec);
  const bool pm = prec_pm(prec);
  const int64_t ld = pm ? Npad : row_ld(Npad, es);
  auto srow = [&](int64_t r) { return r < 0 ? nullptr : (const void*)((const char*)saved + r * ld * es); };
  // point-major (bf16): sections at byte offsets, some in fp8 (pm_save)
  auto psec = [&](int64_t r, int* u8, const float** scale) -> const void* {
    *u8 = 0;
    *scale = nullptr;
    if (r < 0) return nullptr;
    int b = 2;
    int64_t so = -1;
    const int64_t off = pm_sec_bytes(L.L, Npad, r, &b, &so, L.s16);
    *u8 = b == 1;
    if (so >= 0) *scale = (const float*)((const char*)saved + so);
    return (const void*)((const char*)saved + off);
  };
  auto grow = [&](int64_t r) { return (const void*)((const char*)gradbuf + r * ld * es); };
  int a_es = (int)es;  // point-major gradient section bytes per element (pm_grad)
  auto gsec = [&](int64_t r, const float** scale) -> const void* {
    int64_t so = -1;
    const int64_t off = pm_grad_sec(L.L, Npad, r, &a_es, &so, L.s16);
    *scale = so < 0 ? nullptr : (const float*)((const char*)gradbuf + so);
    return (const void*)((const char*)gradbuf + off);
  };
  D.n = 0;
  D.total_tiles = 0;
  D.slab_elems = 0;
  for_each_dw_job(L, pm, [&](const DwSpec& sp) {
    DwJob& j = D.j[D.n++];
    j.ext = 0;
    j.wg_base = 0;
    j.ext_slab_off = 0;
    j.ext_a = j.ext_x = nullptr;
    j.ext_rows = j.ext_ktot = 0;
    j.gi = sp.gi;
    j.A = grow(sp.arow); j.a_rows = sp.a_rows;
    j.x0_u8 = j.x1_u8 = 0;
    j.a_u8 = 0;
    j.a_scale = nullptr;
    j.x_scale = nullptr;
    a_es = (int)es;
    if (pm) {
      j.A = gsec(sp.arow, &j.a_scale);
      j.a_u8 = a_es == 1;
      const float* x1s = nullptr;  // (never scaled: the second inputs are the PE sections)
      int u0 = 0, u1 = 0;
      j.X0 = psec(sp.x0, &u0, &j.x_scale);
      j.X1 = psec(sp.x1, &u1, &x1s);
      j.x0_u8 = (int16_t)u0;
      j.x1_u8 = (int16_t)u1;
    } else {
      j.X0 = srow(sp.x0);
      j.X1 = srow(sp.x1);
    }
    j.x0_rows = sp.x0_rows; j.x1_rows = sp.x1_rows;
    j.ktot = sp.x0_rows + sp.x1_rows;
    // the colour layer without its dirPE columns still writes rows of hid + dir_dim weights
    j.w_ld = (dir_by_ray && sp.gi == 2 * L.L + 4) ? j.ktot + L.dir_dim : j.ktot;
    j.a_ld = sp.a_w; j.x0_ld = sp.x0_w; j.x1_ld = sp.x1_w;
    if (pm) j.A = (const char*)j.A + (int64_t)sp.a_col * a_es;
    j.a_chunks = (sp.a_w - sp.a_col) * a_es / 16;
    j.x0p = dw_x0p(L, pm, sp);
    j.ktot_v = j.x0p + sp.x1_rows;
    j.bn = dw_bn(sp.a_rows);
    int kf = 0, bt = 0, kt = 0;
    dw_ktiles(j.ktot_v, j.bn, prec, &kf, &bt, &kt);
    j.k_full = (int16_t)kf;
    j.bk_tail = (int16_t)bt;
    j.k_tiles = (int16_t)kt;
    D.total_tiles += j.k_tiles;
    j.slab_off = D.slab_elems;
    D.slab_elems += (int64_t)sp.a_rows * (j.ktot + 1);
    j.W = grads[sp.gi];
    j.b = grads[sp.gi + 1];
  }, dir_by_ray);
  D.slab_stride = dw_slab_pad(D.slab_elems);
  if (prec == YANERF_PREC_F32) {
    // the density row rides in the intermediate_linear tiles (dw_tile EXT) when its gradient row directly follows the
    // intermediate's 256 gradient rows (fp32 grad_rows: dY then dsigma) and both read the same H_{L-1} rows
    // and the colour-output rows (dU, at most 8) ride in the first k-tile of color_layer.0 (128 rows, 128-wide tiles),
    // which stages C's 128 rows for them beside its own operands
    DwJob *in = nullptr, *de = nullptr, *co = nullptr, *c2 = nullptr;
    for (int i = 0; i < D.n; ++i) {
      if (D.j[i].gi == 2 * L.L + 0) in = &D.j[i];
      if (D.j[i].gi == 2 * L.L + 2) de = &D.j[i];
      if (D.j[i].gi == 2 * L.L + 4) co = &D.j[i];
      if (D.j[i].gi == 2 * L.L + 6) c2 = &D.j[i];
    }
    bool changed = false;
    if (in && de && in->bn == 256 && in->a_rows == 256 && in->ktot == 256 && in->k_tiles == 2 && !in->X1 &&
        de->a_rows == 1 && de->X0 == in->X0 && de->ktot == in->ktot &&
        (const char*)de->A == (const char*)in->A + 256 * ld * (int64_t)es) {
      in->ext = 1;
      in->ext_slab_off = de->slab_off;
      in->ext_rows = 1;
      in->ext_ktot = de->ktot;
      de->k_full = de->k_tiles = 0;
      changed = true;
    }
    if (co && c2 && co->bn == 128 && co->k_tiles >= 1 && co->k_full >= 1 && c2->a_rows >= 1 && c2->a_rows <= 4 &&
        c2->ktot == 128 && !c2->X1) {
      co->ext = 2;
      co->ext_slab_off = c2->slab_off;
      co->ext_a = c2->A;
      co->ext_x = c2->X0;
      co->ext_rows = c2->a_rows;
      co->ext_ktot = c2->ktot;
      c2->k_full = c2->k_tiles = 0;
      changed = true;
    }
    if (changed) {
      D.total_tiles = 0;
      for (int i = 0; i < D.n; ++i) D.total_tiles += D.j[i].k_tiles;
    }
  }
}

// every job's first workgroup (k_tiles * S workgroups per job, in job order) and the launch's workgroup count
static void dw_plan(DwJobs& D, int S) {
  D.S = S;
  int wg = 0;
  for (int i = 0; i < D.n; ++i) {
    D.j[i].wg_base = wg;
    wg += D.j[i].k_tiles * S;
  }
  D.total_wg = wg;
}

static int64_t dw_slab_elems_for(const MlpLayout& L, int prec, int* total_tiles) {
  int64_t e = 0;
  int tiles = 0;
  const bool pm = prec_pm(prec);
  for_each_dw_job(L, pm, [&](const DwSpec& sp) {
    const int ktot = sp.x0_rows + sp.x1_rows;
    const int ktot_v = dw_x0p(L, pm, sp) + sp.x1_rows;
    e += (int64_t)sp.a_rows * (ktot + 1);
    int kf, bt, kt;
    dw_ktiles(ktot_v, dw_bn(sp.a_rows), prec, &kf, &bt, &kt);
    tiles += kt;
  });
  if (total_tiles) *total_tiles = tiles;
  return dw_slab_pad(e);
}

// the training (saved != null) and inference instantiations of the forward
template <typename T>
static int launch_fwd(const MlpLayout& L, int prec, const void* packed, const float* o, const float* d, const float* t,
                      int64_t R, int64_t P, float* sigma, float* rgb, void* saved, hipStream_t st) {
  typedef typename Cfg<T>::st_t ST;
  const int64_t N = R * P;
  const int64_t Npad = npad_of(prec, N);
  const typename Cfg<T>::w_t* Wt = (const typename Cfg<T>::w_t*)packed;
  const float* Wf = (const float*)((const char*)packed + L.f_base);
  dim3 grid((unsigned)(Npad / Cfg<T>::M)), block(Cfg<T>::WAVES * 64);
  if (saved) {
    uint64_t* masks = (uint64_t*)((char*)saved + saved_t_bytes(L.L, Npad, sizeof(ST), Cfg<T>::PM, L.s16));
    if constexpr (Cfg<T>::PM) {
      if (L.s16) {
        hipLaunchKernelGGL((mlp_fwd_kernel<T, true, true>), grid, block, 0, st, L, Wt, Wf, o, d, t, R, P, sigma, rgb,
                           (ST*)saved, masks, Npad);
        YN_LAUNCH_CHECK("mlp_forward");
        return 0;
      }
    }
    hipLaunchKernelGGL((mlp_fwd_kernel<T, true>), grid, block, 0, st, L, Wt, Wf, o, d, t, R, P, sigma, rgb, (ST*)saved,
                       masks, Npad);
  } else
    hipLaunchKernelGGL((mlp_fwd_kernel<T, false>), grid, block, 0, st, L, Wt, Wf, o, d, t, R, P, sigma, rgb, nullptr,
                       nullptr, Npad);
  YN_LAUNCH_CHECK("mlp_forward");
  return 0;
}

template <typename T>
static int launch_bwd(const MlpLayout& L, int prec, const void* packed, const void* saved, const float* rgb,
                      const float* gs, const float* gr, int64_t R, int64_t P, float* const* grads, void* ws,
                      hipStream_t st, int phase) {
  typedef typename Cfg<T>::st_t ST;
  const int64_t N = R * P;
  const int64_t Npad = npad_of(prec, N);
  const typename Cfg<T>::w_t* Wt = (const typename Cfg<T>::w_t*)packed;
  const float* Wf = (const float*)((const char*)packed + L.f_base);
  ST* gradbuf = (ST*)ws;
  const int64_t grad_bytes = grad_t_bytes(L.L, Npad, sizeof(ST), Cfg<T>::PM, L.s16);
  float* slab = (float*)((char*)ws + grad_bytes);
  // the point splits and slab size are those of the full job set (yanerf_mlp_bwd_workspace_bytes)
  int tiles_all = 0;
  const int64_t slab_all = dw_slab_elems_for(L, prec, &tiles_all);
  const int S = dw_splits(tiles_all, Npad / dw_stage_pts(prec), Cfg<T>::PM, L.s16);
  // the dirPE weight gradient by rays: per-ray dZc partials after the slabs, then the block partials
  constexpr int CH = dzc_chunk<T>();
  // (fp32 only, where it measured -0.21 ms of 15.2 ms per Lego fine backward; bf16 and fp32x3 gained less in dW than
  // the per-ray sums cost in dX)
  const bool dir_by_ray = std::is_same<T, float>::value && P >= CH && L.dir_dim <= KDIR && L.hdir <= HC &&
                          Npad < (1ll << 31);
  float* dzc_part = (float*)((char*)slab + (int64_t)S * slab_all * 4);
  float* blockp = dzc_part + 2 * (Npad / CH) * HC;
  const uint64_t* masks =
      (const uint64_t*)((const char*)saved + saved_t_bytes(L.L, Npad, sizeof(ST), Cfg<T>::PM, L.s16));
  if (phase & 1) {
    bool s16 = false;
    if constexpr (Cfg<T>::PM) {
      if (L.s16) {
        hipLaunchKernelGGL((mlp_bwd_dx_kernel<T, true>), dim3((unsigned)(Npad / Cfg<T>::M)), dim3(Cfg<T>::DXWAVES * 64),
                           0, st, L, Wt, Wf, masks, rgb, gs, gr, N, Npad, gradbuf, P, nullptr);
        s16 = true;
      }
    }
    if (!s16)
    hipLaunchKernelGGL(mlp_bwd_dx_kernel<T>, dim3((unsigned)(Npad / Cfg<T>::M)), dim3(Cfg<T>::DXWAVES * 64), 0, st, L,
                       Wt, Wf, masks, rgb, gs, gr, N, Npad, gradbuf, P, dir_by_ray ? dzc_part : nullptr);
    YN_LAUNCH_CHECK("mlp_backward_dx");
  }
  // phase 2 = dW + reduce; 4 = the dW kernel alone, 8 = the slab reduce alone (4 then 8 == 2: for timing probes)
  const bool dw = (phase & 2) || (phase & 4), red = (phase & 2) || (phase & 8);
  if (!dw && !red) return 0;
  DwJobs D;
  build_dw_jobs(L, prec, saved, gradbuf, Npad, grads, D, dir_by_ray);
  dw_plan(D, S);
  for (int i = 0; i < D.n; ++i)  // a point-major k-tile reads one X format: mixed sections must split at a tile edge
    YN_CHECK(!D.j[i].X1 || D.j[i].x0_u8 == D.j[i].x1_u8 || D.j[i].x0p % dw_bkmax(prec) == 0,
             "mlp_backward: dW job %d mixes fp8 and bf16 columns inside a tile", i);
  if (Cfg<T>::PM)  // every k-tile's images fit the stage buffer (run_pm)
    for (int i = 0; i < D.n; ++i)
      for (int kt = 0; kt < D.j[i].k_tiles; ++kt) {
        const DwJob& j = D.j[i];
        const int k0 = kt * dw_bkmax(prec), bk = kt < j.k_full ? dw_bkmax(prec) : j.bk_tail;
        const bool x8 = (k0 < j.x0p) ? j.x0_u8 : j.x1_u8;
        YN_CHECK(pm_tile_bytes(j.bn, bk, x8, j.a_u8, L.s16 ? 32 : PM_SPTS) <= PM_STAGE_BYTES,
                 "mlp_backward: dW job %d k-tile %d needs %d B per stage (> %d)", i, kt,
                 pm_tile_bytes(j.bn, bk, x8, j.a_u8, L.s16 ? 32 : PM_SPTS), PM_STAGE_BYTES);
      }
  for (int i = 0; i < D.n; ++i)  // the dW tile's A format follows its row tile (dw_tile_pm's A8)
    YN_CHECK(!Cfg<T>::PM || D.j[i].bn == 64 || D.j[i].a_u8 != L.s16,
             "mlp_backward: dW job %d: gradient format %d does not match its %d-row tile", i, D.j[i].a_u8, D.j[i].bn);
  YN_CHECK(D.slab_stride <= dw_slab_pad(slab_all), "mlp_backward: dW slab larger than its workspace");
  if (dw) {
    bool s16 = false;
    if constexpr (Cfg<T>::PM) {
      if (L.s16) {
        hipLaunchKernelGGL((mlp_dw_kernel<T, true>), dim3((unsigned)D.total_wg), dim3(DW_THREADS), 0, st, D, Npad, slab);
        s16 = true;
      }
    }
    if (!s16) hipLaunchKernelGGL(mlp_dw_kernel<T>, dim3((unsigned)D.total_wg), dim3(DW_THREADS), 0, st, D, Npad, slab);
    YN_LAUNCH_CHECK("mlp_backward_dw");
  }
  if (red) {
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((D.slab_elems + 1023) / 1024)), dim3(256), 0, st, D, slab);
    YN_LAUNCH_CHECK("mlp_backward_reduce");
    if (dir_by_ray) {
      const int gi = 2 * L.L + 4;  // color_layer.0 weight [hdir][hid + dir_dim]
      const SavedRows SR = saved_rows(L.L);
      const PmSave PS = pm_save(L.L, Npad, L.s16);
      const bool pm = Cfg<T>::PM;
      const void* dpe = pm ? (const void*)((const char*)saved + PS.dpe)
                           : (const void*)((const char*)saved + SR.dpe * row_ld(Npad, sizeof(ST)) * sizeof(ST));
      const int nblk = (int)((R + DIRB - 1) / DIRB);
      hipLaunchKernelGGL(dirpe_dw_block_kernel, dim3((unsigned)nblk), dim3(256), 0, st, dzc_part, (int)R, (int)P, CH, dpe,
                         pm ? 1 : 0, row_ld(Npad, sizeof(ST)), L.dir_dim, blockp);
      YN_LAUNCH_CHECK("mlp_backward_dirpe_block");
      hipLaunchKernelGGL(dirpe_dw_final_kernel, dim3((unsigned)L.hdir), dim3(256), 0, st, blockp, nblk, L.dir_dim,
                         grads[gi], L.hid + L.dir_dim, L.hid);
      YN_LAUNCH_CHECK("mlp_backward_dirpe_final");
    }
  }
  return 0;
}

}  // namespace yanerf

using namespace yanerf;

extern "C" {

int yanerf_mlp_num_params(const yanerf_mlp_desc* d) {
  if (check_desc(d)) return -1;
  return num_params(d);
}

int64_t yanerf_mlp_packed_bytes(const yanerf_mlp_desc* d, int precision) {
  if (check_desc(d)) return -1;
  return make_layout(d, precision).bytes;
}

static int launch_pack(const PackJobs& J, int precision, void* stream) {
  if (J.total == 0) return 0;
  dim3 grid((unsigned)((J.total / 4 + 255) / 256)), block(256);
  if (precision == YANERF_PREC_F32)
    hipLaunchKernelGGL(pack_kernel<float>, grid, block, 0, as_stream(stream), J);
  else if (prec_bf16(precision))
    hipLaunchKernelGGL(pack_kernel<bf16_t>, grid, block, 0, as_stream(stream), J);
  else
    hipLaunchKernelGGL(pack_kernel<x3_t>, grid, block, 0, as_stream(stream), J);
  YN_LAUNCH_CHECK("mlp_pack");
  return 0;
}

int yanerf_mlp_pack(const yanerf_mlp_desc* d, int precision, const float* const* params, void* packed, void* stream) {
  return yanerf_mlp_pack_multi(1, d, precision, &params, &packed, stream);
}

int yanerf_mlp_pack_multi(int n_models, const yanerf_mlp_desc* d, int precision, const float* const* const* params,
                          void* const* packed, void* stream) {
  YN_CHECK(n_models >= 1 && d && params && packed, "mlp_pack_multi: bad arguments");
  YN_CHECK(precision == YANERF_PREC_F32 || prec_bf16(precision) || precision == YANERF_PREC_F32X3,
           "mlp_pack: bad precision %d", precision);
  for (int m = 0; m < n_models; ++m) {
    if (check_desc(d + m)) return 1;
    YN_CHECK(params[m] && packed[m], "mlp_pack: null pointer (model %d)", m);
    for (int i = 0; i < num_params(d + m); ++i) YN_CHECK(params[m][i], "mlp_pack: parameter %d is null", i);
  }
  PackJobs J;
  J.n = 0;
  J.total = 0;
  for (int m = 0; m < n_models; ++m) {
    const MlpLayout L = make_layout(d + m, precision);
    const PackJobs before = J;
    if (build_pack_jobs(d + m, L, precision, params[m], packed[m], J)) {
      // this model's jobs do not fit beside the ones already collected: flush those, then retry it alone
      YN_CHECK(before.n > 0, "mlp_pack: one model's jobs exceed a launch");
      if (launch_pack(before, precision, stream)) return 1;
      J.n = 0;
      J.total = 0;
      YN_CHECK(!build_pack_jobs(d + m, L, precision, params[m], packed[m], J), "mlp_pack: jobs exceed a launch");
    }
  }
  return launch_pack(J, precision, stream);
}

int64_t yanerf_mlp_saved_bytes(const yanerf_mlp_desc* d, int precision, int64_t n_points) {
  if (check_desc(d)) return -1;
  const int64_t Npad = npad_of(precision, n_points);
  return saved_t_bytes(d->n_layers, Npad, elem_size(precision), prec_pm(precision), precision == YANERF_PREC_BF16S) +
         (d->n_layers * trunk_mask_words_prec(precision, Npad) + mask_words_per_slot(Npad)) * 8;
}

int64_t yanerf_mlp_bwd_workspace_bytes(const yanerf_mlp_desc* d, int precision, int64_t n_points) {
  if (check_desc(d)) return -1;
  MlpLayout L = make_layout(d, precision);
  const int64_t Npad = npad_of(precision, n_points);
  const int64_t grad_bytes =
      grad_t_bytes(d->n_layers, Npad, elem_size(precision), prec_pm(precision), precision == YANERF_PREC_BF16S);
  int tiles = 0;
  int64_t se = dw_slab_elems_for(L, precision, &tiles);
  int S = dw_splits(tiles, Npad / dw_stage_pts(precision), prec_pm(precision), precision == YANERF_PREC_BF16S);
  // + the per-ray dZc partials (two slots per dZc chunk) and the dirPE block partials (rays >= chunks when used)
  const int CH = precision == YANERF_PREC_F32 ? dzc_chunk<float>()
                 : prec_bf16(precision) ? dzc_chunk<bf16_t>() : dzc_chunk<x3_t>();
  const int64_t nblk = (Npad / CH + DIRB - 1) / DIRB + 1;
  return grad_bytes + (int64_t)S * se * 4 + (2 * (Npad / CH) * HC + nblk * HC * KDIR) * 4;
}

int yanerf_mlp_dw_plan(const yanerf_mlp_desc* d, int precision, int64_t n_points, int* tiles, int* splits,
                       int64_t* stage_points, int64_t* stages_min, int64_t* stages_max) {
  if (check_desc(d)) return 1;
  YN_CHECK(n_points >= 0, "mlp_dw_plan: bad n_points %lld", (long long)n_points);
  YN_CHECK(tiles && splits && stage_points && stages_min && stages_max, "mlp_dw_plan: null pointer");
  const MlpLayout L = make_layout(d, precision);
  const int64_t Npad = npad_of(precision, n_points);
  int t = 0;
  dw_slab_elems_for(L, precision, &t);
  const int64_t nst = Npad / dw_stage_pts(precision);
  const int S = dw_splits(t, nst, prec_pm(precision), precision == YANERF_PREC_BF16S);
  *tiles = t;
  *splits = S;
  *stage_points = dw_stage_pts(precision);
  *stages_min = nst / S;  // split s covers stages [nst s / S, nst (s + 1) / S) (dw tile kernels)
  *stages_max = (nst + S - 1) / S;
  return 0;
}

int yanerf_mlp_forward(const yanerf_mlp_desc* d, int precision, const void* packed, const float* origins,
                       const float* directions, const float* lengths, int64_t R, int64_t P, float* sigma_raw,
                       float* rgb, void* saved, void* stream) {
  if (check_desc(d)) return 1;
  YN_CHECK(R >= 0 && P >= 1, "mlp_forward: bad sizes R=%lld P=%lld", (long long)R, (long long)P);
  if (R == 0) return 0;  // an empty bundle: no outputs (its buffers may be NULL)
  YN_CHECK(packed && origins && directions && lengths && sigma_raw && rgb, "mlp_forward: null pointer");
  MlpLayout L = make_layout(d, precision);
  if (precision == YANERF_PREC_F32)
    return launch_fwd<float>(L, precision, packed, origins, directions, lengths, R, P, sigma_raw, rgb, saved,
                             as_stream(stream));
  if (prec_bf16(precision))
    return launch_fwd<bf16_t>(L, precision, packed, origins, directions, lengths, R, P, sigma_raw, rgb, saved,
                              as_stream(stream));
  if (precision == YANERF_PREC_F32X3)
    return launch_fwd<x3_t>(L, precision, packed, origins, directions, lengths, R, P, sigma_raw, rgb, saved,
                            as_stream(stream));
  YN_CHECK(false, "mlp_forward: bad precision %d", precision);
}

int yanerf_mlp_backward(const yanerf_mlp_desc* d, int precision, const void* packed, const void* saved,
                        const float* rgb, const float* g_sigma, const float* g_rgb, int64_t R, int64_t P,
                        float* const* grads, void* workspace, void* stream) {
  return yanerf_mlp_backward_phase(d, precision, packed, saved, rgb, g_sigma, g_rgb, R, P, grads, workspace, 3,
                                   stream);
}

int yanerf_mlp_backward_phase(const yanerf_mlp_desc* d, int precision, const void* packed, const void* saved,
                              const float* rgb, const float* g_sigma, const float* g_rgb, int64_t R, int64_t P,
                              float* const* grads, void* workspace, int phase, void* stream) {
  if (check_desc(d)) return 1;
  YN_CHECK(phase == 1 || phase == 2 || phase == 3 || phase == 4 || phase == 8, "mlp_backward: bad phase %d", phase);
  YN_CHECK(R >= 0 && P >= 1, "mlp_backward: bad sizes R=%lld P=%lld", (long long)R, (long long)P);
  YN_CHECK(grads, "mlp_backward: null pointer");
  for (int i = 0; i < num_params(d); ++i) YN_CHECK(grads[i], "mlp_backward: grad %d is null", i);
  if (R == 0) {
    // no points: every parameter gradient is an empty sum (torch's Linear backward over an empty batch gives zeros),
    // written by the phases that write gradients (2, 3, 8); the point buffers may be NULL
    if (phase == 2 || phase == 3 || phase == 8) {
      const MlpLayout L = make_layout(d, precision);
      for (int i = 0; i < num_params(d); ++i) {
        const hipError_t e = hipMemsetAsync(grads[i], 0, (size_t)param_numel(L, i) * sizeof(float), as_stream(stream));
        YN_CHECK(e == hipSuccess, "mlp_backward: zeroing grad %d failed: %s", i, hipGetErrorString(e));
      }
    }
    return 0;
  }
  YN_CHECK(packed && saved && rgb && g_sigma && g_rgb && workspace, "mlp_backward: null pointer");
  MlpLayout L = make_layout(d, precision);
  if (precision == YANERF_PREC_F32)
    return launch_bwd<float>(L, precision, packed, saved, rgb, g_sigma, g_rgb, R, P, grads, workspace,
                             as_stream(stream), phase);
  if (prec_bf16(precision))
    return launch_bwd<bf16_t>(L, precision, packed, saved, rgb, g_sigma, g_rgb, R, P, grads, workspace,
                              as_stream(stream), phase);
  if (precision == YANERF_PREC_F32X3)
    return launch_bwd<x3_t>(L, precision, packed, saved, rgb, g_sigma, g_rgb, R, P, grads, workspace,
                            as_stream(stream), phase);
  YN_CHECK(false, "mlp_backward: bad precision %d", precision);
}

}  // extern "C"
