/*
 * yanerf_hip.h — C ABI of libyanerf_hip.so, the MI355X (gfx950) volumetric-rendering hot path of
 * yet-another-nerf.
 *
 * The reference (xk-huang/yet-another-nerf @ v0) has no FFI: its hot path is three registered torch
 * modules (RaySampler, NeRFMLP, MultipassEmissionAbsorpsionRenderer). Each entry point below replaces
 * the aten-op sequence of one reference function, cited as path:line into the reference tree. The
 * host-side registry mirror (yet-another-nerf_amd/pipelines) binds these through ctypes
 * (yet-another-nerf_amd/_C.py); INTEGRATION.md shows the binding a maintainer adds to the reference.
 *
 * Conventions (every entry point):
 *   - Plain pointers to DEVICE memory, int64 sizes, and a hipStream_t passed as `void*` (NULL = the
 *     default stream). No torch types. Launches are stream-ordered, asynchronous and capture-safe:
 *     no allocation, no host synchronisation, no memcpy from pageable memory.
 *   - Return 0 on success; non-zero on a bad argument or launch failure, with a message available from
 *     yanerf_last_error() (thread-local).
 *   - Floating point tensors are fp32, row-major and contiguous with the reference's shapes, so torch
 *     tensors pass through without copies. Index tensors are int64.
 *   - Empty bundles (zero rays / points / elements) are valid, as empty tensors are in the reference: the call
 *     returns 0 before touching its per-ray buffers, which may then be NULL (torch gives an empty CUDA tensor a
 *     NULL data pointer). yanerf_mlp_backward with zero points writes all-zero parameter gradients (nn.Linear's
 *     gradient over an empty batch); yanerf_scatter_rays with zero rays writes the background image.
 *   - Randomness: a counter-based Philox4x32-10 stream keyed by (seed, offset); every random draw can
 *     instead be INJECTED by passing the uniforms/normals the reference consumed (test mode).
 */
#ifndef YANERF_HIP_H
#define YANERF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YANERF_PREC_F32 0  /* exact fp32: f32-input MFMA (v_mfma_f32_16x16x4_f32), fp32 activations */
#define YANERF_PREC_BF16 1 /* bf16 MFMA (v_mfma_f32_16x16x32_bf16), fp32 accumulate, bf16 activations */
/* fp32 split into three bf16 terms (x = x0 + x1 + x2 exactly): six bf16 MFMAs per product (all terms down to
   2^-24 relative), fp32 accumulate, fp32 saved activations / gradients. fp32-class accuracy at ~2.6x the fp32
   MFMA rate. */
#define YANERF_PREC_F32X3 2
/* bf16 with bf16 storage throughout: the BF16 mode's kernels (bf16 MFMA forward and input-gradient walk, fp32
   accumulate), but the saved activations and the gradient rows stay bf16 (no fp8 e4m3 sections) and the weight
   gradients run on the bf16 MFMA over 32-point stages. The reference's own reduced precision (torch.autocast bf16 keeps
   every Linear's operands bf16); YANERF_PREC_BF16 is the faster bf16 + fp8-storage mode. */
#define YANERF_PREC_BF16S 3

const char* yanerf_last_error(void);
int yanerf_version(void);
/* First 16 hex digits of the SHA-256 of the sources this library was compiled from (render.hip, mlp.hip,
   common.hpp, this header, the Makefile, in that order): the Python binding refuses a library whose id does not
   match the sources beside it (a stale prebuilt .so). Not a reference entry point. */
const char* yanerf_build_id(void);

/* ------------------------------------------------------------------------------------------------
 * Ray generation. Replaces _RaySampler.forward + _xy_to_ray_bundle + _jiggle_within_stratas
 * (yanerf/pipelines/ray_samplers/ray_sampler.py:149-246, 249-314, 361-386).
 *   poses [B][3][4] (pose[:, :3, :4]), focal [B].
 *   Pixel source, exactly one of:
 *     xy         [B][R][2] float pixel coordinates (x = column, y = row), or
 *     pixel_ids  [B][R] int64 flat ids into a grid of width grid_w (id = y * grid_w + x), or
 *     both NULL: sample R distinct pixels per image uniformly without replacement from the
 *                grid_w x grid_h grid (keyed Philox permutation; replaces torch.multinomial with
 *                uniform weights, ray_sampler.py:187-220); the chosen ids are written to ids_out.
 *   cfg_w/cfg_h: the CONFIGURED image size used for the principal point (reference quirk:
 *     ray_sampler.py:236-246, 302-303 use self._image_width/_height even under overrides).
 *   Depths: torch.linspace(near, far, P) (ray_sampler.py:285-291); jitter_mode 0 = none,
 *     1 = injected uniforms jitter_u [B][R][P], 2 = Philox(seed, offset).
 *   Outputs: origins [B][R][3], directions [B][R][3] (unnormalised, as the reference), lengths
 *     [B][R][P], xys [B][R][2]; ids_out [B][R] (may be NULL).
 *   bounds: NULL, or 2 device floats (near, far) that replace near/far -- LLFF's per-image bounds averaged on the
 *     device (ray_sampler.py:280-283 reads them with .item(), a host sync per step).
 *   rng_base: NULL, or 1 device u64 added to `offset` (a graph-captured step advances it on the device).
 * ---------------------------------------------------------------------------------------------- */
int yanerf_raygen(const float* poses, const float* focal, const float* xy, const int64_t* pixel_ids,
                  int64_t B, int64_t R, int64_t grid_w, int64_t grid_h, float cfg_w, float cfg_h,
                  float near, float far, int64_t P, int jitter_mode, const float* jitter_u,
                  uint64_t seed, uint64_t offset, float* origins, float* directions, float* lengths,
                  float* xys, int64_t* ids_out, const float* bounds, const uint64_t* rng_base, void* stream);

/* ------------------------------------------------------------------------------------------------
 * NeRF MLP (NeRFMLP.forward, yanerf/pipelines/models/nerf_mlp.py:117-177, incl. MLPWithInputSkips
 * :267-289, HarmonicEmbedding models/utils.py:90-103, LinearWithRepeat models/utils.py:207-211).
 * ---------------------------------------------------------------------------------------------- */
typedef struct yanerf_mlp_desc {
  int32_t n_layers;         /* trunk layers, 1..16 (nerf_mlp.py:16)                                   */
  uint32_t skip_mask;       /* bit i: layer i consumes cat(h, PE(x)) (input_skips, nerf_mlp.py:248-252) */
  int32_t n_freq_xyz;       /* n_harmonic_functions_xyz; 3*(2f+append) <= 64                           */
  int32_t n_freq_dir;       /* n_harmonic_functions_dir; 3*(2f+append) <= 32                           */
  int32_t append_xyz;       /* harmonic_functions_xyz_append_intput                                    */
  int32_t append_dir;       /* harmonic_functions_dir_append_intput                                    */
  int32_t hidden_xyz;       /* n_hidden_neurons_xyz (<= 256; the trunk itself is always 256 wide)      */
  int32_t hidden_dir;       /* n_hidden_neurons_dir (<= 128)                                           */
  int32_t color_dim;        /* <= 4                                                                    */
} yanerf_mlp_desc;

/* Number of reference parameter tensors (state_dict order of NeRFMLP: for each trunk layer weight, bias;
 * then intermediate_linear.{weight,bias}, density_layer.{weight,bias}, color_layer.0.{weight,bias},
 * color_layer.2.{weight,bias}). */
int yanerf_mlp_num_params(const yanerf_mlp_desc* d);
/* Bytes of the packed (kernel-layout) weight buffer for a precision. */
int64_t yanerf_mlp_packed_bytes(const yanerf_mlp_desc* d, int precision);
/* Pack reference-layout fp32 parameters (device pointers, in the order above) into the packed buffer:
 * padded row-major W [NOUT][Kpad] and transposed W^T for the backward, in fp32 or bf16, plus fp32 bias
 * and head sections. Call after every optimizer step (cost: one pass over 1.2 M parameters). */
int yanerf_mlp_pack(const yanerf_mlp_desc* d, int precision, const float* const* params, void* packed,
                    void* stream);
/* yanerf_mlp_pack for several MLPs of one precision in ONE launch (the trainer's coarse and fine models every step):
 * d[m], params[m], packed[m] as yanerf_mlp_pack's for model m. Same bytes as n_models separate calls. Not a reference
 * entry point: the parameters are the two NeRFMLPs' (nerf_mlp.py:14-83) that the reference's renderer runs in turn
 * (renderer.py:55-117). */
int yanerf_mlp_pack_multi(int n_models, const yanerf_mlp_desc* d, int precision, const float* const* const* params,
                          void* const* packed, void* stream);
/* Bytes of the per-call activation store kept from forward to backward for N points (0 for inference). */
int64_t yanerf_mlp_saved_bytes(const yanerf_mlp_desc* d, int precision, int64_t n_points);
/* Bytes of the backward workspace for N points (gradient rows + split-K partial slabs). */
int64_t yanerf_mlp_bwd_workspace_bytes(const yanerf_mlp_desc* d, int precision, int64_t n_points);
/* The split-K plan of the weight gradients for N points (host-only query, no device work): dW tiles per launch, point
 * splits per tile, points per stage, and the fewest / most stages one split reduces (split s covers stages
 * [n s / S, n (s + 1) / S)). Not a reference entry point: the reduction over points the reference's autograd does
 * inside each Linear backward (nerf_mlp.py:267-289) -- reported by the full-size parity tests so the regime they
 * exercise is visible. */
int yanerf_mlp_dw_plan(const yanerf_mlp_desc* d, int precision, int64_t n_points, int* tiles, int* splits,
                       int64_t* stage_points, int64_t* stages_min, int64_t* stages_max);

/* Forward over R rays x P samples (point p = r*P + j at x = o_r + t_rj * d_r, models/utils.py:244).
 *   origins/directions [R][3], lengths [R][P] -> sigma_raw [R][P] (density before ReLU), rgb [R][P][C].
 *   saved: NULL for inference, else yanerf_mlp_saved_bytes(...) of scratch kept for the backward. */
int yanerf_mlp_forward(const yanerf_mlp_desc* d, int precision, const void* packed, const float* origins,
                       const float* directions, const float* lengths, int64_t R, int64_t P, float* sigma_raw,
                       float* rgb, void* saved, void* stream);

/* Backward: given dL/dsigma_raw [R][P] and dL/drgb [R][P][C] (and rgb from the forward), write the
 * parameter gradients into `grads` (device pointers, same order/shapes as yanerf_mlp_pack's params;
 * OVERWRITTEN, not accumulated). No input gradient is produced: rays carry no grad in the reference. */
int yanerf_mlp_backward(const yanerf_mlp_desc* d, int precision, const void* packed, const void* saved,
                        const float* rgb, const float* g_sigma, const float* g_rgb, int64_t R, int64_t P,
                        float* const* grads, void* workspace, void* stream);

/* yanerf_mlp_backward in two halves, so that a caller can order the two passes' halves across streams:
 * phase 1 = the input-side walk (every layer's pre-activation gradient into `workspace`), phase 2 = the weight and
 * bias gradients from those (into `grads`), 3 = both (= yanerf_mlp_backward). Phase 2 must follow phase 1 of the
 * same call arguments, stream-ordered; `saved` and `workspace` must be unchanged in between. Phase 2 is itself two
 * launches, available separately for timing: 4 = the split-K weight-gradient kernel (partial slabs in `workspace`),
 * then 8 = the deterministic slab reduction into `grads` (4 followed by 8 == 2). */
int yanerf_mlp_backward_phase(const yanerf_mlp_desc* d, int precision, const void* packed, const void* saved,
                              const float* rgb, const float* g_sigma, const float* g_rgb, int64_t R, int64_t P,
                              float* const* grads, void* workspace, int phase, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Emission-absorption compositing (EmissionAbsorptionRaymarcher.forward,
 * yanerf/pipelines/renderers/multipass_emission_absorpsion_renderer.py:154-239).
 * ---------------------------------------------------------------------------------------------- */
typedef struct yanerf_raymarch_opts {
  int32_t capping;          /* 0 exponential (1-exp(-x)), 1 cap1 (min(x,1))           renderer.py:144-147 */
  int32_t weight_fn;        /* 0 product, 1 minimum                                   renderer.py:149-152 */
  int32_t blend_output;     /* features = alpha*F + (1-alpha)*bg  vs  F + (1-alpha)*bg renderer.py:226-234 */
  int32_t hard_background;  /*                                                        renderer.py:235-237 */
  int32_t density_relu;
  float background_opacity; /* last delta (1e10)                                      renderer.py:194-200 */
  float background_density_bias; /* added after ReLU                                  renderer.py:207    */
  float bg_default[4];      /* the raymarcher's _bg_color, used when bg == NULL (broadcast if bg_default_n==1) */
  int32_t bg_default_n;
  int32_t noise_mode;       /* 0 none, 1 injected normals noise[R][P], 2 Philox(seed, offset) normals  */
  float noise_std;          /* density_noise_std (renderer.py:204-205)                                */
  uint64_t seed, offset;
  const uint64_t* rng_base; /* NULL, or a device u64 added to offset (graph replay)                   */
} yanerf_raymarch_opts;

/* sigma_raw [R][P], rgb [R][P][C], lengths [R][P], directions [R][3], bg [R][C] or NULL,
 * noise [R][P] (N(0,1) draws, multiplied by noise_std inside) or NULL ->
 * features [R][C], depths [R], alpha [R], weights [R][P]. */
int yanerf_composite_forward(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                             const float* lengths, const float* directions, const float* bg,
                             const float* noise, int64_t R, int64_t P, int64_t C, float* features,
                             float* depths, float* alpha, float* weights, void* stream);
/* Reverse mode of the above: upstream g_features [R][C], g_depths [R] or NULL, g_alpha [R] or NULL ->
 * g_sigma [R][P], g_rgb [R][P][C]. Same inputs/options as the forward (noise regenerated identically). */
int yanerf_composite_backward(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                              const float* lengths, const float* directions, const float* bg,
                              const float* noise, const float* g_features, const float* g_depths,
                              const float* g_alpha, int64_t R, int64_t P, int64_t C, float* g_sigma,
                              float* g_rgb, void* stream);

/* The fused trainer's per-pass composite: yanerf_composite_forward, yanerf_rgb_loss (L = scale * sum((features -
 * gt)^2), gt gathered from image [B][H][W][C] at xys [R][2], R / B rays per image) and yanerf_composite_backward from
 * dL/dfeatures (no depth / alpha gradient) in one launch, bit-identical to those three calls; replaces
 * EmissionAbsorptionRaymarcher.forward + the rgb_mse term + their autograd backward on the training step
 * (renderer.py:146-278; pipelines/utils.py:189-196; nerf_pipeline.py:284-305). sq_err_per_ray and g_features
 * (the loss's intermediate values) may be NULL. */
int yanerf_composite_train(const yanerf_raymarch_opts* o, const float* sigma_raw, const float* rgb,
                           const float* lengths, const float* directions, const float* bg, const float* noise,
                           const float* image, const float* xys, int64_t B, int64_t R, int64_t P, int64_t C,
                           int64_t H, int64_t W, float scale, float* features, float* depths, float* alpha,
                           float* weights, float* sq_err_per_ray, float* g_features, float* g_sigma, float* g_rgb,
                           void* stream);

/* ------------------------------------------------------------------------------------------------
 * Importance sampling (sample_pdf_python, yanerf/pipelines/renderers/utils.py:83-158) and the
 * refiner (RayPointRefiner.forward, renderers/utils.py:48-69).
 * ---------------------------------------------------------------------------------------------- */
/* bins [R][nb+1], weights [R][nb] -> samples [R][N]. det != 0: u = linspace(0, 1, N); else u injected
 * ([R][N], may be unsorted) or Philox when u == NULL. */
int yanerf_sample_pdf(const float* bins, const float* weights, int64_t R, int64_t nb, int64_t N, int det,
                      const float* u, uint64_t seed, uint64_t offset, float* samples, void* stream);
/* lengths [R][P], ray_weights [R][P] -> sorted lengths_out [R][P + n_fine] (add_input != 0) or
 * [R][n_fine]: midpoints (torch.lerp(z[1:], z[:-1], 0.5)), sample_pdf on ray_weights[..., 1:-1], merge. */
int yanerf_refine(const float* lengths, const float* ray_weights, int64_t R, int64_t P, int64_t n_fine,
                  int det, const float* u, uint64_t seed, uint64_t offset, int add_input,
                  float* lengths_out, const uint64_t* rng_base, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Photometric loss of the training objective (pipelines/utils.py:189-196; nerf_pipeline.py:284-305):
 * per-ray squared error against gathered ground truth (sample_grid, pipelines/utils.py:272-296) and
 * dL/dfeatures for L = scale * sum((pred - gt)^2). image [B][H][W][C], xys [B][R][2] integer-valued.
 * ---------------------------------------------------------------------------------------------- */
int yanerf_rgb_loss(const float* pred, const float* image, const float* xys, int64_t B, int64_t R,
                    int64_t H, int64_t W, int64_t C, float scale, float* sq_err_per_ray, float* g_pred,
                    void* stream);

/* ------------------------------------------------------------------------------------------------
 * The Monte-Carlo rays' outputs splatted onto full-size images: replaces scatter_rays_to_image
 * (pipelines/utils.py:299-323) as NeRFPipeline._rasterize_mc_samples calls it for rendered_images /
 * rendered_depths / rendered_alpha_masks on every training step with output_rasterized_mc
 * (nerf_pipeline.py:196-201, 307-324). values [B][R][C], xys [B][R][2] (integer-valued floats, pixel
 * x + W * y) -> out [B][H][W][C] = bg[c] (C floats; NULL = 0) everywhere, values at the rays' pixels.
 * Two rays on one pixel: one of them is written (torch's scatter_ leaves that order unspecified too).
 * The pixel index is computed in float and truncated, as the reference's `.long()` of x + W * y (so images of 2^24
 * pixels and more get the reference's own rounded indices). A ray whose index falls outside [0, H * W) -- where the
 * reference's scatter_ raises -- is not written and sets *oob = 1 (a device int, may be NULL; never cleared here):
 * the caller decides when to read it back (ops.scatter_rays raises like the reference).
 * ---------------------------------------------------------------------------------------------- */
int yanerf_scatter_rays(const float* values, const float* xys, int64_t B, int64_t R, int64_t C, int64_t H,
                        int64_t W, const float* bg, float* out, int* oob, void* stream);

/* Fused Adam step over a flat fp32 parameter buffer: torch.optim.Adam (run.py:158-160) with torch's arithmetic, one
 * element per lane. The scalars are doubles, as torch holds them in Python: bias corrections 1 - beta**step, the step
 * size lr / bc1 and sqrt(bc2) are computed on the host in double and rounded to float once, as torch passes them to
 * its kernels. `step` is the 1-based step count after this update (Adam's state["step"]). */
int yanerf_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream);
/* Host function: the two per-step scalars yanerf_adam passes its kernel, (-lr / (1 - beta1^step),
 * sqrt(1 - beta2^step)) rounded to float, into out2[2]. */
int yanerf_adam_scalars(double lr, double beta1, double beta2, int64_t step, float* out2);
/* yanerf_adam with the step's scalars read on the device: row *index of table [K][2] (filled with
 * yanerf_adam_scalars), so a captured step (hipGraph) replays with each step's learning rate and bias corrections.
 * Bit-identical to yanerf_adam with the same scalars. avg_over > 1: `grads` holds the SUM over that many
 * data-parallel ranks and is first averaged in place (grads / avg_over, the division DDP applies after its
 * all-reduce, run.py:162-166); 1 = as given. Not a reference entry point (scripts/run.py:158-160's torch.optim.Adam,
 * as yanerf_adam). */
int yanerf_adam_table(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const float* table, const int64_t* index, double beta1, double beta2, double eps,
                      double weight_decay, int64_t avg_over, void* stream);
/* The device-side step state of a graph-capturable training step: state[0] (the Philox offset base read through the
 * rng_base pointers of yanerf_raygen / yanerf_refine / yanerf_raymarch_opts) += rng_delta, state[1] (the Adam table
 * index) += 1. One thread, stream-ordered. */
int yanerf_step_advance(uint64_t* state, uint64_t rng_delta, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* YANERF_HIP_H */
