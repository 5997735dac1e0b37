// Probe: can the f32 VALU (v_pk_fma_f32) run beside the f32 MFMA (v_mfma_f32_16x16x4_f32) on gfx950, i.e. does a
// SIMD sustain more than the 64 FLOP/clk of either pipe alone when one wave feeds each? Four cases, 512-thread
// workgroups (two waves per SIMD), 4 workgroups per CU worth of grid:
//   mfma   every wave: chains of 8 independent 16x16x4 f32 MFMAs
//   valu   every wave: 16 independent v_pk_fma_f32 accumulators
//   split  waves 0-3 MFMA, waves 4-7 VALU (one of each per SIMD)
//   mixed  every wave interleaves 8 MFMAs with NV v_pk_fma_f32
// Prints TFLOP/s per case (f32 FLOPs counted: MFMA 2*16*16*4 per instruction, pk_fma 2*2*64 per instruction).
//   hipcc --offload-arch=gfx950 -O3 -o probe_mfma_valu probe_mfma_valu.hip && ./probe_mfma_valu
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int ITERS = 2048;

__device__ __forceinline__ void mfma8(v4f (&c)[8], float a, float b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
}
template <int NV>
__device__ __forceinline__ void valu(v2f (&v)[16], v2f x, v2f y) {
#pragma unroll
  for (int i = 0; i < NV; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(v[i % 16]) : "v"(x), "v"(y));
}

// OP (MODE 3 only): 0 v_pk_fma_f32, 1 v_add_u32, 2 v_mov_b32, 3 v_fma_f32, 4 v_xor_b32 -- which VALU ops take issue
// slots from the f32 MFMA
template <int OP, int NV>
__device__ __forceinline__ void valu_op(v2f (&v)[16], v2f x, v2f y) {
  if constexpr (OP == 0) {
    valu<NV>(v, x, y);
  } else {
    float f[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = v[i].x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float& d = f[i % 16];
      if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(y.x));
      if constexpr (OP == 2) asm volatile("v_mov_b32 %0, %1" : "=v"(d) : "v"(f[(i + 1) % 16]));
      if constexpr (OP == 3) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(d) : "v"(x.x), "v"(y.x));
      if constexpr (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(y.x));
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i].x = f[i];
  }
}

template <int MODE, int NV, int OP = 0>
__global__ void __launch_bounds__(512) k(float* out, float s) {
  const int wave = threadIdx.x >> 6;
  v4f c[8];
  v2f v[16];
  for (int i = 0; i < 8; ++i) c[i] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 16; ++i) v[i] = v2f{(float)i, s};
  const float a = s * threadIdx.x, b = s + threadIdx.x;
  const v2f x{s, 0.999f}, y{1e-3f, s};
  const bool do_mfma = MODE == 0 || MODE == 3 || (MODE == 2 && wave < 4);
  const bool do_valu = MODE == 1 || MODE == 3 || (MODE == 2 && wave >= 4);
  if (do_mfma && do_valu) {
    for (int it = 0; it < ITERS; ++it) {
      mfma8(c, a, b);
      valu_op<OP, NV>(v, x, y);
    }
  } else if (do_mfma) {
    for (int it = 0; it < ITERS; ++it) mfma8(c, a, b);
  } else {
    for (int it = 0; it < ITERS; ++it) valu<NV>(v, x, y);
  }
  float r = 0.f;
  for (int i = 0; i < 8; ++i) r += c[i].x + c[i].y + c[i].z + c[i].w;
  for (int i = 0; i < 16; ++i) r += v[i].x + v[i].y;
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int MODE, int NV, int OP = 0>
static void run(const char* name, float* out, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<MODE, NV, OP><<<grid, 512>>>(out, 1.0f);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k<MODE, NV, OP><<<grid, 512>>>(out, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  // per wave: mfma waves 8 * ITERS MFMAs (2048 FLOP each), valu waves NV * ITERS pk_fma (256 FLOP each)
  double mf_waves = 0, va_waves = 0;
  const double waves = (double)grid * 8;
  if (MODE == 0) mf_waves = waves;
  if (MODE == 1) va_waves = waves;
  if (MODE == 2) mf_waves = va_waves = waves / 2;
  if (MODE == 3) mf_waves = va_waves = waves;
  const double fl_m = mf_waves * 8.0 * ITERS * 2048.0, fl_v = va_waves * (double)NV * ITERS * 256.0;
  printf("{\"case\": \"%s\", \"op\": %d, \"nv\": %d, \"ms\": %.4f, \"mfma_tflops\": %.2f, \"valu_tflops\": %.2f, \"total_tflops\": %.2f}\n",
         name, OP, NV, ms, fl_m / ms / 1e9, fl_v / ms / 1e9, (fl_m + fl_v) / ms / 1e9);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu * 4;
  float* out;
  hipMalloc(&out, (size_t)grid * 512 * sizeof(float));
  run<0, 16>("mfma", out, grid);
  run<1, 16>("valu", out, grid);
  run<2, 16>("split", out, grid);
  run<2, 32>("split", out, grid);
  run<3, 4>("mixed", out, grid);
  run<3, 8>("mixed", out, grid);
  run<3, 16>("mixed", out, grid);
  run<3, 32>("mixed", out, grid);
  // MFMA throughput with 8 and 16 VALU ops of each kind per 8 MFMAs (valu_tflops only meaningful for op 0 / 3)
  run<3, 8, 1>("mixed", out, grid);
  run<3, 16, 1>("mixed", out, grid);
  run<3, 8, 2>("mixed", out, grid);
  run<3, 16, 2>("mixed", out, grid);
  run<3, 8, 3>("mixed", out, grid);
  run<3, 16, 3>("mixed", out, grid);
  run<3, 8, 4>("mixed", out, grid);
  run<3, 16, 4>("mixed", out, grid);
  hipFree(out);
  return 0;
}
