// Probe: the bf16 MLP GEMM loop skeleton (mlp.hip gemm_run, MT == 8 path) with 16x16x32 vs 32x32x16 bf16 MFMAs.
// Per wave: a 64-feature x 128-point accumulator tile (128 fp32 registers either way); per 32-wide K-block 4 weight
// fragments from global memory (a 2-deep register ring, L2-resident table), 8 point fragments by ds_read_b128 from an
// 80 KB LDS image (two 256-thread workgroups per CU, as the forward), then 32 (16x16x32) or 16 (32x32x16) MFMAs and V
// independent v_add_f32 fillers. Every 8 K-blocks (a layer) the tile is packed to bf16 and written back to LDS between
// two barriers (the epilogue). Prints TFLOP/s per (shape, V) on random operands.
//   hipcc --offload-arch=gfx950 -O3 -o probe_gemm_shape probe_gemm_shape.hip && ./probe_gemm_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;

constexpr int M = 128, ROWB = 640;  // points per tile, LDS row bytes (320 bf16)
constexpr int LAYERS = 8, KBL = 8;  // layers per launch, K-blocks per layer

__device__ __forceinline__ int swz(int m, int c) { return c ^ ((m >> 1) & 7); }

template <int SHAPE, int V>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
k(const f4* __restrict__ W, float* __restrict__ out, int iters) {
  __shared__ __attribute__((aligned(16))) char act[M * ROWB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < M * ROWB / 16; i += 256) ((f4*)act)[i] = f4{0.01f * (i & 7), 0.02f, -0.03f, 0.04f};
  __syncthreads();
  float fill[8];
  for (int i = 0; i < 8; ++i) fill[i] = lane * 0.001f + i;
  // weights: 64 rows per wave in fragment order, 64 lanes x 16 B per fragment, a table of 16 row tiles x 8 K-blocks
  const f4* wp = W + (size_t)wave * 4 * KBL * 64 + lane;
  if constexpr (SHAPE == 16) {
    f4 acc[4][8];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4, li = lane & 15;
    for (int it = 0; it < iters; ++it) {
      #pragma unroll 1
      for (int l = 0; l < LAYERS; ++l) {
        f4 a0[4], a1[4];
        for (int nt = 0; nt < 4; ++nt) a0[nt] = wp[(nt * KBL + 0) * 64];
        for (int nt = 0; nt < 4; ++nt) a1[nt] = wp[(nt * KBL + 1) * 64];
#pragma unroll 1
        for (int kb = 0; kb < KBL; ++kb) {
          int ln = lane;
          asm volatile("" : "+v"(ln));
          const int g = ln >> 4, li = ln & 15;
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            f4 b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int m = 16 * (4 * hf + q) + li;
              b[q] = *(const f4*)(act + m * ROWB + swz(m, kb * 4 + g) * 16);
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int mt = 4 * hf + q;
                acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a0[nt]),
                                                                      __builtin_bit_cast(bf8, b[q]), acc[nt][mt], 0, 0, 0);
                if constexpr (V > 0)
                  if ((nt * 8 + mt) % (32 / (V < 32 ? V : 32)) == 0)
#pragma unroll
                    for (int v = 0; v < (V > 32 ? V / 32 : 1); ++v) fill[v & 7] += 1.0f;
              }
          }
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            a0[nt] = a1[nt];
            a1[nt] = wp[(nt * KBL + ((kb + 2) & (KBL - 1))) * 64];
          }
        }
        __syncthreads();
        // epilogue: pack to bf16 and write the tile back (each wave its 64 features of all 128 points)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int mt = 0; mt < 8; ++mt) {
            const int m = 16 * mt + li, n = wave * 64 + 16 * nt + 4 * g;
            const f4 v = acc[nt][mt];
            typedef __bf16 bh4 __attribute__((ext_vector_type(4)));
            bh4 h = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
            *(bh4*)(act + m * ROWB + swz(m, n >> 3) * 16 + (n & 7) * 2) = h;
          }
        __syncthreads();
      }
    }
    float r = 0.f;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) r += acc[i][j].x + acc[i][j].y + acc[i][j].z + acc[i][j].w;
    for (int i = 0; i < 8; ++i) r += fill[i];
    out[blockIdx.x * 256 + tid] = r;
  } else {
    // 32x32x16: acc[2 feature tiles][4 point tiles] of 16 registers; per K-block 2 k-steps of 16
    f16v acc[2][4];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int h = lane >> 5, li = lane & 31;
    for (int it = 0; it < iters; ++it) {
      #pragma unroll 1
      for (int l = 0; l < LAYERS; ++l) {
        f4 a0[4], a1[4];  // [feature tile][k-step] flattened as 2 x 2
        for (int nt = 0; nt < 4; ++nt) a0[nt] = wp[(nt * KBL + 0) * 64];
        for (int nt = 0; nt < 4; ++nt) a1[nt] = wp[(nt * KBL + 1) * 64];
#pragma unroll 1
        for (int kb = 0; kb < KBL; ++kb) {
          int ln = lane;
          asm volatile("" : "+v"(ln));
          const int h = ln >> 5, li = ln & 31;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            f4 b[4];  // [point tile] of this k-step
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
              const int m = 32 * mt + li;
              b[mt] = *(const f4*)(act + m * ROWB + swz(m, kb * 4 + ks * 2 + h) * 16);
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
              for (int mt = 0; mt < 4; ++mt) {
                acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a0[nt * 2 + ks]),
                                                                      __builtin_bit_cast(bf8, b[mt]), acc[nt][mt], 0, 0, 0);
                if constexpr (V > 0)
                  if ((ks * 8 + nt * 4 + mt) % (16 / (V < 16 ? V : 16)) == 0)
#pragma unroll
                    for (int v = 0; v < (V > 16 ? V / 16 : 1); ++v) fill[v & 7] += 1.0f;
              }
          }
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            a0[nt] = a1[nt];
            a1[nt] = wp[(nt * KBL + ((kb + 2) & (KBL - 1))) * 64];
          }
        }
        __syncthreads();
        // epilogue: lane (h, li) holds point 32 mt + li, features 8 j + 4 h + r of tile nt (j = reg / 4, r = reg % 4)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = 32 * mt + li, n = wave * 64 + 32 * nt + 8 * j + 4 * h;
              typedef __bf16 bh4 __attribute__((ext_vector_type(4)));
              bh4 hv = {(__bf16)acc[nt][mt][4 * j], (__bf16)acc[nt][mt][4 * j + 1], (__bf16)acc[nt][mt][4 * j + 2],
                        (__bf16)acc[nt][mt][4 * j + 3]};
              *(bh4*)(act + m * ROWB + swz(m, n >> 3) * 16 + (n & 7) * 2) = hv;
            }
        __syncthreads();
      }
    }
    float r = 0.f;
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 4; ++j)
        for (int q = 0; q < 16; ++q) r += acc[i][j][q];
    for (int i = 0; i < 8; ++i) r += fill[i];
    out[blockIdx.x * 256 + tid] = r;
  }
}

template <int SHAPE, int V>
static void run(const f4* W, float* out, int grid) {
  const int iters = 4;
  k<SHAPE, V><<<grid, 256>>>(W, out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k<SHAPE, V><<<grid, 256>>>(W, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  // per workgroup: 256 features x 128 points x 256 K per layer
  const double fl = 2.0 * grid * (double)iters * LAYERS * 256.0 * 128.0 * 256.0;
  printf("{\"shape\": \"%dx%d\", \"valu_per_kblock\": %d, \"ms\": %.4f, \"tflops\": %.1f}\n", SHAPE, SHAPE, V, ms,
         fl / ms / 1e9);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu * 2 * 12;
  const size_t wn = 16 * KBL * 64;
  f4* hw = (f4*)malloc(wn * sizeof(f4));
  for (size_t i = 0; i < wn; ++i) {
    u16 u[8];
    for (int j = 0; j < 8; ++j) u[j] = (u16)(0x3c00 + (rand() & 0x3ff) - 0x200) | (rand() & 1 ? 0x8000 : 0);
    hw[i] = *(f4*)u;
  }
  f4* W;
  float* out;
  (void)hipMalloc(&W, wn * sizeof(f4));
  (void)hipMalloc(&out, (size_t)grid * 256 * sizeof(float));
  (void)hipMemcpy(W, hw, wn * sizeof(f4), hipMemcpyHostToDevice);
  run<16, 0>(W, out, grid);
  run<32, 0>(W, out, grid);
  run<16, 16>(W, out, grid);
  run<32, 16>(W, out, grid);
  run<16, 32>(W, out, grid);
  run<32, 32>(W, out, grid);
  run<16, 64>(W, out, grid);
  run<32, 64>(W, out, grid);
  run<16, 0>(W, out, grid);
  run<32, 0>(W, out, grid);
  (void)hipFree(W);
  (void)hipFree(out);
  free(hw);
  return 0;
}
