// Register-only throughput probe: is an int8-MFMA Q4_K x q8 GEMM (ggml mmq numerics: per-32-k
// weight scales d*sc_j and per-32-k activation scales, applied to the int32 partial sums) faster
// than the bf16-MFMA tile GEMM on gfx950?  Every variant computes the same 16x16 output tiles over
// the same K; only the inner-loop arithmetic differs:
//   bf16 : 2 x v_mfma_f32_16x16x32_bf16 per 64 k (dequantised weights, the shipped path's MFMA work)
//   i8   : 1 x v_mfma_i32_16x16x64_i8 per 64 k, no scales (an upper bound, wrong numerics for Q4_K)
//   i8s  : 2 x v_mfma_i32_16x16x32_i8 per 64 k (one per 32-k scale block) + the per-block epilogue
//          acc += float(i32) * (dw[col] * dx[row]) on the 4 outputs of every lane
//   i8s64: 1 x 16x16x64_i8 per 64 k with the epilogue once per 64 k (scales shared by 2 blocks:
//          not Q4_K-exact either, shows the epilogue cost at half the rate)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/i8_epilogue_probe.hip -o /tmp/i8probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

constexpr int NT = 8;  // independent accumulator tiles per wave

template <int MODE>
__global__ __launch_bounds__(256) void probe(const int* __restrict__ seed, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  int s = seed[lane];
  f32x4 acc[NT];
  for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a16, b16;
  for (int j = 0; j < 8; ++j) {
    a16[j] = (__bf16)(float)((s >> j) & 7);
    b16[j] = (__bf16)(float)((s >> (j + 3)) & 7);
  }
  // per-tile operands, perturbed every iteration (one v_xor per tile) so the compiler can neither
  // hoist the zero-initialised i8 MFMAs out of the loop nor merge identical tiles
  i32x2 a8[NT];
  i32x4v a8w[NT];
  for (int t = 0; t < NT; ++t) {
    a8[t] = i32x2{(s >> t) & 0x07070707, (s >> (t + 1)) & 0x07070707};
    a8w[t] = i32x4v{(s >> t) & 0x07070707, (s >> 1) & 0x07070707, (s >> 2) & 0x07070707, (s >> 3) & 0x07070707};
  }
  float dw = 0.001f * (float)(lane + 1), dx[4];
  for (int i = 0; i < 4; ++i) dx[i] = 0.002f * (float)(i + 1 + (s & 3));
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (MODE == 0) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16, b16, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b16, a16, acc[t], 0, 0, 0);
      } else if constexpr (MODE == 1) {
        a8w[t].x ^= it;
        i32x4 z = __builtin_bit_cast(i32x4, acc[t]);
        z = __builtin_amdgcn_mfma_i32_16x16x64_i8(a8w[t], a8w[t], z, 0, 0, 0);
        acc[t] = __builtin_bit_cast(f32x4, z);
      } else if constexpr (MODE == 2) {
        a8[t].x ^= it;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          i32x4 z = {0, 0, 0, 0};
          const long op = __builtin_bit_cast(long, a8[t]) + h;
          z = __builtin_amdgcn_mfma_i32_16x16x32_i8(op, op, z, 0, 0, 0);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[t][i] = fmaf((float)z[i], dw * dx[i], acc[t][i]);
        }
      } else {
        a8w[t].x ^= it;
        i32x4 z = {0, 0, 0, 0};
        z = __builtin_amdgcn_mfma_i32_16x16x64_i8(a8w[t], a8w[t], z, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = fmaf((float)z[i], dw * dx[i], acc[t][i]);
      }
    }
    dw *= 1.0000001f;
  }
  float r = 0.f;
  for (int t = 0; t < NT; ++t) r += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int MODE>
static double run(const int* seed, float* out, int iters, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE><<<grid, 256>>>(seed, out, iters);  // warm-up
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) probe<MODE><<<grid, 256>>>(seed, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5.0;
}

int main() {
  const int grid = 256 * 8, iters = 4096;  // 8 WGs of 4 waves per CU: 8 waves per SIMD
  int* seed;
  float* out;
  hipMalloc(&seed, 64 * sizeof(int));
  hipMalloc(&out, grid * 256 * sizeof(float));
  int h[64];
  for (int i = 0; i < 64; ++i) h[i] = rand();
  hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
  // useful work per (wave, iteration, tile): a 16x16 output over 64 k = 16*16*64*2 "ops"
  const double ops = 16.0 * 16 * 64 * 2 * NT * iters * (grid * 4.0);
  const char* names[4] = {"bf16 2x16x16x32", "i8 16x16x64 (no scales)", "i8 2x16x16x32 + per-32 epilogue",
                          "i8 16x16x64 + per-64 epilogue"};
  double t[4] = {run<0>(seed, out, iters, grid), run<1>(seed, out, iters, grid), run<2>(seed, out, iters, grid),
                 run<3>(seed, out, iters, grid)};
  for (int m = 0; m < 4; ++m)
    printf("%-36s %8.3f ms  %7.1f TOPS  (%.2fx bf16)\n", names[m], t[m], ops / (t[m] * 1e-3) / 1e12, t[0] / t[m]);
  return 0;
}
