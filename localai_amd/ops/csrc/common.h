// Shared device helpers for the gfx950 (CDNA4) kernels of localai_amd.
// Wave64 everywhere: every reduction below assumes 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LA_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// cache policy of the quantised-weight LDS-DMA loads in the GEMM kernels (0 = default, 2 = nt);
// an A/B build flag (-DLA_W_AUX=2)
#ifndef LA_W_AUX
#define LA_W_AUX 0
#endif

// s_setprio(1) around the GEMM kernels' MFMA clusters (an A/B build flag, -DLA_SETPRIO=1)
#ifndef LA_SETPRIO
#define LA_SETPRIO 0
#endif

namespace la {

constexpr int WAVE = 64;

LA_DEV float bf2f(bf16 x) { return (float)x; }
LA_DEV bf16 f2bf(float x) { return (bf16)x; }

LA_DEV float h2f(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}

LA_DEV float bf16_bits_to_f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

LA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
LA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce within aligned groups of `G` lanes (G power of two <= 64)
template <int G>
LA_DEV float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int G>
LA_DEV float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
LA_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  return r;
}
template <int NT>
LA_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

LA_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

// f32 built from a nibble/byte: exact (128 + q) for q < 256 placed at bits 16..23.
LA_DEV float magic128(uint32_t q) { return __uint_as_float(0x43000000u | (q << 16)); }

}  // namespace la
