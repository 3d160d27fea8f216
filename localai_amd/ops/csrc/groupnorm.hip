// GroupNorm (+ optional SiLU) over NHWC bf16 activations, gfx950 -- the Stable Diffusion UNet /
// VAE normalisation (models/sd.py: ResNet norm1/norm2 + SiLU, Transformer2D norm, conv_norm_out).
//
// PyTorch's GroupNorm on these shapes runs three kernels (row moments over one workgroup per
// (batch, group) -- only 64 workgroups for SD's 2 x 32 groups -- fused params, then a separate
// elementwise pass and another one for SiLU).  Here:
//   la_gn_stats : grid (S chunks of pixels, B).  Each workgroup streams its chunk row by row
//                 (a row = C contiguous bf16, read as bf16x2 lanes: coalesced), every thread owning
//                 fixed channel pairs, so per-group fp32 sum / sum-of-squares stay in registers; one
//                 LDS reduction per workgroup writes [B, S, G, 2] partials.  B*S ~ 256 workgroups
//                 (one pass over the tensor; few partials to fold).
//   la_gn_apply : grid (pixel chunks, B); each workgroup folds the S partials (read coalesced by
//                 all lanes, LDS-summed) into mean / rstd,
//                 precomputes per-channel scale / shift (gamma, beta) and writes
//                 y = x * scale + shift, SiLU'd when asked, in one pass.
// Channels per group must be even (a bf16x2 lane never straddles two groups) and C <= 2048.
#include <hip/hip_bfloat16.h>
#include <hip/hip_runtime.h>

namespace la {

constexpr int GN_THREADS = 256;
constexpr int GN_MAXP = 4;  // channel pairs per thread: C <= 2 * 256 * 4
constexpr int GN_MAXG = 64;

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even
  return (unsigned short)(u >> 16);
}

__global__ void __launch_bounds__(GN_THREADS) gn_stats_kernel(const unsigned* __restrict__ x, float* __restrict__ part,
                                                              int HW, int C, int G, int rows_per_chunk, int S) {
  const int s = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int P = C >> 1, cg = C / G;
  const int r0 = s * rows_per_chunk, r1 = min(HW, r0 + rows_per_chunk);
  // C/2 <= 256: several rows per step, one pair per lane; otherwise one row per step
  const int RS = P <= GN_THREADS ? GN_THREADS / P : 1;
  const int tr = P <= GN_THREADS ? t / P : 0, pb = P <= GN_THREADS ? t % P : t;
  float sum[GN_MAXP], sq[GN_MAXP];
#pragma unroll
  for (int i = 0; i < GN_MAXP; ++i) sum[i] = sq[i] = 0.0f;
  const unsigned* xb = x + (long)b * HW * P;
  for (int r = r0 + tr; tr < RS && r < r1; r += RS) {
    const unsigned* row = xb + (long)r * P;
#pragma unroll
    for (int i = 0; i < GN_MAXP; ++i) {
      const int p = pb + i * GN_THREADS;
      if (p < P) {
        const unsigned v = row[p];
        const float a = bf2f((unsigned short)(v & 0xFFFF)), c = bf2f((unsigned short)(v >> 16));
        sum[i] += a + c;
        sq[i] += a * a + c * c;
      }
    }
  }
  // per-group totals in a FIXED order (no LDS float atomics: their arrival order made the sums,
  // and so every SD / SDXL image, differ in the last bits run to run): every thread parks its
  // per-pair partials in LDS, then lane (g, k) walks group g's pairs and row slots in order
  __shared__ float ps[GN_THREADS * GN_MAXP * 2];
#pragma unroll
  for (int i = 0; i < GN_MAXP; ++i) {
    const bool own = tr < RS && pb + i * GN_THREADS < P;
    ps[(t * GN_MAXP + i) * 2] = own ? sum[i] : 0.0f;
    ps[(t * GN_MAXP + i) * 2 + 1] = own ? sq[i] : 0.0f;
  }
  __syncthreads();
  float* out = part + ((long)b * S + s) * G * 2;
  if (t < 2 * G) {
    const int g = t >> 1, k = t & 1, hp = cg >> 1;
    float a = 0.0f;
    for (int p = g * hp; p < (g + 1) * hp; ++p) {
      if (P <= GN_THREADS) {
        for (int r = 0; r < RS; ++r) a += ps[((r * P + p) * GN_MAXP) * 2 + k];
      } else {
        a += ps[((p % GN_THREADS) * GN_MAXP + p / GN_THREADS) * 2 + k];
      }
    }
    out[t] = a;
  }
}

__global__ void __launch_bounds__(GN_THREADS) gn_apply_kernel(const unsigned* __restrict__ x, unsigned* __restrict__ y,
                                                              const unsigned short* __restrict__ gamma,
                                                              const unsigned short* __restrict__ beta,
                                                              const float* __restrict__ part, int HW, int C, int G,
                                                              int rows_per_chunk, int S, float eps, int silu) {
  // rows_per_chunk: this kernel's pixels per workgroup; S: number of stats partials per batch
  const int s = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int P = C >> 1, cg = C / G;
  // fold the S stats partials [S, G, 2] of this batch: all lanes read them coalesced, lane t
  // owning slot t % 2G (2G divides the workgroup), then an LDS sum over the 256 / 2G lanes per slot
  __shared__ float red[GN_THREADS];
  __shared__ float stat[GN_MAXG * 2];
  {
    const int G2 = 2 * G, slot = t % G2, KS = GN_THREADS / G2;
    const float* pp = part + (long)b * S * G2;
    float a = 0.0f;
#pragma unroll 8
    for (int k = t / G2; k < S; k += KS) a += pp[(long)k * G2 + slot];
    red[t] = a;
    __syncthreads();
    if (t < G2) {
      float v = 0.0f;
      for (int j = 0; j < KS; ++j) v += red[j * G2 + t];
      stat[t] = v;
    }
    __syncthreads();
    if (t < G) {
      const float n = (float)HW * cg;
      const float mean = stat[2 * t] / n;
      const float var = fmaxf(stat[2 * t + 1] / n - mean * mean, 0.0f);
      red[2 * t] = mean;
      red[2 * t + 1] = rsqrtf(var + eps);
    }
  }
  __syncthreads();
  const int RS = P <= GN_THREADS ? GN_THREADS / P : 1;
  const int tr = P <= GN_THREADS ? t / P : 0, pb = P <= GN_THREADS ? t % P : t;
  float sc[GN_MAXP][2], sh[GN_MAXP][2];
#pragma unroll
  for (int i = 0; i < GN_MAXP; ++i) {
    const int p = pb + i * GN_THREADS;
    if (p < P) {
      const int g = (2 * p) / cg;
      const float mean = red[2 * g], rstd = red[2 * g + 1];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float ga = gamma ? bf2f(gamma[2 * p + j]) : 1.0f, be = beta ? bf2f(beta[2 * p + j]) : 0.0f;
        sc[i][j] = rstd * ga;
        sh[i][j] = be - mean * rstd * ga;
      }
    }
  }
  const int r0 = s * rows_per_chunk, r1 = min(HW, r0 + rows_per_chunk);
  const long base = (long)b * HW * P;
  for (int r = r0 + tr; tr < RS && r < r1; r += RS) {
    const unsigned* row = x + base + (long)r * P;
    unsigned* orow = y + base + (long)r * P;
#pragma unroll
    for (int i = 0; i < GN_MAXP; ++i) {
      const int p = pb + i * GN_THREADS;
      if (p < P) {
        const unsigned v = row[p];
        float a = bf2f((unsigned short)(v & 0xFFFF)) * sc[i][0] + sh[i][0];
        float c = bf2f((unsigned short)(v >> 16)) * sc[i][1] + sh[i][1];
        if (silu) {
          a = a / (1.0f + __expf(-a));
          c = c / (1.0f + __expf(-c));
        }
        orow[p] = (unsigned)f2bf(a) | ((unsigned)f2bf(c) << 16);
      }
    }
  }
}

}  // namespace la

// x, y: [B, HW, C] bf16 (NHWC); gamma / beta: [C] bf16 or null; part: fp32 workspace of B*S*G*2.
// rows_stats / rows_apply: pixels per workgroup of the two kernels (the statistics pass uses
// coarser chunks so the apply pass has few partials to fold).
extern "C" int la_groupnorm_nhwc(const void* x, void* y, const void* gamma, const void* beta, float* part, int B,
                                 int HW, int C, int G, int rows_stats, int rows_apply, float eps, int silu,
                                 void* stream) {
  if (B <= 0 || HW <= 0 || C <= 0 || G <= 0 || G > la::GN_MAXG || C % G || (C / G) % 2 ||
      la::GN_THREADS % (2 * G) || C > 2 * la::GN_THREADS * la::GN_MAXP || rows_stats <= 0 || rows_apply <= 0)
    return (int)hipErrorInvalidValue;
  const int S = (HW + rows_stats - 1) / rows_stats;
  const int SA = (HW + rows_apply - 1) / rows_apply;
  hipLaunchKernelGGL(la::gn_stats_kernel, dim3((unsigned)S, (unsigned)B), dim3(la::GN_THREADS), 0,
                     (hipStream_t)stream, (const unsigned*)x, part, HW, C, G, rows_stats, S);
  hipLaunchKernelGGL(la::gn_apply_kernel, dim3((unsigned)SA, (unsigned)B), dim3(la::GN_THREADS), 0,
                     (hipStream_t)stream, (const unsigned*)x, (unsigned*)y, (const unsigned short*)gamma,
                     (const unsigned short*)beta, part, HW, C, G, rows_apply, S, eps, silu);
  return (int)hipGetLastError();
}
