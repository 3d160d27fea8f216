// Quantised "skinny" GEMM for decode / small batches:  out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]
//
// Replaces ggml-cuda's mmvq/mmq ([external]).  MI355X-first design:
//  * B operand = weights, read ONCE from HBM straight into VGPRs (16-byte loads,
//    one super-block of prefetch in flight), dequantised in-register to bf16 and fed
//    to v_mfma_f32_16x16x32_bf16.  No LDS round trip for weights (guide §5:
//    "GEMV / M <= 16 decode weights: load straight to VGPRs").
//  * A operand = activations (M <= 64 rows), staged per super-block through LDS
//    (shared by the 4 waves of the workgroup, each wave owns 16 output columns),
//    issue-early / write-late (T14) so the L2 latency of X hides under the MFMAs.
//  * Split-K over grid.y gives >= 2 workgroups per CU; partial fp32 slabs are summed by
//    the consuming kernel (rmsnorm / rope / silu-mul prologue), never by atomics.
#include "qweight.h"

namespace la {

constexpr int SK_WAVES = 4;
constexpr int SK_THREADS = 64 * SK_WAVES;
constexpr int SK_LDS_STRIDE = 256 + 8;  // bf16 elements per LDS row (16 B pad: spreads banks)

template <int FMT, int MT>
__global__ __launch_bounds__(SK_THREADS, 2) void qgemm_skinny_kernel(
    QW w, const bf16* __restrict__ X, int ldx, int M, int k_per_split, float* __restrict__ out, int ldo,
    long slab) {
  constexpr int MP = 16 * MT;
  __shared__ __attribute__((aligned(16))) bf16 xs[MP * SK_LDS_STRIDE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int N = w.N, K = w.K;
  const int split = blockIdx.y;
  const int kbeg = split * k_per_split;
  const int nsb = min(k_per_split, K - kbeg) >> 8;
  const int n = blockIdx.x * (16 * SK_WAVES) + wave * 16 + r;
  const int nl = min(n, N - 1);  // clamp: out-of-range lanes compute garbage, never stored

  // ---- X staging: MP rows x 256 cols bf16 = MP*32 16-byte chunks per super-block
  constexpr int XCH = MP * 32;
  constexpr int XPT = (XCH + SK_THREADS - 1) / SK_THREADS;
  bf16x8 xr[XPT];
  auto x_issue = [&](int sb) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * SK_THREADS;
      const int row = c >> 5, col = (c & 31) * 8;
      bf16x8 v = {};
      if (c < XCH && row < M) v = *(const bf16x8*)(X + (size_t)row * ldx + kbeg + sb * 256 + col);
      xr[i] = v;
    }
  };
  auto x_store = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * SK_THREADS;
      if (c < XCH) {
        const int row = c >> 5, col = (c & 31) * 8;
        *(bf16x8*)(xs + row * SK_LDS_STRIDE + col) = xr[i];
      }
    }
  };

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int sb0 = kbeg >> 8;
  WFrag<FMT> fa, fb;
  x_issue(0);
  fa.load(w, nl, sb0, g);

  auto compute = [&](WFrag<FMT>& f) {
    f.prep(g);
#define SK_STEP(S)                                                                         \
  {                                                                                        \
    const bf16x8 b = f.template deq<S>();                                                  \
    const int kp = kphys<FMT>(S, g);                                                       \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                    \
      const bf16x8 a = *(const bf16x8*)(xs + (mt * 16 + r) * SK_LDS_STRIDE + kp);          \
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[mt], 0, 0, 0);           \
    }                                                                                      \
  }
    SK_STEP(0) SK_STEP(1) SK_STEP(2) SK_STEP(3) SK_STEP(4) SK_STEP(5) SK_STEP(6) SK_STEP(7)
#undef SK_STEP
  };

  // two super-blocks per iteration with statically named fragments (no runtime-indexed arrays)
  for (int sb = 0; sb < nsb; sb += 2) {
    // --- super-block sb (fragment fa)
    __syncthreads();  // previous readers of xs done
    x_store();
    __syncthreads();
    if (sb + 1 < nsb) {
      x_issue(sb + 1);
      fb.load(w, nl, sb0 + sb + 1, g);
    }
    compute(fa);
    if (sb + 1 >= nsb) break;
    // --- super-block sb+1 (fragment fb)
    __syncthreads();
    x_store();
    __syncthreads();
    if (sb + 2 < nsb) {
      x_issue(sb + 2);
      fa.load(w, nl, sb0 + sb + 2, g);
    }
    compute(fb);
  }

  if (n < N) {
    float* o = out + (size_t)split * slab;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mt * 16 + 4 * g + i;
        if (m < M) o[(size_t)m * ldo + n] = acc[mt][i];
      }
    }
  }
}

template <int FMT, int MT>
static void launch_skinny_t(const QW& w, const bf16* X, int ldx, int M, int splits, float* out, int ldo,
                            long slab, hipStream_t st) {
  const int nsb_total = w.K >> 8;
  const int per = nsb_total / splits;
  dim3 grid((w.N + 16 * SK_WAVES - 1) / (16 * SK_WAVES), splits);
  hipLaunchKernelGGL((qgemm_skinny_kernel<FMT, MT>), grid, dim3(SK_THREADS), 0, st, w, X, ldx, M,
                     per * 256, out, ldo, slab);
}

template <int FMT>
static void launch_skinny_f(const QW& w, const bf16* X, int ldx, int M, int splits, float* out, int ldo,
                            long slab, hipStream_t st) {
  if (M <= 16) launch_skinny_t<FMT, 1>(w, X, ldx, M, splits, out, ldo, slab, st);
  else if (M <= 32) launch_skinny_t<FMT, 2>(w, X, ldx, M, splits, out, ldo, slab, st);
  else launch_skinny_t<FMT, 4>(w, X, ldx, M, splits, out, ldo, slab, st);
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
extern "C" int la_qgemm_skinny(int fmt, const void* p0, const void* p1, const void* p2, const void* p3,
                               int N, int K, const void* X, int ldx, int M, int splits, void* out,
                               int ldo, long slab, void* stream) {
  using namespace la;
  if (M < 1 || M > 64 || (K & 255) || splits < 1 || ((K >> 8) % splits) || ldo < N || slab < (long)M * ldo) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)p2, (const uint8_t*)p3, N, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
  switch (fmt) {
    case FMT_Q4_K: launch_skinny_f<FMT_Q4_K>(w, x, ldx, M, splits, o, ldo, slab, st); break;
    case FMT_Q6_K: launch_skinny_f<FMT_Q6_K>(w, x, ldx, M, splits, o, ldo, slab, st); break;
    case FMT_Q8_0: launch_skinny_f<FMT_Q8_0>(w, x, ldx, M, splits, o, ldo, slab, st); break;
    case FMT_BF16: launch_skinny_f<FMT_BF16>(w, x, ldx, M, splits, o, ldo, slab, st); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}
