// Quantised mid-M GEMM (batched decode, 64 < M <= a few hundred rows):
//   out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]      (fp32 split-K slabs)
//
// Replaces the bf16 hipBLASLt call on a dequantised weight copy that the engine used
// for 64 < M (SURVEY §2.8 K5/K6 mmq, [external]).  Why a second kernel next to the skinny
// one: at M = 128..256 the in-register dequant of the skinny kernel (each wave dequantises
// the fragments it multiplies) costs ~22 VALU ops per 8 weights, which only hides under
// the MFMAs when ONE dequantised fragment feeds >= ~11 of them.  Here the weight tile is
// dequantised ONCE per workgroup into LDS (16-weight units, 16-B raw loads) and shared by
// all waves, like the activation tile:
//   * tile BM (M) x BN (N) x 64 (K), BM in {128, 256}, BN in {64, 128} (autotuned per shape);
//     default BM = 128 (4 waves, 2x2) for M <= 128 and BM = 256
//     (8 waves, 4x2) above, so the dequant cost per MFMA halves as M grows; each wave owns a
//     64x64 output tile = 4x4 v_mfma_f32_16x16x32_bf16 accumulators;
//   * both operands staged through padded LDS rows (row stride 160 B: the 16 rows a
//     ds_read_b128 lane group touches land on 16 distinct 16-B bank slots);
//   * a 4-deep register ring feeds a 2-buffer LDS pipeline: the raw quant bytes + X chunks
//     of K-step t+4 are in flight while the MFMAs of step t run; dequant/LDS write after;
//   * split-K over grid.y, M tiles over grid.z; the fp32 slabs are summed by the
//     consuming kernel's prologue (same contract as the skinny GEMM).
#include "qraw.h"

namespace la {

constexpr int MD_BN = 128, MD_BK = 64;
#ifndef MID_DEPTH
#define MID_DEPTH 4
#endif
constexpr int MD_LDS = MD_BK + 16;  // bf16 per LDS row: 160 B = 10 16-B slots, conflict-free ds_read_b128 for the (row r, k-chunk g) fragment pattern (stride 144 B was 2-way)

// Tile BM x BN, (BM/64) x (BN/64) waves; every wave owns a 64x64 output tile.  BN = 64 tiles
// double the workgroup count of the small-N projections (o / down / qkv: N = 4096-6144) at
// batch-decode M, where BN = 128 leaves most CUs idle.
template <int FMT, int BM, int BN>
__global__ __launch_bounds__((BM / 64) * (BN / 64) * 64) void qgemm_mid_kernel(
    QW w, const bf16* __restrict__ X, int ldx, int M, int ksteps_per_split, float* __restrict__ out, int ldo,
    long slab) {
  constexpr int WN = BN / 64;                   // waves along N
  constexpr int NT = (BM / 64) * WN * 64;       // threads
  constexpr int XU = BM * MD_BK / 8 / NT;       // 16-B X chunks per thread per K-step
  constexpr int WU = BN * 4 / NT;               // 16-weight W units per thread
  static_assert(XU >= 1 && WU >= 1 && BM * MD_BK / 8 % NT == 0 && BN * 4 % NT == 0, "tile/thread mismatch");
  constexpr int BUF = (BM + BN) * MD_LDS;       // bf16 per stage buffer
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 15, g = lane >> 4;
  const int N = w.N;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.z * BM;
  const int total_ks = w.K / MD_BK;
  const int ks0 = blockIdx.y * ksteps_per_split;
  const int ks1 = min(total_ks, ks0 + ksteps_per_split);
  if (ks0 >= ks1) return;  // uniform per block

  // Register ring stages: the raw quant bytes + X chunks of one K-step.  Loads are never
  // predicated (clamped instead) so hipcc emits counted vmcnt waits, not vmcnt(0).
  struct Stage {
    MidRaw<FMT> raw[WU];
    bf16x8 xr[XU];
  };
  typename MidRaw<FMT>::Addr wad[WU];
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int id = tid + u * NT;
    wad[u].init(w, min(n0 + (id >> 2), N - 1), id & 3);  // clamped rows: garbage, never stored
  }
  uint32_t xoff[XU];
#pragma unroll
  for (int i = 0; i < XU; ++i) {
    const int c = tid + i * NT;
    xoff[i] = (uint32_t)min(m0 + (c >> 3), M - 1) * ldx + (c & 7) * 8;  // rows >= M: never stored
  }
  auto issue = [&](Stage& S, int ks) {
#pragma unroll
    for (int u = 0; u < WU; ++u) S.raw[u].load(w, wad[u], ks);
    const bf16* xk = X + ks * MD_BK;
#pragma unroll
    for (int i = 0; i < XU; ++i) {
      S.xr[i] = *(const bf16x8*)(xk + xoff[i]);
    }
  };
  auto commit = [&](const Stage& S, int ks, int buf) {
    bf16* xs = lds + buf * BUF;
    bf16* ws = xs + BM * MD_LDS;
#pragma unroll
    for (int i = 0; i < XU; ++i) {
      const int c = tid + i * NT;
      *(bf16x8*)(xs + (c >> 3) * MD_LDS + (c & 7) * 8) = S.xr[i];
    }
#pragma unroll
    for (int u = 0; u < WU; ++u) {
      const int id = tid + u * NT;
      bf16x8 d[2];
      S.raw[u].deq(wad[u], ks, d);
      bf16* dst = ws + (id >> 2) * MD_LDS + 16 * (id & 3);
      *(bf16x8*)dst = d[0];
      *(bf16x8*)(dst + 8) = d[1];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16* xs = lds + buf * BUF;
    const bf16* ws = xs + BM * MD_LDS;
#pragma unroll
    for (int kk = 0; kk < MD_BK; kk += 32) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = *(const bf16x8*)(xs + (wm * 64 + t * 16 + r) * MD_LDS + kk + 8 * g);
        b[t] = *(const bf16x8*)(ws + (wn * 64 + t * 16 + r) * MD_LDS + kk + 8 * g);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
  };

  // D-deep ring (MID_DEPTH stages): vmcnt retires in issue order, so the X chunks (L2) and
  // the raw weights (HBM) share one prefetch distance; at ~1 WG per CU the weight stream
  // needs ~3-4 K-steps of loads in flight to cover HBM latency (measured: the ablated kernel
  // with no MFMA/dequant/X still ran at 1 TB/s with a 3-deep ring).
  constexpr int D = MID_DEPTH;
  const int last = ks1 - 1;
  Stage st[D];
#pragma unroll
  for (int i = 0; i < D; ++i) issue(st[i], min(ks0 + i, last));
  commit(st[0], ks0, 0);
  __syncthreads();
  const int nks = ks1 - ks0;
  for (int j = 0; j < nks; j += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      // step t = j + i: buffer (t & 1) holds K-step t; slot i refills with t + D; slot i+1
      // (K-step t + 1) is committed to the other buffer
      const int t = j + i;
      issue(st[i], min(ks0 + t + D, last));
      compute(t & 1);
      commit(st[(i + 1) % D], min(ks0 + t + 1, last), (t + 1) & 1);
      __syncthreads();
      if (t + 1 >= nks) break;
    }
  }


  float* o = out + (size_t)blockIdx.y * slab;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = n0 + wn * 64 + nt * 16 + r;
    if (n >= N) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + mt * 16 + 4 * g + i;
        if (m < M) o[(size_t)m * ldo + n] = acc[mt][nt][i];
      }
    }
  }
}

template <int FMT, int BM, int BN>
static void launch_mid_t(const QW& w, const bf16* X, int ldx, int M, int per, int splits, float* out, int ldo,
                         long slab, hipStream_t st) {
  dim3 grid((w.N + BN - 1) / BN, splits, (M + BM - 1) / BM);
  hipLaunchKernelGGL((qgemm_mid_kernel<FMT, BM, BN>), grid, dim3((BM / 64) * (BN / 64) * 64), 0, st, w, X, ldx, M,
                     per, out, ldo, slab);
}

// tile: 0 = auto (BM by M, BN 128); else 10 * (BM / 64) + (BN / 64), e.g. 42 = 256 x 128, 41 = 256 x 64,
// 22 = 128 x 128, 21 = 128 x 64
template <int FMT>
static int launch_mid(const QW& w, const bf16* X, int ldx, int M, int splits, int tile, float* out, int ldo,
                      long slab, hipStream_t st) {
  const int total = w.K / MD_BK;
  const int per = (total + splits - 1) / splits;
  if (tile == 0) tile = (M <= 128) ? 22 : 42;
  switch (tile) {
    case 42: launch_mid_t<FMT, 256, 128>(w, X, ldx, M, per, splits, out, ldo, slab, st); break;
    case 41: launch_mid_t<FMT, 256, 64>(w, X, ldx, M, per, splits, out, ldo, slab, st); break;
    case 22: launch_mid_t<FMT, 128, 128>(w, X, ldx, M, per, splits, out, ldo, slab, st); break;
    case 21: launch_mid_t<FMT, 128, 64>(w, X, ldx, M, per, splits, out, ldo, slab, st); break;
    default: return -1;
  }
  return 0;
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// splits must satisfy ceil(K/64 / splits) * (splits-1) < K/64 so every slab is written.
extern "C" int la_qgemm_mid(int fmt, const void* p0, const void* p1, const void* p2, const void* p3, int N, int K,
                            const void* X, int ldx, int M, int splits, void* out, int ldo, long slab, int tile,
                            void* stream) {
  using namespace la;
  if (M < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || slab < (long)M * ldo) return -1;
  if ((long)N * K >= (1L << 31) || (long)M * ldx >= (1L << 31)) return -1;  // 32-bit staging offsets
  const int total = K / MD_BK, per = (total + splits - 1) / splits;
  if (per * (splits - 1) >= total) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)p2, (const uint8_t*)p3, N, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
  switch (fmt) {
    case FMT_Q4_K: if (launch_mid<FMT_Q4_K>(w, x, ldx, M, splits, tile, o, ldo, slab, st)) return -1; break;
    case FMT_Q6_K: if (launch_mid<FMT_Q6_K>(w, x, ldx, M, splits, tile, o, ldo, slab, st)) return -1; break;
    case FMT_Q8_0: if (launch_mid<FMT_Q8_0>(w, x, ldx, M, splits, tile, o, ldo, slab, st)) return -1; break;
    default: return -2;
  }
  return (int)hipGetLastError();
}
