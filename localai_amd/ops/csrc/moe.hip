// Mixture-of-experts for decode-sized batches (ggml MUL_MAT_ID [external]),
// graph-capturable: routing, grouping and the expert GEMMs never leave the device.
//
//  moe_route   : one workgroup; from top-k expert ids [T][topk] build a pair list grouped by expert
//                (order[], off[E+1]; pair p = t*topk + slot), deterministic (stable by pair id).
//  grouped GEMM: the skinny quantised GEMM with blockIdx.z = expert.  The expert's QW descriptor
//                comes from a device array; its rows are gathered through order[] (so each expert's
//                weights stream from HBM once per step however many tokens picked it).  Two output
//                modes:
//                  GATE_UP: out[split][pair][n]                      (X row = token of the pair)
//                  DOWN   : out[split*topk + slot][token][n] * w[pair]  (X row = pair)
//                DOWN writes the routing-weighted expert outputs as extra split-K slabs, so the
//                next kernel's slab-sum prologue (add_norm) performs the top-k combine for free.
#include <cmath>

#include "qweight.h"

namespace la {

constexpr int MOE_WAVES = 4;
constexpr int MOE_THREADS = 64 * MOE_WAVES;
constexpr int MOE_LDS_STRIDE = 256 + 8;

__global__ __launch_bounds__(1024) void moe_route_kernel(const int* __restrict__ ids, int T, int topk, int E,
                                                         int* __restrict__ order, int* __restrict__ off) {
  __shared__ int cnt[256];
  __shared__ int base[257];
  const int P = T * topk;
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) atomicAdd(&cnt[min(max(ids[p], 0), E - 1)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    base[0] = 0;
    for (int e = 0; e < E; ++e) base[e + 1] = base[e] + cnt[e];
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E; e += blockDim.x) off[e] = base[e];
  // stable placement, one wave per expert: 64 pairs per ballot, each hit's slot = its rank
  // among the hits of lower lanes (expert e's pairs land in increasing pair order)
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int e = threadIdx.x >> 6; e < E; e += nw) {
    int o = base[e];
    for (int p0 = 0; p0 < P; p0 += 64) {
      const int p = p0 + lane;
      const bool hit = p < P && min(max(ids[p], 0), E - 1) == e;
      const unsigned long long m = __ballot(hit);
      if (hit) order[o + __popcll(m & ((1ull << lane) - 1ull))] = p;
      o += __popcll(m);
    }
  }
}

// Fused router for decode-sized batches: one workgroup per token.  Each wave takes experts
// e = wave, wave + 4, ...: a 64-lane dot of the token's bf16 hidden row with the fp32 router row
// (shuffle reduction), logits into LDS; then one lane does softmax over E, top-k by probability
// (lowest id first on ties), optional renormalisation and scale, and writes the expert ids --
// remapped to this rank's local ids under expert parallelism (others -> E_local) -- and weights.
// Replaces the router GEMM, softmax, top-k sort, renorm and dtype-copy launches (about ten small
// kernels per MoE layer at batch 1).
// The block has min(E, 16) waves (one expert each when E <= 16) and the dot product's loads are
// issued 4 chunks at a time before any FMA, so a batch-1 router costs about one memory latency
// per expert instead of one per 512-wide chunk (Mixtral-8x7B C=1: 11.8 us per layer with 4 waves
// walking 2 experts each, chunk by chunk).
__global__ __launch_bounds__(1024) void moe_router_kernel(const bf16* __restrict__ x, int ldx,
                                                          const float* __restrict__ wr, int E, int D, int topk,
                                                          int renorm, float scale, int ep_base, int ep_local,
                                                          int* __restrict__ ids, float* __restrict__ wts) {
  __shared__ float lg[256];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const bf16* xr = x + (size_t)t * ldx;
  for (int e = wave; e < E; e += nw) {
    const float* w = wr + (size_t)e * D;
    float acc = 0.0f;
    int i = lane * 8;
    for (; i + 3 * 512 < D; i += 4 * 512) {
      bf16x8 xv[4];
      float4 w0[4], w1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[u] = *(const bf16x8*)(xr + i + u * 512);
        w0[u] = *(const float4*)(w + i + u * 512);
        w1[u] = *(const float4*)(w + i + u * 512 + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc += bf2f(xv[u][0]) * w0[u].x + bf2f(xv[u][1]) * w0[u].y + bf2f(xv[u][2]) * w0[u].z +
               bf2f(xv[u][3]) * w0[u].w + bf2f(xv[u][4]) * w1[u].x + bf2f(xv[u][5]) * w1[u].y +
               bf2f(xv[u][6]) * w1[u].z + bf2f(xv[u][7]) * w1[u].w;
    }
    for (; i < D; i += 512) {
      const bf16x8 xv = *(const bf16x8*)(xr + i);
      const float4 w0 = *(const float4*)(w + i), w1 = *(const float4*)(w + i + 4);
      acc += bf2f(xv[0]) * w0.x + bf2f(xv[1]) * w0.y + bf2f(xv[2]) * w0.z + bf2f(xv[3]) * w0.w +
             bf2f(xv[4]) * w1.x + bf2f(xv[5]) * w1.y + bf2f(xv[6]) * w1.z + bf2f(xv[7]) * w1.w;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) lg[e] = acc;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, lg[e]);
  float z = 0.0f;
  for (int e = 0; e < E; ++e) {
    lg[e] = __expf(lg[e] - mx);
    z += lg[e];
  }
  const float inv = 1.0f / z;
  unsigned long long taken[4] = {0ull, 0ull, 0ull, 0ull};  // E <= 256
  float sel[16];
  int sid[16];
  float sum = 0.0f;
  for (int k = 0; k < topk; ++k) {
    int best = -1;
    float bv = -1.0f;
    for (int e = 0; e < E; ++e) {
      if ((taken[e >> 6] >> (e & 63)) & 1ull) continue;
      if (lg[e] > bv) { bv = lg[e]; best = e; }
    }
    taken[best >> 6] |= 1ull << (best & 63);
    sid[k] = best;
    sel[k] = bv * inv;
    sum += sel[k];
  }
  for (int k = 0; k < topk; ++k) {
    const float wv = (renorm ? sel[k] / sum : sel[k]) * scale;
    const int loc = sid[k] - ep_base;
    ids[t * topk + k] = (loc >= 0 && loc < ep_local) ? loc : ep_local;
    wts[t * topk + k] = wv;
  }
}

// NW waves per workgroup, 16 output columns each: the X tile staged in LDS per super-block serves
// 16 * NW columns, so NW = 8 halves the L2 -> LDS activation traffic of a wide batch (where every
// column block of an expert re-stages the same gathered rows) and doubles the waves per CU.
template <int FMT, int MT, bool DOWN, int NW = MOE_WAVES, bool W3 = false>
__global__ __launch_bounds__(64 * NW, W3 ? 2 : (NW > 8 ? 1 : 8 / NW)) void moe_gemm_kernel(
    const QW* __restrict__ qws, const int* __restrict__ order, const int* __restrict__ off, int topk,
    const bf16* __restrict__ X, int ldx, int k_per_split, const float* __restrict__ wts, float* __restrict__ out,
    int ldo, long slab, int T, int nchunk) {
  constexpr int MP = 16 * MT;
  __shared__ __attribute__((aligned(16))) bf16 xs[MP * MOE_LDS_STRIDE];
  __shared__ int prow[MP];

  // blockIdx.z = expert * nchunk + chunk: chunk c takes the expert's rows [c*MP, c*MP + MP), so any
  // batch size is one fixed-shape launch (chunks past an expert's row count exit at once)
  const int e = blockIdx.z / nchunk, chunk = blockIdx.z - e * nchunk;
  const int o0 = off[e] + chunk * MP;
  const int M = min(off[e + 1] - o0, MP);
  if (M <= 0) return;
  const QW w = qws[e];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int N = w.N, K = w.K;
  const int split = blockIdx.y;
  const int kbeg = split * k_per_split;
  const int nsb = min(k_per_split, K - kbeg) >> 8;
  constexpr int NT = 64 * NW;
  const int n = blockIdx.x * (16 * NW) + wave * 16 + r;
  const int nl = min(n, N - 1);
  if (tid < MP) prow[tid] = tid < M ? order[o0 + tid] : 0;
  __syncthreads();

  constexpr int XCH = MP * 32;
  constexpr int XPT = (XCH + NT - 1) / NT;
  bf16x8 xr[XPT];
  auto x_issue = [&](int sb) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT;
      const int row = min(c >> 5, MP - 1), col = (c & 31) * 8;
      const int p = prow[row];
      const int xrow = DOWN ? p : p / topk;
      bf16x8 v = *(const bf16x8*)(X + (size_t)xrow * ldx + kbeg + sb * 256 + col);
      if (row >= M) v = bf16x8{};
      xr[i] = v;
    }
  };
  auto x_store = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT;
      if (c < XCH) *(bf16x8*)(xs + (c >> 5) * MOE_LDS_STRIDE + (c & 31) * 8) = xr[i];
    }
  };

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int sb0 = kbeg >> 8;
  WFrag<FMT> fa, fb;
  x_issue(0);
  fa.load(w, nl, sb0, g);
  WFrag<FMT> fc;
  if constexpr (W3) {
    if (nsb > 1) fb.load(w, nl, sb0 + 1, g);
  }
  auto compute = [&](WFrag<FMT>& f) {
    f.prep(g);
#define MOE_STEP(S)                                                                          \
  {                                                                                          \
    const bf16x8 b = f.template deq<S>();                                                    \
    const int kp = kphys<FMT>(S, g);                                                         \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                      \
      const bf16x8 a = *(const bf16x8*)(xs + (mt * 16 + r) * MOE_LDS_STRIDE + kp);           \
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[mt], 0, 0, 0);             \
    }                                                                                        \
  }
    MOE_STEP(0) MOE_STEP(1) MOE_STEP(2) MOE_STEP(3) MOE_STEP(4) MOE_STEP(5) MOE_STEP(6) MOE_STEP(7)
#undef MOE_STEP
  };
  if constexpr (W3) {
    // three-slot weight ring: super-block s + 2 is requested while s computes, so each HBM weight
    // round trip has two compute phases to land instead of one (the gathered activation rows come
    // from L2 and keep the one-ahead register stage)
    auto step = [&](int s, WFrag<FMT>& cur, WFrag<FMT>& nxt2) {
      __syncthreads();
      x_store();
      __syncthreads();
      if (s + 1 < nsb) x_issue(s + 1);
      if (s + 2 < nsb) nxt2.load(w, nl, sb0 + s + 2, g);
      compute(cur);
    };
    for (int sb = 0; sb < nsb; sb += 3) {
      step(sb, fa, fc);
      if (sb + 1 >= nsb) break;
      step(sb + 1, fb, fa);
      if (sb + 2 >= nsb) break;
      step(sb + 2, fc, fb);
    }
  } else {
  for (int sb = 0; sb < nsb; sb += 2) {
    __syncthreads();
    x_store();
    __syncthreads();
    if (sb + 1 < nsb) {
      x_issue(sb + 1);
      fb.load(w, nl, sb0 + sb + 1, g);
    }
    compute(fa);
    if (sb + 1 >= nsb) break;
    __syncthreads();
    x_store();
    __syncthreads();
    if (sb + 2 < nsb) {
      x_issue(sb + 2);
      fa.load(w, nl, sb0 + sb + 2, g);
    }
    compute(fb);
  }
  }
  if (n >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * g + i;
      if (m >= M) continue;
      const int p = prow[m];
      if (DOWN) {
        const int t = p / topk, slot = p - t * topk;
        out[((size_t)split * topk + slot) * slab + (size_t)t * ldo + n] = acc[mt][i] * wts[p];
      } else {
        out[(size_t)split * slab + (size_t)p * ldo + n] = acc[mt][i];
      }
    }
  }
}

static int g_moe_mt = 0;  // 0: auto; else the row tile (MT x 16 rows) for batches past 64 rows
static int g_moe_nw = 8;  // waves (16 columns each) per workgroup for batches past 64 rows
static int g_moe_w3 = 0;  // three-slot weight ring (A/B)
static int g_moe_mid8 = 1;   // 8-wave workgroups for 33..64-row batches too
static int g_moe_small8 = 0; // ... and for 17..32-row batches (A/B)

template <int FMT, bool DOWN>
static void launch_moe(const QW* qws, int N, int K, int E, const int* order, const int* off, int topk,
                       const bf16* X, int ldx, int maxM, int splits, const float* wts, float* out, int ldo, long slab,
                       int T, hipStream_t st) {
  const int per = (K >> 8) / splits;
#define MOE_LW(MT, NW, W3)                                                                                        \
  {                                                                                                               \
    const int gx = (N + 16 * (NW)-1) / (16 * (NW));                                                               \
    const int nch = (maxM + 16 * (MT)-1) / (16 * (MT));                                                           \
    hipLaunchKernelGGL((moe_gemm_kernel<FMT, MT, DOWN, NW, W3>), dim3(gx, splits, E * nch), dim3(64 * (NW)), 0,  \
                       st, qws, order, off, topk, X, ldx, per * 256, wts, out, ldo, slab, T, nch);                \
  }
#define MOE_L(MT, NW) MOE_LW(MT, NW, false)
  if (maxM <= 16) MOE_L(1, 4)
  else if (maxM <= 32) {
    if (g_moe_small8) MOE_L(2, 8) else MOE_L(2, 4)
  } else if (maxM <= 64) {
    // 8-wave workgroups here too: Mixtral-8x7B engine C=64 3309 / 3311 tok/s vs 3047 / 3043
    // with 4 waves (scripts/gpu_r4_t.sh)
    if (g_moe_mid8) MOE_L(4, 8) else MOE_L(4, 4)
  }
  else {
    // wide batch: 64-row tiles in 8-wave workgroups, whatever the batch.  Mixtral-8x7B, engine
    // C=256 (decode + the prefill chunks, one box): 64-row / 8 waves 3951 tok/s; 128-row / 4 waves
    // (round 3) 3461; 128 / 8: 3475; 96 / 8: 3346-3592; 80 / 8: 3119 (scripts/gpu_r4_m.sh).  The
    // 64-row tile keeps two workgroups (16 waves) per CU -- occupancy outweighs streaming the
    // weights of an expert with more rows once per extra chunk (they come back from L2 / MALL)
    const int mt = g_moe_mt > 0 ? g_moe_mt : 4;
    if (g_moe_w3 && mt == 4 && g_moe_nw == 8) MOE_LW(4, 8, true)
    else if (g_moe_nw == 16 && mt == 4) MOE_L(4, 16)
    else if (g_moe_nw >= 8) {
      if (mt <= 4) MOE_L(4, 8) else if (mt <= 5) MOE_L(5, 8) else if (mt <= 6) MOE_L(6, 8) else MOE_L(8, 8)
    } else {
      if (mt <= 4) MOE_L(4, 4) else if (mt <= 5) MOE_L(5, 4) else if (mt <= 6) MOE_L(6, 4) else MOE_L(8, 4)
    }
  }
#undef MOE_L
#undef MOE_LW
}

}  // namespace la

extern "C" int la_moe_router(const void* x, int ldx, const float* wr, int E, int D, int T, int topk, int renorm,
                             float scale, int ep_base, int ep_local, int* ids, float* wts, void* stream) {
  if (E < 1 || E > 256 || topk < 1 || topk > 16 || topk > E || (D & 7) || T < 1) return -1;
  const int nw = E < 4 ? 4 : (E > 16 ? 16 : E);
  hipLaunchKernelGGL(la::moe_router_kernel, dim3(T), dim3(64 * nw), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                     wr, E, D, topk, renorm, scale, ep_base, ep_local, ids, wts);
  return (int)hipGetLastError();
}

extern "C" int la_moe_route(const int* ids, int T, int topk, int E, int* order, int* off, void* stream) {
  if (E > 256 || E < 1) return -1;
  hipLaunchKernelGGL(la::moe_route_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, ids, T, topk, E, order, off);
  return (int)hipGetLastError();
}

// qws: device array of E QW descriptors (all experts share fmt, N, K).  maxM = max rows per expert
// (<= T for GATE_UP / DOWN since a token picks an expert at most once); above 64 the launch covers
// ceil(maxM / 128) row chunks per expert.
extern "C" int la_moe_gemm(int fmt, int down, const void* qws, int N, int K, int E, const int* order, const int* off,
                           int topk, const void* X, int ldx, int maxM, int splits, const float* wts, void* out,
                           int ldo, long slab, int T, void* stream) {
  using namespace la;
  if (maxM < 1 || E * ((maxM + 127) / 128) > 65535 || (K & 255) || splits < 1 || ((K >> 8) % splits) || ldo < N) return -1;
  hipStream_t st = (hipStream_t)stream;
  const QW* q = (const QW*)qws;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
#define MOE_F(F)                                                                                     \
  if (down) launch_moe<F, true>(q, N, K, E, order, off, topk, x, ldx, maxM, splits, wts, o, ldo, slab, T, st); \
  else launch_moe<F, false>(q, N, K, E, order, off, topk, x, ldx, maxM, splits, wts, o, ldo, slab, T, st);
  switch (fmt) {
    case FMT_Q4_K: MOE_F(FMT_Q4_K) break;
    case FMT_Q6_K: MOE_F(FMT_Q6_K) break;
    case FMT_Q8_0: MOE_F(FMT_Q8_0) break;
    case FMT_BF16: MOE_F(FMT_BF16) break;
    default: return -2;
  }
#undef MOE_F
  return (int)hipGetLastError();
}

extern "C" int la_qw_size() { return (int)sizeof(la::QW); }

// Tuning hook (A/B): wide-batch row tile (0 auto, 4..8) and waves per workgroup (4 or 8).
extern "C" int la_moe_tune(int mt, int nw) {
  // nw 9: 8 waves + weight ring; nw 10: 4 waves for 33..64-row batches (round-3 shape);
  // nw 11: 8 waves also for 17..32-row batches
  if (mt < 0 || mt > 8 || (nw != 4 && nw != 8 && nw != 9 && nw != 10 && nw != 11 && nw != 16)) return -1;
  la::g_moe_mid8 = nw != 10;
  la::g_moe_small8 = nw == 11;
  if (nw == 10 || nw == 11) nw = 8;
  la::g_moe_mt = mt;
  la::g_moe_nw = nw == 9 ? 8 : nw;
  la::g_moe_w3 = nw == 9;
  return 0;
}
