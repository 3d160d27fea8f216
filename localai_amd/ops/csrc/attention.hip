// Paged attention for the engine (replaces ggml-cuda fattn*.cu / softmax.cu / the KQ,KQV
// batched GEMMs of the non-FA path; SURVEY §2.8 K7, K11, K12, K15 [external]).
//
// KV cache layout (per layer): K, V each [num_blocks][Hkv][BS][Dh] bf16, so one page of one
// kv-head is BS*Dh*2 contiguous bytes (8 KiB at BS=32, Dh=128).
//
// * attn_decode: one query row per sequence.  Workgroup = (partition of <=PS keys, kv head,
//   sequence); the G = Hq/Hkv query heads sharing a kv head are packed so K/V are read from
//   HBM once (GQA packing).  Split-KV partials are merged by attn_decode_combine.
// * attn_prefill: causal flash attention on MFMA (v_mfma_f32_16x16x32_bf16) for chunks of new
//   tokens appended to a (possibly prefix-cached) context; K/V tiles of 32 keys come from the
//   paged cache, so prefix reuse and chunked prefill need no special casing.
#include "common.h"

namespace la {

// ----------------------------------------------------------------------------- decode
constexpr int DEC_T = 256;
constexpr int DEC_PS = 256;  // keys per partition

template <int DH, int G>
__global__ __launch_bounds__(DEC_T) void attn_decode_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ seq_lens, int Hkv, int BS,
    float scale, bf16* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml, int P) {
  constexpr int NC = DH / 8;  // 16-byte chunks per row
  static_assert(NC <= 16, "head dim <= 128");
  __shared__ float qs[G][DH];
  __shared__ float sc[G][DEC_PS];
  __shared__ float red[DEC_T / 64][G][DH];
  __shared__ float stat[G][2];

  const int p = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int Hq = Hkv * G;
  const int L = seq_lens[b];
  const int t0 = p * DEC_PS;
  if (t0 >= L) {
    // empty partition: publish a neutral partial
    if (P > 1 && threadIdx.x < G) {
      const int h = kvh * G + threadIdx.x;
      float* ml = part_ml + (((long)b * Hq + h) * P + p) * 2;
      ml[0] = -INFINITY;
      ml[1] = 0.f;
    }
    if (P > 1) {
      for (int i = threadIdx.x; i < G * DH; i += DEC_T) {
        const int h = kvh * G + i / DH;
        part_o[(((long)b * Hq + h) * P + p) * DH + (i % DH)] = 0.f;
      }
    }
    return;
  }
  const int t1 = min(L, t0 + DEC_PS);
  const int* bt = block_tables + (long)b * max_blocks;

  for (int i = threadIdx.x; i < G * DH; i += DEC_T) {
    const int h = i / DH, d = i % DH;
    qs[h][d] = (float)q[((long)b * Hq + kvh * G + h) * DH + d] * scale;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane >> 4, c = lane & 15;  // 4 token-groups per wave, 16 lanes each
  const int gid = wave * 4 + grp;             // 0..15

  // ---- scores
  for (int t = t0 + gid; t < t1; t += 16) {
    const int blk = bt[t / BS], off = t % BS;
    float s[G];
#pragma unroll
    for (int h = 0; h < G; ++h) s[h] = 0.f;
    if (c < NC) {
      const bf16x8 kv = *(const bf16x8*)(kc + (((long)blk * Hkv + kvh) * BS + off) * DH + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float kf = (float)kv[j];
#pragma unroll
        for (int h = 0; h < G; ++h) s[h] = fmaf(qs[h][8 * c + j], kf, s[h]);
      }
    }
#pragma unroll
    for (int h = 0; h < G; ++h) s[h] = group_sum<16>(s[h]);
    if (c == 0) {
#pragma unroll
      for (int h = 0; h < G; ++h) sc[h][t - t0] = s[h];
    }
  }
  __syncthreads();

  // ---- softmax per head (wave w handles heads w, w+4, ...)
  const int n = t1 - t0;
  for (int h = wave; h < G; h += DEC_T / 64) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, sc[h][i]);
    m = wave_max(m);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float e = __expf(sc[h][i] - m);
      sc[h][i] = e;
      l += e;
    }
    l = wave_sum(l);
    if (lane == 0) {
      stat[h][0] = m;
      stat[h][1] = l;
    }
  }
  __syncthreads();

  // ---- P.V : lane chunk c owns d in [8c, 8c+8)
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  if (c < NC) {
    for (int t = t0 + gid; t < t1; t += 16) {
      const int blk = bt[t / BS], off = t % BS;
      const bf16x8 vv = *(const bf16x8*)(vc + (((long)blk * Hkv + kvh) * BS + off) * DH + 8 * c);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float pr = sc[h][t - t0];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[h][j] = fmaf(pr, (float)vv[j], acc[h][j]);
      }
    }
  }
  // reduce over the 4 token groups of the wave (lanes c, c+16, c+32, c+48)
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[h][j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[h][j] = v;
    }
  if (grp == 0 && c < NC) {
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wave][h][8 * c + j] = acc[h][j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * DH; i += DEC_T) {
    const int h = i / DH, d = i % DH;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < DEC_T / 64; ++w) v += red[w][h][d];
    const int hq = kvh * G + h;
    if (P == 1) {
      out[((long)b * Hq + hq) * DH + d] = (bf16)(v / stat[h][1]);
    } else {
      part_o[(((long)b * Hq + hq) * P + p) * DH + d] = v;
      if (d == 0) {
        float* ml = part_ml + (((long)b * Hq + hq) * P + p) * 2;
        ml[0] = stat[h][0];
        ml[1] = stat[h][1];
      }
    }
  }
}

__global__ __launch_bounds__(128) void attn_decode_combine_kernel(const float* __restrict__ part_o,
                                                                  const float* __restrict__ part_ml, int P, int DH,
                                                                  bf16* __restrict__ out) {
  const int hq = blockIdx.x, b = blockIdx.y, Hq = gridDim.x;
  const long base = ((long)b * Hq + hq) * P;
  float M = -INFINITY;
  for (int i = 0; i < P; ++i) M = fmaxf(M, part_ml[(base + i) * 2]);
  float den = 0.f;
  for (int i = 0; i < P; ++i) {
    const float m = part_ml[(base + i) * 2];
    if (m > -INFINITY) den += __expf(m - M) * part_ml[(base + i) * 2 + 1];
  }
  for (int d = threadIdx.x; d < DH; d += blockDim.x) {
    float num = 0.f;
    for (int i = 0; i < P; ++i) {
      const float m = part_ml[(base + i) * 2];
      if (m > -INFINITY) num += __expf(m - M) * part_o[(base + i) * DH + d];
    }
    out[((long)b * Hq + hq) * DH + d] = (bf16)(num / den);
  }
}

// ----------------------------------------------------------------------------- prefill
// Workgroup = 64 query rows (4 waves x 16) of one sequence x one query head.
constexpr int PF_T = 256;
constexpr int PF_KT = 32;  // keys per tile

template <int DH>
__global__ __launch_bounds__(PF_T) void attn_prefill_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ tiles,          // [ntiles][2] = (seq, first query row within seq)
    const int* __restrict__ cu_q,           // [nseq+1] token offsets of each seq's queries
    const int* __restrict__ ctx_lens,       // [nseq] total keys (cached + new)
    const int* __restrict__ block_tables, int max_blocks, int Hq, int Hkv, int BS, float scale,
    bf16* __restrict__ out) {
  constexpr int DP = (DH + 31) / 32 * 32;  // padded head dim for the MFMA k loop
  constexpr int KC = DP / 32;               // k-chunks of 32
  constexpr int ND = DP / 16;               // 16-wide output column tiles
  constexpr int KS = DP + 8;                // K tile LDS stride (elements)
  constexpr int VS = PF_KT + 8;             // V^T tile LDS stride
  __shared__ __attribute__((aligned(16))) bf16 ks[PF_KT * KS];
  __shared__ __attribute__((aligned(16))) bf16 vt[DP * VS];
  __shared__ __attribute__((aligned(16))) bf16 ps[4][16 * VS];

  const int tile = blockIdx.x, h = blockIdx.y;
  const int s = tiles[2 * tile], r0 = tiles[2 * tile + 1];
  const int G = Hq / Hkv, kvh = h / G;
  const int qbeg = cu_q[s], qlen = cu_q[s + 1] - qbeg;
  const int L = ctx_lens[s];
  const int pos0 = L - qlen;  // absolute position of query row 0
  const int* bt = block_tables + (long)s * max_blocks;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  // Q fragments (A operand): row = wave*16 + fr, k = 32*kc + 8*fq
  const int qrow = r0 + wave * 16 + fr;
  bf16x8 qa[KC];
#pragma unroll
  for (int kc2 = 0; kc2 < KC; ++kc2) {
    bf16x8 v = {};
    const int d = 32 * kc2 + 8 * fq;
    if (qrow < qlen && d < DH) v = *(const bf16x8*)(q + ((long)(qbeg + qrow) * Hq + h) * DH + d);
    qa[kc2] = v;
  }

  f32x4 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }

  const float sl2 = scale * 1.4426950408889634f;
  const int last_row = min(qlen, r0 + 64) - 1;
  const int kend = min(L, pos0 + last_row + 1);  // exclusive

  for (int k0 = 0; k0 < kend; k0 += PF_KT) {
    __syncthreads();
    // stage K tile rows and V^T tile: PF_KT keys x DP dims, 16-byte chunks
    for (int cidx = tid; cidx < PF_KT * (DP / 8); cidx += PF_T) {
      const int kr = cidx / (DP / 8), d = (cidx % (DP / 8)) * 8;
      const int key = k0 + kr;
      bf16x8 kv = {}, vv = {};
      if (key < kend && d < DH) {
        const int blk = bt[key / BS], off = key % BS;
        const long base = (((long)blk * Hkv + kvh) * BS + off) * DH + d;
        kv = *(const bf16x8*)(kc + base);
        vv = *(const bf16x8*)(vc + base);
      }
      *(bf16x8*)(ks + kr * KS + d) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) vt[(d + j) * VS + kr] = vv[j];
    }
    __syncthreads();

    // S = Q K^T : two 16-key sub-tiles
    f32x4 sacc[2];
#pragma unroll
    for (int ns = 0; ns < 2; ++ns) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc2 = 0; kc2 < KC; ++kc2) {
        const bf16x8 kb = *(const bf16x8*)(ks + (16 * ns + fr) * KS + 32 * kc2 + 8 * fq);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[kc2], kb, a, 0, 0, 0);
      }
      sacc[ns] = a;
    }
    // mask + online softmax.  lane holds rows 4*fq+i, keys 16*ns+fr
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qr = r0 + wave * 16 + 4 * fq + i;
      const int qpos = pos0 + qr;
      float v0 = sacc[0][i] * sl2, v1 = sacc[1][i] * sl2;
      const int key0 = k0 + fr, key1 = k0 + 16 + fr;
      if (key0 > qpos || key0 >= kend || qr >= qlen) v0 = -INFINITY;
      if (key1 > qpos || key1 >= kend || qr >= qlen) v1 = -INFINITY;
      float mx = group_max<16>(fmaxf(v0, v1));
      const float mnew = fmaxf(mrow[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      const float p0 = exp2f(v0 - msafe), p1 = exp2f(v1 - msafe);
      alpha[i] = exp2f(mrow[i] - msafe);
      lrow[i] = lrow[i] * alpha[i] + group_sum<16>(p0 + p1);
      mrow[i] = mnew;
      ps[wave][(4 * fq + i) * VS + fr] = (bf16)p0;
      ps[wave][(4 * fq + i) * VS + 16 + fr] = (bf16)p1;
    }
#pragma unroll
    for (int nd = 0; nd < ND; ++nd)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[nd][i] *= alpha[i];
    __syncthreads();
    // O += P V : A = P[16 q][32 keys], B = V[32 keys][16 d]
    const bf16x8 pa = *(const bf16x8*)(&ps[wave][fr * VS + 8 * fq]);
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const bf16x8 vb = *(const bf16x8*)(vt + (16 * nd + fr) * VS + 8 * fq);
      o[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[nd], 0, 0, 0);
    }
  }

  // epilogue: out[token][h][d] = O / l
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qr = r0 + wave * 16 + 4 * fq + i;
    if (qr >= qlen) continue;
    const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const int d = 16 * nd + fr;
      if (d < DH) out[((long)(qbeg + qr) * Hq + h) * DH + d] = (bf16)(o[nd][i] * inv);
    }
  }
}

}  // namespace la

// C ABI ------------------------------------------------------------------------------------
template <int DH, int G>
static void dec_launch(dim3 grid, hipStream_t st, const void* q, const void* kc, const void* vc, const int* bt,
                       int maxb, const int* sl, int Hkv, int BS, float scale, void* out, float* po, float* pml,
                       int P) {
  hipLaunchKernelGGL((la::attn_decode_kernel<DH, G>), grid, dim3(la::DEC_T), 0, st, (const bf16*)q,
                     (const bf16*)kc, (const bf16*)vc, bt, maxb, sl, Hkv, BS, scale, (bf16*)out, po, pml, P);
}

template <int DH>
static int dec_dispatch_g(int G, dim3 grid, hipStream_t st, const void* q, const void* kc, const void* vc,
                          const int* bt, int maxb, const int* sl, int Hkv, int BS, float scale, void* out, float* po,
                          float* pml, int P) {
  switch (G) {
    case 1: dec_launch<DH, 1>(grid, st, q, kc, vc, bt, maxb, sl, Hkv, BS, scale, out, po, pml, P); break;
    case 2: dec_launch<DH, 2>(grid, st, q, kc, vc, bt, maxb, sl, Hkv, BS, scale, out, po, pml, P); break;
    case 4: dec_launch<DH, 4>(grid, st, q, kc, vc, bt, maxb, sl, Hkv, BS, scale, out, po, pml, P); break;
    case 8: dec_launch<DH, 8>(grid, st, q, kc, vc, bt, maxb, sl, Hkv, BS, scale, out, po, pml, P); break;
    default: return -3;
  }
  return 0;
}

extern "C" int la_attn_decode(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                              const int* seq_lens, int B, int Hq, int Hkv, int Dh, int BS, float scale, int P,
                              void* out, void* part_o, void* part_ml, void* stream) {
  if (Hq % Hkv) return -1;
  const int G = Hq / Hkv;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(P, Hkv, B);
  float* po = (float*)part_o;
  float* pml = (float*)part_ml;
  int rc;
  switch (Dh) {
    case 64: rc = dec_dispatch_g<64>(G, grid, st, q, kc, vc, block_tables, max_blocks, seq_lens, Hkv, BS, scale, out, po, pml, P); break;
    case 80: rc = dec_dispatch_g<80>(G, grid, st, q, kc, vc, block_tables, max_blocks, seq_lens, Hkv, BS, scale, out, po, pml, P); break;
    case 96: rc = dec_dispatch_g<96>(G, grid, st, q, kc, vc, block_tables, max_blocks, seq_lens, Hkv, BS, scale, out, po, pml, P); break;
    case 128: rc = dec_dispatch_g<128>(G, grid, st, q, kc, vc, block_tables, max_blocks, seq_lens, Hkv, BS, scale, out, po, pml, P); break;
    default: return -2;
  }
  if (rc) return rc;
  if (P > 1)
    hipLaunchKernelGGL(la::attn_decode_combine_kernel, dim3(Hq, B), dim3(128), 0, st, po, pml, P, Dh, (bf16*)out);
  return (int)hipGetLastError();
}

extern "C" int la_attn_prefill(const void* q, const void* kc, const void* vc, const int* tiles, int ntiles,
                               const int* cu_q, const int* ctx_lens, const int* block_tables, int max_blocks, int Hq,
                               int Hkv, int Dh, int BS, float scale, void* out, void* stream) {
  if (Hq % Hkv) return -1;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(ntiles, Hq);
#define PF(D)                                                                                                     \
  hipLaunchKernelGGL(la::attn_prefill_kernel<D>, grid, dim3(la::PF_T), 0, st, (const bf16*)q, (const bf16*)kc,    \
                     (const bf16*)vc, tiles, cu_q, ctx_lens, block_tables, max_blocks, Hq, Hkv, BS, scale,       \
                     (bf16*)out)
  switch (Dh) {
    case 64: PF(64); break;
    case 80: PF(80); break;
    case 96: PF(96); break;
    case 128: PF(128); break;
    default: return -2;
  }
#undef PF
  return (int)hipGetLastError();
}
