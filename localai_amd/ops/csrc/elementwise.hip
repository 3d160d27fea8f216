// Memory-bound fused kernels: residual-add + RMSNorm/LayerNorm, RoPE + paged-KV append,
// gated activations, embedding gather with dequant, weight materialisation.
// Replaces ggml-cuda norm.cu / rope.cu / cpy.cu / unary.cu / binbcast.cu / getrows.cu
// ([external]).
//
// Every kernel that consumes a GEMM output takes a `Src`: either S fp32 split-K slabs
// (summed here, in the prologue -- the skinny GEMM never reduces) or one bf16 matrix
// (the hipBLASLt prefill path).  All loads are 16-byte vectors (guide §6 G13).
#include "qweight.h"

namespace la {

struct Src {
  const void* p;
  long slab;   // elements between split-K slabs
  int S;       // number of fp32 slabs; 0 => p is a single bf16 matrix
  const float* bias;  // optional per-column bias (length = row width), may be null
};

// Sum of up to SMAX slabs with every load issued before the first add: the slab index is
// clamped (duplicate loads hit L2) and masked, never branched on, so hipcc keeps all the
// loads in flight instead of waiting vmcnt(0) per slab (guide §5 trap (c)).
template <int SMAX>
LA_DEV float4 sum_slabs(const float* f, long slab, int S) {
  float4 b[SMAX];
#pragma unroll
  for (int i = 0; i < SMAX; ++i) b[i] = *(const float4*)(f + (long)min(i, S - 1) * slab);
  float4 a = b[0];
#pragma unroll
  for (int i = 1; i < SMAX; ++i) {
    const float m = (i < S) ? 1.f : 0.f;
    a.x = fmaf(m, b[i].x, a.x); a.y = fmaf(m, b[i].y, a.y);
    a.z = fmaf(m, b[i].z, a.z); a.w = fmaf(m, b[i].w, a.w);
  }
  return a;
}

LA_DEV void load4(const Src& s, long idx, int col, float v[4]) {
  if (s.S == 0) {
    const bf16x4 b = *(const bf16x4*)((const bf16*)s.p + idx);
    v[0] = (float)b[0]; v[1] = (float)b[1]; v[2] = (float)b[2]; v[3] = (float)b[3];
  } else {
    const float* f = (const float*)s.p + idx;
    float4 a;
    if (s.S == 1) a = *(const float4*)f;
    else if (s.S <= 2) a = sum_slabs<2>(f, s.slab, s.S);
    else if (s.S <= 4) a = sum_slabs<4>(f, s.slab, s.S);
    else if (s.S <= 8) a = sum_slabs<8>(f, s.slab, s.S);
    else {
      a = sum_slabs<8>(f, s.slab, min(s.S, 8));
      for (int i0 = 8; i0 < s.S; i0 += 8) {
        const float4 c = sum_slabs<8>(f + (long)i0 * s.slab, s.slab, min(s.S - i0, 8));
        a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
      }
    }
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  if (s.bias) {
    const float4 b = *(const float4*)(s.bias + col);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
}

// ------------------------------------------------------------------------------------
// residual[t] += sum(src[t]) (optional);  out[t] = norm(residual[t]) * w (+ b)
// mode 0 = RMSNorm, 1 = LayerNorm.  One workgroup per row, row cached in VGPRs: 256 threads,
// or 1024 when there are few rows (batch-1/-small decode: a single 256-thread workgroup
// reading the row plus up to 8 split-K slabs (~150 KB) is latency-bound at ~6.6 us; 16 waves
// keep 4x the loads in flight).
constexpr int NORM_T = 256;
constexpr int NORM_MAXV = 8;  // float4 per thread => D <= 8192

// IT = ceil(D/4 / NORM_T) float4 chunks per thread, a compile-time count so every load of
// the row (and of all its split-K slabs) is issued before the first use.
template <int IT, int NT = NORM_T>
__global__ __launch_bounds__(NT) void add_norm_kernel(float* __restrict__ residual, Src add, int has_add,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      bf16* __restrict__ out, int D, float eps, int mode,
                                                      float* __restrict__ out_f32) {
  __shared__ float red[NT / 64];
  const int t = blockIdx.x;
  const int nv = D >> 2;
  float* rrow = residual + (long)t * D;
  float v[IT][4];
  // the norm weight/bias loads do not depend on the reduction: issue them with the row loads so
  // their HBM round trip overlaps the residual/slab fetch instead of following the block barrier
  float4 ww[IT], bb[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = min(threadIdx.x + i * NT, nv - 1);  // clamped: loads never branch
    ww[i] = out ? *(const float4*)(w + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
    bb[i] = b ? *(const float4*)(b + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 r = *(const float4*)(rrow + 4 * c);
    v[i][0] = r.x; v[i][1] = r.y; v[i][2] = r.z; v[i][3] = r.w;
    if (has_add) {
      float a[4];
      load4(add, (long)t * D + 4 * c, 4 * c, a);
      v[i][0] += a[0]; v[i][1] += a[1]; v[i][2] += a[2]; v[i][3] += a[3];
    }
  }
  float s1 = 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nv) {
      if (has_add) *(float4*)(rrow + 4 * c) = make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
      s1 += (mode == 0) ? (v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3])
                        : (v[i][0] + v[i][1] + v[i][2] + v[i][3]);
    }
  }
  float mean = 0.f, rstd;
  if (mode == 0) {
    const float ss = block_sum<NT>(s1, red);
    rstd = rsqrtf(ss / (float)D + eps);
  } else {
    mean = block_sum<NT>(s1, red) / (float)D;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = threadIdx.x + i * NT;
      if (c < nv) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { const float d = v[i][j] - mean; s2 += d * d; }
      }
    }
    rstd = rsqrtf(block_sum<NT>(s2, red) / (float)D + eps);
  }
  if (!out) return;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nv) {
      float o[4] = {(v[i][0] - mean) * rstd * ww[i].x + bb[i].x, (v[i][1] - mean) * rstd * ww[i].y + bb[i].y,
                    (v[i][2] - mean) * rstd * ww[i].z + bb[i].z, (v[i][3] - mean) * rstd * ww[i].w + bb[i].w};
      bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      *(bf16x4*)(out + (long)t * D + 4 * c) = ob;
      if (out_f32) *(float4*)(out_f32 + (long)t * D + 4 * c) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// ------------------------------------------------------------------------------------
// add_norm + the MoE router of the same row (replaces add_norm + moe_router_kernel before a
// sparse-MoE FFN: one launch less per layer, the normed row never re-read).  The router reads the
// bf16-ROUNDED normed values, as the unfused router reads the bf16 activation; its logits are
// reduced across the block 8 experts at a time; thread 0 then takes softmax / top-k / renorm /
// EP remap exactly as moe_router_kernel (moe.hip).  E <= 64, 1024 threads, D <= 8192.
struct NormRouter {
  const float* wr;  // [E][D] fp32
  int E, topk, renorm;
  float scale;
  int ep_base, ep_local;
  int* ids;         // [T][topk]
  float* wts;       // [T * topk]
};

template <int IT>
__global__ __launch_bounds__(1024) void add_norm_router_kernel(float* __restrict__ residual, Src add, int has_add,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ b, bf16* __restrict__ out,
                                                               int D, float eps, int mode, NormRouter R) {
  constexpr int NT = 1024, NWV = NT / 64;
  __shared__ float red[NWV];
  __shared__ float rl[NWV][8];
  __shared__ float lg[64];
  const int t = blockIdx.x;
  const int nv = D >> 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* rrow = residual + (long)t * D;
  float v[IT][4];
  float4 ww[IT], bb[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = min(threadIdx.x + i * NT, nv - 1);
    ww[i] = *(const float4*)(w + 4 * c);
    bb[i] = b ? *(const float4*)(b + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 r = *(const float4*)(rrow + 4 * c);
    v[i][0] = r.x; v[i][1] = r.y; v[i][2] = r.z; v[i][3] = r.w;
    if (has_add) {
      float a[4];
      load4(add, (long)t * D + 4 * c, 4 * c, a);
      v[i][0] += a[0]; v[i][1] += a[1]; v[i][2] += a[2]; v[i][3] += a[3];
    }
  }
  float s1 = 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nv) {
      if (has_add) *(float4*)(rrow + 4 * c) = make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
      s1 += (mode == 0) ? (v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3])
                        : (v[i][0] + v[i][1] + v[i][2] + v[i][3]);
    }
  }
  float mean = 0.f, rstd;
  if (mode == 0) {
    rstd = rsqrtf(block_sum<NT>(s1, red) / (float)D + eps);
  } else {
    mean = block_sum<NT>(s1, red) / (float)D;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = threadIdx.x + i * NT;
      if (c < nv) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { const float d = v[i][j] - mean; s2 += d * d; }
      }
    }
    rstd = rsqrtf(block_sum<NT>(s2, red) / (float)D + eps);
  }
  float xb[IT][4];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = threadIdx.x + i * NT;
    const float o[4] = {(v[i][0] - mean) * rstd * ww[i].x + bb[i].x, (v[i][1] - mean) * rstd * ww[i].y + bb[i].y,
                        (v[i][2] - mean) * rstd * ww[i].z + bb[i].z, (v[i][3] - mean) * rstd * ww[i].w + bb[i].w};
    const bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) xb[i][j] = (c < nv) ? (float)ob[j] : 0.f;
    if (c < nv) *(bf16x4*)(out + (long)t * D + 4 * c) = ob;
  }
  // router logits, 8 experts per round: per-thread partial dots -> wave sums -> block sums
  for (int e0 = 0; e0 < R.E; e0 += 8) {
    float p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      p[u] = 0.f;
      const int e = min(e0 + u, R.E - 1);  // clamped: loads never branch (extra rows unused)
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int c = min(threadIdx.x + i * NT, nv - 1);
        const float4 wv = *(const float4*)(R.wr + (size_t)e * D + 4 * c);
        p[u] += xb[i][0] * wv.x + xb[i][1] * wv.y + xb[i][2] * wv.z + xb[i][3] * wv.w;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) p[u] += __shfl_xor(p[u], o, 64);
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < 8; ++u) rl[wave][u] = p[u];
    }
    __syncthreads();
    if (threadIdx.x < 8 && e0 + (int)threadIdx.x < R.E) {
      float sacc = 0.f;
#pragma unroll
      for (int wv = 0; wv < NWV; ++wv) sacc += rl[wv][threadIdx.x];
      lg[e0 + threadIdx.x] = sacc;
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  float mx = -INFINITY;
  for (int e = 0; e < R.E; ++e) mx = fmaxf(mx, lg[e]);
  float z = 0.0f;
  for (int e = 0; e < R.E; ++e) {
    lg[e] = __expf(lg[e] - mx);
    z += lg[e];
  }
  const float inv = 1.0f / z;
  unsigned long long taken = 0ull;  // E <= 64
  float sel[16];
  int sid[16];
  float sum = 0.0f;
  for (int k = 0; k < R.topk; ++k) {
    int best = -1;
    float bv = -1.0f;
    for (int e = 0; e < R.E; ++e) {
      if ((taken >> e) & 1ull) continue;
      if (lg[e] > bv) { bv = lg[e]; best = e; }
    }
    taken |= 1ull << best;
    sid[k] = best;
    sel[k] = bv * inv;
    sum += sel[k];
  }
  for (int k = 0; k < R.topk; ++k) {
    const float wv = (R.renorm ? sel[k] / sum : sel[k]) * R.scale;
    const int loc = sid[k] - R.ep_base;
    R.ids[t * R.topk + k] = (loc >= 0 && loc < R.ep_local) ? loc : R.ep_local;
    R.wts[t * R.topk + k] = wv;
  }
}

// ------------------------------------------------------------------------------------
// RoPE on q,k + append k,v into the paged cache.
// qkv row layout: [Hq*Dh | Hkv*Dh | Hkv*Dh].  K cache [num_blocks][Hkv][BS][Dh], V cache transposed
// in groups of 8 keys: [num_blocks][Hkv][BS/8][Dh][8] (bf16, see attention.hip).
// cos_sin: [max_pos][rot/2][2] f32 (host-precomputed table: guide App. B "trig tables").
// mode 0 = NORM (adjacent pairs, llama/mistral GGUF), 1 = NEOX (half-split, phi-2).
__global__ __launch_bounds__(256) void rope_kv_kernel(Src qkv, const int* __restrict__ pos,
                                                      const int* __restrict__ slots,
                                                      const float* __restrict__ cos_sin, int Hq, int Hkv,
                                                      int Dh, int rot, int mode, bf16* __restrict__ q_out,
                                                      bf16* __restrict__ kc, bf16* __restrict__ vc, int BS) {
  const int t = blockIdx.x;
  const int W = (Hq + 2 * Hkv) * Dh;
  const int p = pos[t];
  const int slot = slots ? slots[t] : -1;
  const long row = (long)t * W;
  const float* cs = cos_sin + (long)p * rot;  // rot/2 pairs x (cos, sin)
  // work unit = 4 consecutive elements of one head (Dh % 4 == 0)
  const int units = W >> 2;
  // one thread per 4-element unit; grid.y spreads a row over several workgroups so a
  // single decode token still fills more than one CU
  for (int u = blockIdx.y * blockDim.x + threadIdx.x; u < units; u += blockDim.x * gridDim.y) {
    const int col = u * 4;
    const int head = col / Dh, d0 = col - head * Dh;
    float v[4];
    load4(qkv, row + col, col, v);
    bf16* dst;
    if (head < Hq) {
      dst = q_out + ((long)t * Hq + head) * Dh + d0;
    } else if (head < Hq + Hkv) {
      if (slot < 0) continue;
      const int kh = head - Hq, blk = slot / BS, off = slot - blk * BS;
      dst = kc + (((long)blk * Hkv + kh) * BS + off) * Dh + d0;
    } else {
      if (slot < 0) continue;
      const int vh = head - Hq - Hkv, blk = slot / BS, off = slot - blk * BS;
      dst = vc + ((long)blk * Hkv + vh) * Dh * BS + ((off >> 3) * Dh + d0) * 8 + (off & 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[8 * j] = (bf16)v[j];
      continue;
    }
    if (mode == 0) {
      // pairs (d0,d0+1), (d0+2,d0+3)
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int pi = (d0 + j) >> 1;
        if (d0 + j < rot) {
          const float c = cs[2 * pi], s = cs[2 * pi + 1];
          const float x0 = v[j], x1 = v[j + 1];
          v[j] = x0 * c - x1 * s;
          v[j + 1] = x0 * s + x1 * c;
        }
      }
    } else {
      // NEOX: pair (i, i + rot/2) for i < rot/2.  Each unit of the first half handles both halves.
      const int half = rot >> 1;
      if (d0 < half) {
        float w2[4];
        load4(qkv, row + col + half, col + half, w2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pi = d0 + j;
          const float c = cs[2 * pi], s = cs[2 * pi + 1];
          const float x0 = v[j], x1 = w2[j];
          v[j] = x0 * c - x1 * s;
          w2[j] = x0 * s + x1 * c;
        }
        bf16x4 o2 = {(bf16)w2[0], (bf16)w2[1], (bf16)w2[2], (bf16)w2[3]};
        *(bf16x4*)(dst + half) = o2;
      } else if (d0 < rot) {
        continue;  // written by its partner unit
      }
    }
    bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *(bf16x4*)dst = o;
  }
}

// Fast path of rope_kv: NORM (adjacent-pair) rotary over the whole head, DH in {64, 128}.  One
// thread per 8 consecutive elements of a row (16-byte source loads, two float4 cos/sin loads,
// 16-byte q / k stores; the 8 V values of a unit land in one 128-byte line of the grouped-
// transposed V page).  The block's token position and slot are read once.
LA_DEV void load8(const Src& s, long idx, int col, float v[8]) {
  if (s.S == 0) {
    const bf16x8 b = *(const bf16x8*)((const bf16*)s.p + idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
    if (s.bias) {
      const float4 b0 = *(const float4*)(s.bias + col), b1 = *(const float4*)(s.bias + col + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
  } else {
    load4(s, idx, col, v);
    load4(s, idx + 4, col + 4, v + 4);
  }
}

template <int DH>
__global__ __launch_bounds__(256) void rope_kv8_kernel(Src qkv, const int* __restrict__ pos,
                                                       const int* __restrict__ slots,
                                                       const float* __restrict__ cos_sin, int Hq, int Hkv,
                                                       bf16* __restrict__ q_out, bf16* __restrict__ kc,
                                                       bf16* __restrict__ vc, int BS) {
  const int t = blockIdx.x;
  const int W = (Hq + 2 * Hkv) * DH;
  const int p = pos[t];
  const int slot = slots ? slots[t] : -1;
  const long row = (long)t * W;
  const float* cs = cos_sin + (long)p * DH;  // DH/2 pairs x (cos, sin)
  const int units = W >> 3;
  const int u = blockIdx.y * blockDim.x + threadIdx.x;
  if (u >= units) return;
  const int col = u * 8;
  const int head = col / DH, d0 = col - head * DH;
  float v[8];
  load8(qkv, row + col, col, v);
  if (head >= Hq + Hkv) {  // v: no rotation
    if (slot < 0) return;
    const int vh = head - Hq - Hkv, blk = slot / BS, off = slot - blk * BS;
    bf16* dst = vc + ((long)blk * Hkv + vh) * DH * BS + ((off >> 3) * DH + d0) * 8 + (off & 7);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[8 * j] = (bf16)v[j];
    return;
  }
  const float4 c0 = *(const float4*)(cs + d0), c1 = *(const float4*)(cs + d0 + 4);  // pairs d0/2 .. d0/2+3
  const float cc[4] = {c0.x, c0.z, c1.x, c1.z}, sn[4] = {c0.y, c0.w, c1.y, c1.w};
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = v[2 * j], x1 = v[2 * j + 1];
    o[2 * j] = (bf16)(x0 * cc[j] - x1 * sn[j]);
    o[2 * j + 1] = (bf16)(x0 * sn[j] + x1 * cc[j]);
  }
  if (head < Hq) {
    *(bf16x8*)(q_out + ((long)t * Hq + head) * DH + d0) = o;
  } else if (slot >= 0) {
    const int kh = head - Hq, blk = slot / BS, off = slot - blk * BS;
    *(bf16x8*)(kc + (((long)blk * Hkv + kh) * BS + off) * DH + d0) = o;
  }
}

// ------------------------------------------------------------------------------------
// Activations.  mode 0: SwiGLU  out[t][i] = silu(x[t][i]) * x[t][F+i]   (src width 2F)
//               mode 1: GELU(tanh) out[t][i] = gelu(x[t][i])             (src width F)
//               mode 2: GELU-quick (CLIP)  x * sigmoid(1.702 x)
//               mode 3: GeGLU (Gemma)  out[t][i] = gelu(x[t][i]) * x[t][F+i]   (src width 2F)
LA_DEV float gelu_tanh(float x) { return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))); }

__global__ __launch_bounds__(256) void act_kernel(Src src, bf16* __restrict__ out, int F, int mode) {
  const int t = blockIdx.y;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (c >= F) return;
  const int W = (mode == 0 || mode == 3) ? 2 * F : F;
  float a[4];
  load4(src, (long)t * W + c, c, a);
  float o[4];
  if (mode == 0 || mode == 3) {
    float b[4];
    load4(src, (long)t * W + F + c, F + c, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (mode == 0 ? silu(a[j]) : gelu_tanh(a[j])) * b[j];
  } else if (mode == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = a[j];
      o[j] = 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = a[j] / (1.f + __expf(-1.702f * a[j]));
  }
  bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
  *(bf16x4*)(out + (long)t * F + c) = ob;
}

// bf16 source without bias (the hipBLASLt gate|up output at batch decode / prefill): 8 elements
// per thread so every load and store is a 16-byte vector (halves the memory instructions of
// act_kernel, which moves 4-wide 8-byte vectors)
__global__ __launch_bounds__(256) void act8_kernel(const bf16* __restrict__ src, bf16* __restrict__ out, int F,
                                                   int mode) {
  const int t = blockIdx.y;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c >= F) return;
  const int W = (mode == 0 || mode == 3) ? 2 * F : F;
  const bf16x8 a = *(const bf16x8*)(src + (long)t * W + c);
  bf16x8 ob;
  if (mode == 0) {
    const bf16x8 b = *(const bf16x8*)(src + (long)t * W + F + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) ob[j] = (bf16)(silu((float)a[j]) * (float)b[j]);
  } else if (mode == 3) {
    const bf16x8 b = *(const bf16x8*)(src + (long)t * W + F + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) ob[j] = (bf16)(gelu_tanh((float)a[j]) * (float)b[j]);
  } else if (mode == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = (float)a[j];
      ob[j] = (bf16)(0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = (float)a[j];
      ob[j] = (bf16)(x / (1.f + __expf(-1.702f * x)));
    }
  }
  *(bf16x8*)(out + (long)t * F + c) = ob;
}

// sum split-K slabs (+bias) -> f32 or bf16 matrix [T][N]
__global__ __launch_bounds__(256) void reduce_slabs_kernel(Src src, int N, float* __restrict__ out_f32,
                                                           bf16* __restrict__ out_bf16) {
  const int t = blockIdx.y;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (c >= N) return;
  float a[4];
  load4(src, (long)t * N + c, c, a);
  if (out_f32) *(float4*)(out_f32 + (long)t * N + c) = make_float4(a[0], a[1], a[2], a[3]);
  if (out_bf16) {
    bf16x4 ob = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
    *(bf16x4*)(out_bf16 + (long)t * N + c) = ob;
  }
}

// ------------------------------------------------------------------------------------
// Embedding gather with on-the-fly dequant: out[t][:] = W[tok[t]][:] * scale   (f32 out)
template <int FMT>
__global__ __launch_bounds__(256) void embed_kernel(QW w, const int* __restrict__ tok, float* __restrict__ out,
                                                    float scale) {
  const int t = blockIdx.x;
  const int n = tok[t];
  for (int k = threadIdx.x * 8; k < w.K; k += blockDim.x * 8) {
    float v[8];
    deq8_natural<FMT>(w, n, k, v);
    float* o = out + (long)t * w.K + k;
    *(float4*)o = make_float4(v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale);
    *(float4*)(o + 4) = make_float4(v[4] * scale, v[5] * scale, v[6] * scale, v[7] * scale);
  }
}

// W (any format) -> bf16 [N][K]   (prefill path keeps an HBM-resident bf16 copy)
template <int FMT>
__global__ __launch_bounds__(256) void dequant_kernel(QW w, bf16* __restrict__ out, long total8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total8) return;
  const int kc = w.K >> 3;
  const int n = (int)(i / kc), k = (int)(i - (long)n * kc) * 8;
  float v[8];
  deq8_natural<FMT>(w, n, k, v);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  *(bf16x8*)(out + (long)n * w.K + k) = o;
}

// ------------------------------------------------------------------------------------
// Row gather with a fill row: out[t] = idx[t] >= 0 ? src[idx[t]] : fill  (any 2-byte or 4-byte
// element type, rows of C elements, 16-byte vectors when C allows).  The LLaVA-1.6 anyres image
// assembly (base tile, grid tiles permuted to row-major, spatial unpadding, an
// image_newline row after every feature row) is one precomputed index vector and this one launch,
// where the torch path ran a permute copy, a slice, an expand + cat and a final cat.
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* __restrict__ src, const long* __restrict__ idx,
                                                          const uint8_t* __restrict__ fill, uint8_t* __restrict__ out,
                                                          long row_bytes) {
  const long t = blockIdx.x;
  const long i = idx[t];
  const uint8_t* s = i >= 0 ? src + i * row_bytes : fill;
  uint8_t* d = out + t * row_bytes;
  if ((row_bytes & 15) == 0) {
    for (long b = (long)threadIdx.x * 16; b < row_bytes; b += 256 * 16) *(u32x4*)(d + b) = *(const u32x4*)(s + b);
  } else {
    for (long b = threadIdx.x; b < row_bytes; b += 256) d[b] = s[b];
  }
}

}  // namespace la

// C ABI ------------------------------------------------------------------------------
using la::Src;

extern "C" int la_gather_rows(const void* src, const long* idx, long T, const void* fill, void* out, long row_bytes,
                               void* stream) {
  if (T < 1 || row_bytes < 1 || !src || !idx || !out) return -1;
  hipLaunchKernelGGL(la::gather_rows_kernel, dim3(T), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src, idx,
                     (const uint8_t*)(fill ? fill : src), (uint8_t*)out, row_bytes);
  return (int)hipGetLastError();
}

extern "C" int la_add_norm(void* residual, const void* add_p, long add_slab, int add_S, const void* add_bias,
                           int has_add, const void* w, const void* b, void* out, int T, int D, float eps,
                           int mode, void* out_f32, void* stream) {
  if ((D & 3) || D > la::NORM_T * la::NORM_MAXV * 4) return -1;
  Src s{add_p, add_slab, add_S, (const float*)add_bias};
  const int it = (D / 4 + la::NORM_T - 1) / la::NORM_T;
#define LA_NORM_CASE(I)                                                                                     \
  case I:                                                                                                   \
    hipLaunchKernelGGL(la::add_norm_kernel<I>, dim3(T), dim3(la::NORM_T), 0, (hipStream_t)stream,          \
                       (float*)residual, s, has_add, (const float*)w, (const float*)b, (bf16*)out, D, eps,  \
                       mode, (float*)out_f32);                                                            \
    break;
  // one 1024-thread workgroup per row whenever the row fits two float4 per thread: a 256-row
  // decode batch then puts 16 waves on every CU instead of 4 (the 256-thread variants below are
  // left for very wide rows)
  if (D <= 1024 * 4 * 2) {
    const int it4 = (D / 4 + 1023) / 1024;
    if (it4 == 1)
      hipLaunchKernelGGL((la::add_norm_kernel<1, 1024>), dim3(T), dim3(1024), 0, (hipStream_t)stream,
                         (float*)residual, s, has_add, (const float*)w, (const float*)b, (bf16*)out, D, eps, mode,
                         (float*)out_f32);
    else
      hipLaunchKernelGGL((la::add_norm_kernel<2, 1024>), dim3(T), dim3(1024), 0, (hipStream_t)stream,
                         (float*)residual, s, has_add, (const float*)w, (const float*)b, (bf16*)out, D, eps, mode,
                         (float*)out_f32);
    return (int)hipGetLastError();
  }
  switch (it) {
    LA_NORM_CASE(1) LA_NORM_CASE(2) LA_NORM_CASE(3) LA_NORM_CASE(4)
    LA_NORM_CASE(5) LA_NORM_CASE(6) LA_NORM_CASE(7) LA_NORM_CASE(8)
    default: return -1;
  }
#undef LA_NORM_CASE
  return (int)hipGetLastError();
}

// add_norm (RMS / LayerNorm, always writing the bf16 row) + the MoE router of every row; -1 when
// the shape is outside the fused kernel (caller runs add_norm + la_moe_router)
extern "C" int la_add_norm_router(void* residual, const void* add_p, long add_slab, int add_S, const void* add_bias,
                                  int has_add, const void* w, const void* b, void* out, int T, int D, float eps,
                                  int mode, const float* wr, int E, int topk, int renorm, float scale, int ep_base,
                                  int ep_local, int* ids, float* wts, void* stream) {
  if ((D & 3) || D > 1024 * 4 * 2 || T < 1 || !out || !wr || !ids || !wts || E < 1 || E > 64 || topk < 1 ||
      topk > 16 || topk > E)
    return -1;
  Src s{add_p, add_slab, add_S, (const float*)add_bias};
  la::NormRouter R{wr, E, topk, renorm, scale, ep_base, ep_local, ids, wts};
  if ((D / 4 + 1023) / 1024 == 1)
    hipLaunchKernelGGL((la::add_norm_router_kernel<1>), dim3(T), dim3(1024), 0, (hipStream_t)stream, (float*)residual,
                       s, has_add, (const float*)w, (const float*)b, (bf16*)out, D, eps, mode, R);
  else
    hipLaunchKernelGGL((la::add_norm_router_kernel<2>), dim3(T), dim3(1024), 0, (hipStream_t)stream, (float*)residual,
                       s, has_add, (const float*)w, (const float*)b, (bf16*)out, D, eps, mode, R);
  return (int)hipGetLastError();
}

extern "C" int la_rope_kv(const void* qkv_p, long slab, int S, const void* bias, const int* pos, const int* slots,
                          const float* cos_sin, int T, int Hq, int Hkv, int Dh, int rot, int mode, void* q_out,
                          void* kc, void* vc, int BS, void* stream) {
  if ((Dh & 3) || (rot & 3) || rot > Dh) return -1;
  Src s{qkv_p, slab, S, (const float*)bias};
  if (mode == 0 && rot == Dh && (Dh == 128 || Dh == 64) && (BS & 7) == 0) {
    const int units8 = (Hq + 2 * Hkv) * Dh / 8;
    dim3 grid(T, (units8 + 255) / 256);
    if (Dh == 128)
      hipLaunchKernelGGL(la::rope_kv8_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, s, pos, slots, cos_sin,
                         Hq, Hkv, (bf16*)q_out, (bf16*)kc, (bf16*)vc, BS);
    else
      hipLaunchKernelGGL(la::rope_kv8_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, s, pos, slots, cos_sin,
                         Hq, Hkv, (bf16*)q_out, (bf16*)kc, (bf16*)vc, BS);
    return (int)hipGetLastError();
  }
  const int units = (Hq + 2 * Hkv) * Dh / 4;
  hipLaunchKernelGGL(la::rope_kv_kernel, dim3(T, (units + 255) / 256), dim3(256), 0, (hipStream_t)stream, s, pos,
                     slots, cos_sin, Hq,
                     Hkv, Dh, rot, mode, (bf16*)q_out, (bf16*)kc, (bf16*)vc, BS);
  return (int)hipGetLastError();
}

extern "C" int la_act(const void* p, long slab, int S, const void* bias, void* out, int T, int F, int mode,
                      void* stream) {
  if ((F & 3) || mode < 0 || mode > 3) return -1;
  if (S == 0 && bias == nullptr && (F & 7) == 0 && ((uintptr_t)p & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    dim3 grid((F / 8 + 255) / 256, T);
    hipLaunchKernelGGL(la::act8_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)p, (bf16*)out, F,
                       mode);
    return (int)hipGetLastError();
  }
  Src s{p, slab, S, (const float*)bias};
  dim3 grid((F / 4 + 255) / 256, T);
  hipLaunchKernelGGL(la::act_kernel, grid, dim3(256), 0, (hipStream_t)stream, s, (bf16*)out, F, mode);
  return (int)hipGetLastError();
}

extern "C" int la_reduce_slabs(const void* p, long slab, int S, const void* bias, int T, int N, void* out_f32,
                               void* out_bf16, void* stream) {
  if (N & 3) return -1;
  Src s{p, slab, S, (const float*)bias};
  dim3 grid((N / 4 + 255) / 256, T);
  hipLaunchKernelGGL(la::reduce_slabs_kernel, grid, dim3(256), 0, (hipStream_t)stream, s, N, (float*)out_f32,
                     (bf16*)out_bf16);
  return (int)hipGetLastError();
}

extern "C" int la_embed(int fmt, const void* p0, const void* p1, const void* p2, const void* p3, int N, int K,
                        const int* tok, int T, void* out, float scale, void* stream) {
  using namespace la;
  if (K & 7) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)p2, (const uint8_t*)p3, N, K};
  hipStream_t st = (hipStream_t)stream;
  switch (fmt) {
    case FMT_Q4_K: hipLaunchKernelGGL(embed_kernel<FMT_Q4_K>, dim3(T), dim3(256), 0, st, w, tok, (float*)out, scale); break;
    case FMT_Q6_K: hipLaunchKernelGGL(embed_kernel<FMT_Q6_K>, dim3(T), dim3(256), 0, st, w, tok, (float*)out, scale); break;
    case FMT_Q8_0: hipLaunchKernelGGL(embed_kernel<FMT_Q8_0>, dim3(T), dim3(256), 0, st, w, tok, (float*)out, scale); break;
    case FMT_BF16: hipLaunchKernelGGL(embed_kernel<FMT_BF16>, dim3(T), dim3(256), 0, st, w, tok, (float*)out, scale); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int la_dequant(int fmt, const void* p0, const void* p1, const void* p2, const void* p3, int N, int K,
                          void* out, void* stream) {
  using namespace la;
  if (K & 7) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)p2, (const uint8_t*)p3, N, K};
  const long total8 = (long)N * (K >> 3);
  dim3 grid((unsigned)((total8 + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  switch (fmt) {
    case FMT_Q4_K: hipLaunchKernelGGL(dequant_kernel<FMT_Q4_K>, grid, dim3(256), 0, st, w, (bf16*)out, total8); break;
    case FMT_Q6_K: hipLaunchKernelGGL(dequant_kernel<FMT_Q6_K>, grid, dim3(256), 0, st, w, (bf16*)out, total8); break;
    case FMT_Q8_0: hipLaunchKernelGGL(dequant_kernel<FMT_Q8_0>, grid, dim3(256), 0, st, w, (bf16*)out, total8); break;
    case FMT_BF16: hipLaunchKernelGGL(dequant_kernel<FMT_BF16>, grid, dim3(256), 0, st, w, (bf16*)out, total8); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}
