// Batch-1..4 decode GEMV on packed int8 dot products (v_dot4_i32_i8), Q4_K and Q6_K weights.
//
// Why not MFMA here: at M <= 4 the bf16 MFMA path (gemm_skinny.hip) spends ~4.35 VALU lane-ops
// per weight dequantising to bf16 (profiles/decode_gemv_study.md, skinny_pmc.md) and wastes
// 15/16 of every 16x16 tile.  This kernel instead quantises the activation row once per
// workgroup to int8 with one scale per 32 elements (ggml's q8_1 activation blocks, which is
// what the reference's GPU build feeds its k-quant mmvq dot products) and multiplies the weights' raw
// 4-/6-bit codes with 4-way int8 dots: ~1 VALU op per weight, so the kernel is left to stream.
//
// Work mapping (wave64): a row's super-block is 128 contiguous quant bytes, read by 8 adjacent
// lanes x 16 B (fully used 128 B runs: 5.0 TB/s class access pattern, decode_gemv_study.md §1).
// A wave covers 8 rows per load instruction, RS row slots per wave, 4 waves per workgroup,
// so a workgroup owns 64 rows and one K split; grid.y = split-K, partials go to fp32 slabs
// [S][M][ldo] which the consumer (add_norm / rope_kv / act) sums -- the same contract as the
// other GEMMs (ops.Partial).
//
// Activation image in LDS (per row m of x, for this split's K range):
//   xq  int8 [kper]       q = round(x * 127 / absmax_32)   (ggml q8_1 blocks of 32)
//   bs  int32 [kper/16]   sum of q over each 16-run (Q4_K min term, Q6_K -32 offset)
//   dx  f32  [kper/32]    absmax_32 / 127
// Weight side: Q4_K uses the qs plane plus two planes made at load time (ops.QWeight.from_raw):
//   scm u8 [N][K/256][16]  (sc0,m0,sc1,m1, sc2,m2,...): the 6-bit scales/mins unpacked
//   dd  u8 [N][K/256][4]   f16 d, f16 dmin
// Q6_K uses its ql / qh / sc / d planes unchanged.
// Reference semantics: ggml dequantize_row_q4_K / q6_K and ggml_vec_dot_q4_K_q8_K
// [external, llama.cpp @ d5cb868 ggml/src/ggml-quants.c]; used for the decode MUL_MAT of
// SURVEY.md §2.8 K5 (mmvq.cu in the reference build).
// One launch may cover up to GV_SEGS weights of different formats sharing K (e.g. a Q4_K q|k
// and a Q6_K v): grid.x walks the row blocks of all segments, each block branches (uniformly)
// on its segment's format, and writes its columns side by side into the same slabs.
//
// The first super-block of weights is requested BEFORE the activation image is built, so the
// weight stream's first HBM round trip overlaps the x load / quantisation prologue.
#include "qweight.h"

namespace la {

constexpr int GV_THREADS = 256;
// row slots (of 8 rows) per wave: 2 by default, 1 or 4 in the tuning variants (VAR bits 2/3)
template <int VAR>
constexpr int gv_rs() { return (VAR & 4) ? 1 : ((VAR & 8) ? 4 : 2); }
constexpr int GV_SEGS = 3;

struct GVArgs {
  QW w[GV_SEGS];
  int fmt[GV_SEGS];
  int blk_end[GV_SEGS];  // exclusive prefix sum of row blocks
  int col0[GV_SEGS];     // first output column of each segment
  int nseg;
};


LA_DEV int dot4(uint32_t a, uint32_t b, int c) { return __builtin_amdgcn_sdot4((int)a, (int)b, c, false); }

template <int NT>
LA_DEV u32x4 ldg16(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load((const u32x4*)p);
  else return *(const u32x4*)p;
}

// Optional fused-activation source: instead of a bf16 x, the GEMV reads the fp32 split-K
// slabs of the preceding gate|up GEMM and applies the activation while quantising, so the
// decode MLP runs gate_up GEMV -> down GEMV with no activation launch in between
// ("fused into the GEMM" -- here into the consumer's prologue).
//   mode 0: x = silu(g) * u with g = row[k], u = row[F + k] (SwiGLU, row width 2F)
//   mode 1: x = gelu_tanh(row[k]);  mode 2: x = quick_gelu(row[k])      (row width F)
//   mode 3: x = gelu_tanh(g) * u (GeGLU, row width 2F)
//   mode 4 (GV_NORM): x = rmsnorm(res + sum(slabs) + bias) * nw over the whole row (width F = K):
//     the residual-add + RMSNorm of the layer boundary (K2 + K14) folded into the consuming GEMV,
//     so a batch-1/2 decode step has no add_norm launch between the down projection and the next
//     q|k|v GEMV.  Every workgroup recomputes the row statistics (one 16-32 KiB row from L2, its
//     loads in flight together with the first weight super-blocks); workgroup (0, 0) writes the
//     updated residual to res_out (a different buffer: the other workgroups still read res).
constexpr int GV_NORM = 4;
constexpr int GV_NORM_IT = 8;  // float4 per thread per row: K <= 8192

struct GVAct {
  const float* p;      // [S][M][W] fp32 slabs, W = 2F (mode 0) or F; null = plain bf16 x
  long slab;           // elements between slabs
  int S;
  const float* bias;   // optional per-column bias of the gate|up output (length W)
  int mode, F;
  float scale = 1.f;   // x multiplied by this (an MoE routing weight: down(w x) = w down(x))
  const float* res = nullptr;  // GV_NORM: fp32 residual [M][F]
  float* res_out = nullptr;    // GV_NORM: residual + add, [M][F] (null: not written)
  const float* nw = nullptr;   // GV_NORM: norm weight [F]
  float eps = 0.f;
};

// x prologues that read fp32 sources (act / norm) issue the first weight loads before them
LA_DEV bool gv_late(const GVAct& a) { return a.p != nullptr; }

// every slab load issued before the first add (clamped index, masked add: no per-slab wait)
LA_DEV float4 gv_sum_slabs(const GVAct& a, long idx, int col) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s0 = 0; s0 < a.S; s0 += 4) {
    float4 b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = *(const float4*)(a.p + (long)min(s0 + i, a.S - 1) * a.slab + idx);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float m = (s0 + i < a.S) ? 1.f : 0.f;
      v.x = fmaf(m, b[i].x, v.x); v.y = fmaf(m, b[i].y, v.y); v.z = fmaf(m, b[i].z, v.z); v.w = fmaf(m, b[i].w, v.w);
    }
  }
  if (a.bias) {
    const float4 b = *(const float4*)(a.bias + col);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  return v;
}

LA_DEV float gv_act1(float x, int mode) {
  if (mode == 1) return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x)));
  return x / (1.f + __expf(-1.702f * x));
}

// x[m, k .. k+3] from the activation source (in fp32, never rounded to bf16)
LA_DEV void gv_act_x(const GVAct& a, int m, int k, float v[4]) {
  const bool glu = a.mode == 0 || a.mode == 3;
  const long W = glu ? 2L * a.F : (long)a.F;
  const float4 g = gv_sum_slabs(a, m * W + k, k);
  if (a.mode == 0) {
    const float4 u = gv_sum_slabs(a, m * W + a.F + k, a.F + k);
    v[0] = silu(g.x) * u.x; v[1] = silu(g.y) * u.y; v[2] = silu(g.z) * u.z; v[3] = silu(g.w) * u.w;
  } else if (a.mode == 3) {
    const float4 u = gv_sum_slabs(a, m * W + a.F + k, a.F + k);
    v[0] = gv_act1(g.x, 1) * u.x; v[1] = gv_act1(g.y, 1) * u.y; v[2] = gv_act1(g.z, 1) * u.z;
    v[3] = gv_act1(g.w, 1) * u.w;
  } else {
    v[0] = gv_act1(g.x, a.mode); v[1] = gv_act1(g.y, a.mode); v[2] = gv_act1(g.z, a.mode); v[3] = gv_act1(g.w, a.mode);
  }
}

// Quantise x[m, k0 : k0+kper] into the LDS image (ggml q8_1 granularity: one scale per 32).
// Wave w handles super-blocks w, w+4, ...; lane l owns elements 4l..4l+3 of the super-block,
// so 8 lanes share a 32-block and 4 lanes a 16-run.
// One 32-block of x (4 elements per lane, 8 lanes per block) into the int8 image.
LA_DEV void gv_quant4(float v0, float v1, float v2, float v3, int l, int8_t* q, int* b, float* d) {
  const float amax = group_max<8>(fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
  const float inv = amax > 0.f ? 127.f / amax : 0.f;
  const int q0 = __float2int_rn(v0 * inv), q1 = __float2int_rn(v1 * inv);
  const int q2 = __float2int_rn(v2 * inv), q3 = __float2int_rn(v3 * inv);
  *(uint32_t*)(q + 4 * l) = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
                            ((uint32_t)(q3 & 0xFF) << 24);
  int s = q0 + q1 + q2 + q3;
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  if ((l & 3) == 0) b[l >> 2] = s;
  if ((l & 7) == 0) d[l >> 3] = amax / 127.f;
}

// GV_NORM prologue.  Thread (wave w, lane l) holds float4 chunks c = tid + 256 i of the row, which
// is exactly super-block sb = w + 4 i, elements 4l..4l+3 -- the quantiser's own mapping -- so the
// normed values go from registers to the int8 image with no LDS round trip; only the row's sum of
// squares crosses the waves.
template <int MT>
LA_DEV void norm_quantize_x(const GVAct& a, int M, int k0, int kper, int8_t* xq, int* bs, float* dx) {
  __shared__ float red[MT][GV_THREADS / 64];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int K = a.F, nv = K >> 2;
  const bool wr = a.res_out && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;
  float v[MT][GV_NORM_IT][4];
  float4 wgt[GV_NORM_IT];
#pragma unroll
  for (int i = 0; i < GV_NORM_IT; ++i) {
    const int c = min(tid + GV_THREADS * i, nv - 1);
    wgt[i] = *(const float4*)(a.nw + 4 * c);
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < GV_NORM_IT; ++i) {
      const int c = tid + GV_THREADS * i;
      v[m][i][0] = v[m][i][1] = v[m][i][2] = v[m][i][3] = 0.f;
      if (m < M && c < nv) {
        float4 r = *(const float4*)(a.res + (long)m * K + 4 * c);
        if (a.p) {
          const float4 s = gv_sum_slabs(a, (long)m * K + 4 * c, 4 * c);
          r.x += s.x; r.y += s.y; r.z += s.z; r.w += s.w;
        } else if (a.bias) {
          const float4 b = *(const float4*)(a.bias + 4 * c);
          r.x += b.x; r.y += b.y; r.z += b.z; r.w += b.w;
        }
        if (wr) *(float4*)(a.res_out + (long)m * K + 4 * c) = r;
        v[m][i][0] = r.x; v[m][i][1] = r.y; v[m][i][2] = r.z; v[m][i][3] = r.w;
        ss += r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (l == 0) red[m][wv] = ss;
  }
  __syncthreads();
  const int sb_lo = k0 >> 8, sb_hi = (k0 + kper) >> 8;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m >= M) break;
    const float rstd = rsqrtf((red[m][0] + red[m][1] + red[m][2] + red[m][3]) / (float)K + a.eps);
#pragma unroll
    for (int i = 0; i < GV_NORM_IT; ++i) {
      const int sb = wv + 4 * i;  // uniform per wave
      if (sb < sb_lo || sb >= sb_hi) continue;
      const int ls = sb - sb_lo;
      gv_quant4(v[m][i][0] * rstd * wgt[i].x, v[m][i][1] * rstd * wgt[i].y, v[m][i][2] * rstd * wgt[i].z,
                v[m][i][3] * rstd * wgt[i].w, l, xq + m * kper + ls * 256, bs + m * (kper >> 4) + ls * 16,
                dx + m * (kper >> 5) + ls * 8);
    }
  }
}

template <int MT, int NM = 0>
LA_DEV void quantize_x(const bf16* X, int ldx, const GVAct& act, int M, int k0, int kper, int8_t* xq, int* bs,
                       float* dx) {
  if constexpr (NM && MT <= 2) {  // its own kernel instantiation (VAR bit 5): the row lives in VGPRs
    norm_quantize_x<MT>(act, M, k0, kper, xq, bs, dx);
    return;
  }
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nsb = kper >> 8;
  for (int m = 0; m < MT; ++m) {
    if (m >= M) break;
    const bf16* xr = X + (size_t)m * ldx + k0;
    int8_t* q = xq + m * kper;
    int* b = bs + m * (kper >> 4);
    float* d = dx + m * (kper >> 5);
    for (int sb = wv; sb < nsb; sb += 4) {
      float v0, v1, v2, v3;
      if (act.p) {
        float v[4];
        gv_act_x(act, m, k0 + sb * 256 + 4 * l, v);
        v0 = v[0] * act.scale; v1 = v[1] * act.scale; v2 = v[2] * act.scale; v3 = v[3] * act.scale;
      } else {
        const u32x2 raw = *(const u32x2*)(xr + sb * 256 + 4 * l);
        v0 = bf16_bits_to_f(raw.x & 0xFFFFu); v1 = bf16_bits_to_f(raw.x >> 16);
        v2 = bf16_bits_to_f(raw.y & 0xFFFFu); v3 = bf16_bits_to_f(raw.y >> 16);
      }
      const float amax = group_max<8>(fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
      const float inv = amax > 0.f ? 127.f / amax : 0.f;
      const int q0 = __float2int_rn(v0 * inv), q1 = __float2int_rn(v1 * inv);
      const int q2 = __float2int_rn(v2 * inv), q3 = __float2int_rn(v3 * inv);
      const uint32_t packed = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) |
                              ((uint32_t)(q2 & 0xFF) << 16) | ((uint32_t)(q3 & 0xFF) << 24);
      *(uint32_t*)(q + sb * 256 + 4 * l) = packed;
      int s = q0 + q1 + q2 + q3;
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if ((l & 3) == 0) b[sb * 16 + (l >> 2)] = s;
      if ((l & 7) == 0) d[sb * 8 + (l >> 3)] = amax / 127.f;
    }
  }
}

// Register-staged variant of quantize_x for the common decode case (bf16 x, at most GV_XI
// (row, super-block) items per thread): x_issue() only issues the loads, so the caller can put
// the first weight loads behind them and the two HBM round trips overlap; x_commit() waits for
// x alone (loads retire in issue order) and writes the LDS image.
constexpr int GV_XI = 4;

template <int MT>
LA_DEV bool x_staged_ok(const GVAct& act, int kper) {
  return !act.p && MT * (((kper >> 8) + 3) >> 2) <= GV_XI;
}

template <int MT>
LA_DEV void x_issue(const bf16* X, int ldx, int M, int k0, int kper, u32x2 (&xr)[GV_XI]) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nsb = kper >> 8, per = (nsb + 3) >> 2;
#pragma unroll
  for (int it = 0; it < GV_XI; ++it) {
    const int m = it / per, sb = wv + 4 * (it - m * per);
    const bool ok = m < M && m < MT && sb < nsb;
    xr[it] = *(const u32x2*)(X + (size_t)(ok ? m : 0) * ldx + k0 + (ok ? sb : 0) * 256 + 4 * l);
  }
}

template <int MT>
LA_DEV void x_commit(int M, int kper, const u32x2 (&xr)[GV_XI], int8_t* xq, int* bs, float* dx) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nsb = kper >> 8, per = (nsb + 3) >> 2;
#pragma unroll
  for (int it = 0; it < GV_XI; ++it) {
    const int m = it / per, sb = wv + 4 * (it - m * per);
    if (m >= M || m >= MT || sb >= nsb) continue;
    const float v0 = bf16_bits_to_f(xr[it].x & 0xFFFFu), v1 = bf16_bits_to_f(xr[it].x >> 16);
    const float v2 = bf16_bits_to_f(xr[it].y & 0xFFFFu), v3 = bf16_bits_to_f(xr[it].y >> 16);
    const float amax = group_max<8>(fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
    const float inv = amax > 0.f ? 127.f / amax : 0.f;
    const int q0 = __float2int_rn(v0 * inv), q1 = __float2int_rn(v1 * inv);
    const int q2 = __float2int_rn(v2 * inv), q3 = __float2int_rn(v3 * inv);
    *(uint32_t*)(xq + m * kper + sb * 256 + 4 * l) = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) |
                                                    ((uint32_t)(q2 & 0xFF) << 16) | ((uint32_t)(q3 & 0xFF) << 24);
    int sm = q0 + q1 + q2 + q3;
    sm += __shfl_xor(sm, 1, 64);
    sm += __shfl_xor(sm, 2, 64);
    if ((l & 3) == 0) bs[m * (kper >> 4) + sb * 16 + (l >> 2)] = sm;
    if ((l & 7) == 0) dx[m * (kper >> 5) + sb * 8 + (l >> 3)] = amax / 127.f;
  }
}

// Fused RoPE + paged-KV append epilogue for the decode q|k|v GEMV (split-K 1): the GEMV's
// output row n of the fused [q | k | v] projection is complete in the 8 lanes of its row group,
// and NORM rotary pairs adjacent rows (2i, 2i+1) = adjacent row groups of one wave (lane ^ 8),
// so the rotation is one shuffle.  q goes to q_out (bf16, [M][Hq][Dh]), k / v of token m to its
// cache slot (V in the grouped-transposed page layout of attention.hip).  Replaces the rope_kv
// launch of a batch-1/2 decode step (SURVEY §2.8 K9 + K10 fused into K5).
struct GVRope {
  const int* pos;        // [M] rotary position of each token
  const int* slots;      // [M] cache slot (< 0: no append)
  const float* cos_sin;  // [max_pos][Dh/2][2]
  bf16* q_out;           // null: plain fp32 slab epilogue
  bf16* kc;
  bf16* vc;
  int Hq, Hkv, Dh, BS;
};

template <int MT, int RS>
LA_DEV void gv_store(const float (&acc)[MT][RS], const int (&n)[RS], int N, int M, int t, float* o,
                     int ldo, int col0, const GVRope& rp) {
  if (rp.q_out) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < M) {
        const int p = rp.pos[m], slot = rp.slots[m];
        const float* cs = rp.cos_sin + (long)p * rp.Dh;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          const float v = group_sum<8>(acc[m][s]);
          const float partner = __shfl_xor(v, 8, 64);  // row n ^ 1
          const int col = col0 + n[s];
          const int head = col / rp.Dh, d = col - head * rp.Dh;
          float y = v;
          if (head < rp.Hq + rp.Hkv) {
            const float c = cs[d & ~1], sn = cs[(d & ~1) + 1];
            y = (d & 1) ? fmaf(partner, sn, v * c) : fmaf(-partner, sn, v * c);
          }
          if (t != 0 || n[s] >= N || (lane & 7)) continue;
          if (head < rp.Hq) {
            rp.q_out[((long)m * rp.Hq + head) * rp.Dh + d] = (bf16)y;
          } else if (slot >= 0) {
            const int blk = slot / rp.BS, off = slot - blk * rp.BS;
            if (head < rp.Hq + rp.Hkv) {
              rp.kc[(((long)blk * rp.Hkv + head - rp.Hq) * rp.BS + off) * rp.Dh + d] = (bf16)y;
            } else {
              const int vh = head - rp.Hq - rp.Hkv;
              rp.vc[((long)blk * rp.Hkv + vh) * rp.Dh * rp.BS + ((off >> 3) * rp.Dh + d) * 8 + (off & 7)] = (bf16)y;
            }
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m < M) {
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        const float v = group_sum<8>(acc[m][s]);
        if (t == 0 && n[s] < N) o[(size_t)m * ldo + col0 + n[s]] = v;
      }
    }
  }
}

template <int MT, int NT, int EARLY, int RS, int PD = 0, int NM = 0>
LA_DEV void gv_q4k(const QW& w, int row0, const bf16* X, int ldx, const GVAct& act, int M, int kper, float* o,
                   int ldo, int col0,
                   int8_t* xq, int* bs, float* dx, const GVRope& rp) {
  const int k0 = blockIdx.y * kper, nsb = kper >> 8, sb0 = k0 >> 8;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane >> 3, t = lane & 7;
  const int j = t >> 1, h = t & 1;
  const int xlo = 64 * j + 16 * h;  // element offset of this lane's low-nibble run (high: +32)
  const int blo = 4 * j + h;        // its 16-run index (high-nibble run: blo + 2)
  const size_t qrow = (size_t)(w.K >> 1), srow = (size_t)(w.K >> 8) * 16, drow = (size_t)(w.K >> 8) * 4;
  int n[RS];
  const uint8_t* qp[RS];
  const uint8_t* sp[RS];
  const uint8_t* dp[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    n[s] = row0 + wv * (8 * RS) + s * 8 + r;
    const size_t nc = n[s] < w.N ? n[s] : w.N - 1;  // clamped row for loads
    qp[s] = w.p0 + nc * qrow + (size_t)sb0 * 128 + 16 * t;
    sp[s] = w.p2 + nc * srow + (size_t)sb0 * 16 + 4 * j;
    dp[s] = w.p3 + nc * drow + (size_t)sb0 * 4;
  }
  const bool staged = !EARLY && !NM && x_staged_ok<MT>(act, kper);
  const bool late = EARLY || NM || gv_late(act);  // fused prologues: first weight round trip goes out first
  u32x2 xr[GV_XI];
  if (staged) x_issue<MT>(X, ldx, M, k0, kper, xr);
  if (!staged && !late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }
  u32x4 qa[RS];
  uint32_t sa[RS], da[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    qa[s] = ldg16<NT>(qp[s]);
    sa[s] = *(const uint32_t*)sp[s];
    da[s] = *(const uint32_t*)dp[s];
  }
  if (staged) {
    x_commit<MT>(M, kper, xr, xq, bs, dx);
    __syncthreads();
  }
  if (late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }

  float acc[MT][RS];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[m][s] = 0.f;
  if constexpr (PD > 0) {
    // PD-deep register ring (nsb % PD == 0, host-checked): super-block sb lives in slot sb % PD and
    // the slot is refilled with sb + PD right after use, so PD super-blocks stay in flight (a
    // split-K-1 workgroup walks all 16 super-blocks of a 4096-wide row serially)
    u32x4 qr[PD][RS];
    uint32_t sr[PD][RS], dr[PD][RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      qr[0][s] = qa[s];
      sr[0][s] = sa[s];
      dr[0][s] = da[s];
    }
#pragma unroll
    for (int i = 1; i < PD; ++i)
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        qr[i][s] = ldg16<NT>(qp[s] + i * 128);
        sr[i][s] = *(const uint32_t*)(sp[s] + i * 16);
        dr[i][s] = *(const uint32_t*)(dp[s] + i * 4);
      }
    for (int sb0 = 0; sb0 < nsb; sb0 += PD) {
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int sb = sb0 + i;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          qa[s] = qr[i][s];
          sa[s] = sr[i][s];
          da[s] = dr[i][s];
        }
        const int nx = min(sb + PD, nsb - 1);  // clamped tail reload: harmless, keeps the ring uniform
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          qr[i][s] = ldg16<NT>(qp[s] + nx * 128);
          sr[i][s] = *(const uint32_t*)(sp[s] + nx * 16);
          dr[i][s] = *(const uint32_t*)(dp[s] + nx * 4);
        }
        // unpack the nibbles once, reuse for every activation row
        u32x4 lo[RS], hi[RS];
    #pragma unroll
        for (int s = 0; s < RS; ++s) {
    #pragma unroll
          for (int i = 0; i < 4; ++i) {
            lo[s][i] = qa[s][i] & 0x0F0F0F0Fu;
            hi[s][i] = (qa[s][i] >> 4) & 0x0F0F0F0Fu;
          }
        }
    #pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (m < M) {
            const int8_t* xm = xq + m * kper + sb * 256;
            const u32x4 xl = *(const u32x4*)(xm + xlo);
            const u32x4 xh = *(const u32x4*)(xm + xlo + 32);
            const int* bm = bs + m * (kper >> 4) + sb * 16;
            const float* dm = dx + m * (kper >> 5) + sb * 8;
            const float dxl = dm[2 * j], dxh = dm[2 * j + 1];
            const float bl = (float)bm[blo] * dxl, bh = (float)bm[blo + 2] * dxh;
    #pragma unroll
            for (int s = 0; s < RS; ++s) {
              int dl = dot4(lo[s][0], xl[0], 0), dh = dot4(hi[s][0], xh[0], 0);
              dl = dot4(lo[s][1], xl[1], dl); dh = dot4(hi[s][1], xh[1], dh);
              dl = dot4(lo[s][2], xl[2], dl); dh = dot4(hi[s][2], xh[2], dh);
              dl = dot4(lo[s][3], xl[3], dl); dh = dot4(hi[s][3], xh[3], dh);
              const uint32_t sc = sa[s];
              const float fs = fmaf((float)(dl * (int)(sc & 0xFFu)), dxl, (float)(dh * (int)((sc >> 16) & 0xFFu)) * dxh);
              const float fm = fmaf((float)((sc >> 8) & 0xFFu), bl, (float)(sc >> 24) * bh);
              const float d = h2f((uint16_t)(da[s] & 0xFFFFu)), dmin = h2f((uint16_t)(da[s] >> 16));
              acc[m][s] = fmaf(d, fs, fmaf(-dmin, fm, acc[m][s]));
            }
          }
        }

      }
    }
  } else {
  for (int sb = 0; sb < nsb; ++sb) {
    u32x4 qn[RS];
    uint32_t sn[RS], dn[RS];
    if (sb + 1 < nsb) {
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        qn[s] = ldg16<NT>(qp[s] + (sb + 1) * 128);
        sn[s] = *(const uint32_t*)(sp[s] + (sb + 1) * 16);
        dn[s] = *(const uint32_t*)(dp[s] + (sb + 1) * 4);
      }
    }
    // unpack the nibbles once, reuse for every activation row
    u32x4 lo[RS], hi[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo[s][i] = qa[s][i] & 0x0F0F0F0Fu;
        hi[s][i] = (qa[s][i] >> 4) & 0x0F0F0F0Fu;
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < M) {
        const int8_t* xm = xq + m * kper + sb * 256;
        const u32x4 xl = *(const u32x4*)(xm + xlo);
        const u32x4 xh = *(const u32x4*)(xm + xlo + 32);
        const int* bm = bs + m * (kper >> 4) + sb * 16;
        const float* dm = dx + m * (kper >> 5) + sb * 8;
        const float dxl = dm[2 * j], dxh = dm[2 * j + 1];
        const float bl = (float)bm[blo] * dxl, bh = (float)bm[blo + 2] * dxh;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          int dl = dot4(lo[s][0], xl[0], 0), dh = dot4(hi[s][0], xh[0], 0);
          dl = dot4(lo[s][1], xl[1], dl); dh = dot4(hi[s][1], xh[1], dh);
          dl = dot4(lo[s][2], xl[2], dl); dh = dot4(hi[s][2], xh[2], dh);
          dl = dot4(lo[s][3], xl[3], dl); dh = dot4(hi[s][3], xh[3], dh);
          const uint32_t sc = sa[s];
          const float fs = fmaf((float)(dl * (int)(sc & 0xFFu)), dxl, (float)(dh * (int)((sc >> 16) & 0xFFu)) * dxh);
          const float fm = fmaf((float)((sc >> 8) & 0xFFu), bl, (float)(sc >> 24) * bh);
          const float d = h2f((uint16_t)(da[s] & 0xFFFFu)), dmin = h2f((uint16_t)(da[s] >> 16));
          acc[m][s] = fmaf(d, fs, fmaf(-dmin, fm, acc[m][s]));
        }
      }
    }
    if (sb + 1 < nsb) {
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        qa[s] = qn[s];
        sa[s] = sn[s];
        da[s] = dn[s];
      }
    }
  }
  }
  gv_store<MT, RS>(acc, n, w.N, M, t, o, ldo, col0, rp);
}

template <int MT, int NT, int EARLY, int RS, int PD = 0, int NM = 0>
LA_DEV void gv_q6k(const QW& w, int row0, const bf16* X, int ldx, const GVAct& act, int M, int kper, float* o,
                   int ldo, int col0,
                   int8_t* xq, int* bs, float* dx, const GVRope& rp) {
  const int k0 = blockIdx.y * kper, nsb = kper >> 8, sb0 = k0 >> 8;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane >> 3, t = lane & 7;
  const int hh = t >> 2, u = t & 3, s2 = u >> 1;
  const int xlo = 128 * hh + 32 * s2 + 16 * (u & 1);  // low-nibble run; high run at +64
  const int blo = xlo >> 4;                             // 16-run index; high run at +4
  const int shl = 4 - 2 * s2, shr = 2 * s2;
  const int scb = 8 * (2 * s2 + (u & 1));               // bit offset of this lane's scale byte
  const size_t lrow = (size_t)(w.K >> 1), hrow = (size_t)(w.K >> 2), crow = (size_t)(w.K >> 4),
               drow = (size_t)(w.K >> 8) * 2;
  int n[RS];
  const uint8_t* lp[RS];
  const uint8_t* hp[RS];
  const uint8_t* cp[RS];
  const uint8_t* dp[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    n[s] = row0 + wv * (8 * RS) + s * 8 + r;
    const size_t nc = n[s] < w.N ? n[s] : w.N - 1;
    lp[s] = w.p0 + nc * lrow + (size_t)sb0 * 128 + 64 * hh + 16 * u;
    hp[s] = w.p1 + nc * hrow + (size_t)sb0 * 64 + 32 * hh + 16 * (u & 1);
    cp[s] = w.p2 + nc * crow + (size_t)sb0 * 16 + 8 * hh;
    dp[s] = w.p3 + nc * drow + (size_t)sb0 * 2;
  }
  const bool staged = !EARLY && !NM && x_staged_ok<MT>(act, kper);
  const bool late = EARLY || NM || gv_late(act);  // fused prologues: first weight round trip goes out first
  u32x2 xr[GV_XI];
  if (staged) x_issue<MT>(X, ldx, M, k0, kper, xr);
  if (!staged && !late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }
  u32x4 la_[RS], ha[RS];
  u32x2 ca[RS];
  uint32_t da[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    la_[s] = ldg16<NT>(lp[s]);
    ha[s] = ldg16<NT>(hp[s]);
    ca[s] = *(const u32x2*)cp[s];
    da[s] = *(const uint16_t*)dp[s];
  }
  if (staged) {
    x_commit<MT>(M, kper, xr, xq, bs, dx);
    __syncthreads();
  }
  if (late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }

  float acc[MT][RS];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[m][s] = 0.f;
  if constexpr (PD > 0) {
    // PD-deep register ring, as in gv_q4k
    u32x4 lr[PD][RS], hr[PD][RS];
    u32x2 cr[PD][RS];
    uint32_t dr[PD][RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      lr[0][s] = la_[s];
      hr[0][s] = ha[s];
      cr[0][s] = ca[s];
      dr[0][s] = da[s];
    }
#pragma unroll
    for (int i = 1; i < PD; ++i)
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        lr[i][s] = ldg16<NT>(lp[s] + i * 128);
        hr[i][s] = ldg16<NT>(hp[s] + i * 64);
        cr[i][s] = *(const u32x2*)(cp[s] + i * 16);
        dr[i][s] = *(const uint16_t*)(dp[s] + i * 2);
      }
    for (int sb0 = 0; sb0 < nsb; sb0 += PD) {
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int sb = sb0 + i;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          la_[s] = lr[i][s];
          ha[s] = hr[i][s];
          ca[s] = cr[i][s];
          da[s] = dr[i][s];
        }
        const int nx = min(sb + PD, nsb - 1);
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          lr[i][s] = ldg16<NT>(lp[s] + nx * 128);
          hr[i][s] = ldg16<NT>(hp[s] + nx * 64);
          cr[i][s] = *(const u32x2*)(cp[s] + nx * 16);
          dr[i][s] = *(const uint16_t*)(dp[s] + nx * 2);
        }
    u32x4 lo[RS], hi[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo[s][i] = (la_[s][i] & 0x0F0F0F0Fu) | ((ha[s][i] << shl) & 0x30303030u);
        hi[s][i] = ((la_[s][i] >> 4) & 0x0F0F0F0Fu) | ((ha[s][i] >> shr) & 0x30303030u);
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < M) {
        const int8_t* xm = xq + m * kper + sb * 256;
        const u32x4 xl = *(const u32x4*)(xm + xlo);
        const u32x4 xh = *(const u32x4*)(xm + xlo + 64);
        const int* bm = bs + m * (kper >> 4) + sb * 16;
        const int bl = -32 * bm[blo], bh = -32 * bm[blo + 4];
        const float* dm = dx + m * (kper >> 5) + sb * 8;
        const float dxl = dm[xlo >> 5], dxh = dm[(xlo >> 5) + 2];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          int dl = dot4(lo[s][0], xl[0], bl), dh = dot4(hi[s][0], xh[0], bh);
          dl = dot4(lo[s][1], xl[1], dl); dh = dot4(hi[s][1], xh[1], dh);
          dl = dot4(lo[s][2], xl[2], dl); dh = dot4(hi[s][2], xh[2], dh);
          dl = dot4(lo[s][3], xl[3], dl); dh = dot4(hi[s][3], xh[3], dh);
          const int sl = __builtin_amdgcn_sbfe((int)ca[s].x, scb, 8);
          const int sh = __builtin_amdgcn_sbfe((int)ca[s].y, scb, 8);
          const float d = h2f((uint16_t)da[s]);
          acc[m][s] = fmaf(d, fmaf((float)(dl * sl), dxl, (float)(dh * sh) * dxh), acc[m][s]);
        }
      }
    }
      }
    }
  } else {
  for (int sb = 0; sb < nsb; ++sb) {
    u32x4 ln[RS], hn[RS];
    u32x2 cn[RS];
    uint32_t dn[RS];
    if (sb + 1 < nsb) {
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        ln[s] = ldg16<NT>(lp[s] + (sb + 1) * 128);
        hn[s] = ldg16<NT>(hp[s] + (sb + 1) * 64);
        cn[s] = *(const u32x2*)(cp[s] + (sb + 1) * 16);
        dn[s] = *(const uint16_t*)(dp[s] + (sb + 1) * 2);
      }
    }
    u32x4 lo[RS], hi[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo[s][i] = (la_[s][i] & 0x0F0F0F0Fu) | ((ha[s][i] << shl) & 0x30303030u);
        hi[s][i] = ((la_[s][i] >> 4) & 0x0F0F0F0Fu) | ((ha[s][i] >> shr) & 0x30303030u);
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < M) {
        const int8_t* xm = xq + m * kper + sb * 256;
        const u32x4 xl = *(const u32x4*)(xm + xlo);
        const u32x4 xh = *(const u32x4*)(xm + xlo + 64);
        const int* bm = bs + m * (kper >> 4) + sb * 16;
        const int bl = -32 * bm[blo], bh = -32 * bm[blo + 4];
        const float* dm = dx + m * (kper >> 5) + sb * 8;
        const float dxl = dm[xlo >> 5], dxh = dm[(xlo >> 5) + 2];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          int dl = dot4(lo[s][0], xl[0], bl), dh = dot4(hi[s][0], xh[0], bh);
          dl = dot4(lo[s][1], xl[1], dl); dh = dot4(hi[s][1], xh[1], dh);
          dl = dot4(lo[s][2], xl[2], dl); dh = dot4(hi[s][2], xh[2], dh);
          dl = dot4(lo[s][3], xl[3], dl); dh = dot4(hi[s][3], xh[3], dh);
          const int sl = __builtin_amdgcn_sbfe((int)ca[s].x, scb, 8);
          const int sh = __builtin_amdgcn_sbfe((int)ca[s].y, scb, 8);
          const float d = h2f((uint16_t)da[s]);
          acc[m][s] = fmaf(d, fmaf((float)(dl * sl), dxl, (float)(dh * sh) * dxh), acc[m][s]);
        }
      }
    }
    if (sb + 1 < nsb) {
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        la_[s] = ln[s];
        ha[s] = hn[s];
        ca[s] = cn[s];
        da[s] = dn[s];
      }
    }
  }
  }
  gv_store<MT, RS>(acc, n, w.N, M, t, o, ldo, col0, rp);
}

// Q8_0 (ggml block_q8_0: f16 d + 32 int8 per 32 weights; planes p0 = qs [N][K] int8, p1 = d
// [N][K/32] f16): lane t of a row group takes the 32-weight block t of each 256-weight chunk
// (two 16-B loads), 8 v_dot4 against the int8 activation block, one scale product per block --
// symmetric codes, so no 16-run sums.  Reference: ggml_vec_dot_q8_0_q8_0 [external, llama.cpp @
// d5cb868 ggml/src/ggml-quants.c].
template <int MT, int NT, int EARLY, int RS, int PD = 0, int NM = 0>
LA_DEV void gv_q8(const QW& w, int row0, const bf16* X, int ldx, const GVAct& act, int M, int kper, float* o,
                  int ldo, int col0, int8_t* xq, int* bs, float* dx, const GVRope& rp) {
  const int k0 = blockIdx.y * kper, nsb = kper >> 8, sb0 = k0 >> 8;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane >> 3, t = lane & 7;
  const size_t qrow = (size_t)w.K, drow = (size_t)(w.K >> 5) * 2;
  int n[RS];
  const uint8_t* qp[RS];
  const uint8_t* dp[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    n[s] = row0 + wv * (8 * RS) + s * 8 + r;
    const size_t nc = n[s] < w.N ? n[s] : w.N - 1;  // clamped row for loads
    qp[s] = w.p0 + nc * qrow + (size_t)sb0 * 256 + 32 * t;
    dp[s] = w.p1 + nc * drow + ((size_t)sb0 * 8 + t) * 2;
  }
  const bool staged = !EARLY && !NM && x_staged_ok<MT>(act, kper);
  const bool late = EARLY || NM || gv_late(act);  // fused prologues: first weight round trip goes out first
  u32x2 xr[GV_XI];
  if (staged) x_issue<MT>(X, ldx, M, k0, kper, xr);
  if (!staged && !late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }
  // PD-deep register ring over 256-weight chunks (PD 0: a 2-deep double buffer)
  constexpr int D = PD > 0 ? PD : 2;
  u32x4 qa[D][RS][2];
  uint32_t da[D][RS];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      const int sb = min(i, nsb - 1);
      qa[i][s][0] = ldg16<NT>(qp[s] + sb * 256);
      qa[i][s][1] = ldg16<NT>(qp[s] + sb * 256 + 16);
      da[i][s] = *(const uint16_t*)(dp[s] + sb * 16);
    }
  if (staged) {
    x_commit<MT>(M, kper, xr, xq, bs, dx);
    __syncthreads();
  }
  if (late) {
    quantize_x<MT, NM>(X, ldx, act, M, k0, kper, xq, bs, dx);
    __syncthreads();
  }
  float acc[MT][RS];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[m][s] = 0.f;
  for (int sb0i = 0; sb0i < nsb; sb0i += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int sb = sb0i + i;
      if (sb >= nsb) break;
      u32x4 q0[RS], q1[RS];
      uint32_t dd[RS];
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        q0[s] = qa[i][s][0];
        q1[s] = qa[i][s][1];
        dd[s] = da[i][s];
      }
      const int nx = min(sb + D, nsb - 1);  // clamped tail reload: harmless, keeps the ring uniform
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        qa[i][s][0] = ldg16<NT>(qp[s] + nx * 256);
        qa[i][s][1] = ldg16<NT>(qp[s] + nx * 256 + 16);
        da[i][s] = *(const uint16_t*)(dp[s] + nx * 16);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (m < M) {
          const int8_t* xm = xq + m * kper + sb * 256 + 32 * t;
          const u32x4 x0 = *(const u32x4*)xm;
          const u32x4 x1 = *(const u32x4*)(xm + 16);
          const float dxm = dx[m * (kper >> 5) + sb * 8 + t];
#pragma unroll
          for (int s = 0; s < RS; ++s) {
            int di = dot4(q0[s][0], x0[0], 0);
            di = dot4(q0[s][1], x0[1], di);
            di = dot4(q0[s][2], x0[2], di);
            di = dot4(q0[s][3], x0[3], di);
            di = dot4(q1[s][0], x1[0], di);
            di = dot4(q1[s][1], x1[1], di);
            di = dot4(q1[s][2], x1[2], di);
            di = dot4(q1[s][3], x1[3], di);
            acc[m][s] = fmaf(h2f((uint16_t)dd[s]) * dxm, (float)di, acc[m][s]);
          }
        }
      }
    }
  }
  gv_store<MT, RS>(acc, n, w.N, M, t, o, ldo, col0, rp);
}

// Segments [0, nA) are format FA, [nA, nseg) format FB (a q|k + v fusion is (Q4_K, Q6_K)).
// VAR bit 0: non-temporal weight loads; bit 1: weights requested before the x prologue.
template <int MT, int FA, int FB, int VAR>
__global__ __launch_bounds__(GV_THREADS) void qgemv_dp4_kernel(GVArgs a, const bf16* __restrict__ X, int ldx,
                                                               GVAct act, int M, int kper, float* __restrict__ out,
                                                               int ldo, long slab, GVRope rp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gv_lds[];
  int8_t* xq = (int8_t*)gv_lds;                                      // [MT][kper]
  int* bs = (int*)(gv_lds + MT * kper);                              // [MT][kper/16]
  float* dx = (float*)(gv_lds + MT * kper + MT * (kper >> 4) * 4);   // [MT][kper/32]
  int seg = 0, blk = blockIdx.x;
#pragma unroll
  for (int i = 0; i < GV_SEGS - 1; ++i)
    if (seg < a.nseg - 1 && blk >= a.blk_end[seg]) ++seg;
  constexpr int RS = gv_rs<VAR>();
  const int row0 = (blk - (seg ? a.blk_end[seg - 1] : 0)) * (32 * RS);
  float* o = out + (size_t)blockIdx.y * slab;
  constexpr int NT = VAR & 1, EARLY = (VAR >> 1) & 1, PD = (VAR & 16) ? 4 : 0, NM = (VAR >> 5) & 1;
  const bool fa = FA == FB || a.fmt[seg] == FA;
  if constexpr (FA == FMT_Q8_0) {  // Q8_0 launches are homogeneous (host-checked)
    gv_q8<MT, NT, EARLY, RS, PD, NM>(a.w[seg], row0, X, ldx, act, M, kper, o, ldo, a.col0[seg], xq, bs, dx, rp);
  } else if (fa) {
    if constexpr (FA == FMT_Q4_K) gv_q4k<MT, NT, EARLY, RS, PD, NM>(a.w[seg], row0, X, ldx, act, M, kper, o, ldo, a.col0[seg], xq, bs, dx, rp);
    else gv_q6k<MT, NT, EARLY, RS, PD, NM>(a.w[seg], row0, X, ldx, act, M, kper, o, ldo, a.col0[seg], xq, bs, dx, rp);
  } else if constexpr (FA != FB) {
    if constexpr (FB == FMT_Q4_K) gv_q4k<MT, NT, EARLY, RS, PD, NM>(a.w[seg], row0, X, ldx, act, M, kper, o, ldo, a.col0[seg], xq, bs, dx, rp);
    else gv_q6k<MT, NT, EARLY, RS, PD, NM>(a.w[seg], row0, X, ldx, act, M, kper, o, ldo, a.col0[seg], xq, bs, dx, rp);
  }
}

// MoE decode (1-2 tokens): the routed experts' projections as GEMVs on the int8-dot path.  One
// workgroup = (32-row block, K split, routed pair p = token t x slot); the expert is read from
// the device routing (ids[p], local ids, >= E_local: another rank's expert -> zero rows), its
// planes from the device QW descriptors, so the launch is graph-capturable with no host routing.
//   gate|up (down = 0): x = X[t]           -> out [S][P][N]        (row p)
//   down    (down = 1): x = wts[p] * act(gate|up slab row p) -> out [S*topk][T][N] (slab
//                       split*topk + slot, row t): summing the slabs is the weighted combine.
template <int FMT, int VAR>
__global__ __launch_bounds__(GV_THREADS) void moe_gemv_kernel(const QW* __restrict__ qws, const int* __restrict__ ids,
                                                              int E_local, int topk, const bf16* __restrict__ X,
                                                              int ldx, GVAct act, const float* __restrict__ wts,
                                                              int down, int kper, float* __restrict__ out, int ldo,
                                                              long slab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gv_lds[];
  int8_t* xq = (int8_t*)gv_lds;
  int* bs = (int*)(gv_lds + kper);
  float* dx = (float*)(gv_lds + kper + (kper >> 4) * 4);
  constexpr int RS = gv_rs<VAR>();
  constexpr int NT = VAR & 1, EARLY = (VAR >> 1) & 1, PD = (VAR & 16) ? 4 : 0;
  const int p = blockIdx.z, t = p / topk, slot = p - t * topk;
  const int row0 = blockIdx.x * (32 * RS);
  float* o = down ? out + ((size_t)blockIdx.y * topk + slot) * slab + (size_t)t * ldo
                  : out + (size_t)blockIdx.y * slab + (size_t)p * ldo;
  const int e = ids[p];
  if (e < 0 || e >= E_local) {  // not computed here: its rows read as zero
    const int N = qws[0].N;
    for (int i = threadIdx.x; i < 32 * RS; i += GV_THREADS)
      if (row0 + i < N) o[row0 + i] = 0.f;
    return;
  }
  const QW w = qws[e];
  GVAct a = act;
  const bf16* xp = X;
  if (down) {
    a.p = act.p + (size_t)p * ((act.mode == 0 || act.mode == 3) ? 2L * act.F : (long)act.F);
    a.scale = wts[p];
  } else {
    xp = X + (size_t)t * ldx;
  }
  const GVRope rp{};
  if constexpr (FMT == FMT_Q8_0) gv_q8<1, NT, EARLY, RS, PD>(w, row0, xp, ldx, a, 1, kper, o, 0, 0, xq, bs, dx, rp);
  else if constexpr (FMT == FMT_Q4_K) gv_q4k<1, NT, EARLY, RS, PD>(w, row0, xp, ldx, a, 1, kper, o, 0, 0, xq, bs, dx, rp);
  else gv_q6k<1, NT, EARLY, RS, PD>(w, row0, xp, ldx, a, 1, kper, o, 0, 0, xq, bs, dx, rp);
}

static inline size_t gv_lds_bytes(int MT, int kper) {
  return (size_t)MT * kper + (size_t)MT * (kper >> 4) * 4 + (size_t)MT * (kper >> 5) * 4;
}

static int g_gv_variant = 5;  // non-temporal weight loads, x staged first, one 8-row slot per wave (fastest overall)

template <int MT, int FA, int FB>
static int launch_gv(const GVArgs& a, int nblk, int K, const bf16* X, int ldx, const GVAct& act, int M, int splits,
                     float* out, int ldo, long slab, hipStream_t st, const GVRope& rp, int cvar) {
  const int kper = K / splits;
  const size_t lds = gv_lds_bytes(MT, kper);
  if (lds > 64 * 1024) return -3;
  dim3 grid(nblk, splits);
  // the fused-RoPE launch runs split-K 1: each workgroup walks the whole row, so it takes the
  // 4-deep weight ring (VAR bit 4) of the default variant
  int var = (rp.q_out && cvar == 5) ? 21 : cvar;
  if ((var & 16) && ((kper >> 8) % 4)) var &= ~16;  // the ring walks whole groups of 4 super-blocks
  if (act.mode == GV_NORM) {
    if (MT > 2 || (var != 5 && var != 21)) return -4;
    var |= 32;  // the fused-norm prologue's own instantiation
  }
  switch (var) {
#define GV_CASE(V) \
    case V: hipLaunchKernelGGL((qgemv_dp4_kernel<MT, FA, FB, V>), grid, dim3(GV_THREADS), lds, st, a, X, ldx, act, M, kper, out, ldo, slab, rp); break;
    GV_CASE(0) GV_CASE(1) GV_CASE(2) GV_CASE(3) GV_CASE(5) GV_CASE(9) GV_CASE(21) GV_CASE(37) GV_CASE(53)
#undef GV_CASE
    default: return -4;
  }
  return 0;
}

template <int FA, int FB>
static int launch_gv_m(const GVArgs& a, int nblk, int K, const bf16* X, int ldx, const GVAct& act, int M, int splits,
                       float* out, int ldo, long slab, hipStream_t st, const GVRope& rp, int cvar) {
  if (M == 1) return launch_gv<1, FA, FB>(a, nblk, K, X, ldx, act, M, splits, out, ldo, slab, st, rp, cvar);
  if (M == 2) return launch_gv<2, FA, FB>(a, nblk, K, X, ldx, act, M, splits, out, ldo, slab, st, rp, cvar);
  return launch_gv<4, FA, FB>(a, nblk, K, X, ldx, act, M, splits, out, ldo, slab, st, rp, cvar);
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// nseg weights side by side: fmts[i], planes[4*i .. 4*i+3], Ns[i]; all share K.
// Q4_K planes: p0 = qs, p2 = scm, p3 = dd (p1, the packed header, is unused here).
// Q6_K planes: p0 = ql, p1 = qh, p2 = sc, p3 = d.
// act_p != null: x is act(gate|up) computed from fp32 slabs act_p [act_S][M][W] (X unused),
// W = 2K for act_mode 0 (SwiGLU) / 3 (GeGLU) else K; act_bias optional [W].
static int qgemv_dp4_impl(int nseg, const int* fmts, const void* const* planes, const int* Ns, int K,
                          const void* X, int ldx, int M, int splits, void* out, int ldo, long slab,
                          const void* act_p, long act_slab, int act_S, const void* act_bias, int act_mode,
                          void* stream, const la::GVRope& rp, const la::GVAct* norm = nullptr) {
  using namespace la;
  if (nseg < 1 || nseg > GV_SEGS || M < 1 || M > 4 || (K & 255) || splits < 1 || ((K >> 8) % splits) ||
      slab < (long)M * ldo)
    return -1;
  GVAct act{(const float*)act_p, act_slab, act_S, (const float*)act_bias, act_mode, K};
  if (norm) {
    // fused residual-add + RMSNorm prologue: M <= 2, K <= 8192 (row in VGPRs), slabs optional
    act = *norm;
    if (M > 2 || K > GV_THREADS * GV_NORM_IT * 4 || !act.res || !act.nw || act.mode != GV_NORM || act.F != K ||
        (act.p && (act.S < 1 || act.S > 16 || act.slab < (long)M * K)) || act.res_out == act.res)
      return -1;
  } else if (act_p) {
    if (act_S < 1 || act_S > 16 || act_mode < 0 || act_mode > 3 ||
        act_slab < (long)M * ((act_mode == 0 || act_mode == 3) ? 2L * K : (long)K))
      return -1;
  } else if (!X || ldx < K) {
    return -1;
  }
  GVArgs a{};
  int nblk = 0, col = 0;
  // per-call variant: the default (5) except the widest batch-1 plain GEMVs (gate|up, N >= 16384),
  // where four 8-row slots per wave measured faster (28672 x 4096 Q4_K: 18.2 vs 18.9 us,
  // scripts/gpu_r4_gv.sh); every other shape keeps 5
  int Nsum = 0;
  for (int i = 0; i < nseg; ++i) Nsum += Ns[i];
  // (at M = 2 variant 1 timed faster per GEMV -- gate|up 20.9 vs 22.0 us -- but engine C=2 did
  // not confirm it: 733-734 tok/s; M = 2 keeps 5)
  const bool plain = g_gv_variant == 5 && !rp.q_out && !norm && !act_p;
  const int cvar = (plain && M == 1 && Nsum >= 16384) ? 9 : g_gv_variant;
  const int rows = 32 * ((cvar & 4) ? 1 : ((cvar & 8) ? 4 : 2));  // rows per workgroup
  for (int i = 0; i < nseg; ++i) {
    const int f = fmts[i], N = Ns[i];
    const void* const* p = planes + 4 * i;
    if (f == FMT_Q8_0) {
      if (N < 1 || !p[0] || !p[1]) return -2;
    } else if (N < 1 || !p[0] || !p[2] || !p[3] || (f != FMT_Q4_K && f != FMT_Q6_K) || (f == FMT_Q6_K && !p[1])) {
      return -2;
    }
    a.w[i] = QW{(const uint8_t*)p[0], (const uint8_t*)p[1], (const uint8_t*)p[2], (const uint8_t*)p[3], N, K};
    a.fmt[i] = f;
    a.col0[i] = col;
    nblk += (N + rows - 1) / rows;
    a.blk_end[i] = nblk;
    col += N;
  }
  a.nseg = nseg;
  if (ldo < col) return -1;
  // formats must form at most two runs: [FA ...][FB ...]
  int fa = a.fmt[0], fb = a.fmt[nseg - 1];
  for (int i = 0; i < nseg; ++i)
    if (a.fmt[i] != fa && a.fmt[i] != fb) return -2;
  for (int i = 1; i < nseg; ++i)
    if (a.fmt[i - 1] == fb && a.fmt[i] == fa && fa != fb) return -2;
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
  int rc;
  if ((fa == FMT_Q8_0) != (fb == FMT_Q8_0)) return -2;  // Q8_0 weights launch on their own
  if (fa == FMT_Q8_0) rc = launch_gv_m<FMT_Q8_0, FMT_Q8_0>(a, nblk, K, x, ldx, act, M, splits, o, ldo, slab, st, rp, cvar);
  else if (fa == FMT_Q4_K && fb == FMT_Q4_K) rc = launch_gv_m<FMT_Q4_K, FMT_Q4_K>(a, nblk, K, x, ldx, act, M, splits, o, ldo, slab, st, rp, cvar);
  else if (fa == FMT_Q6_K && fb == FMT_Q6_K) rc = launch_gv_m<FMT_Q6_K, FMT_Q6_K>(a, nblk, K, x, ldx, act, M, splits, o, ldo, slab, st, rp, cvar);
  else if (fa == FMT_Q4_K) rc = launch_gv_m<FMT_Q4_K, FMT_Q6_K>(a, nblk, K, x, ldx, act, M, splits, o, ldo, slab, st, rp, cvar);
  else rc = launch_gv_m<FMT_Q6_K, FMT_Q4_K>(a, nblk, K, x, ldx, act, M, splits, o, ldo, slab, st, rp, cvar);
  if (rc) return rc;
  return (int)hipGetLastError();
}

extern "C" int la_qgemv_dp4(int nseg, const int* fmts, const void* const* planes, const int* Ns, int K,
                            const void* X, int ldx, int M, int splits, void* out, int ldo, long slab,
                            const void* act_p, long act_slab, int act_S, const void* act_bias, int act_mode,
                            void* stream) {
  la::GVRope rp{};
  return qgemv_dp4_impl(nseg, fmts, planes, Ns, K, X, ldx, M, splits, out, ldo, slab, act_p, act_slab, act_S,
                        act_bias, act_mode, stream, rp);
}

// Decode q|k|v projection with RoPE (NORM pairs over the whole head) and the paged K/V append
// fused into the GEMV epilogue: no split-K (each output row is complete in one workgroup), q to
// q_out [M][Hq][Dh] bf16, k / v of token m to cache slot slots[m] (skipped when < 0).
extern "C" int la_qgemv_dp4_rope(int nseg, const int* fmts, const void* const* planes, const int* Ns, int K,
                                 const void* X, int M, const int* pos, const int* slots, const float* cos_sin,
                                 int Hq, int Hkv, int Dh, void* q_out, void* kc, void* vc, int BS, void* stream) {
  if (!q_out || !kc || !vc || !pos || !slots || !cos_sin || (Dh & 1) || Dh < 2 || BS < 8 || (BS & 7)) return -1;
  if ((K >> 8) % 4) return -1;  // the 4-deep weight ring walks whole groups of 4 super-blocks
  int W = 0;
  for (int i = 0; i < nseg; ++i) W += Ns[i];
  if (W != (Hq + 2 * Hkv) * Dh) return -1;
  la::GVRope rp{pos, slots, cos_sin, (__bf16*)q_out, (__bf16*)kc, (__bf16*)vc, Hq, Hkv, Dh, BS};
  // out / slab are unused by the rope epilogue; pass a non-null dummy that passes the checks
  return qgemv_dp4_impl(nseg, fmts, planes, Ns, K, X, K, M, 1, q_out, W, (long)M * W, nullptr, 0, 0, nullptr, 0,
                        stream, rp);
}

// The same two launches with the layer-boundary residual-add + RMSNorm as their x prologue
// (GV_NORM): x = rmsnorm(res + sum(add slabs) + add_bias) * nw, res_out = res + ... (written
// once, by workgroup (0, 0); must not alias res).  add_p may be null (no add: the first layer).
static la::GVAct gv_norm_args(int K, const void* res, const void* add_p, long add_slab, int add_S,
                              const void* add_bias, const void* nw, float eps, void* res_out) {
  la::GVAct a{(const float*)add_p, add_slab, add_S, (const float*)add_bias, la::GV_NORM, K};
  a.res = (const float*)res;
  a.res_out = (float*)res_out;
  a.nw = (const float*)nw;
  a.eps = eps;
  return a;
}

extern "C" int la_qgemv_dp4_norm(int nseg, const int* fmts, const void* const* planes, const int* Ns, int K, int M,
                                 int splits, void* out, int ldo, long slab, const void* res, const void* add_p,
                                 long add_slab, int add_S, const void* add_bias, const void* nw, float eps,
                                 void* res_out, void* stream) {
  la::GVRope rp{};
  const la::GVAct na = gv_norm_args(K, res, add_p, add_slab, add_S, add_bias, nw, eps, res_out);
  return qgemv_dp4_impl(nseg, fmts, planes, Ns, K, nullptr, K, M, splits, out, ldo, slab, nullptr, 0, 0, nullptr, 0,
                        stream, rp, &na);
}

extern "C" int la_qgemv_dp4_rope_norm(int nseg, const int* fmts, const void* const* planes, const int* Ns, int K,
                                      int M, const int* pos, const int* slots, const float* cos_sin, int Hq, int Hkv,
                                      int Dh, void* q_out, void* kc, void* vc, int BS, const void* res,
                                      const void* add_p, long add_slab, int add_S, const void* add_bias,
                                      const void* nw, float eps, void* res_out, void* stream) {
  if (!q_out || !kc || !vc || !pos || !slots || !cos_sin || (Dh & 1) || Dh < 2 || BS < 8 || (BS & 7)) return -1;
  if ((K >> 8) % 4) return -1;
  int W = 0;
  for (int i = 0; i < nseg; ++i) W += Ns[i];
  if (W != (Hq + 2 * Hkv) * Dh) return -1;
  la::GVRope rp{pos, slots, cos_sin, (__bf16*)q_out, (__bf16*)kc, (__bf16*)vc, Hq, Hkv, Dh, BS};
  const la::GVAct na = gv_norm_args(K, res, add_p, add_slab, add_S, add_bias, nw, eps, res_out);
  return qgemv_dp4_impl(nseg, fmts, planes, Ns, K, nullptr, K, M, 1, q_out, W, (long)M * W, nullptr, 0, 0, nullptr, 0,
                        stream, rp, &na);
}

// MoE decode GEMV (see moe_gemv_kernel): fmt / N / K shared by the E_local experts of `qws`
// (device QW descriptors); ids [P = T*topk] local expert ids; down: act_p = the gate|up fp32
// slabs [act_S][P][2F] (SwiGLU, act_mode 0 / GeGLU 3) or [..][P][F], wts [P] routing weights.
extern "C" int la_moe_gemv(int fmt, int down, const void* qws, int N, int K, int E_local, const int* ids, int T,
                           int topk, const void* X, int ldx, int splits, const void* act_p, long act_slab, int act_S,
                           int act_mode, const float* wts, void* out, int ldo, long slab, void* stream) {
  using namespace la;
  if (T < 1 || topk < 1 || N < 1 || (K & 255) || splits < 1 || ((K >> 8) % splits) || E_local < 1 || !qws || !ids)
    return -1;
  if (fmt != FMT_Q4_K && fmt != FMT_Q6_K && fmt != FMT_Q8_0) return -2;
  if (down ? (!act_p || !wts || act_S < 1 || act_S > 16 || (act_mode != 0 && act_mode != 3 && act_mode != 1 &&
                                                             act_mode != 2))
           : (!X || ldx < K))
    return -1;
  const int kper = K / splits;
  const size_t lds = gv_lds_bytes(1, kper);
  if (lds > 64 * 1024) return -3;
  GVAct act{(const float*)act_p, act_slab, act_S, nullptr, act_mode, K};
  hipStream_t st = (hipStream_t)stream;
  // variant 1: non-temporal weights, x staged first, two 8-row slots per wave -- Mixtral C=1 312.8 /
  // 313.2 vs 306.4 tok/s with one slot, C=2 413.3 / 412.8 vs 404.0 (profiles/r5_logs/r5_mv2_*.log)
  constexpr int V = 1;
  const int rows = 32 * gv_rs<V>();
  dim3 grid((N + rows - 1) / rows, splits, T * topk);
#define MG(F)                                                                                                 \
  hipLaunchKernelGGL((moe_gemv_kernel<F, V>), grid, dim3(GV_THREADS), lds, st, (const QW*)qws, ids, E_local,   \
                     topk, (const bf16*)X, ldx, act, wts, down, kper, (float*)out, ldo, slab);
  if (fmt == FMT_Q4_K) MG(FMT_Q4_K)
  else if (fmt == FMT_Q6_K) MG(FMT_Q6_K)
  else MG(FMT_Q8_0)
#undef MG
  return (int)hipGetLastError();
}

// Tuning hook: select the kernel variant (bit 0 non-temporal loads, bit 1 early weight prefetch).
extern "C" int la_gemv_variant(int v) {
  if (!(v >= 0 && v <= 3) && v != 5 && v != 9 && v != 21) return -1;
  la::g_gv_variant = v;
  return 0;
}
