// Paged attention for the engine (replaces ggml-cuda fattn*.cu / softmax.cu / the KQ,KQV
// batched GEMMs of the non-FA path; SURVEY §2.8 K7, K11, K12, K15 [external]).
//
// KV cache layout (per layer): K [num_blocks][Hkv][BS][Dh] and V [num_blocks][Hkv][BS/8][Dh][8]
// bf16: one page of one kv-head is BS*Dh*2 contiguous bytes (8 KiB at BS=32, Dh=128).  V is
// stored transposed in groups of 8 keys ([key group][d][8 keys]), so the PV MFMA's B operand (8
// consecutive keys at one d) is one 16-byte load, and appending one token touches 16-byte
// segments of ONE 2 KiB group run instead of every 64-byte row of the page (a fully transposed
// [Dh][BS] page made each decode append a 2-byte write into 128 separate cache lines).
//
// * attn_decode: one query row per sequence.  Workgroup = (partition of <=PS keys, kv head,
//   sequence); the G = Hq/Hkv query heads sharing a kv head are packed so K/V are read from
//   HBM once (GQA packing).  Split-KV partials are merged by attn_decode_combine.
// * attn_prefill: causal flash attention on MFMA (v_mfma_f32_16x16x32_bf16) for chunks of new
//   tokens appended to a (possibly prefix-cached) context; K/V tiles of 32 keys come from the
//   paged cache, so prefix reuse and chunked prefill need no special casing.
#include <cstdlib>

#include "common.h"

namespace la {

// ----------------------------------------------------------------------------- decode
// MFMA flash-decoding.  Workgroup = (partition of <= PS keys, kv head, sequence), 4 waves; wave w
// takes the partition's 32-key tiles w, w+4, ...
//   S^T[16 keys x 16 heads] = K[16 keys x Dh] . Q^T[Dh x 16 heads]   (keys on MFMA rows)
//   -> MFMA t (of 2 per 32-key tile) puts key 8(m>>2) + 4t + (m&3) on row m, so lane l ends up
//      with the scores of head l&15 for the 8 CONSECUTIVE keys 8(l>>4) .. +7: the running max
//      needs only two cross-lane shuffles (xor 16, 32) and P is already the lane's A fragment;
//   O[16 heads x Dh] += P[16 heads x 32 keys] . V[32 keys x Dh]
//   -> V is stored transposed per page ([Dh][BS]) so the B fragment (8 consecutive keys at one
//      d) is ONE 16-byte load; 16 lanes x 64 B full rows per instruction, no LDS, no transposes.
// Latency structure (decode attention is latency-bound: a few KB per wave):
//   * the partition's block-table slice is staged in LDS once (no bt -> K/V load chains);
//   * every K and V load of tile i+1 is issued before tile i is computed (register double
//     buffer); keys past the sequence end are clamped to a valid key and masked in the scores,
//     so no load sits behind a branch;
//   * split-KV partials are merged IN the kernel by the last-arriving partition (agent-scope
//     release/acquire ticket per (sequence, kv head); the ticket resets itself for the next
//     launch / graph replay), so there is no separate combine launch.
// Scores live in the log2 domain (scale * log2 e folded in): every exponential is one v_exp_f32.
// Workgroup = NW waves of one (partition, kv head, sequence).  NW = 4 splits a partition's tiles
// over 4 waves (few sequences: more waves in flight per key); NW = 1 gives every wave a whole
// partition (batch decode: B x Hkv >= 1024 single-wave workgroups fill the chip in ONE residency
// round, so the seq_len -> block table -> first tile latency chain is paid once per CU instead
// of once per 4-wave round, and no cross-wave LDS merge is needed).
constexpr int DEC_MAXBT = 2048;  // block-table entries of one partition staged in LDS
constexpr int DEC_ONE_PART = 256;  // sequences up to this many keys run as a single partition

template <int DH, int GT, int NW>
struct DecShared {
  float ow[NW < 2 ? 2 : NW][GT][DH];  // wave partials (NW > 1); the split-KV merge weights reuse it
  float mw[NW][16], lw[NW][16];
  int bt[DEC_MAXBT];
  int last;
};

template <int DH>
struct DecTile {
  bf16x8 k[2][(DH + 31) / 32];
  bf16x8 v[DH / 16];
};

// Fused RoPE + KV append for decode (replaces the rope_kv launch of a decode step): the kernel
// reads the q|k|v GEMM output itself (fp32 split-K slabs or one bf16 matrix, optional bias),
// rotates q for its heads, and the workgroup whose partition holds the newest key rotates k
// and writes k / v of that token into the paged cache before its own tile loads read them.
// NORM (adjacent-pair) rotary over the full head only; anything else uses rope_kv.
struct DecRope {
  const void* p;         // null: q comes pre-rotated in `q` (unfused path)
  long slab;             // elements between fp32 slabs
  int S;                 // fp32 slabs (0: p is one bf16 [B][W] matrix)
  const float* bias;     // [W] or null
  const int* pos;        // [B] rotary position of the new token
  const int* slots;      // [B] cache slot of the new token (< 0: no append)
  const float* cos_sin;  // [max_pos][DH/2][2]
  int W;                 // row width (Hq + 2 Hkv) * DH
};

// x[b, col .. col+N) of the q|k|v source, summed over slabs (+bias), in fp32.  N in {1, 2, 8};
// col is a multiple of N.  Every slab load of a group of 8 is issued before the first add
// (clamped slab index, masked -- never a branch), so the slabs cost one memory round trip.
template <int N>
LA_DEV void rope_src_load(const DecRope& R, int b, int col, float (&v)[N]) {
  typedef float fvec __attribute__((ext_vector_type(N)));
  typedef __bf16 bvec __attribute__((ext_vector_type(N)));
  const long idx = (long)b * R.W + col;
  if (R.S == 0) {
    const bvec s = *(const bvec*)((const bf16*)R.p + idx);
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = (float)s[j];
  } else {
    const float* f = (const float*)R.p + idx;
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = 0.f;
    for (int s0 = 0; s0 < R.S; s0 += 8) {
      fvec t[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = *(const fvec*)(f + (long)min(s0 + i, R.S - 1) * R.slab);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float m = (s0 + i < R.S) ? 1.f : 0.f;
#pragma unroll
        for (int j = 0; j < N; ++j) v[j] = fmaf(m, t[i][j], v[j]);
      }
    }
  }
  if (R.bias) {
    const fvec bb = *(const fvec*)(R.bias + col);
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] += bb[j];
  }
}

// K/V are streamed once per decode step: non-temporal loads (the default) read them 12-14 %
// faster at batch 256 (5.05 -> 5.70 TB/s at 256 keys, 5.21 -> 5.98 at 384;
// profiles/r4_attn_decode_nt.md).  VAR bit 0 = ordinary cached loads (A/B only); bit 1 = keys
// two tiles ahead (measured no faster; kept for the A/B).
template <int DH, int GT, int NW, int VAR = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void attn_decode_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ seq_lens, int Hkv, int G,
    int BS, float scale_log2, int PS_grid, bf16* __restrict__ out, float* __restrict__ part_o,
    float* __restrict__ part_ml, int P, int* __restrict__ tickets, DecRope R, float cap_l2, float cap_mul,
    int window, int one_part) {
  constexpr int KC = (DH + 31) / 32;  // 32-wide k chunks of the QK^T product
  constexpr int ND = DH / 16;         // 16-wide d tiles of the PV product
  constexpr int NT = NW * 64;
  __shared__ DecShared<DH, GT, NW> sh;

  const int p = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int Hq = Hkv * G;
  const int L = seq_lens[b];
  // The grid's partitioning is fixed when a decode graph is captured (for the context bound);
  // a short sequence takes ONE partition of DEC_ONE_PART keys instead, so it skips the split-KV
  // merge round trip (partials + ticket + last-arriver reduction) -- worth more than the
  // parallelism at a few hundred keys.  Decided per sequence, uniformly for its workgroups.
  const int PS = (L <= one_part && PS_grid < one_part) ? one_part : PS_grid;
  const int t0 = p * PS;
  if (t0 >= L) return;  // empty partition: the combiner only waits for ceil(L / PS) of them
  const int wlo = window > 0 ? L - window : 0;  // first key inside the sliding window
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int kend = min(L, t0 + PS);
  const int nbt = (kend - t0 + BS - 1) / BS;
  const int* bt = block_tables + (long)b * max_blocks + t0 / BS;
  for (int i = tid; i < nbt; i += NT) sh.bt[i] = bt[i];

  // Q^T fragments: lane holds Q[head r][d = 32c + 8g .. +8]
  bf16x8 qf[KC];
  if (R.p) {
    const float* cs = R.cos_sin + (long)R.pos[b] * DH;  // DH/2 (cos, sin) pairs
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int d = 32 * c + 8 * g;
      bf16x8 v = {};
      if (r < G) {
        float x[8];
        rope_src_load<8>(R, b, (kvh * G + r) * DH + d, x);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float cc = cs[d + j], sn = cs[d + j + 1];  // pair (d+j)/2: (cos, sin) at d+j, d+j+1
          v[j] = (bf16)(x[j] * cc - x[j + 1] * sn);
          v[j + 1] = (bf16)(x[j] * sn + x[j + 1] * cc);
        }
      }
      qf[c] = v;
    }
    // the partition holding the newest key appends its k (rotated) and v to the cache
    const int slot = R.slots[b];
    if (slot >= 0 && L - 1 >= t0 && L - 1 < kend) {
      const int blk = slot / BS, off = slot - blk * BS;
      for (int j = tid; j < DH / 2 + DH; j += NT) {
        if (j < DH / 2) {
          float x[2];
          rope_src_load<2>(R, b, (Hq + kvh) * DH + 2 * j, x);
          const float cc = cs[2 * j], sn = cs[2 * j + 1];
          bf16* kd = (bf16*)kc + (((long)blk * Hkv + kvh) * BS + off) * DH + 2 * j;
          kd[0] = (bf16)(x[0] * cc - x[1] * sn);
          kd[1] = (bf16)(x[0] * sn + x[1] * cc);
        } else {
          const int d = j - DH / 2;
          float x[1];
          rope_src_load<1>(R, b, (Hq + Hkv + kvh) * DH + d, x);
          ((bf16*)vc)[((long)blk * Hkv + kvh) * DH * BS + ((off >> 3) * DH + d) * 8 + (off & 7)] = (bf16)x[0];
        }
      }
      // Only this workgroup reads the appended key back (pages never straddle partitions, and
      // L1 starts each launch clean), so same-CU ordering suffices: the stores reach the XCD's
      // L2 before the barrier below; no agent-scope fence (MI355X_MICROARCH: ~3.5 us each).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int d = 32 * c + 8 * g;
      bf16x8 v = {};
      if (r < G && d < DH) v = *(const bf16x8*)(q + ((long)b * Hq + kvh * G + r) * DH + d);
      qf[c] = v;
    }
  }
  __syncthreads();

  const long head_off = (long)kvh * BS * DH;  // inside a page: [Hkv][BS][Dh] / [Hkv][Dh][BS]
  constexpr bool NTL = !(VAR & 1);
  auto ld16 = [](const bf16* p) -> bf16x8 {
    if constexpr (NTL) return __builtin_nontemporal_load((const bf16x8*)p);
    else return *(const bf16x8*)p;
  };
  auto load_k = [&](int kb, bf16x8 (&K)[2][(DH + 31) / 32]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // K row r of MFMA t: key kb + 8(r>>2) + 4t + (r&3) (clamped to a real key)
      const int kk = min(kb + 8 * (r >> 2) + 4 * t + (r & 3), kend - 1);
      const long pk = (long)sh.bt[(kk - t0) / BS] * Hkv * BS * DH + head_off;
      const bf16* krow = kc + pk + (long)(kk % BS) * DH;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const int d = min(32 * c + 8 * g, DH - 8);
        K[t][c] = ld16(krow + d);
      }
    }
  };
  auto load_v = [&](int kb, bf16x8 (&V)[DH / 16]) {
    // V^T: keys kb + 8g .. +7 at d (an 8-aligned run inside one page, clamped to a real key)
    const int kv = min(kb + 8 * g, kend - 1) & ~7;
    const long pv = (long)sh.bt[(kv - t0) / BS] * Hkv * BS * DH + head_off;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const int d = 16 * nd + r;
      V[nd] = ld16(vc + pv + ((long)((kv % BS) >> 3) * DH + d) * 8);
    }
  };
  auto load_tile = [&](int kb, DecTile<DH>& T) {
    load_k(kb, T.k);
    load_v(kb, T.v);
  };

  f32x4 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;

  // register double buffer up to Dh 128; a Dh-256 tile (Gemma) is 128 VGPRs on its own, so it
  // is loaded at the top of each iteration instead (no prefetch, no spills)
  constexpr bool DB = DH <= 128;
  // K2: keys two tiles ahead (V stays one ahead: a whole second tile does not fit in 256 VGPRs)
  constexpr bool K2 = (VAR & 2) != 0;
  int kb = t0 + 32 * wave;
  if (kb < kend) {
    DecTile<DH> cur, nxt;
    bf16x8 k2[2][(DH + 31) / 32];
    if constexpr (DB) {
      load_tile(kb, cur);
      if constexpr (K2)
        if (kb + 32 * NW < kend) load_k(kb + 32 * NW, nxt.k);
    }
    for (; kb < kend; kb += 32 * NW) {
      if constexpr (DB) {
        if constexpr (K2) {
          if (kb + 2 * 32 * NW < kend) load_k(kb + 2 * 32 * NW, k2);
          if (kb + 32 * NW < kend) load_v(kb + 32 * NW, nxt.v);
        } else {
          if (kb + 32 * NW < kend) load_tile(kb + 32 * NW, nxt);
        }
      } else {
        load_tile(kb, cur);
      }
      float s[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          bf16x8 a = cur.k[t][c];
          if (32 * c + 8 * g >= DH) a = bf16x8{};  // Dh % 32 != 0: zero the tail chunk
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[c], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = kb + 8 * g + 4 * t + i;
          // Gemma-2 logit soft-capping cap * tanh(s / cap) (cap_l2 = cap * log2 e, 0: off) and
          // sliding-window attention (keys at least `window` positions behind the query masked)
          const float sv = cap_l2 > 0.f ? cap_l2 * tanhf(acc[i] * cap_mul) : acc[i] * scale_log2;
          s[t][i] = (key < kend && key >= wlo) ? sv : -INFINITY;
        }
      }
      // online softmax for head r over this 32-key tile
      float mx = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                       fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = exp2f(m - msafe);
      bf16x8 pa;
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = exp2f(s[t][i] - msafe);
          ps += e;
          pa[4 * t + i] = (bf16)e;
        }
      lsum = lsum * alpha + ps;
      m = mnew;
      // O rows are heads 4g+i: fetch each row's alpha from the lane that owns that head
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float f = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
        for (int nd = 0; nd < ND; ++nd) o[nd][i] *= f;
      }
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) o[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, cur.v[nd], o[nd], 0, 0, 0);
      if constexpr (DB) {
        cur = nxt;
        if constexpr (K2) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int c = 0; c < (DH + 31) / 32; ++c) nxt.k[t][c] = k2[t][c];
        }
      }
    }
  }
  // wave totals: lsum over the 4 lane groups (same head r)
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const int np = (L + PS - 1) / PS;  // partitions holding keys of this sequence
  if constexpr (NW == 1) {
    // one wave per workgroup: its accumulators ARE the partition's result (no LDS merge).
    // o[nd][i] is head 4g+i at d = 16nd + r; that head's (m, l) live in lane 4g+i.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g + i;
      const float lh = __shfl(lsum, h, 64), mh = __shfl(m, h, 64);
      if (h < G) {
        const int hq = kvh * G + h;
        if (np == 1) {
          const float inv = lh > 0.f ? 1.f / lh : 0.f;
#pragma unroll
          for (int nd = 0; nd < ND; ++nd) out[((long)b * Hq + hq) * DH + 16 * nd + r] = (bf16)(o[nd][i] * inv);
        } else {
#pragma unroll
          for (int nd = 0; nd < ND; ++nd) part_o[(((long)b * Hq + hq) * P + p) * DH + 16 * nd + r] = o[nd][i];
          if (r == 0) {
            float* ml = part_ml + (((long)b * Hq + hq) * P + p) * 2;
            ml[0] = mh;
            ml[1] = lh;
          }
        }
      }
    }
    if (np == 1) return;
  } else {
  if (g == 0) {
    sh.mw[wave][r] = m;
    sh.lw[wave][r] = lsum;
  }
#pragma unroll
  for (int nd = 0; nd < ND; ++nd)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * g + i < GT) sh.ow[wave][min(4 * g + i, GT - 1)][16 * nd + r] = o[nd][i];
  __syncthreads();
  for (int i = tid; i < G * DH; i += NT) {
    const int h = i / DH, d = i % DH;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sh.mw[w][h]);
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = exp2f(sh.mw[w][h] - Ms);
      num += f * sh.ow[w][h][d];
      den += f * sh.lw[w][h];
    }
    const int hq = kvh * G + h;
    if (np == 1) {
      out[((long)b * Hq + hq) * DH + d] = (bf16)(den > 0.f ? num / den : 0.f);
    } else {
      part_o[(((long)b * Hq + hq) * P + p) * DH + d] = num;
      if (d == 0) {
        float* ml = part_ml + (((long)b * Hq + hq) * P + p) * 2;
        ml[0] = M;
        ml[1] = den;
      }
    }
  }
  if (np == 1) return;
  }
  // ---- split-KV merge by the last-arriving partition of (b, kvh)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* tk = tickets + (long)b * Hkv + kvh;
    const int prev = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (prev == np - 1);
    if (last) {
      *tk = 0;  // self-resetting ticket (next launch / graph replay starts from 0)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sh.last = last;
  }
  __syncthreads();
  if (!sh.last) return;
  // merge weights per (partition, head) staged in LDS (reuses the wave-merge arrays), then every
  // (head, d) output sums its np partials with independent, unrolled loads
  float* wts = &sh.ow[0][0][0];  // [np][G] weights, then [G] 1/den
  const long hb = ((long)b * Hq + kvh * G) * P;
  if (tid < G) {
    const long base = hb + (long)tid * P;
    float M = -INFINITY;
    for (int j = 0; j < np; ++j) M = fmaxf(M, part_ml[(base + j) * 2]);
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float den = 0.f;
    for (int j = 0; j < np; ++j) {
      const float f = exp2f(part_ml[(base + j) * 2] - Ms);
      wts[j * G + tid] = f;
      den += f * part_ml[(base + j) * 2 + 1];
    }
    wts[np * G + tid] = den > 0.f ? 1.f / den : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < G * DH; i += NT) {
    const int h = i / DH, d = i % DH;
    const float* po = part_o + (hb + (long)h * P) * DH + d;
    float num = 0.f;
    for (int j0 = 0; j0 < np; j0 += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = po[(long)min(j0 + j, np - 1) * DH];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j0 + j < np) num += wts[(j0 + j) * G + h] * v[j];
    }
    out[((long)b * Hq + kvh * G + h) * DH + d] = (bf16)(num * wts[np * G + h]);
  }
}

// ----------------------------------------------------------------------------- prefill
// Workgroup = 64 query rows (4 waves x 16) of one sequence x one query head.
// DENSE = false: causal, K/V from the paged cache (engine prefill).  DENSE = true: non-causal
// over K/V rows of the same tokens in plain strided matrices -- a vision tower's bidirectional
// self-attention (CLIP ViT, SURVEY K12 "non-causal variant"): q/k/v/out row t, head h at
// ptr + t * ld + h * DH (the fused q|k|v projection output read in place).
constexpr int PF_T = 256;
constexpr int PF_KT = 32;  // keys per tile

template <int DH, bool DENSE = false>
__global__ __launch_bounds__(PF_T) void attn_prefill_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ tiles,          // [ntiles][2] = (seq, first query row within seq)
    const int* __restrict__ cu_q,           // [nseq+1] token offsets of each seq's queries
    const int* __restrict__ ctx_lens,       // [nseq] total keys (cached + new)
    const int* __restrict__ block_tables, int max_blocks, int Hq, int Hkv, int BS, float scale,
    bf16* __restrict__ out, float cap, int window, long ldq = 0, long ldk = 0, long ldv = 0, long ldo = 0) {
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
  const int L = DENSE ? qlen : ctx_lens[s];
  const int pos0 = L - qlen;  // absolute position of query row 0
  const int* bt = DENSE ? nullptr : block_tables + (long)s * max_blocks;
  if constexpr (!DENSE) ldq = ldo = (long)Hq * DH;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  // Q fragments (A operand): row = wave*16 + fr, k = 32*kc + 8*fq
  const int qrow = r0 + wave * 16 + fr;
  bf16x8 qa[KC];
#pragma unroll
  for (int kc2 = 0; kc2 < KC; ++kc2) {
    bf16x8 v = {};
    const int d = 32 * kc2 + 8 * fq;
    if (qrow < qlen && d < DH) v = *(const bf16x8*)(q + (long)(qbeg + qrow) * ldq + (long)h * DH + d);
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
  const int kend = DENSE ? L : min(L, pos0 + last_row + 1);  // exclusive

  for (int k0 = 0; k0 < kend; k0 += PF_KT) {
    __syncthreads();
    // stage the K tile (row-major) and the V^T tile ([d][key], copied from the transposed cache)
    for (int cidx = tid; cidx < PF_KT * (DP / 8); cidx += PF_T) {
      const int kr = cidx / (DP / 8), d = (cidx % (DP / 8)) * 8;
      const int key = k0 + kr;
      bf16x8 kv = {};
      if (key < kend && d < DH) {
        if constexpr (DENSE) {
          kv = *(const bf16x8*)(kc + (long)(qbeg + key) * ldk + (long)kvh * DH + d);
        } else {
          const int blk = bt[key / BS], off = key % BS;
          kv = *(const bf16x8*)(kc + (((long)blk * Hkv + kvh) * BS + off) * DH + d);
        }
      }
      *(bf16x8*)(ks + kr * KS + d) = kv;
    }
    if constexpr (DENSE) {
      // V rows are key-major: 16 B (8 d) per load, transposed into V^T[d][key] by scalar writes
      for (int cidx = tid; cidx < PF_KT * (DP / 8); cidx += PF_T) {
        const int kr = cidx / (DP / 8), d = (cidx % (DP / 8)) * 8;
        const int key = k0 + kr;
        bf16x8 vv = {};
        if (key < kend && d < DH) vv = *(const bf16x8*)(vc + (long)(qbeg + key) * ldv + (long)kvh * DH + d);
#pragma unroll
        for (int j = 0; j < 8; ++j) vt[(d + j) * VS + kr] = vv[j];
      }
    }
    for (int cidx = tid; !DENSE && cidx < DP * (PF_KT / 8); cidx += PF_T) {
      const int d = cidx % DP, q8 = (cidx / DP) * 8;  // consecutive threads: consecutive d of one key group
      const int key = k0 + q8;
      bf16x8 vv = {};
      if (key < kend && d < DH) {
        const int blk = bt[key / BS], off = key % BS;
        vv = *(const bf16x8*)(vc + ((long)blk * Hkv + kvh) * DH * BS + ((off >> 3) * DH + d) * 8);
        if (key + 8 > kend) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (key + j >= kend) vv[j] = (bf16)0.f;
        }
      }
      *(bf16x8*)(vt + d * VS + q8) = vv;
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
      if (cap > 0.f) {  // soft-capping (Gemma-2): cap * tanh(s / cap), in the log2 domain
        v0 = cap * 1.4426950408889634f * tanhf(sacc[0][i] * scale / cap);
        v1 = cap * 1.4426950408889634f * tanhf(sacc[1][i] * scale / cap);
      }
      const int key0 = k0 + fr, key1 = k0 + 16 + fr;
      const int wlo = window > 0 ? qpos - window + 1 : 0;
      const bool causal = !DENSE;
      if ((causal && key0 > qpos) || key0 >= kend || qr >= qlen || key0 < wlo) v0 = -INFINITY;
      if ((causal && key1 > qpos) || key1 >= kend || qr >= qlen || key1 < wlo) v1 = -INFINITY;
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
      if (d < DH) out[(long)(qbeg + qr) * ldo + (long)h * DH + d] = (bf16)(o[nd][i] * inv);
    }
  }
}

}  // namespace la

// C ABI ------------------------------------------------------------------------------------
static int g_dec_one_part = la::DEC_ONE_PART;  // tuning hook (la_dec_one_part)

// Sequences of up to n keys run as one partition per kv head (no split-KV merge); n % 128 == 0.
extern "C" int la_dec_one_part(int n) {
  if (n < 0 || n > 2048 * 16 || n % 128) return -1;
  g_dec_one_part = n;
  return 0;
}

extern "C" int la_attn_decode(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                              const int* seq_lens, int B, int Hq, int Hkv, int Dh, int BS, float scale, int P, int PS,
                              void* out, void* part_o, void* part_ml, void* tickets, const void* rope_p,
                              long rope_slab, int rope_S, const void* rope_bias, const int* pos, const int* slots,
                              const float* cos_sin, float softcap, int window, int nw, void* stream) {
  // nw bit 8: split even short sequences over the grid's partitions (few sequences: the
  // parallelism is worth the merge); otherwise a sequence of <= DEC_ONE_PART keys is one partition
  const int one_part = (nw & 256) ? 0 : g_dec_one_part;
  nw &= 255;
  if (Hq % Hkv || Hq / Hkv > 16 || (BS % 16) || (128 % BS && BS % 128) || (PS % 32) || (PS % BS) || P < 1 ||
      (nw != 1 && nw != 4) ||
      PS / BS > la::DEC_MAXBT || P > 64 || (P > 1 && !tickets))
    return -1;
  // rope_p != null: fused RoPE + KV append from the q|k|v GEMM output (q unused)
  if (rope_p && ((Dh & 31) || !pos || !slots || !cos_sin || rope_S < 0)) return -1;
  if (!rope_p && !q) return -1;
  const la::DecRope R{rope_p, rope_slab, rope_S, (const float*)rope_bias, pos, slots, cos_sin, (Hq + 2 * Hkv) * Dh};
  const int G = Hq / Hkv;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(P, Hkv, B);
  float* po = (float*)part_o;
  float* pml = (float*)part_ml;
  int* tk = (int*)tickets;
  const float sl2 = scale * 1.4426950408889634f;
  const float cap_l2 = softcap > 0.f ? softcap * 1.4426950408889634f : 0.f;
  const float cap_mul = softcap > 0.f ? scale / softcap : 0.f;
  static const int var = [] {
    const char* e = getenv("LOCALAI_AMD_ATTN_VAR");
    return e ? atoi(e) & 3 : 0;
  }();
#define DEC_LAUNCH(D, GT, NW, V)                                                                                  \
  hipLaunchKernelGGL((la::attn_decode_kernel<D, GT, NW, V>), grid, dim3(NW * 64), 0, st, (const bf16*)q,        \
                     (const bf16*)kc, (const bf16*)vc, block_tables, max_blocks, seq_lens, Hkv, G, BS, sl2, PS,  \
                     (bf16*)out, po, pml, P, tk, R, cap_l2, cap_mul, window, one_part)
#define DEC_NW(D, GT, NW)                                                  \
  do {                                                                     \
    if constexpr (D == 128 && GT == 4 && NW == 1) {                        \
      if (var == 1) DEC_LAUNCH(D, GT, NW, 1);                              \
      else if (var == 2) DEC_LAUNCH(D, GT, NW, 2);                         \
      else if (var == 3) DEC_LAUNCH(D, GT, NW, 3);                         \
      else DEC_LAUNCH(D, GT, NW, 0);                                       \
    } else {                                                               \
      DEC_LAUNCH(D, GT, NW, 0);                                            \
    }                                                                      \
  } while (0)
#define DEC(D, GT)          \
  do {                      \
    if (nw == 1)            \
      DEC_NW(D, GT, 1);     \
    else                    \
      DEC_NW(D, GT, 4);     \
  } while (0)
#define DEC_G(D)                          \
  if (G == 1) DEC(D, 1);                  \
  else if (G == 2) DEC(D, 2);             \
  else if (G <= 4) DEC(D, 4);             \
  else if (G <= 8) DEC(D, 8);             \
  else DEC(D, 16);
  switch (Dh) {
    case 64: DEC_G(64); break;
    case 80: DEC_G(80); break;
    case 96: DEC_G(96); break;
    case 128: DEC_G(128); break;
    case 192: DEC_G(192); break;  // DeepSeek-V2 latent attention keys (128 nope + 64 rope)
    case 256: DEC_G(256); break;
    default: return -2;
  }
#undef DEC_G
#undef DEC
#undef DEC_NW
#undef DEC_LAUNCH
  return (int)hipGetLastError();
}

// Non-causal attention over strided q / k / v rows of the same tokens (vision towers): sequence s
// holds tokens cu_q[s] .. cu_q[s+1]; tiles as la_attn_prefill's (seq, first query row).
extern "C" int la_attn_dense(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, void* out,
                             long ldo, const int* tiles, int ntiles, const int* cu_q, int Hq, int Hkv, int Dh,
                             float scale, void* stream) {
  if (Hq % Hkv || (ldq & 7) || (ldk & 7) || (ldv & 7) || ntiles < 1) return -1;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(ntiles, Hq);
#define DENSE_CASE(D)                                                                                              \
  case D:                                                                                                          \
    hipLaunchKernelGGL((la::attn_prefill_kernel<D, true>), grid, dim3(la::PF_T), 0, st, (const bf16*)q,          \
                       (const bf16*)k, (const bf16*)v, tiles, cu_q, nullptr, nullptr, 0, Hq, Hkv, 0, scale,       \
                       (bf16*)out, 0.f, 0, ldq, ldk, ldv, ldo);                                                   \
    break;
  switch (Dh) {
    DENSE_CASE(64) DENSE_CASE(80) DENSE_CASE(96) DENSE_CASE(128)
    default: return -2;
  }
#undef DENSE_CASE
  return (int)hipGetLastError();
}

extern "C" int la_attn_prefill(const void* q, const void* kc, const void* vc, const int* tiles, int ntiles,
                               const int* cu_q, const int* ctx_lens, const int* block_tables, int max_blocks, int Hq,
                               int Hkv, int Dh, int BS, float scale, void* out, float softcap, int window,
                               void* stream) {
  if (Hq % Hkv) return -1;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(ntiles, Hq);
#define PF(D)                                                                                                     \
  hipLaunchKernelGGL(la::attn_prefill_kernel<D>, grid, dim3(la::PF_T), 0, st, (const bf16*)q, (const bf16*)kc,    \
                     (const bf16*)vc, tiles, cu_q, ctx_lens, block_tables, max_blocks, Hq, Hkv, BS, scale,       \
                     (bf16*)out, softcap, window)
  switch (Dh) {
    case 64: PF(64); break;
    case 80: PF(80); break;
    case 96: PF(96); break;
    case 128: PF(128); break;
    case 192: PF(192); break;
    case 256: PF(256); break;
    default: return -2;
  }
#undef PF
  return (int)hipGetLastError();
}
