// Device-side views of the repacked GGUF weight formats.
//
// Runtime layouts (built on the GPU from raw GGUF blocks by localai_amd/ops/qweight.py):
//   Q4_K : qs  u8  [N][K/2]      (the 128 quant bytes of each 256-block, ggml order)
//          hdr u8  [N][K/256][16] (f16 d, f16 dmin, 12 packed 6-bit scales/mins)
//   Q6_K : ql  u8  [N][K/2], qh u8 [N][K/4], sc i8 [N][K/16], d f16 [N][K/256]
//   Q8_0 : qs  i8  [N][K],   d  f16 [N][K/32]
//   BF16 : w   bf16[N][K]
// Splitting the 144/210/34-byte blocks into per-field planes makes every fragment
// load a 16-byte (or 8-byte) aligned vector load; the arithmetic is bit-exact with
// ggml's dequantize_row_* (reference: llama.cpp @ d5cb868, [external]).
//
// A "fragment" is what ONE lane of a wave needs for one 256-wide K super-block of one
// weight row when the wave runs v_mfma_f32_16x16x32_bf16 with B = W^T: lane l owns
// row n = l&15 and k-group g = l>>4.  Each format fixes a permutation kphys(s,g) of
// the 8-element groups inside the super-block (s = MFMA k-step 0..7) chosen so the
// lane's quant bytes are contiguous; the activation (A) operand is read with the same
// permutation, so the dot product is unchanged.
#pragma once
#include "common.h"

namespace la {

enum WFmt : int { FMT_Q8_0 = 8, FMT_Q4_K = 12, FMT_Q6_K = 14, FMT_BF16 = 30 };

struct QW {
  const uint8_t* p0;  // Q4_K: qs   | Q6_K: ql | Q8_0: qs | BF16: w
  const uint8_t* p1;  // Q4_K: hdr  | Q6_K: qh | Q8_0: d  | -
  const uint8_t* p2;  // Q6_K: sc
  const uint8_t* p3;  // Q6_K: d
  int N, K;
};

// physical k offset (inside a 256 super-block) of k-step s, lane group g
template <int FMT>
LA_DEV int kphys(int s, int g) {
  if constexpr (FMT == FMT_Q6_K) return 128 * (g >> 1) + 32 * (s >> 1) + 16 * (g & 1) + 8 * (s & 1);
  else return 64 * g + 32 * (s >> 2) + 8 * (s & 3);
}

LA_DEV uint32_t byte_of12(uint32_t a, uint32_t b, uint32_t c, int i) {
  const uint32_t w = (i < 4) ? a : ((i < 8) ? b : c);
  return (w >> (8 * (i & 3))) & 0xFFu;
}

// ggml get_scale_min_k4 on the 12 packed bytes (a,b,c little-endian dwords).  Branch-free:
// j is per-lane in the GEMV kernels, and an exec-masked if/else there makes hipcc drain
// the weight-load ring (vmcnt) around each arm.
LA_DEV void q4k_scale_min(uint32_t a, uint32_t b, uint32_t c, int j, uint32_t& sc, uint32_t& m) {
  const bool lo = j < 4;
  const uint32_t bj = byte_of12(a, b, c, j);                  // j < 4: scale byte
  const uint32_t bj4 = byte_of12(a, b, c, j + 4);             // j < 4: min byte; j >= 4: low nibbles
  const uint32_t bjm4 = byte_of12(a, b, c, lo ? j : j - 4);   // j >= 4: high bits of the scale
  const uint32_t sc_hi = (bj4 & 0xFu) | ((bjm4 >> 6) << 4);
  const uint32_t m_hi = (bj4 >> 4) | ((bj >> 6) << 4);
  sc = lo ? (bj & 63u) : sc_hi;
  m = lo ? (bj4 & 63u) : m_hi;
}

template <int FMT> struct WFrag;

// ---------------------------------------------------------------- Q4_K
template <> struct WFrag<FMT_Q4_K> {
  u32x4 q0, q1, hdr;
  float D[2], Mn[2];
  LA_DEV void load(const QW& w, int n, int sb, int g) {
    const uint8_t* qs = w.p0 + (size_t)n * (w.K >> 1) + sb * 128 + 32 * g;
    q0 = *(const u32x4*)qs;
    q1 = *(const u32x4*)(qs + 16);
    hdr = *(const u32x4*)(w.p1 + ((size_t)n * (w.K >> 8) + sb) * 16);
  }
  LA_DEV void prep(int g) {
    const float d = h2f(hdr.x & 0xFFFFu), dmin = h2f(hdr.x >> 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t sc, m;
      q4k_scale_min(hdr.y, hdr.z, hdr.w, 2 * g + h, sc, m);
      D[h] = d * (float)sc;
      Mn[h] = dmin * (float)m;
    }
  }
  template <int S>
  LA_DEV bf16x8 deq() const {
    constexpr int h = S >> 2, t = S & 3;
    const uint32_t lo = (t == 0) ? q0.x : (t == 1) ? q0.z : (t == 2) ? q1.x : q1.z;
    const uint32_t hi = (t == 0) ? q0.y : (t == 1) ? q0.w : (t == 2) ? q1.y : q1.w;
    const uint32_t a = (lo >> (4 * h)) & 0x0F0F0F0Fu, b = (hi >> (4 * h)) & 0x0F0F0F0Fu;
    const float Dv = D[h], Mv = -Mn[h];
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = (bf16)fmaf(Dv, (float)((a >> (8 * j)) & 0xFu), Mv);
      r[j + 4] = (bf16)fmaf(Dv, (float)((b >> (8 * j)) & 0xFu), Mv);
    }
    return r;
  }
};

// ---------------------------------------------------------------- Q6_K
template <> struct WFrag<FMT_Q6_K> {
  u32x4 la, lb, qh;
  u32x2 sc8;
  float dd;
  float S[4];
  LA_DEV void load(const QW& w, int n, int sb, int g) {
    const int hh = g >> 1, o = 16 * (g & 1);
    const uint8_t* ql = w.p0 + (size_t)n * (w.K >> 1) + sb * 128 + 64 * hh + o;
    la = *(const u32x4*)ql;
    lb = *(const u32x4*)(ql + 32);
    qh = *(const u32x4*)(w.p1 + (size_t)n * (w.K >> 2) + sb * 64 + 32 * hh + o);
    sc8 = *(const u32x2*)(w.p2 + (size_t)n * (w.K >> 4) + sb * 16 + 8 * hh);
    const uint16_t dbits = *(const uint16_t*)(w.p3 + ((size_t)n * (w.K >> 8) + sb) * 2);
    dd = h2f(dbits);
  }
  LA_DEV void prep(int g) {
    const int o = g & 1;
#pragma unroll
    for (int qi = 0; qi < 4; ++qi) {
      const int idx = 2 * qi + o;  // byte inside the 8 loaded scale bytes
      const uint32_t w = (idx < 4) ? sc8.x : sc8.y;
      const int8_t s = (int8_t)((w >> (8 * (idx & 3))) & 0xFFu);
      S[qi] = dd * (float)s;
    }
  }
  template <int St>
  LA_DEV bf16x8 deq() const {
    constexpr int qi = St >> 1, jh = St & 1;
    const u32x4& L = (qi & 1) ? lb : la;
    const uint32_t l0 = jh ? L.z : L.x, l1 = jh ? L.w : L.y;
    const uint32_t h0 = jh ? qh.z : qh.x, h1 = jh ? qh.w : qh.y;
    constexpr int ls = 4 * (qi >> 1), hs = 2 * qi;
    const float sc = S[qi];
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int q0 = (int)(((l0 >> (8 * j + ls)) & 0xFu) | (((h0 >> (8 * j + hs)) & 3u) << 4)) - 32;
      int q1 = (int)(((l1 >> (8 * j + ls)) & 0xFu) | (((h1 >> (8 * j + hs)) & 3u) << 4)) - 32;
      r[j] = (bf16)(sc * (float)q0);
      r[j + 4] = (bf16)(sc * (float)q1);
    }
    return r;
  }
};

// ---------------------------------------------------------------- Q8_0
template <> struct WFrag<FMT_Q8_0> {
  u32x4 a0, a1, a2, a3;
  uint32_t dpair;
  float d[2];
  LA_DEV void load(const QW& w, int n, int sb, int g) {
    const uint8_t* qs = w.p0 + (size_t)n * w.K + sb * 256 + 64 * g;
    a0 = *(const u32x4*)qs;
    a1 = *(const u32x4*)(qs + 16);
    a2 = *(const u32x4*)(qs + 32);
    a3 = *(const u32x4*)(qs + 48);
    dpair = *(const uint32_t*)(w.p1 + ((size_t)n * (w.K >> 5) + sb * 8 + 2 * g) * 2);
  }
  LA_DEV void prep(int) {
    d[0] = h2f(dpair & 0xFFFFu);
    d[1] = h2f(dpair >> 16);
  }
  template <int S>
  LA_DEV bf16x8 deq() const {
    constexpr int h = S >> 2, t = S & 3;
    // bytes [32h + 8t, +8) of the lane's 64 bytes
    const u32x4& A = (h == 0) ? ((t < 2) ? a0 : a1) : ((t < 2) ? a2 : a3);
    const uint32_t lo = (t & 1) ? A.z : A.x, hi = (t & 1) ? A.w : A.y;
    const float dv = d[h];
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = (bf16)(dv * (float)(int8_t)((lo >> (8 * j)) & 0xFFu));
      r[j + 4] = (bf16)(dv * (float)(int8_t)((hi >> (8 * j)) & 0xFFu));
    }
    return r;
  }
};

// ---------------------------------------------------------------- BF16
template <> struct WFrag<FMT_BF16> {
  bf16x8 v[8];
  LA_DEV void load(const QW& w, int n, int sb, int g) {
    const bf16x8* p = (const bf16x8*)(w.p0 + ((size_t)n * w.K + sb * 256 + 64 * g) * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = p[i];
  }
  LA_DEV void prep(int) {}
  template <int S>
  LA_DEV bf16x8 deq() const {
    return v[S];  // kphys(s,g) = 64g + 8s when s is decomposed as (s>>2, s&3)
  }
};

// Dequantise 8 consecutive weights (natural k order, k % 8 == 0) of row n to floats.
// Used by the embedding gather and the bf16 materialisation kernels (not hot).
template <int FMT>
LA_DEV void deq8_natural(const QW& w, int n, int k, float* out) {
  if constexpr (FMT == FMT_Q4_K) {
    const int sb = k >> 8, kk = k & 255, c = kk >> 6, h = (kk >> 5) & 1, off = kk & 31;
    const uint8_t* qs = w.p0 + (size_t)n * (w.K >> 1) + sb * 128 + 32 * c + off;
    const u32x4 hdr = *(const u32x4*)(w.p1 + ((size_t)n * (w.K >> 8) + sb) * 16);
    uint32_t sc, m;
    q4k_scale_min(hdr.y, hdr.z, hdr.w, 2 * c + h, sc, m);
    const float D = h2f(hdr.x & 0xFFFFu) * (float)sc, Mv = h2f(hdr.x >> 16) * (float)m;
    const u32x2 q = *(const u32x2*)qs;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t byte = ((j < 4 ? q.x : q.y) >> (8 * (j & 3))) & 0xFFu;
      out[j] = D * (float)((byte >> (4 * h)) & 0xFu) - Mv;
    }
  } else if constexpr (FMT == FMT_Q6_K) {
    const int sb = k >> 8, kk = k & 255, hh = kk >> 7, e = kk & 127, qi = e >> 5, l0 = e & 31;
    const uint8_t* ql = w.p0 + (size_t)n * (w.K >> 1) + sb * 128 + 64 * hh + ((qi & 1) ? 32 : 0) + l0;
    const uint8_t* qh = w.p1 + (size_t)n * (w.K >> 2) + sb * 64 + 32 * hh + l0;
    const int8_t s = *(const int8_t*)(w.p2 + (size_t)n * (w.K >> 4) + sb * 16 + 8 * hh + 2 * qi + (l0 >> 4));
    const float D = h2f(*(const uint16_t*)(w.p3 + ((size_t)n * (w.K >> 8) + sb) * 2)) * (float)s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = (int)(((ql[j] >> (4 * (qi >> 1))) & 0xF) | (((qh[j] >> (2 * qi)) & 3) << 4)) - 32;
      out[j] = D * (float)q;
    }
  } else if constexpr (FMT == FMT_Q8_0) {
    const int8_t* qs = (const int8_t*)(w.p0 + (size_t)n * w.K + k);
    const float d = h2f(*(const uint16_t*)(w.p1 + ((size_t)n * (w.K >> 5) + (k >> 5)) * 2));
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = d * (float)qs[j];
  } else {
    const bf16x8 v = *(const bf16x8*)(w.p0 + ((size_t)n * w.K + k) * 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (float)v[j];
  }
}

}  // namespace la
