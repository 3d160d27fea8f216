// Staging units of the quantised GEMMs that dequantise a weight tile into LDS (gemm_mid.hip,
// gemm_ws.hip): one unit = 16 consecutive weights (natural k order) of one weight row, read
// as raw quant bytes and expanded to bf16 (bit-exact with ggml's dequantize_row_*).
#pragma once
#include "qweight.h"

namespace la {

// Raw bytes for one staging unit = 16 weights of row n at k = 64*ks + 16*q .. +16 (q = 0..3).
// Addressing is split into a per-thread 32-bit offset (fixed for the whole K loop, set by
// init) and a wave-uniform per-K-step base, so every staging load is a saddr+voffset
// global_load with no per-step 64-bit address VALU work.
template <int FMT> struct MidRaw;

template <> struct MidRaw<FMT_Q4_K> {
  struct Addr {
    uint32_t qs, hdr;
    int half;
    LA_DEV void init(const QW& w, int n, int q) {
      qs = (uint32_t)n * (w.K >> 1) + 16 * (q & 1);
      hdr = (uint32_t)n * (w.K >> 8) * 16;
      half = q >> 1;
    }
  };
  u32x4 qs;
  u32x4 hdr;
  LA_DEV void load(const QW& w, const Addr& a, int ks) {
    qs = *(const u32x4*)(w.p0 + 32 * ks + a.qs);
    hdr = *(const u32x4*)(w.p1 + 16 * (ks >> 2) + a.hdr);
  }
  LA_DEV void deq(const Addr& ad, int ks, bf16x8 out[2]) const {
    const int half = ad.half;
    uint32_t sc, m;
    q4k_scale_min(hdr.y, hdr.z, hdr.w, 2 * (ks & 3) + half, sc, m);
    const float D = h2f(hdr.x & 0xFFFFu) * (float)sc, Mv = -h2f(hdr.x >> 16) * (float)m;
    const uint32_t v[4] = {qs.x, qs.y, qs.z, qs.w};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t a = (v[2 * j] >> (4 * half)) & 0x0F0F0F0Fu, b = (v[2 * j + 1] >> (4 * half)) & 0x0F0F0F0Fu;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        out[j][i] = (bf16)fmaf(D, (float)((a >> (8 * i)) & 0xFFu), Mv);
        out[j][i + 4] = (bf16)fmaf(D, (float)((b >> (8 * i)) & 0xFFu), Mv);
      }
    }
  }
};

template <> struct MidRaw<FMT_Q6_K> {
  struct Addr {
    uint32_t ql, qh, sc, d;
    int qhi;
    LA_DEV void init(const QW& w, int n, int q) {
      qhi = q >> 1;
      ql = (uint32_t)n * (w.K >> 1) + 32 * qhi + 16 * (q & 1);
      qh = (uint32_t)n * (w.K >> 2) + 16 * (q & 1);
      sc = (uint32_t)n * (w.K >> 4) + 2 * qhi + (q & 1);
      d = (uint32_t)n * (w.K >> 8) * 2;
    }
  };
  u32x4 ql, qh;
  int8_t sc;
  uint16_t dbits;
  LA_DEV void load(const QW& w, const Addr& a, int ks) {
    // sb*128 + 64*hh == 64*(ks>>1);  sb*64 + 32*hh == 32*(ks>>1);  sb*16 + 8*hh + 4*(c&1) == 8*(ks>>1) + 4*(ks&1)
    ql = *(const u32x4*)(w.p0 + 64 * (ks >> 1) + a.ql);
    qh = *(const u32x4*)(w.p1 + 32 * (ks >> 1) + a.qh);
    sc = *(const int8_t*)(w.p2 + 8 * (ks >> 1) + 4 * (ks & 1) + a.sc);
    dbits = *(const uint16_t*)(w.p3 + 2 * (ks >> 2) + a.d);
  }
  LA_DEV void deq(const Addr& ad, int ks, bf16x8 out[2]) const {
    const int qi = 2 * (ks & 1) + ad.qhi;
    const int ls = 4 * (qi >> 1), hs = 2 * qi;
    const float s = h2f(dbits) * (float)sc;
    const uint32_t L[4] = {ql.x, ql.y, ql.z, ql.w};
    const uint32_t H[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t lw = L[2 * j + (i >> 2)], hw = H[2 * j + (i >> 2)];
        const int sh = 8 * (i & 3);
        const int v = (int)(((lw >> (sh + ls)) & 0xFu) | (((hw >> (sh + hs)) & 3u) << 4)) - 32;
        out[j][i] = (bf16)(s * (float)v);
      }
    }
  }
};

template <> struct MidRaw<FMT_Q8_0> {
  struct Addr {
    uint32_t qs, d;
    LA_DEV void init(const QW& w, int n, int q) {
      qs = (uint32_t)n * w.K + 16 * q;
      d = ((uint32_t)n * (w.K >> 5) + (q >> 1)) * 2;
    }
  };
  u32x4 qs;
  uint16_t dbits;
  LA_DEV void load(const QW& w, const Addr& a, int ks) {
    qs = *(const u32x4*)(w.p0 + 64 * ks + a.qs);
    dbits = *(const uint16_t*)(w.p1 + 4 * ks + a.d);
  }
  LA_DEV void deq(const Addr&, int, bf16x8 out[2]) const {
    const float d = h2f(dbits);
    const uint32_t v[4] = {qs.x, qs.y, qs.z, qs.w};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) out[j][i] = (bf16)(d * (float)(int8_t)((v[2 * j + (i >> 2)] >> (8 * (i & 3))) & 0xFFu));
    }
  }
};

}  // namespace la
