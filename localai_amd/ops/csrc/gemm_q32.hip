// Quantised GEMM on v_mfma_f32_32x32x16_bf16 for decode batches (M = 65..256) and prefill
// chunks (M up to 8192):
//   out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]   (fp32 split-K slabs, or bf16 [M][N] at S = 1)
//   GLU form: out[m][j] = act(x Wg[j]^T) * (x Wu[j]^T), bf16 [M][F]
// W stays in its GGUF quantisation (Q4_K, Q6_K, Q8_0).  SURVEY §2.8 K6 (the reference reaches
// this through ggml's mmq / dequant + BLAS inside llama_decode, backend/cpp/llama/grpc-server.cpp:1910).
//
// Why this shape (MI355X, profiles/r3_pmc_decode_gemms.md): the 16x16x32 tile kernel of
// gemm_q.hip spends ~2.75 VALU per weight on dequantisation and a 16x16x32 MFMA leaves only 8 of
// its 16 issue cycles to the vector pipe, so its loop was issue/latency bound at 28 % MFMA-busy.
// Here:
//   * one workgroup of 4 waves per CU, ONE wave per SIMD (the whole 512-entry register file);
//   * wave w owns the WN columns [w*WN, (w+1)*WN) of the tile and ALL BM rows (BM = 256 or 128):
//     each dequantised B fragment feeds BM/32 MFMAs and no two waves dequantise the same column,
//     so dequant costs ~2.5 VALU per 32x32x16 MFMA, well inside the 24 free vector-issue cycles
//     of each 32-cycle MFMA;
//   * X (bf16 rows of 128 B per K-step) arrives by LDS-DMA into an NS-slot ring, XOR-swizzled on
//     the SOURCE address so the A-fragment ds_read_b128 is conflict-free; each wave DMAs the raw
//     code bytes and the 8-byte scale records of ITS columns only (no other wave reads them);
//   * counted vmcnt + raw s_barrier, one barrier per 64-deep K-step; all LDS in one array;
//   * K permutation: lane half h of MFMA sub-step s reads the 8 k's of logical chunk
//     chunk(s, h) of the K-step, chosen so a lane's quant bytes for the whole K-step are one
//     16-byte run; A is read with the same permutation, so the dot product is unchanged.
#include <type_traits>

#include "qweight.h"

namespace la {

typedef float f32x16_t __attribute__((ext_vector_type(16)));

LA_DEV void q32_glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
LA_DEV void q32_glds16w(const void* g, void* l) {  // quantised weight bytes
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, LA_W_AUX);
}
LA_DEV void q32_glds4(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 4, 0, 0);
}

template <int N>
LA_DEV void q32_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int L>
LA_DEV void q32_wait_stages(int ahead) {
  // at most `ahead` stages (L DMAs each) still in flight; vmcnt holds 6 bits
  if (ahead <= 0) q32_vmwait<0>();
  else if (ahead == 1) q32_vmwait<L>();
  else if (ahead == 2) q32_vmwait<2 * L>();
  else if (ahead == 3 || 4 * L > 63) q32_vmwait<3 * L <= 63 ? 3 * L : 0>();
  else if (ahead == 4 || 5 * L > 63) q32_vmwait<4 * L>();
  else if (ahead == 5 || 6 * L > 63) q32_vmwait<5 * L <= 63 ? 5 * L : 0>();
  else if (ahead == 6 || 7 * L > 63) q32_vmwait<6 * L <= 63 ? 6 * L : 0>();
  else q32_vmwait<7 * L <= 63 ? 7 * L : 0>();
}

// One wave's columns: weight planes + row map (local column c -> weight row).
struct Q32Cols {
  const uint8_t* p0;
  const uint8_t* p1;
  const uint8_t* gsc;
  int K;
  int base, jbase, lim;  // row = base + min(jbase + c, lim)
  LA_DEV int n(int c) const { return base + min(jbase + c, lim); }
};

// 8-byte scale record of (row n, K-step ks) in the blocked plane [ceil(N/16)][K/64][16][8 B]
LA_DEV const uint8_t* q32_scale_rec(const Q32Cols& cm, int n, int ks) {
  return cm.gsc + ((size_t)((n >> 4) * (cm.K >> 6) + ks) * 16 + (n & 15)) * 8;
}

// ---------------------------------------------------------------- per-format traits
template <int FMT> struct Q32F;

// Q4_K: 32 B per column per K-step (byte i: k = i low nibble, k = 32 + i high nibble); lane half
// h reads bytes 16h .. 16h+15: sub-step s -> bytes 16h + 8(s&1) .., nibble s>>1.
template <> struct Q32F<FMT_Q4_K> {
  static constexpr int RAW = 32;
  LA_DEV static int chunk(int s, int h) { return 2 * h + (s & 1) + 4 * (s >> 1); }
  LA_DEV static int xk(int ks) { return 64 * ks; }
  LA_DEV static int kofs(int c) { return 8 * c; }
  // raw piece p (1 KiB: 32 columns x 32 B); 16-B halves swapped on columns with bit 3 set
  LA_DEV static void issue(const Q32Cols& cm, int ks, int p, uint8_t* dst, int lane) {
    const int c = 32 * p + (lane >> 1);
    const int lh = (lane & 1) ^ ((c >> 3) & 1);
    q32_glds16w(cm.p0 + (size_t)cm.n(c) * (cm.K >> 1) + 32 * ks + 16 * lh, dst + p * 1024);
  }
  static constexpr int PIECES(int WN) { return WN * RAW / 1024; }
  struct St {
    u32x4 q;
    float D0, M0, D1, M1;
  };
  LA_DEV static void load(const uint8_t* raw, const uint8_t* scl, int c, int h, int, St& st) {
    st.q = *(const u32x4*)(raw + c * 32 + 16 * (h ^ ((c >> 3) & 1)));
    const u32x2 s = *(const u32x2*)(scl + c * 8);  // f16 D0, -M0, D1, -M1 (la_gemm_scales)
    st.D0 = h2f(s.x & 0xFFFFu);
    st.M0 = h2f(s.x >> 16);
    st.D1 = h2f(s.y & 0xFFFFu);
    st.M1 = h2f(s.y >> 16);
  }
  template <int S>
  LA_DEV static bf16x8 deq(const St& st) {
    const uint32_t w0 = (S & 1) ? st.q.z : st.q.x, w1 = (S & 1) ? st.q.w : st.q.y;
    uint32_t lo, hi;
    // opaque masks: one v_cvt_f32_ubyteN per weight (a packed v_cvt_pk_f32_fp8 + v_pk_fma_f32 form,
    // 1.75 VALU per weight, was no faster on moe32 / the C=256 step and miscomputed the 64-column
    // variants: profiles/r6_moe_live.md)
    if constexpr (S < 2) {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(lo) : "v"(w0));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(hi) : "v"(w1));
    } else {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(lo) : "v"(w0 >> 4));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(hi) : "v"(w1 >> 4));
    }
    const float D = S < 2 ? st.D0 : st.D1, Mn = S < 2 ? st.M0 : st.M1;
    bf16x8 r;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      r[b] = (bf16)fmaf(D, (float)((lo >> (8 * b)) & 0xFFu), Mn);
      r[b + 4] = (bf16)fmaf(D, (float)((hi >> (8 * b)) & 0xFFu), Mn);
    }
    return r;
  }
};

// Q6_K: K-step (hh, part) of a super-block covers k in [128hh + 32part, +32) (run 0: ql low
// nibbles) and [128hh + 64 + 32part, +32) (run 1: ql high nibbles); the 32 qh bytes of half hh
// carry both runs' 2-bit fields (shifts 2part and 4 + 2part).  Per column per K-step: 32 B ql +
// 32 B qh, stored [ql: WN x 32][qh: WN x 32].
template <> struct Q32F<FMT_Q6_K> {
  static constexpr int RAW = 64;
  LA_DEV static int chunk(int s, int h) { return 2 * h + (s & 1) + 4 * (s >> 1); }
  LA_DEV static int xk(int ks) { return 256 * (ks >> 2) + 128 * ((ks >> 1) & 1) + 32 * (ks & 1); }
  LA_DEV static int kofs(int c) { return 8 * (c & 3) + 64 * (c >> 2); }
  static constexpr int PIECES(int WN) { return WN * RAW / 1024; }
  LA_DEV static void issue(const Q32Cols& cm, int ks, int p, uint8_t* dst, int lane) {
    const int sb = ks >> 2, hh = (ks >> 1) & 1, part = ks & 1;
    // pieces [0, P/2): ql of columns 32p ..; [P/2, P): qh
    const int half = p & 1;  // caller passes p = 2 * cb + half
    const int cb = p >> 1;
    const int c = 32 * cb + (lane >> 1);
    const int lh = (lane & 1) ^ ((c >> 3) & 1);
    const int n = cm.n(c);
    const uint8_t* src = half == 0 ? cm.p0 + (size_t)n * (cm.K >> 1) + 128 * sb + 64 * hh + 32 * part + 16 * lh
                                   : cm.p1 + (size_t)n * (cm.K >> 2) + 64 * sb + 32 * hh + 16 * lh;
    q32_glds16w(src, dst + p * 1024);
  }
  struct St {
    u32x4 ql, qh;
    float S0, S1;
    int sh;
  };
  // raw layout per wave: piece 2cb = ql of columns 32cb.., piece 2cb+1 = qh of the same columns
  LA_DEV static void load(const uint8_t* raw, const uint8_t* scl, int c, int h, int ks, St& st) {
    const int cb = c >> 5, cl = c & 31;
    const int o = cl * 32 + 16 * (h ^ ((cl >> 3) & 1));
    st.ql = *(const u32x4*)(raw + (2 * cb) * 1024 + o);
    st.qh = *(const u32x4*)(raw + (2 * cb + 1) * 1024 + o);
    const u32x2 s = *(const u32x2*)(scl + c * 8);  // f16 d*sc: run0 g0, run0 g1, run1 g0, run1 g1
    st.S0 = h2f(h ? (s.x >> 16) : (s.x & 0xFFFFu));
    st.S1 = h2f(h ? (s.y >> 16) : (s.y & 0xFFFFu));
    st.sh = 2 * (ks & 1);
  }
  template <int S>
  LA_DEV static bf16x8 deq(const St& st) {
    const uint32_t l0 = (S & 1) ? st.ql.z : st.ql.x, l1 = (S & 1) ? st.ql.w : st.ql.y;
    const uint32_t h0 = (S & 1) ? st.qh.z : st.qh.x, h1 = (S & 1) ? st.qh.w : st.qh.y;
    const int sh = st.sh + (S < 2 ? 0 : 4);
    uint32_t n0, n1, q0, q1;
    if constexpr (S < 2) {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n0) : "v"(l0));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n1) : "v"(l1));
    } else {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n0) : "v"(l0 >> 4));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n1) : "v"(l1 >> 4));
    }
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q0) : "v"((h0 >> sh) << 4), "s"(0x30303030u), "v"(n0));
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q1) : "v"((h1 >> sh) << 4), "s"(0x30303030u), "v"(n1));
    const float Sc = S < 2 ? st.S0 : st.S1, O = -32.0f * Sc;
    bf16x8 r;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      r[b] = (bf16)fmaf(Sc, (float)((q0 >> (8 * b)) & 0xFFu), O);
      r[b + 4] = (bf16)fmaf(Sc, (float)((q1 >> (8 * b)) & 0xFFu), O);
    }
    return r;
  }
};

// Q8_0: 64 B per column per K-step (two 32-blocks); lane half h reads block h (bytes 32h ..
// 32h+31): sub-step s -> bytes 32h + 8s.  16-B chunk q of a column stored at q ^ ((c >> 2) & 3).
template <> struct Q32F<FMT_Q8_0> {
  static constexpr int RAW = 64;
  LA_DEV static int chunk(int s, int h) { return 4 * h + s; }
  LA_DEV static int xk(int ks) { return 64 * ks; }
  LA_DEV static int kofs(int c) { return 8 * c; }
  static constexpr int PIECES(int WN) { return WN * RAW / 1024; }
  LA_DEV static void issue(const Q32Cols& cm, int ks, int p, uint8_t* dst, int lane) {
    const int c = 16 * p + (lane >> 2);
    const int lc = (lane & 3) ^ ((c >> 2) & 3);
    q32_glds16w(cm.p0 + (size_t)cm.n(c) * cm.K + 64 * ks + 16 * lc, dst + p * 1024);
  }
  struct St {
    u32x4 q0, q1;
    float d, o;
  };
  LA_DEV static void load(const uint8_t* raw, const uint8_t* scl, int c, int h, int, St& st) {
    const int sw = (c >> 2) & 3;
    st.q0 = *(const u32x4*)(raw + c * 64 + 16 * ((2 * h) ^ sw));
    st.q1 = *(const u32x4*)(raw + c * 64 + 16 * ((2 * h + 1) ^ sw));
    const uint32_t s = *(const uint32_t*)(scl + c * 8);  // f16 d0, d1
    st.d = h2f(h ? (s >> 16) : (s & 0xFFFFu));
    st.o = -128.0f * st.d;
  }
  template <int S>
  LA_DEV static bf16x8 deq(const St& st) {
    const u32x4& Q = S < 2 ? st.q0 : st.q1;
    const uint32_t w0 = (S & 1) ? Q.z : Q.x, w1 = (S & 1) ? Q.w : Q.y;
    uint32_t lo, hi;  // int8 -> q + 128 as an unsigned byte
    asm("v_xor_b32 %0, 0x80808080, %1" : "=v"(lo) : "v"(w0));
    asm("v_xor_b32 %0, 0x80808080, %1" : "=v"(hi) : "v"(w1));
    bf16x8 r;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      r[b] = (bf16)fmaf(st.d, (float)((lo >> (8 * b)) & 0xFFu), st.o);
      r[b + 4] = (bf16)fmaf(st.d, (float)((hi >> (8 * b)) & 0xFFu), st.o);
    }
    return r;
  }
};

template <int FMT, int BM, int WN, int NW_ = 4>
struct Q32Geo {
  static constexpr int NW = NW_;
  static constexpr int BN = NW * WN;
  static constexpr int XB = BM * 128;                      // X bytes per slot
  static constexpr int RW = WN * Q32F<FMT>::RAW;            // raw bytes per wave per slot
  static constexpr int SW = WN * 8;                         // scale bytes per wave per slot
  static constexpr int SLOT = XB + NW * (RW + SW);
  static constexpr int PX = BM / 8 / NW;                    // X DMA pieces per wave
  static constexpr int PR = RW / 1024;                      // raw pieces per wave
  static constexpr int PS = SW / 256;                       // scale dword pieces per wave
  static constexpr int L = PX + PR + PS;                    // DMAs per wave per stage
};

template <int FMT, int BM, int WN, int NW = 4>
constexpr int q32_ns() {
  // deepest ring (<= 4 slots) that fits 160 KiB
  constexpr int s = Q32Geo<FMT, BM, WN, NW>::SLOT;
  return (4 * s <= 163840) ? 4 : (3 * s <= 163840) ? 3 : 2;
}

struct Q32Glu {
  QW b;
  int oa, ob, F, act;
};

// Grouped (MoE) tiles: MOE 1 gathers X row m from rows[m] / rdiv (a routed pair's token), MOE 2
// scatters output row m to slab (split * rdiv + slot) row t of pair p = rows[m] (t = p / rdiv,
// slot = p % rdiv), scaled by the routing weight wts[p].
struct Q32Moe {
  const int* rows;
  int rdiv;
  const float* wts;
};

LA_DEV float q32_gelu_tanh(float x) { return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))); }

// One (M tile, N tile, K split).  GLU: columns [0, BN/2) of the tile are gate rows, [BN/2, BN)
// the matching up rows; no split.
// MBL (<= BM / 32): row blocks that hold rows of this tile; the MFMAs and A-fragment reads of the
// blocks past it are not issued (grouped MoE tiles: an expert's last row chunk is often short).
template <int FMT, int BM, int WN, int NS, bool GLU, int PIPE = 0, int NW_ = 4, int ABL = 0, int MOE = 0,
          int MBL = BM / 32>
LA_DEV void q32_tile(uint8_t* __restrict__ lds, const QW& w, int tile, const bf16* __restrict__ X, int ldx, int M,
                     int per_split, int m_tiles, int n_tiles, float* __restrict__ out, bf16* __restrict__ outb,
                     int ldo, long slab, const Q32Glu& glu, const Q32Moe& moe = Q32Moe{}) {
  using F = Q32F<FMT>;
  using G = Q32Geo<FMT, BM, WN, NW_>;
  constexpr int NW = G::NW, BN = G::BN, MB = BM / 32, CB = WN / 32;
  constexpr int XB = G::XB, SLOT = G::SLOT, PX = G::PX, PR = G::PR, PS = G::PS, L = G::L;
  static_assert(WN % 32 == 0 && BM % 32 == 0 && PR * 1024 == G::RW && PS * 256 == G::SW, "geometry");
  static_assert(MBL >= 1 && MBL <= MB, "live row blocks");
  static_assert(NS >= 2 && NS <= 8 && NS * SLOT <= 163840, "ring");

  const int mt_i = tile % m_tiles;
  const int rest = tile / m_tiles;
  const int nt_i = rest % n_tiles;
  const int split = rest / n_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = mt_i * BM;
  const int KS = w.K >> 6;
  const int ks0 = split * per_split;
  const int nk = min(KS, ks0 + per_split) - ks0;
  if (nk <= 0) return;

  // this wave's columns
  Q32Cols cm;
  if constexpr (GLU) {
    const bool up = wave >= NW / 2;
    const QW& q = up ? glu.b : w;
    cm = Q32Cols{q.p0, q.p1, q.p2, q.K, up ? glu.ob : glu.oa, nt_i * (BN / 2) + (up ? wave - NW / 2 : wave) * WN,
                 glu.F - 1};
  } else {
    cm = Q32Cols{w.p0, w.p1, w.p2, w.K, 0, nt_i * BN + wave * WN, w.N - 1};
  }

  // X DMA: piece j of this wave = rows 8(wave*PX + j) .. +8; lane -> (row, physical 16-B chunk)
  uint32_t xoff[PX];
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int r = 8 * (wave * PX + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);  // logical chunk stored at this physical chunk
    const int mr = min(m0 + r, M - 1);
    xoff[j] = (uint32_t)(MOE == 1 ? moe.rows[mr] / moe.rdiv : mr) * ldx + F::kofs(c);
  }
  // scale records of this wave's columns: piece p = columns 32p .. 32p+31, lane -> (column, dword)
  const uint8_t* srec[PS];
#pragma unroll
  for (int p = 0; p < PS; ++p) srec[p] = q32_scale_rec(cm, cm.n(32 * p + (lane >> 1)), 0) + 4 * (lane & 1);

  auto issue = [&](int t) {
    if constexpr (ABL & 4) return;  // probe: no DMA
    const int ks = ks0 + t;
    uint8_t* sl = lds + (t % NS) * SLOT;
    const bf16* xk = X + F::xk(ks);
#pragma unroll
    for (int j = 0; j < PX; ++j) q32_glds16(xk + xoff[j], sl + (wave * PX + j) * 1024);
    uint8_t* rw = sl + XB + wave * G::RW;
#pragma unroll
    for (int p = 0; p < PR; ++p) F::issue(cm, ks, p, rw, lane);
    uint8_t* sw = sl + XB + NW * G::RW + wave * G::SW;
#pragma unroll
    for (int p = 0; p < PS; ++p) q32_glds4(srec[p] + (size_t)ks * 128, sw + p * 256);
  };

  f32x16_t acc[MB][CB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  int aoff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) aoff[s] = r32 * 128 + 16 * (F::chunk(s, h) ^ ((r32 >> 1) & 7));

  // Software pipeline (one barrier per K-step, in the MIDDLE of the step).  A fragments live in
  // two fixed register sets: alo = sub-steps 0, 1 and ahi = sub-steps 2, 3 of a K-step.
  //   step t start : issue the LDS reads of A(t) sub-steps 2, 3 -> ahi
  //   first half   : MFMA sub-steps 0, 1 on alo (read half a step ago)
  //   mid barrier  : this wave's DMAs of stage t+1 landed (counted vmcnt) -> s_barrier -> slot
  //                  t % NS is free (every wave's reads of A(t) / B(t) completed: lgkmcnt(0)
  //                  before the barrier) -> issue the DMAs of stage t+NS into it -> LDS reads of
  //                  B(t+1) and of A(t+1) sub-steps 0, 1 -> alo
  //   second half  : MFMA sub-steps 2, 3 on ahi
  // Every LDS read hides under half a K-step of MFMAs; the DMA ring runs NS-1 stages ahead.
  auto read_a = [&](bf16x8 (&dst)[2][MB], int t, int s0) {
    const uint8_t* sl = lds + (t % NS) * SLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mb = 0; mb < MBL; ++mb) {
        if constexpr (ABL & 8) asm volatile("; probe: no A read" : "=v"(dst[s][mb]));
        else dst[s][mb] = *(const bf16x8*)(sl + mb * 4096 + aoff[s0 + s]);
      }
  };
  auto read_b = [&](typename F::St (&dst)[CB], int t) {
    const uint8_t* sl = lds + (t % NS) * SLOT;
    const uint8_t* rw = sl + XB + wave * G::RW;
    const uint8_t* sw = sl + XB + NW * G::RW + wave * G::SW;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) F::load(rw, sw, cb * 32 + r32, h, ks0 + t, dst[cb]);
  };
  auto mm = [&](const bf16x8 (&a)[MB], const bf16x8 (&b)[CB]) {
    if constexpr (LA_SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mb = 0; mb < MBL; ++mb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        if constexpr (ABL & 1) asm volatile("; probe: no MFMA" ::"v"(a[mb]), "v"(b[cb]));
        else acc[mb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mb], b[cb], acc[mb][cb], 0, 0, 0);
      }
    if constexpr (LA_SETPRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto deqs = [&](bf16x8 (&b)[CB], const typename F::St (&st)[CB], auto S_) {
    constexpr int S = decltype(S_)::value;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      if constexpr (ABL & 2) asm volatile("; probe: no dequant" : "=v"(b[cb]) : "v"(st[cb].q));
      else b[cb] = F::template deq<S>(st[cb]);
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;
  auto mid = [&](int t, bf16x8 (&alo)[2][MB], typename F::St (&st)[CB]) {
    if constexpr (!(ABL & 16)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of slot t done
      q32_wait_stages<L>(min(NS - 2, nk - 2 - t));        // this wave's DMAs of stage t+1 landed
      __builtin_amdgcn_s_barrier();                       // ... everyone's; slot t free everywhere
    }
    asm volatile("" ::: "memory");
    read_b(st, t + 1);
    if (t + NS < nk) issue(t + NS);
    read_a(alo, t + 1, 0);
  };

  bf16x8 alo[2][MB], ahi[2][MB];
  typename F::St st[CB];
  // prologue: all NS slots in flight, then stage 0's B and A sub-steps 0, 1 into registers
#pragma unroll
  for (int i = 0; i < NS; ++i)
    if (i < nk) issue(i);
  q32_wait_stages<L>(min(NS - 1, nk - 1));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_b(st, 0);
  read_a(alo, 0, 0);

  if constexpr (PIPE == 0) {
    auto step = [&](int t, bool more) {
      read_a(ahi, t, 2);
      bf16x8 b[CB], b2[CB], b3[CB];
      deqs(b, st, S0{});
      mm(alo[0], b);
      deqs(b, st, S1{});
      mm(alo[1], b);
      deqs(b2, st, S2{});
      deqs(b3, st, S3{});
      if (more) mid(t, alo, st);
      mm(ahi[0], b2);
      mm(ahi[1], b3);
    };
    for (int t = 0; t + 1 < nk; ++t) step(t, true);
    step(nk - 1, false);
  } else {
    // Interleaved (sched_group_barrier): the B fragments of the next sub-step are dequantised
    // between the MFMAs of the current one, and the LDS reads are threaded between MFMAs, so
    // neither the dequant VALU nor the read issue serialises with the matrix pipe.  The last
    // K-step is peeled so the loop body has no branch around MFMAs (the accumulators stay put).
    constexpr int NM = MBL * CB;                     // MFMAs per sub-step
    constexpr int VPM = (24 * CB + NM - 1) / NM;     // dequant VALU per MFMA slot
    constexpr int RPM = (2 * MBL + NM - 1) / NM;     // LDS reads per MFMA slot
    bf16x8 b0[CB];
    deqs(b0, st, S0{});
    auto first_half = [&](int t, bf16x8 (&b2)[CB], bf16x8 (&b3)[CB]) {
      bf16x8 b1[CB];
      read_a(ahi, t, 2);
      deqs(b1, st, S1{});
      mm(alo[0], b0);
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);  // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
      deqs(b2, st, S2{});
      deqs(b3, st, S3{});
      mm(alo[1], b1);
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x002, 2 * VPM, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    for (int t = 0; t + 1 < nk; ++t) {
      bf16x8 b2[CB], b3[CB];
      first_half(t, b2, b3);
      mid(t, alo, st);
      mm(ahi[0], b2);
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        __builtin_amdgcn_sched_group_barrier(0x100, RPM + 1, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      deqs(b0, st, S0{});
      mm(ahi[1], b3);
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 3);
        __builtin_amdgcn_sched_group_barrier(0x002, VPM, 3);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      bf16x8 b2[CB], b3[CB];
      first_half(nk - 1, b2, b3);
      mm(ahi[0], b2);
      mm(ahi[1], b3);
    }
  }

  // ---- epilogue through LDS: acc[mb][cb] reg j = (row mb*32 + (j&3) + 8(j>>2) + 4h, col cb*32 + r32)
  // each wave parks ER rows x WN of its columns in [ER][WN] f32 (conflict-free for both the
  // per-register ds_write_b32 and the 16-B row reads), then every lane stores 16 B of one row.
  constexpr int ERF = (NS * SLOT) / (NW * WN * 4) / 32 * 32;
  constexpr int ER = ERF >= BM ? BM : ERF >= BM / 2 ? BM / 2 : BM / 4;
  constexpr int EP = (BM + ER - 1) / ER;
  static_assert(ER >= 32 && BM % ER == 0, "epilogue image");
  constexpr int CH = WN / 4;  // 16-B chunks per image row
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave has finished reading the ring
  asm volatile("" ::: "memory");
  float* img = (float*)lds + wave * ER * WN;
  const bool f32out = outb == nullptr;
  float* o = f32out ? out + (size_t)split * slab : nullptr;
#pragma unroll
  for (int pass = 0; pass < EP; ++pass) {
#pragma unroll
    for (int mb = pass * (ER / 32); mb < (pass + 1) * (ER / 32); ++mb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          img[((mb % (ER / 32)) * 32 + (j & 3) + 8 * (j >> 2) + 4 * h) * WN + cb * 32 + r32] = acc[mb][cb][j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (GLU) {
      __builtin_amdgcn_s_barrier();  // the partner wave's rows are parked
      asm volatile("" ::: "memory");
      if (wave < NW / 2) {
        const float* pimg = (const float*)lds + (wave + NW / 2) * ER * WN;
        const int cbase = nt_i * (BN / 2) + wave * WN;
#pragma unroll 4
        for (int it = 0; it < ER * CH / 64; ++it) {
          const int idx = it * 64 + lane;
          const int r = idx / CH, c4 = idx % CH;
          const int m = m0 + pass * ER + r, j = cbase + 4 * c4;
          if (m < M) {
            const f32x4 gv = *(const f32x4*)(img + r * WN + 4 * c4);
            const f32x4 uv = *(const f32x4*)(pimg + r * WN + 4 * c4);
            bf16x4 hv;
#pragma unroll
            for (int e = 0; e < 4; ++e) hv[e] = (bf16)((glu.act == 0 ? silu(gv[e]) : q32_gelu_tanh(gv[e])) * uv[e]);
            if (j + 3 < glu.F) {
              *(bf16x4*)(outb + (size_t)m * ldo + j) = hv;
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (j + e < glu.F) outb[(size_t)m * ldo + j + e] = hv[e];
            }
          }
        }
      }
    } else {
      const int cbase = nt_i * BN + wave * WN;
#pragma unroll 4
      for (int it = 0; it < ER * CH / 64; ++it) {
        const int idx = it * 64 + lane;
        const int r = idx / CH, c4 = idx % CH;
        const f32x4 v = *(const f32x4*)(img + r * WN + 4 * c4);
        const int m = m0 + pass * ER + r, n = cbase + 4 * c4;
        if (MOE == 2 && m < M) {
          // routed pair -> (slot slab, token row), weighted: the consumer's slab sum is the combine
          const int p = moe.rows[m], t = p / moe.rdiv, slot = p - t * moe.rdiv;
          const float sc = moe.wts[p];
          float* dst = out + ((size_t)split * moe.rdiv + slot) * slab + (size_t)t * ldo + n;
          if (n + 3 < w.N) {
            *(f32x4*)dst = f32x4{v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < w.N) dst[e] = v[e] * sc;
          }
        } else if (m < M) {
          if (n + 3 < w.N) {
            if (f32out) {
              *(f32x4*)(o + (size_t)m * ldo + n) = v;
            } else {
              bf16x4 bv;
              bv[0] = (bf16)v[0]; bv[1] = (bf16)v[1]; bv[2] = (bf16)v[2]; bv[3] = (bf16)v[3];
              *(bf16x4*)(outb + (size_t)m * ldo + n) = bv;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < w.N) {
                if (f32out) o[(size_t)m * ldo + n + e] = v[e];
                else outb[(size_t)m * ldo + n + e] = (bf16)v[e];
              }
          }
        }
      }
    }
    if (EP > 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // images read before the next pass overwrites them
      asm volatile("" ::: "memory");
    }
  }
}

template <int FMT, int BM, int WN, int NW = 4>
constexpr int q32_lds() {
  return q32_ns<FMT, BM, WN, NW>() * Q32Geo<FMT, BM, WN, NW>::SLOT;
}

// Kernel configurations: tile BM x (NW * WN), NW waves (1 or 2 per SIMD), schedule PIPE.
template <int BM_, int WN_, int NW_, int PIPE_>
struct Q32Cfg {
  static constexpr int BM = BM_, WN = WN_, NW = NW_, PIPE = PIPE_, BN = NW_ * WN_;
};

// Tiles (M fastest, then N, then split) in XCD-contiguous runs: blocks b, b + 8, ... share an
// XCD, and each XCD takes a contiguous run, so the tiles of one K split share X's slice in L2.
template <int FMT, class C, int ABL = 0>
__global__ __launch_bounds__(C::NW * 64, 1) __attribute__((amdgpu_waves_per_eu(C::NW / 4, C::NW / 4))) void qgemm32_kernel(QW w, const bf16* __restrict__ X, int ldx, int M,
                                                                int per_split, int m_tiles, int n_tiles,
                                                                int real_tiles, float* __restrict__ out,
                                                                bf16* __restrict__ outb, int ldo, long slab) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[q32_lds<FMT, C::BM, C::WN, C::NW>()];
  const int tile = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (tile >= real_tiles) return;  // grid padded to a multiple of 8
  q32_tile<FMT, C::BM, C::WN, q32_ns<FMT, C::BM, C::WN, C::NW>(), false, C::PIPE, C::NW, ABL>(
      lds, w, tile, X, ldx, M, per_split, m_tiles, n_tiles, out, outb, ldo, slab, Q32Glu{});
}

// Two weights of one fused output (Q4_K q|k beside a Q6_K v): segment B's tiles follow A's.
template <int FA, int FB, class C>
__global__ __launch_bounds__(C::NW * 64, 1) __attribute__((amdgpu_waves_per_eu(C::NW / 4, C::NW / 4))) void qgemm32_2_kernel(QW wa, QW wb, int col_b, const bf16* __restrict__ X,
                                                                  int ldx, int M, int per_split, int m_tiles,
                                                                  int n_tiles_a, int n_tiles_b, int tiles_a,
                                                                  int real_tiles, float* __restrict__ out,
                                                                  bf16* __restrict__ outb, int ldo, long slab) {
  constexpr int LA_ = q32_lds<FA, C::BM, C::WN, C::NW>(), LB_ = q32_lds<FB, C::BM, C::WN, C::NW>();
  __shared__ __attribute__((aligned(1024))) uint8_t lds[LA_ > LB_ ? LA_ : LB_];
  const int tile = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (tile >= real_tiles) return;
  if (tile < tiles_a) {
    q32_tile<FA, C::BM, C::WN, q32_ns<FA, C::BM, C::WN, C::NW>(), false, C::PIPE, C::NW>(
        lds, wa, tile, X, ldx, M, per_split, m_tiles, n_tiles_a, out, outb, ldo, slab, Q32Glu{});
  } else {
    q32_tile<FB, C::BM, C::WN, q32_ns<FB, C::BM, C::WN, C::NW>(), false, C::PIPE, C::NW>(
        lds, wb, tile - tiles_a, X, ldx, M, per_split, m_tiles, n_tiles_b, out ? out + col_b : nullptr,
        outb ? outb + col_b : nullptr, ldo, slab, Q32Glu{});
  }
}

template <int FMT, class C>
__global__ __launch_bounds__(C::NW * 64, 1) __attribute__((amdgpu_waves_per_eu(C::NW / 4, C::NW / 4))) void qgemm32_glu_kernel(QW wa, Q32Glu glu, const bf16* __restrict__ X,
                                                                    int ldx, int M, int m_tiles, int n_tiles,
                                                                    int real_tiles, bf16* __restrict__ outb, int ldo) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[q32_lds<FMT, C::BM, C::WN, C::NW>()];
  const int tile = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (tile >= real_tiles) return;
  q32_tile<FMT, C::BM, C::WN, q32_ns<FMT, C::BM, C::WN, C::NW>(), true, C::PIPE, C::NW>(
      lds, wa, tile, X, ldx, M, wa.K >> 6, m_tiles, n_tiles, nullptr, outb, ldo, 0, glu);
}

// variant ids (shared with ops/__init__.py Q32_VARIANTS): tile BM x BN, waves, schedule
//   0: 256 x 128 (4 waves)   1: 128 x 256 (4)   2: 256 x 256 (4)   3: 128 x 128 (4)
//   8: 128 x 256 (8 waves, 2 per SIMD);  +4 (4 .. 7) / 9: the same with the interleaved schedule (PIPE = 1)
// The 256 x 256 tiles (2, 6) hold 256 accumulator registers per lane: Q4_K only (the larger
// Q6_K / Q8_0 fragment state does not fit beside them without spilling).
template <bool BIG, class Fn>
static int q32_var(int var, Fn&& fn) {
  if constexpr (BIG) {
    if (var == 2) { fn(Q32Cfg<256, 64, 4, 0>{}); return 0; }
    if (var == 6) { fn(Q32Cfg<256, 64, 4, 1>{}); return 0; }
  }
  switch (var) {
    case 0: fn(Q32Cfg<256, 32, 4, 0>{}); break;
    case 1: fn(Q32Cfg<128, 64, 4, 0>{}); break;
    case 3: fn(Q32Cfg<128, 32, 4, 0>{}); break;
    case 4: fn(Q32Cfg<256, 32, 4, 1>{}); break;
    case 5: fn(Q32Cfg<128, 64, 4, 1>{}); break;
    case 7: fn(Q32Cfg<128, 32, 4, 1>{}); break;
    case 8: fn(Q32Cfg<128, 32, 8, 0>{}); break;
    case 9: fn(Q32Cfg<128, 32, 8, 1>{}); break;
    default: return -1;
  }
  return 0;
}

template <int FMT, int ABL, class C>
static void q32_go(C, const QW& w, const bf16* X, int ldx, int M, int splits, float* out, bf16* outb, int ldo,
                   long slab, hipStream_t st) {
  const int KS = w.K >> 6;
  const int per = (KS + splits - 1) / splits;
  const int m_tiles = (M + C::BM - 1) / C::BM, n_tiles = (w.N + C::BN - 1) / C::BN;
  const int real = m_tiles * n_tiles * splits;
  const int grid = (real + 7) / 8 * 8;
  hipLaunchKernelGGL((qgemm32_kernel<FMT, C, ABL>), dim3(grid), dim3(C::NW * 64), 0, st, w, X, ldx, M, per, m_tiles,
                     n_tiles, real, out, outb, ldo, slab);
}

template <int FMT>
static int q32_launch(int var, const QW& w, const bf16* X, int ldx, int M, int splits, float* out, bf16* outb,
                      int ldo, long slab, hipStream_t st) {
  return q32_var<FMT == FMT_Q4_K>(var, [&](auto c) { q32_go<FMT, 0>(c, w, X, ldx, M, splits, out, outb, ldo, slab, st); });
}

template <int ABL>
static int q32_probe_launch(int var, const QW& w, const bf16* X, int ldx, int M, int splits, float* out, int ldo,
                            long slab, hipStream_t st) {
  if (var == 0) q32_go<FMT_Q4_K, ABL>(Q32Cfg<256, 32, 4, 0>{}, w, X, ldx, M, splits, out, nullptr, ldo, slab, st);
  else if (var == 4) q32_go<FMT_Q4_K, ABL>(Q32Cfg<256, 32, 4, 1>{}, w, X, ldx, M, splits, out, nullptr, ldo, slab, st);
  else if (var == 8) q32_go<FMT_Q4_K, ABL>(Q32Cfg<128, 32, 8, 0>{}, w, X, ldx, M, splits, out, nullptr, ldo, slab, st);
  else return -1;
  return 0;
}

template <int FA, int FB>
static int q32_launch2(int var, const QW& wa, const QW& wb, const bf16* X, int ldx, int M, int splits, float* out,
                       bf16* outb, int ldo, long slab, hipStream_t st) {
  const int KS = wa.K >> 6;
  const int per = (KS + splits - 1) / splits;
  return q32_var<false>(var, [&](auto c) {
    using C = decltype(c);
    const int m_tiles = (M + C::BM - 1) / C::BM;
    const int nta = (wa.N + C::BN - 1) / C::BN, ntb = (wb.N + C::BN - 1) / C::BN;
    const int tiles_a = m_tiles * nta * splits;
    const int real = tiles_a + m_tiles * ntb * splits;
    const int grid = (real + 7) / 8 * 8;
    hipLaunchKernelGGL((qgemm32_2_kernel<FA, FB, C>), dim3(grid), dim3(C::NW * 64), 0, st, wa, wb, wa.N, X, ldx, M,
                       per, m_tiles, nta, ntb, tiles_a, real, out, outb, ldo, slab);
  });
}

template <int FMT>
static int q32_launch_glu(int var, const QW& wa, const Q32Glu& glu, const bf16* X, int ldx, int M, bf16* outb,
                          int ldo, hipStream_t st) {
  return q32_var<FMT == FMT_Q4_K>(var, [&](auto c) {
    using C = decltype(c);
    const int m_tiles = (M + C::BM - 1) / C::BM, n_tiles = (glu.F + C::BN / 2 - 1) / (C::BN / 2);
    const int real = m_tiles * n_tiles;
    const int grid = (real + 7) / 8 * 8;
    hipLaunchKernelGGL((qgemm32_glu_kernel<FMT, C>), dim3(grid), dim3(C::NW * 64), 0, st, wa, glu, X, ldx, M, m_tiles,
                       n_tiles, real, outb, ldo);
  });
}

// ---------------------------------------------------------------- grouped MoE GEMM
// The routed rows of every expert through the same per-wave-columns MFMA tile (replaces the
// 16-column-per-wave moe_gemm_kernel of moe.hip for wide batches: there each wave dequantised
// its own 16 columns for 16-row MFMAs, 12.8 VALU per MFMA; here one dequantised 32-column
// fragment feeds BM/32 32x32x16 MFMAs).  Tile id -> (row chunk fastest, column tile, split,
// expert); chunks past an expert's row count exit at once, so any routing is one fixed launch
// (graph-capturable).  MODE 1: gate|up of the expert (gate rows [0, F), up rows [F, 2F) of one
// weight) with the GLU fused, bf16 h rows in grouped order (row off[e] + m); MODE 2: down
// projection of the grouped h rows, routing-weighted fp32 output scattered to slab
// (split * topk + slot) row token.  qws[e] = {codes, aux, blocked scale plane, -, N, K}.
template <class C, int OCC_, int NS_ = 0, bool LIVE_ = false>
struct MoeCfg : C {
  static constexpr int OCC = OCC_;  // workgroups per CU the register budget is sized for
  static constexpr int NS = NS_;    // ring slots (0: q32_ns, <= 4); up to 8 stages of weight bytes in flight
  static constexpr bool LIVE = LIVE_;  // MFMAs of the chunk's live row blocks only (per-tile dispatch)
};

template <int FMT, class C, int MODE, int ABL = 0>
__global__ __launch_bounds__(C::NW * 64) __attribute__((amdgpu_waves_per_eu(C::NW / 4 * C::OCC, C::NW / 4 * C::OCC))) void moe32_kernel(
    const QW* __restrict__ qws, const int* __restrict__ order, const int* __restrict__ off, int topk,
    const bf16* __restrict__ X, int ldx, int mch, int n_tiles, int splits, int per_split, int real_tiles,
    const float* __restrict__ wts, float* __restrict__ out, bf16* __restrict__ outb, int ldo, long slab, int F, int act) {
  constexpr int FIT = 163840 / Q32Geo<FMT, C::BM, C::WN, C::NW>::SLOT;  // Q6_K / Q8_0 slots are larger
  constexpr int NS = C::NS ? (C::NS < FIT ? C::NS : FIT) : q32_ns<FMT, C::BM, C::WN, C::NW>();
  __shared__ __attribute__((aligned(1024))) uint8_t lds[NS * Q32Geo<FMT, C::BM, C::WN, C::NW>::SLOT];
  // expert fastest, then row chunk, column tile, split; XCD-contiguous runs of tiles therefore
  // hold every expert's tiles of a few column tiles: the XCDs stay balanced however the router
  // skews the row counts, and the row chunks of one (expert, column tile) share its weight
  // bytes in one L2
  const int tile = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (tile >= real_tiles) return;
  const int E = real_tiles / (mch * n_tiles * splits);
  const int e = tile % E;
  int r = tile / E;
  const int chunk = r % mch;
  r /= mch;
  const int nt = r % n_tiles, split = r / n_tiles;
  const int o0 = off[e], Me = off[e + 1] - o0;
  if (chunk * C::BM >= Me) return;
  const int mte = (Me + C::BM - 1) / C::BM;
  const int t2 = chunk + mte * (nt + n_tiles * split);
  QW w = qws[e];
  const Q32Moe mo{order + o0, topk, wts};
  // row blocks of this chunk that hold rows: the tile runs only their MFMAs (wave-uniform)
  const int live = min(C::BM / 32, (Me - chunk * C::BM + 31) / 32);
  auto run = [&](auto mbl_) {
    constexpr int MBL = decltype(mbl_)::value;
    if constexpr (MODE == 1) {
      const Q32Glu glu{w, 0, F, F, act};
      QW wg = w;
      wg.N = F;
      q32_tile<FMT, C::BM, C::WN, NS, true, C::PIPE, C::NW, ABL, 1, MBL>(lds, wg, t2, X, ldx, Me, w.K >> 6, mte,
                                                                        n_tiles, nullptr, outb + (size_t)o0 * ldo,
                                                                        ldo, 0, glu, mo);
    } else {
      q32_tile<FMT, C::BM, C::WN, NS, false, C::PIPE, C::NW, ABL, 2, MBL>(lds, w, t2, X + (size_t)o0 * ldx, ldx, Me,
                                                                         per_split, mte, n_tiles, out, nullptr, ldo,
                                                                         slab, Q32Glu{}, mo);
    }
  };
  if constexpr (C::LIVE && C::BM / 32 >= 4) {
    if (live <= 1) run(std::integral_constant<int, 1>{});
    else if (live == 2) run(std::integral_constant<int, 2>{});
    else if (live == 3) run(std::integral_constant<int, 3>{});
    else run(std::integral_constant<int, C::BM / 32>{});
  } else if constexpr (C::LIVE && C::BM / 32 >= 2) {
    if (live <= 1) run(std::integral_constant<int, 1>{});
    else run(std::integral_constant<int, C::BM / 32>{});
  } else {
    run(std::integral_constant<int, C::BM / 32>{});
  }
}

// MoE variant ids (ops/__init__.py MOE32_TILES): row tile x (waves x columns per wave), schedule
template <bool Q4, class Fn>
static int moe32_var(int var, Fn&& fn) {
  switch (var) {
    case 0: fn(MoeCfg<Q32Cfg<64, 32, 4, 0>, 2>{}); break;
    case 1: fn(MoeCfg<Q32Cfg<64, 32, 4, 1>, 2>{}); break;
    case 2: fn(MoeCfg<Q32Cfg<64, 64, 4, 0>, 2>{}); break;
    case 3: fn(MoeCfg<Q32Cfg<64, 64, 4, 1>, 2>{}); break;
    case 4: fn(MoeCfg<Q32Cfg<64, 32, 8, 0>, 2>{}); break;
    case 5: fn(MoeCfg<Q32Cfg<32, 32, 4, 0>, 2>{}); break;
    case 6: fn(MoeCfg<Q32Cfg<128, 32, 4, 1>, 1>{}); break;
    case 7: fn(MoeCfg<Q32Cfg<64, 32, 4, 0>, 3>{}); break;
    case 8: fn(MoeCfg<Q32Cfg<64, 32, 4, 1>, 3>{}); break;
    case 9: fn(MoeCfg<Q32Cfg<32, 32, 4, 0>, 4>{}); break;
    case 10: fn(MoeCfg<Q32Cfg<32, 64, 4, 0>, 2>{}); break;
    case 11: fn(MoeCfg<Q32Cfg<64, 64, 4, 0>, 1, 8>{}); break;
    case 12: fn(MoeCfg<Q32Cfg<32, 64, 4, 0>, 2, 5>{}); break;
    case 13: fn(MoeCfg<Q32Cfg<64, 32, 4, 0>, 1, 8>{}); break;
    case 14: fn(MoeCfg<Q32Cfg<32, 64, 4, 0>, 1, 8>{}); break;
    // live-row-block dispatch: one 96..128-row chunk per expert at decode batches, MFMAs of its
    // live 32-row blocks only (an expert's weights dequantised once, not once per 64 rows)
    case 15: fn(MoeCfg<Q32Cfg<128, 32, 8, 0>, 1, 0, true>{}); break;
    case 16: fn(MoeCfg<Q32Cfg<128, 32, 4, 0>, 1, 0, true>{}); break;
    case 17: fn(MoeCfg<Q32Cfg<64, 32, 8, 0>, 2, 0, true>{}); break;
    case 18: fn(MoeCfg<Q32Cfg<128, 32, 4, 1>, 1, 0, true>{}); break;
    // 64 columns per wave: twice the weight bytes per ring stage against the same X stage (the
    // 128-row X slab is most of a stage), so twice the weight bytes in flight per CU
    case 19: if constexpr (Q4) fn(MoeCfg<Q32Cfg<128, 64, 8, 0>, 1, 0, true>{}); else return -1; break;
    case 20: if constexpr (Q4) fn(MoeCfg<Q32Cfg<128, 64, 4, 0>, 1, 0, true>{}); else return -1; break;
    default: return -1;
  }
  return 0;
}

template <int FMT, int MODE>
static int moe32_launch(int var, const QW* qws, int N, int K, int E, const int* order, const int* off, int topk,
                        const bf16* X, int ldx, int maxM, int splits, const float* wts, float* out, bf16* outb,
                        int ldo, long slab, int act, hipStream_t st) {
  const int KS = K >> 6, per = (KS + splits - 1) / splits;
  // 64 columns per wave at 128 rows spill with Q6_K / Q8_0's larger fragment state: those formats
  // take the 32-column form of the same chunking
  if (FMT != FMT_Q4_K && (var == 19 || var == 20)) var -= 4;
  return moe32_var<FMT == FMT_Q4_K>(var, [&](auto c) {
    using C = decltype(c);
    const int mch = (maxM + C::BM - 1) / C::BM;
    const int n_tiles = MODE == 1 ? (N + C::BN / 2 - 1) / (C::BN / 2) : (N + C::BN - 1) / C::BN;
    const long real = (long)E * mch * n_tiles * splits;
    const int grid = (int)((real + 7) / 8 * 8);
    hipLaunchKernelGGL((moe32_kernel<FMT, C, MODE>), dim3(grid), dim3(C::NW * 64), 0, st, qws, order, off, topk, X,
                       ldx, mch, n_tiles, splits, per, (int)real, wts, out, outb, ldo, slab, N, act);
  });
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// Same operand conventions as la_qgemm_tile (gemm_q.hip): p0/p1 format planes, gsc the blocked
// scale plane (la_gemm_scales); out fp32 slabs [splits][M][ldo] (stride slab) or bf16 [M][ldo].
extern "C" int la_qgemm32(int fmt, const void* p0, const void* p1, const void* gsc, int N, int K, const void* X,
                          int ldx, int M, int splits, void* out, int ldo, long slab, int out_bf16, int var,
                          void* stream) {
  using namespace la;
  if (M < 1 || N < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7) || !gsc) return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  if ((long)M * ldx >= (1L << 31)) return -1;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)gsc, nullptr, N, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = out_bf16 ? nullptr : (float*)out;
  bf16* ob = out_bf16 ? (bf16*)out : nullptr;
  int rc;
  switch (fmt) {
    case FMT_Q4_K: rc = q32_launch<FMT_Q4_K>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    case FMT_Q6_K: rc = q32_launch<FMT_Q6_K>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    case FMT_Q8_0: rc = q32_launch<FMT_Q8_0>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    default: return -2;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Two weights (same K) side by side: columns [0, Na) from (fa, pa*), [Na, Na+Nb) from (fb, pb*).
extern "C" int la_qgemm32_2(int fa, const void* pa0, const void* pa1, const void* ga, int Na, int fb, const void* pb0,
                            const void* pb1, const void* gb, int Nb, int K, const void* X, int ldx, int M, int splits,
                            void* out, int ldo, long slab, int out_bf16, int var, void* stream) {
  using namespace la;
  if (M < 1 || Na < 1 || Nb < 1 || (K & 255) || splits < 1 || ldo < Na + Nb || ldx < K || (ldx & 7)) return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  if ((long)M * ldx >= (1L << 31) || !ga || !gb) return -1;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  QW wa{(const uint8_t*)pa0, (const uint8_t*)pa1, (const uint8_t*)ga, nullptr, Na, K};
  QW wb{(const uint8_t*)pb0, (const uint8_t*)pb1, (const uint8_t*)gb, nullptr, Nb, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = out_bf16 ? nullptr : (float*)out;
  bf16* ob = out_bf16 ? (bf16*)out : nullptr;
  int rc;
  if (fa == FMT_Q4_K && fb == FMT_Q6_K) rc = q32_launch2<FMT_Q4_K, FMT_Q6_K>(var, wa, wb, x, ldx, M, splits, o, ob, ldo, slab, st);
  else if (fa == FMT_Q6_K && fb == FMT_Q4_K) rc = q32_launch2<FMT_Q6_K, FMT_Q4_K>(var, wa, wb, x, ldx, M, splits, o, ob, ldo, slab, st);
  else return -2;
  if (rc) return rc;
  return (int)hipGetLastError();
}

// h = act(x Wg^T) * (x Wu^T) -> bf16 [M][ldo]; gate rows oa .. oa+F of (pa*, ga), up rows ob ..
// ob+F of (pb*, gb).  act: 0 SwiGLU, 3 GeGLU.
extern "C" int la_qgemm32_glu(int fmt, const void* pa0, const void* pa1, const void* ga, int oa, const void* pb0,
                              const void* pb1, const void* gb, int ob, int F, int K, const void* X, int ldx, int M,
                              void* out, int ldo, int act, int var, void* stream) {
  using namespace la;
  if (M < 1 || F < 1 || (K & 255) || ldo < F || ldx < K || (ldx & 7) || (oa & 15) || (ob & 15)) return -1;
  if (act != 0 && act != 3) return -1;
  if ((long)M * ldx >= (1L << 31) || !ga || !gb) return -1;
  QW wa{(const uint8_t*)pa0, (const uint8_t*)pa1, (const uint8_t*)ga, nullptr, oa + F, K};
  Q32Glu glu{QW{(const uint8_t*)pb0, (const uint8_t*)pb1, (const uint8_t*)gb, nullptr, ob + F, K}, oa, ob, F, act};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  bf16* o = (bf16*)out;
  int rc;
  switch (fmt) {
    case FMT_Q4_K: rc = q32_launch_glu<FMT_Q4_K>(var, wa, glu, x, ldx, M, o, ldo, st); break;
    case FMT_Q6_K: rc = q32_launch_glu<FMT_Q6_K>(var, wa, glu, x, ldx, M, o, ldo, st); break;
    case FMT_Q8_0: rc = q32_launch_glu<FMT_Q8_0>(var, wa, glu, x, ldx, M, o, ldo, st); break;
    default: return -2;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Probe (scripts/q32_bench.py --abl): Q4_K, fp32 slabs, ldx = K, ldo = N; variants 0, 4, 8 with
// ablation bits: 1 no MFMA, 2 no dequant, 4 no DMA, 8 no A LDS reads, 16 no mid-step barrier.
extern "C" int la_qgemm32_probe(int var, int abl, const void* p0, const void* gsc, int N, int K, const void* X, int M,
                                int splits, void* out, void* stream) {
  using namespace la;
  QW w{(const uint8_t*)p0, nullptr, (const uint8_t*)gsc, nullptr, N, K};
  const long slab = (long)M * N;
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
  if (var != 0 && var != 4 && var != 8) return -1;
#define Q32_PROBE(A) \
  case A: return q32_probe_launch<A>(var, w, x, K, M, splits, o, N, slab, st) ? -1 : (int)hipGetLastError();
  switch (abl) {
    Q32_PROBE(1) Q32_PROBE(2) Q32_PROBE(3) Q32_PROBE(4) Q32_PROBE(8) Q32_PROBE(16) Q32_PROBE(12) Q32_PROBE(15)
    Q32_PROBE(31) Q32_PROBE(20)
    default: return -1;
  }
#undef Q32_PROBE
}

// Grouped expert GEMM on the 32x32x16 tile (see moe32_kernel).  qws: device array of E QW
// descriptors {p0, p1, blocked scale plane, -, N, K}; order / off: the pair grouping of
// la_moe_route; maxM: most rows any expert can hold (<= T).
//   mode 1: X [T][ldx] tokens -> out bf16 [P][ldo] (row off[e] + m = act(gate) * up of pair
//           order[off[e] + m]); N = F (the expert weight holds 2F rows); splits must be 1.
//   mode 2: X [P][ldx] grouped h rows -> out fp32 [splits * topk][T][ldo] (stride slab), each
//           row scaled by wts[pair].
extern "C" int la_moe32(int fmt, int mode, const void* qws, int N, int K, int E, const int* order, const int* off,
                        int topk, const void* X, int ldx, int maxM, int splits, const float* wts, void* out, int ldo,
                        long slab, int act, int var, void* stream) {
  using namespace la;
  if (maxM < 1 || N < 1 || E < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7) || topk < 1) return -1;
  if (mode == 1 && (splits != 1 || (N & 15) || (act != 0 && act != 3))) return -1;
  if (mode == 2 && (!wts || slab < (long)maxM * ldo)) return -1;
  if (mode != 1 && mode != 2) return -1;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  if ((long)maxM * topk * ldx >= (1L << 31) || (long)E * ((maxM + 31) / 32) * ((N + 63) / 64) * splits >= (1L << 31)) return -1;
  hipStream_t st = (hipStream_t)stream;
  const QW* q = (const QW*)qws;
  const bf16* x = (const bf16*)X;
  float* o = mode == 2 ? (float*)out : nullptr;
  bf16* ob = mode == 1 ? (bf16*)out : nullptr;
  int rc;
#define MOE32_F(F_)                                                                                                \
  rc = mode == 1 ? moe32_launch<F_, 1>(var, q, N, K, E, order, off, topk, x, ldx, maxM, 1, wts, o, ob, ldo, slab, act, st) \
                 : moe32_launch<F_, 2>(var, q, N, K, E, order, off, topk, x, ldx, maxM, splits, wts, o, ob, ldo, slab, act, st);
  switch (fmt) {
    case FMT_Q4_K: MOE32_F(FMT_Q4_K) break;
    case FMT_Q6_K: MOE32_F(FMT_Q6_K) break;
    case FMT_Q8_0: MOE32_F(FMT_Q8_0) break;
    default: return -2;
  }
#undef MOE32_F
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Probe (scripts/moe_bench.py --abl): la_moe32 mode 1, Q4_K, variant 4 geometry, with q32_tile's
// ablation bits (1 no MFMA, 2 no dequant, 4 no DMA, 8 no A LDS reads, 16 no mid-step barrier).
extern "C" int la_moe32_probe(int abl, const void* qws, int N, int K, int E, const int* order, const int* off,
                              int topk, const void* X, int ldx, int maxM, void* out, int ldo, void* stream) {
  using namespace la;
  using C = MoeCfg<Q32Cfg<64, 32, 8, 0>, 2>;
  const int mch = (maxM + C::BM - 1) / C::BM, n_tiles = (N + C::BN / 2 - 1) / (C::BN / 2);
  const long real = (long)E * mch * n_tiles;
  const int grid = (int)((real + 7) / 8 * 8);
  hipStream_t st = (hipStream_t)stream;
#define MOE32_P(A)                                                                                              \
  case A:                                                                                                       \
    hipLaunchKernelGGL((moe32_kernel<FMT_Q4_K, C, 1, A>), dim3(grid), dim3(C::NW * 64), 0, st, (const QW*)qws, order, \
                       off, topk, (const bf16*)X, ldx, mch, n_tiles, 1, K >> 6, (int)real, nullptr, nullptr, (bf16*)out, \
                       ldo, 0L, N, 0);                                                                            \
    break;
  switch (abl) {
    MOE32_P(1) MOE32_P(2) MOE32_P(3) MOE32_P(4) MOE32_P(8) MOE32_P(16) MOE32_P(11)
    default: return -1;
  }
#undef MOE32_P
  return (int)hipGetLastError();
}
