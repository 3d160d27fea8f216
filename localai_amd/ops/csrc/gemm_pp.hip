// Prefill GEMM (M >= ~1024 rows): out[m][n] = sum_k X[m,k] * W[n,k], W in its GGUF quantisation
// (Q4_K, Q6_K) or bf16.  SURVEY §2.8 K6: the reference reaches this through ggml's mmq / dequant +
// hipBLAS GemmEx inside llama_decode (backend/cpp/llama/grpc-server.cpp:1910); here it is one
// hand-written CDNA4 kernel that never materialises a bf16 copy of the weight.
//
// Design (MI355X, cdna_hip_programming.md §5 "The 256^2 8-phase template", T1-T5):
//   * 256 x 256 output tile, BK = 64, 8 waves (512 threads) = 2 per SIMD, one workgroup per CU;
//     wave (wr, wc) = (wave >> 2, wave & 3) owns rows [128 wr, +128) x cols [64 wc, +64);
//   * v_mfma_f32_32x32x16_bf16 with SWAPPED operands (A-slot = W fragment, B-slot = X
//     fragment), so each lane's accumulators come in runs of 4 consecutive output COLUMNS of one
//     row and the epilogue stores 8 / 16 bytes per lane with no LDS transpose.  32x32x16, not
//     16x16x32: an MFMA holds the SIMD's vector issue for 8 cycles either way, so the 32-cycle
//     shape leaves 24 issue cycles per MFMA to the partner wave's dequant / LDS traffic instead
//     of 8 (profiles/r5_prefill_gemm.md: the 16x16x32 build was issue-bound, 0.9 PF/s);
//   * each K-tile is 4 phases (one 64 x 32 quadrant x K = 64 = 8 MFMAs per wave); the two wave
//     groups (wr = 0 / 1) run ONE BARRIER APART (ping-pong): while one group is in its MFMA
//     cluster the other issues its LDS reads, its DMA and its dequantisation;
//   * X (bf16) arrives by LDS-DMA (global_load_lds_dwordx4) into a 3-deep ring, XOR-swizzled on
//     the SOURCE address (chunk c of row r stored at c ^ ((r >> 1) & 7)) so every ds_read_b128
//     fragment read is bank-conflict free;
//   * W: each thread owns (column, k-half) of the tile and streams that column's raw GGUF bytes
//     for K-tile t+2 into registers (inline-asm loads, counted by hand: hipcc would otherwise
//     drain the X DMA ring at every use), dequantises K-tile t+1 with ggml's arithmetic (fp32,
//     rounded once to bf16 -- the same values as the dequant + hipBLASLt path it replaces) and
//     writes it ONCE per workgroup into a double-buffered bf16 LDS image that all 8 waves
//     read: 32 weights / thread / K-tile, ~2.25 VALU each (a Q4_K nibble byte IS an OCP e4m3
//     code of q * 2^-9, so v_cvt_pk_f32_fp8 converts two per instruction), hidden behind the
//     other group's MFMAs; the two lanes of a column read its 32 contiguous code bytes;
//   * counted vmcnt, raw s_barrier, all LDS in one array, s_setprio(1) around the MFMA clusters;
//   * XCD-aware tile order: each XCD takes a contiguous run of tiles, walked in groups of 8 M x
//     4 N tiles, so the ~32 resident workgroups of an XCD share 8 X row panels and 4 weight
//     panels through its L2; split-K into fp32 slabs, GLU (gate|up) epilogue.
//
// Hazard bookkeeping (i = 4 t + p is the global phase; G0 = waves 0-3, G1 = waves 4-7, G1 one
// barrier behind): G0's LDS section of phase i sits between barriers 2i and 2i+1, G1's between
// 2i+1 and 2i+2.  All LDS reads of K-tile t-1 are complete at barrier 8t+1, so buffers of
// tile t-1 are refilled from phase 4t+1 on (both groups); every producer of K-tile t+1 retires
// its writes (vmcnt for the DMA, lgkmcnt for the dequant stores) at the end of its phase-4t+3
// LDS section, which precedes barrier 8t+8 for both groups, and the first reader (G0, phase
// 4t+4) starts after barrier 8t+8.
#include <type_traits>

#include "qweight.h"

namespace la {
namespace pp {

// Ablation build flag (scripts/pp_abl.py; never set in the library): 1 no MFMA, 2 no dequant VALU,
// 4 no X DMA, 8 no W register loads, 16 no fragment LDS reads.
#ifndef LA_PP_ABL
#define LA_PP_ABL 0
#endif


// Diagnostic build (-DLA_PP_STAMP=1, scripts/pp_abl.py): s_memtime stamps around every section of
// K-tiles 10-11 of selected workgroups, written by lane 0 of each wave to pp_dbg.
#ifndef LA_PP_STAMP
#define LA_PP_STAMP 0
#endif
#if LA_PP_STAMP
__device__ unsigned long long* pp_dbg;
#endif

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int ABUF = BM * BK * 2;              // 32 KiB bf16 X image per K-tile
constexpr int BBUF = BN * BK * 2;              // 32 KiB bf16 W image per K-tile
constexpr int LDS_BYTES = 3 * ABUF + 2 * BBUF;  // 160 KiB
// LDS plan per weight kind: quantised W = X ring of 4 + ONE W image (each k-half of it rewritten
// as soon as its last reader is past, the dequant skewed across K-tiles); bf16 W (staged by DMA
// in whole rows) = X ring of 3 + two W images.
template <bool Q> struct Plan {
  static constexpr int XR = Q ? 4 : 3, WB = Q ? 1 : 2;
  static_assert(XR * ABUF + WB * BBUF <= LDS_BYTES, "LDS plan");
};

LA_DEV int swz(int r) { return (r >> 1) & 7; }

LA_DEV void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
template <int N>
LA_DEV void vmwait() {
  // ablation builds that drop loads would under-count: drain instead
  constexpr int n = (LA_PP_ABL & 12) ? 0 : N;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}
LA_DEV void mem_fence() { asm volatile("" ::: "memory"); }
LA_DEV void bar() {
  mem_fence();
  __builtin_amdgcn_s_barrier();
  mem_fence();
}

// Hand-counted register loads (invisible to hipcc's waitcnt bookkeeping; §5.7 item 1 form (ii)):
// the base is a wave-uniform SGPR pair (fresh from readfirstlane: s_nop 4 first), the offset a
// 32-bit VGPR.  The destination is not valid until the matching raw_wait below.
LA_DEV u32x4 ld_x4(const uint8_t* base, uint32_t off) {
  u32x4 r;
  asm volatile("s_nop 4\n\tglobal_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(off), "s"(base) : "memory");
  return r;
}
LA_DEV u32x2 ld_x2(const uint8_t* base, uint32_t off) {
  u32x2 r;
  asm volatile("s_nop 4\n\tglobal_load_dwordx2 %0, %1, %2" : "=v"(r) : "v"(off), "s"(base) : "memory");
  return r;
}

LA_DEV const uint8_t* uni(const uint8_t* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const uint8_t*)(((uint64_t)hi << 32) | lo);
}

// opaque 0x0f0f0f0f mask: keeps one v_cvt_f32_ubyteN per weight
LA_DEV uint32_t nib_lo(uint32_t w) {
  uint32_t r;
  asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(r) : "v"(w));
  return r;
}
LA_DEV uint32_t nib_hi(uint32_t w) {
  uint32_t r;
  asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(r) : "v"(w >> 4));
  return r;
}
LA_DEV bf16x8 deq8(uint32_t a, uint32_t b, float D, float O) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)fmaf(D, (float)((a >> (8 * j)) & 0xFFu), O);
    r[j + 4] = (bf16)fmaf(D, (float)((b >> (8 * j)) & 0xFFu), O);
  }
  return r;
}

// Same from 8 nibble BYTES read as OCP e4m3 codes: byte q (0..15) converts to exactly q * 2^-9
// (subnormal for q < 8, exponent 1 above), two per v_cvt_pk_f32_fp8.
LA_DEV bf16x8 deq8_fp8(uint32_t a, uint32_t b, float D, float O) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 a0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, false), a1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, true);
  const f2 b0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, false), b1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, true);
  bf16x8 r;
  r[0] = (bf16)fmaf(D, a0.x, O);
  r[1] = (bf16)fmaf(D, a0.y, O);
  r[2] = (bf16)fmaf(D, a1.x, O);
  r[3] = (bf16)fmaf(D, a1.y, O);
  r[4] = (bf16)fmaf(D, b0.x, O);
  r[5] = (bf16)fmaf(D, b0.y, O);
  r[6] = (bf16)fmaf(D, b1.x, O);
  r[7] = (bf16)fmaf(D, b1.y, O);
  return r;
}

// The weight rows behind this thread's tile column (wave-uniform plane bases).
struct Src {
  const uint8_t* p0;
  const uint8_t* p1;
  const uint8_t* gsc;
  uint32_t o0, o1, os;  // this thread's byte offsets for K-tile 0
};

// ---------------------------------------------------------------- formats
// Each thread (column c, half h) of a K-tile dequantises 32 weights: chunks (8 k each, logical
// order of the X image row) 2h, 2h+1 (lo nibbles / run 0) and 4+2h, 5+2h (hi nibbles / run 1).
template <int FMT> struct Fmt;

// Q4_K: K-tile ks = bytes [32 ks, +32) of the row's code plane (byte i: k = 64 ks + i low
// nibble, k = 64 ks + 32 + i high nibble); scale record (f16 D0, -M0, D1, -M1) per (row, ks).
template <> struct Fmt<FMT_Q4_K> {
  static constexpr int R = 2;  // register loads per thread per K-tile
  struct Raw {
    u32x4 q;
    u32x2 s;
  };
  LA_DEV static int xk(int ks) { return 64 * ks; }
  LA_DEV static int kofs(int c) { return 8 * c; }
  LA_DEV static void init(Src& s, int n, int h, int K) {
    s.o0 = (uint32_t)n * (uint32_t)(K >> 1) + 16 * h;
    s.os = (uint32_t)(((n >> 4) * (K >> 6)) * 16 + (n & 15)) * 8;
  }
  LA_DEV static void load(Raw& r, const Src& s, int ks) {
    if constexpr (LA_PP_ABL & 8) return;
    r.q = ld_x4(s.p0, s.o0 + 32 * ks);
    r.s = ld_x2(s.gsc, s.os + 128 * ks);
  }
  LA_DEV static void wait_reg(Raw& r) {  // pins the registers at the wait (see raw_wait)
    asm volatile("" : "+v"(r.q), "+v"(r.s));
  }
  // chunk C (0..3): bytes 8 (C & 1) .. +8 of the thread's 16, low nibbles (C < 2) or high
  template <int C>
  LA_DEV static bf16x8 deq(const Raw& r, int) {
    constexpr bool HI = C >= 2, B1 = C & 1;
    const uint32_t sv = HI ? r.s.y : r.s.x;
    // q * 2^-9 from the fp8 conversion: fold 2^9 into D (exact)
    const float D = h2f(sv & 0xFFFFu) * 512.0f, O = h2f(sv >> 16);
    const uint32_t w0 = B1 ? r.q.z : r.q.x, w1 = B1 ? r.q.w : r.q.y;
    return deq8_fp8(HI ? nib_hi(w0) : nib_lo(w0), HI ? nib_hi(w1) : nib_lo(w1), D, O);
  }
};

// Q6_K: K-tile ks = (super-block ks >> 2, half hh = (ks >> 1) & 1, part = ks & 1) covers run 0 =
// k [128 hh + 32 part, +32) (ql low nibbles) and run 1 = k [128 hh + 64 + 32 part, +32) (ql high
// nibbles); ql bytes [32 ks, +32), qh bytes [16 (ks & ~1), +32) with the run's 2-bit fields at
// shift 2 part (run 0) and 4 + 2 part (run 1); scale record = f16 d*sc of (run 0 g0, g1, run 1
// g0, g1), 16 k per group.
template <> struct Fmt<FMT_Q6_K> {
  static constexpr int R = 3;
  struct Raw {
    u32x4 ql, qh;
    u32x2 s;
  };
  LA_DEV static int xk(int ks) { return 256 * (ks >> 2) + 128 * ((ks >> 1) & 1) + 32 * (ks & 1); }
  LA_DEV static int kofs(int c) { return 8 * (c & 3) + 64 * (c >> 2); }
  LA_DEV static void init(Src& s, int n, int h, int K) {
    s.o0 = (uint32_t)n * (uint32_t)(K >> 1) + 16 * h;
    s.o1 = (uint32_t)n * (uint32_t)(K >> 2) + 16 * h;
    s.os = (uint32_t)(((n >> 4) * (K >> 6)) * 16 + (n & 15)) * 8;
  }
  LA_DEV static void load(Raw& r, const Src& s, int ks) {
    if constexpr (LA_PP_ABL & 8) return;
    r.ql = ld_x4(s.p0, s.o0 + 32 * ks);
    r.qh = ld_x4(s.p1, s.o1 + 16 * (ks & ~1));
    r.s = ld_x2(s.gsc, s.os + 128 * ks);
  }
  LA_DEV static void wait_reg(Raw& r) { asm volatile("" : "+v"(r.ql), "+v"(r.qh), "+v"(r.s)); }
  // chunk C (0..3): bytes 8 (C & 1) .. +8 of the thread's 16, run 0 (C < 2) or run 1; this
  // thread's 16-k scale group h arrives folded into bit 30 of ks
  template <int C>
  LA_DEV static bf16x8 deq(const Raw& r, int ks) {
    constexpr bool HI = C >= 2, B1 = C & 1;
    const int h = ks >> 30, sh = 2 * (ks & 1) + (HI ? 4 : 0);
    const uint32_t sv = HI ? r.s.y : r.s.x;
    const float S = h2f(h ? (sv >> 16) : (sv & 0xFFFFu)), O = -32.0f * S;
    const uint32_t l0 = B1 ? r.ql.z : r.ql.x, l1 = B1 ? r.ql.w : r.ql.y;
    const uint32_t h0 = B1 ? r.qh.z : r.qh.x, h1 = B1 ? r.qh.w : r.qh.y;
    uint32_t q0, q1;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q0) : "v"((h0 >> sh) << 4), "s"(0x30303030u), "v"(HI ? nib_hi(l0) : nib_lo(l0)));
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q1) : "v"((h1 >> sh) << 4), "s"(0x30303030u), "v"(HI ? nib_hi(l1) : nib_lo(l1)));
    return deq8(q0, q1, S, O);
  }
};

// bf16 weights: the W image arrives by LDS-DMA like X (no registers, no dequant).
template <> struct Fmt<FMT_BF16> {
  static constexpr int R = 0;
  struct Raw {};
  LA_DEV static int xk(int ks) { return 64 * ks; }
  LA_DEV static int kofs(int c) { return 8 * c; }
};

struct Glu {
  const uint8_t* b0;  // up weight planes (gate = the main planes)
  const uint8_t* b1;
  const uint8_t* bg;
  int oa, ob, F, act;
};

struct Args {
  const uint8_t* p0;
  const uint8_t* p1;
  const uint8_t* gsc;
  int N, K;
  const bf16* X;
  int ldx, M;
  int per_split, m_tiles, n_tiles, real_tiles;
  float* out;   // fp32 slabs [S][M][ldo] (stride slab), or null
  bf16* outb;   // bf16 [M][ldo] (S == 1), or null
  int ldo;
  long slab;
  Glu glu;
};

LA_DEV float gelu_tanh(float x) { return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))); }

// Tile id -> (m tile, n tile, split): splits outermost, then groups of GM m tiles x all n tiles,
// m fastest inside a group, so a window of ~32 consecutive tiles (one XCD's resident set)
// covers GM x 32/GM tiles.
#ifndef LA_PP_GM
#define LA_PP_GM 8
#endif
constexpr int GM = LA_PP_GM;
LA_DEV void tile_coords(const Args& a, int tile, int& mt, int& nt, int& split) {
  const int per = a.m_tiles * a.n_tiles;
  split = tile / per;
  const int i = tile - split * per;
  const int gsz = GM * a.n_tiles;
  const int g = i / gsz, first = g * GM;
  const int gm = min(a.m_tiles - first, GM);
  const int j = i - g * gsz;
  mt = first + j % gm;
  nt = j / gm;
}

template <int FMT, bool GLU>
LA_DEV void tile_run(uint8_t* __restrict__ lds, const Args& a, int tile) {
  using F = Fmt<FMT>;
  constexpr bool Q = FMT != FMT_BF16;
  constexpr int R = F::R;
  int mt, nt, split;
  tile_coords(a, tile, mt, nt, split);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int m0 = mt * BM;
  const int KT = a.K >> 6;
  const int ks0 = split * a.per_split;
  const int nk = min(KT, ks0 + a.per_split) - ks0;  // a multiple of 4 (host guarantees)
  if (nk <= 0) return;

  uint8_t* const Abase = lds;
  constexpr int XR = Plan<Q>::XR, WB = Plan<Q>::WB;
  uint8_t* const Bbase = lds + XR * ABUF;
#if LA_PP_STAMP
  const int sblk = (blockIdx.x == 0) ? 0 : (blockIdx.x == 100 ? 1 : (blockIdx.x == 201 ? 2 : -1));
  auto stamp = [&](int t, int p, int k) {
    if (sblk < 0 || t < 10 || t > 11) return;
    const unsigned long long v = __builtin_amdgcn_s_memtime();
    if (lane == 0) pp_dbg[((sblk * 8 + wave) * 8 + (t - 10) * 4 + p) * 6 + k] = v;
  };
#else
  auto stamp = [](int, int, int) {};
#endif

  // weight row of tile column c (clamped into the matrix; out-of-range columns are not stored)
  auto wrow = [&](int c, const uint8_t*& p0, const uint8_t*& p1, const uint8_t*& gsc) -> int {
    if constexpr (GLU) {
      const bool up = c >= BN / 2;
      p0 = up ? a.glu.b0 : a.p0;
      p1 = up ? a.glu.b1 : a.p1;
      gsc = up ? a.glu.bg : a.gsc;
      return (up ? a.glu.ob : a.glu.oa) + min(nt * (BN / 2) + (c & (BN / 2 - 1)), a.glu.F - 1);
    } else {
      p0 = a.p0;
      p1 = a.p1;
      gsc = a.gsc;
      return min(nt * BN + c, a.N - 1);
    }
  };

  // ---- X DMA: wave w stages rows [32 w, +32) as 4 pieces of 8 rows x 128 B
  uint32_t xoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 32 * wave + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    xoff[j] = (uint32_t)min(m0 + r, a.M - 1) * (uint32_t)a.ldx + F::kofs(c);
  }
  auto issue_x = [&](int t, int j0) {  // pieces j0, j0+1 of K-tile t
    if constexpr (LA_PP_ABL & 4) return;
    uint8_t* dst = Abase + (t % XR) * ABUF + 32 * wave * 128;
    const bf16* xk = a.X + F::xk(ks0 + t);
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j) glds16(xk + xoff[j], dst + j * 1024);
  };

  // ---- W: bf16 weights by DMA (wave w stages tile columns [32 w, +32)); quantised weights by
  // register loads + dequant into the LDS image.  Thread -> (column cw, k-half hh): the two lanes
  // of a pair share a column (its 32 contiguous code bytes), and the pair -> column permutation
  // puts 8 distinct 16-B bank slots under every 8-lane ds_write_b128 group.
  const bf16* wsrc[4];
  Src src{};
  int hh = 0, cw = 0;
  if constexpr (!Q) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 32 * wave + 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ swz(r);
      const uint8_t *p0, *p1, *g;
      const int n = wrow(r, p0, p1, g);
      wsrc[j] = (const bf16*)p0 + (size_t)n * a.K + 8 * c;
    }
  } else {
    hh = lane & 1;
    const int pr = lane >> 1;
    cw = 32 * wave + ((pr & 16) | (((pr >> 3) & 1) << 2) | ((pr >> 2) & 1) | (((pr >> 1) & 1) << 3) | ((pr & 1) << 1));
    const uint8_t *p0, *p1, *g;
    const int n = wrow(cw, p0, p1, g);
    src.p0 = uni(p0);
    src.p1 = uni(p1);
    src.gsc = uni(g);
    F::init(src, n, hh, a.K);
    (void)wsrc;
  }
  auto issue_wb = [&](int t) {  // bf16 W: all 4 pieces of K-tile t
    if constexpr (!Q) {
      uint8_t* dst = Bbase + (t % WB) * BBUF + 32 * wave * 128;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(wsrc[j] + 64 * (ks0 + t), dst + j * 1024);
    }
  };
  // chunk C of the thread's 32 weights lands in logical chunk 2 hh + (C & 1) (+ 4 for C >= 2)
  int wb_off[4];
#pragma unroll
  for (int C = 0; C < 4; ++C) wb_off[C] = cw * 128 + 16 * (((C >= 2 ? 4 : 0) + 2 * hh + (C & 1)) ^ swz(cw));
  auto dequant = [&](auto& raw, int t, auto C_) {
    if constexpr (Q) {
      constexpr int C = decltype(C_)::value;
      bf16x8 v;
      if constexpr (LA_PP_ABL & 2) {
        v = __builtin_bit_cast(bf16x8, u32x4{raw.s.x, raw.s.y, raw.s.x, raw.s.y});
      } else {
        v = F::template deq<C>(raw, (ks0 + t) | (hh << 30));
      }
      *(bf16x8*)(Bbase + (t % WB) * BBUF + wb_off[C]) = v;
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;

  // ---- fragments (32x32x16): lane (r = lane & 31, hk = lane >> 5) reads row 32 blk + r, logical
  // chunk 2 s + hk of k-substep s
  const int fr = lane & 31, fh = lane >> 5;
  int fo[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) fo[s4] = fr * 128 + 16 * ((2 * s4 + fh) ^ swz(fr));

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // phase p of a K-tile = (row half mh = p & 1, k half kh = p >> 1): 2 x 2 tiles of 32 x 32 x
  // K 32 = 8 MFMAs; X fragments (4) are read every phase, W fragments (4) at kh = 0 and 1 only
  bf16x8 xf[2][2], wf[2][2];
  auto read_x = [&](int t, int mh, int kh) {
    const uint8_t* A = Abase + (t % XR) * ABUF + 4096 * (4 * wr + 2 * mh);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if constexpr (LA_PP_ABL & 16) asm volatile("" : "=v"(xf[rt][k]) : "v"(A));
        else xf[rt][k] = *(const bf16x8*)(A + 4096 * rt + fo[2 * kh + k]);
      }
  };
  auto read_w = [&](int t, int kh) {
    const uint8_t* B = Bbase + (t % WB) * BBUF + 4096 * (2 * wc);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if constexpr (LA_PP_ABL & 16) asm volatile("" : "=v"(wf[ct][k]) : "v"(B));
        else wf[ct][k] = *(const bf16x8*)(B + 4096 * ct + fo[2 * kh + k]);
      }
  };
  auto mfma = [&](int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          if constexpr (LA_PP_ABL & 1)
            asm volatile("" : "+v"(acc[2 * mh + rt][ct]) : "v"(wf[ct][k]), "v"(xf[rt][k]));
          else
            acc[2 * mh + rt][ct] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ct][k], xf[rt][k], acc[2 * mh + rt][ct], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mfma_section = [&](int t, int p, int mh) {
    stamp(t, p, 1);
    bar();
    stamp(t, p, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(t, p, 3);
    mfma(mh);
    stamp(t, p, 4);
    bar();
    stamp(t, p, 5);
  };

  typename F::Raw raw0{}, raw1{}, raw2{}, raw3{};
  if constexpr (Q) {
    // ---- quantised W.  Per K-tile t the W image is consumed k-half 0 in phases 0-1 and k-half
    // 1 in phases 2-3, so (barrier arithmetic as in the header) its k-half 1 for tile t is
    // written in phases 0-1 of tile t (chunks 2, 3 of raw(t)) and its k-half 0 for tile t+1 in
    // phases 2-3 of tile t (chunks 0, 1 of raw(t+1)); each writer retires its stores
    // (lgkmcnt(0)) before the barrier that precedes the first reader.  raw(t) lives in register
    // set t % 4 from its load (phase 0 of tile t-3) to phase 1 of tile t: 2.5 K-tiles of
    // latency cover.  X(t+3) goes into the ring slot of X(t-1) in phases 1-2 of tile t and is
    // retired in phase 3 of tile t+2.
    // Per-thread VMEM issue order of tile t: raw(t+3) [p0], X(t+3) pieces 0-1 [p1], 2-3 [p2].
    //   p2 wait for raw(t+1): younger = X(t+1), raw(t+2), X(t+2), raw(t+3), X(t+3) 0-1 -> 2R + 10
    //   p3 wait for X(t+1):   younger = raw(t+2), X(t+2), raw(t+3), X(t+3)            -> 2R + 8
    // ---- prologue: raw(0), X(0), raw(1), X(1), raw(2), X(2); image k-half 0 of tile 0
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < nk) {
        if (i == 0) F::load(raw0, src, ks0 + 0);
        if (i == 1) F::load(raw1, src, ks0 + 1);
        if (i == 2) F::load(raw2, src, ks0 + 2);
        issue_x(i, 0);
        issue_x(i, 2);
      }
    }
    vmwait<0>();  // prologue: simply drain (once per tile)
    F::wait_reg(raw0);
    F::wait_reg(raw1);
    F::wait_reg(raw2);
    dequant(raw0, 0, C0{});
    dequant(raw0, 0, C1{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (wr == 1) bar();  // G1 runs one barrier behind G0

    auto ktile = [&](int t, auto& ra, auto& rb, auto& rn) {
      // ra = raw(t), rb = raw(t+1), rn receives raw(t+3)
      const bool more1 = t + 1 < nk, more3 = t + 3 < nk;
      // phase 0: rows m0, k 0-31; image k-half 1 of tile t: chunk 2; raw(t+3)
      stamp(t, 0, 0);
      read_w(t, 0);
      read_x(t, 0, 0);
      dequant(ra, t, C2{});
      if (more3) F::load(rn, src, ks0 + t + 3);
      mfma_section(t, 0, 0);
      // phase 1: rows m1, k 0-31; chunk 3 (k-half 1 complete before its readers); X(t+3) 0-1
      stamp(t, 1, 0);
      read_x(t, 1, 0);
      dequant(ra, t, C3{});
      if (more3) issue_x(t + 3, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_section(t, 1, 1);
      // phase 2: rows m0, k 32-63; image k-half 0 of tile t+1: chunk 0; X(t+3) 2-3
      stamp(t, 2, 0);
      read_w(t, 1);
      read_x(t, 0, 1);
      if (more1) {
        if (more3) vmwait<2 * R + 10>();
        else vmwait<0>();
        F::wait_reg(rb);
        dequant(rb, t + 1, C0{});
      }
      if (more3) issue_x(t + 3, 2);
      mfma_section(t, 2, 0);
      // phase 3: rows m1, k 32-63; chunk 1; retire X(t+1) and the image k-half 0
      stamp(t, 3, 0);
      read_x(t, 1, 1);
      if (more1) {
        dequant(rb, t + 1, C1{});
        if (more3) vmwait<2 * R + 8>();
        else vmwait<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      mfma_section(t, 3, 1);
    };
    for (int t = 0; t < nk; t += 4) {
      ktile(t, raw0, raw1, raw3);
      ktile(t + 1, raw1, raw2, raw0);
      ktile(t + 2, raw2, raw3, raw1);
      ktile(t + 3, raw3, raw0, raw2);
    }
  } else {
    // ---- bf16 W by DMA, two W images.  Per-thread VMEM issue order of tile t: W(t+1) [p0],
    // X(t+2) pieces 0-1 [p1], 2-3 [p2]; p3 retires X(t+1) and W(t+1) (younger: X(t+2)).
    issue_x(0, 0);
    issue_x(0, 2);
    issue_wb(0);
    if (nk > 1) {
      issue_x(1, 0);
      issue_x(1, 2);
    }
    vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (wr == 1) bar();  // G1 runs one barrier behind G0
    for (int t = 0; t < nk; ++t) {
      const bool more1 = t + 1 < nk, more2 = t + 2 < nk;
      stamp(t, 0, 0);
      read_w(t, 0);
      read_x(t, 0, 0);
      if (more1) issue_wb(t + 1);
      mfma_section(t, 0, 0);
      stamp(t, 1, 0);
      read_x(t, 1, 0);
      if (more2) issue_x(t + 2, 0);
      mfma_section(t, 1, 1);
      stamp(t, 2, 0);
      read_w(t, 1);
      read_x(t, 0, 1);
      if (more2) issue_x(t + 2, 2);
      mfma_section(t, 2, 0);
      stamp(t, 3, 0);
      read_x(t, 1, 1);
      if (more1) {
        if (more2) vmwait<4>();
        else vmwait<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      mfma_section(t, 3, 1);
    }
  }
  if (wr == 0) bar();  // re-align the groups: every wave is past its last LDS read

  // ---- epilogue.  acc[mi][ni][j] = out[m0 + 128 wr + 32 mi + fr][64 wc + 32 ni + 8 (j >> 2) +
  // 4 fh + (j & 3)]: runs of 4 consecutive columns
  const int mrow = m0 + 128 * wr + fr;
  if constexpr (GLU) {
    // up waves (wc 2, 3) park their accumulators; gate waves (wc 0, 1) combine and store
    float* park = (float*)lds;
    const int pw = 2 * wr + (wc & 1);
    if (wc >= 2) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *(f32x4*)(park + (((pw * 8 + mi * 2 + ni) * 4 + q) * 64 + lane) * 4) =
                f32x4{acc[mi][ni][4 * q], acc[mi][ni][4 * q + 1], acc[mi][ni][4 * q + 2], acc[mi][ni][4 * q + 3]};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (wc < 2) {
      const int jb = nt * (BN / 2) + 64 * wc + 4 * fh;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int m = mrow + 32 * mi;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 u = *(const f32x4*)(park + (((pw * 8 + mi * 2 + ni) * 4 + q) * 64 + lane) * 4);
            const int j = jb + 32 * ni + 8 * q;
            bf16x4 hv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float gv = acc[mi][ni][4 * q + e];
              hv[e] = (bf16)((a.glu.act == 0 ? silu(gv) : gelu_tanh(gv)) * u[e]);
            }
            if (m < a.M) {
              if (j + 3 < a.glu.F) {
                *(bf16x4*)(a.outb + (size_t)m * a.ldo + j) = hv;
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  if (j + e < a.glu.F) a.outb[(size_t)m * a.ldo + j + e] = hv[e];
              }
            }
          }
      }
    }
  } else {
    const int nb = nt * BN + 64 * wc + 4 * fh;
    float* o = a.out ? a.out + (size_t)split * a.slab : nullptr;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = mrow + 32 * mi;
      if (m >= a.M) continue;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = nb + 32 * ni + 8 * q;
          const f32x4 v{acc[mi][ni][4 * q], acc[mi][ni][4 * q + 1], acc[mi][ni][4 * q + 2], acc[mi][ni][4 * q + 3]};
          if (n + 3 < a.N) {
            if (o) {
              *(f32x4*)(o + (size_t)m * a.ldo + n) = v;
            } else {
              bf16x4 bv;
#pragma unroll
              for (int e = 0; e < 4; ++e) bv[e] = (bf16)v[e];
              *(bf16x4*)(a.outb + (size_t)m * a.ldo + n) = bv;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < a.N) {
                if (o) o[(size_t)m * a.ldo + n + e] = v[e];
                else a.outb[(size_t)m * a.ldo + n + e] = (bf16)v[e];
              }
          }
        }
    }
  }
}

// XCD-contiguous tile order: blocks b, b + 8, ... share an XCD; each XCD takes a contiguous run
// of tiles (M fastest), so one weight panel serves the ~32 resident workgroups of an XCD from L2.
LA_DEV int xcd_tile(int nwg) {
  const int b = blockIdx.x, x = b & 7, q = nwg >> 3;
  return x * q + (b >> 3);
}

template <int FMT, bool GLU>
__global__ __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_pp_kernel(Args a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];
  const int tile = xcd_tile(gridDim.x);
  if (tile >= a.real_tiles) return;  // grid padded to a multiple of 8
  tile_run<FMT, GLU>(lds, a, tile);
}

// Two weights side by side in one output (a Q4_K q|k beside a Q6_K v): B's tiles follow A's.
template <int FA, int FB>
__global__ __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_pp2_kernel(Args a, Args b,
                                                                                                int tiles_a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];
  const int tile = xcd_tile(gridDim.x);
  if (tile < tiles_a) {
    tile_run<FA, false>(lds, a, tile);
  } else if (tile - tiles_a < b.real_tiles) {
    tile_run<FB, false>(lds, b, tile - tiles_a);
  }
}

}  // namespace pp
}  // namespace la

using la::FMT_BF16;
using la::FMT_Q4_K;
using la::FMT_Q6_K;

static int pp_check(int N, int K, int M, int ldx, int splits) {
  if (M < 1 || N < 1 || K < 256 || (K & 255) || splits < 1 || ldx < K || (ldx & 7)) return -1;
  if ((long)M * ldx >= (1L << 31)) return -1;
  const int KT = K / 64;
  if (KT % splits || (KT / splits) % 4) return -1;  // equal K-tile counts per split, multiples of 4
  return 0;
}

static int pp_fmt_ok(int fmt, const void* p1, const void* gsc) {
  if (fmt == FMT_BF16) return 1;
  if (fmt == FMT_Q4_K) return gsc != nullptr;
  if (fmt == FMT_Q6_K) return gsc != nullptr && p1 != nullptr;
  return 0;
}

static la::pp::Args pp_args(const void* p0, const void* p1, const void* gsc, int N, int K, const void* X, int ldx, int M,
                            int splits, void* out, int ldo, long slab, int out_bf16) {
  la::pp::Args a{};
  a.p0 = (const uint8_t*)p0;
  a.p1 = (const uint8_t*)p1;
  a.gsc = (const uint8_t*)gsc;
  a.N = N;
  a.K = K;
  a.X = (const __bf16*)X;
  a.ldx = ldx;
  a.M = M;
  a.per_split = K / 64 / splits;
  a.m_tiles = (M + la::pp::BM - 1) / la::pp::BM;
  a.n_tiles = (N + la::pp::BN - 1) / la::pp::BN;
  a.real_tiles = a.m_tiles * a.n_tiles * splits;
  a.out = out_bf16 ? nullptr : (float*)out;
  a.outb = out_bf16 ? (__bf16*)out : nullptr;
  a.ldo = ldo;
  a.slab = slab;
  return a;
}

#if LA_PP_STAMP
extern "C" int la_gemm_pp_dbg(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(la::pp::pp_dbg), &p, sizeof(p));
}
#endif

// out = X W^T: fp32 slabs [splits][M][ldo] (stride slab) or bf16 [M][ldo] (splits == 1).
// Weight planes as la_qgemm_tile (p0 / p1 format planes, gsc = la_gemm_scales record plane).
extern "C" int la_gemm_pp(int fmt, const void* p0, const void* p1, const void* gsc, int N, int K, const void* X, int ldx,
                          int M, int splits, void* out, int ldo, long slab, int out_bf16, void* stream) {
  using namespace la::pp;
  if (pp_check(N, K, M, ldx, splits) || ldo < N || !pp_fmt_ok(fmt, p1, gsc)) return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  Args a = pp_args(p0, p1, gsc, N, K, X, ldx, M, splits, out, ldo, slab, out_bf16);
  const int grid = (a.real_tiles + 7) / 8 * 8;
  hipStream_t st = (hipStream_t)stream;
  switch (fmt) {
    case FMT_Q4_K: hipLaunchKernelGGL((gemm_pp_kernel<FMT_Q4_K, false>), dim3(grid), dim3(NT), 0, st, a); break;
    case FMT_Q6_K: hipLaunchKernelGGL((gemm_pp_kernel<FMT_Q6_K, false>), dim3(grid), dim3(NT), 0, st, a); break;
    case FMT_BF16: hipLaunchKernelGGL((gemm_pp_kernel<FMT_BF16, false>), dim3(grid), dim3(NT), 0, st, a); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

// Two weights of one output: columns [0, Na) from (fa, pa*), [Na, Na + Nb) from (fb, pb*).
extern "C" int la_gemm_pp2(int fa, const void* pa0, const void* pa1, const void* ga, int Na, int fb, const void* pb0,
                           const void* pb1, const void* gb, int Nb, int K, const void* X, int ldx, int M, int splits,
                           void* out, int ldo, long slab, int out_bf16, void* stream) {
  using namespace la::pp;
  if (pp_check(Na, K, M, ldx, splits) || Nb < 1 || ldo < Na + Nb) return -1;
  if (!pp_fmt_ok(fa, pa1, ga) || !pp_fmt_ok(fb, pb1, gb)) return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  Args a = pp_args(pa0, pa1, ga, Na, K, X, ldx, M, splits, out, ldo, slab, out_bf16);
  const size_t esz = out_bf16 ? 2 : 4;
  Args b = pp_args(pb0, pb1, gb, Nb, K, X, ldx, M, splits, (uint8_t*)out + (size_t)Na * esz, ldo, slab, out_bf16);
  const int grid = (a.real_tiles + b.real_tiles + 7) / 8 * 8;
  hipStream_t st = (hipStream_t)stream;
  if (fa == FMT_Q4_K && fb == FMT_Q6_K)
    hipLaunchKernelGGL((gemm_pp2_kernel<FMT_Q4_K, FMT_Q6_K>), dim3(grid), dim3(NT), 0, st, a, b, a.real_tiles);
  else if (fa == FMT_Q6_K && fb == FMT_Q4_K)
    hipLaunchKernelGGL((gemm_pp2_kernel<FMT_Q6_K, FMT_Q4_K>), dim3(grid), dim3(NT), 0, st, a, b, a.real_tiles);
  else if (fa == FMT_Q4_K && fb == FMT_Q4_K)
    hipLaunchKernelGGL((gemm_pp2_kernel<FMT_Q4_K, FMT_Q4_K>), dim3(grid), dim3(NT), 0, st, a, b, a.real_tiles);
  else
    return -2;
  return (int)hipGetLastError();
}

// h = act(x Wg^T) * (x Wu^T) -> bf16 [M][ldo]; gate rows oa .. oa+F of (pa*, ga), up rows ob ..
// ob+F of (pb*, gb) (same format).  act: 0 SwiGLU, 3 GeGLU.
extern "C" int la_gemm_pp_glu(int fmt, const void* pa0, const void* pa1, const void* ga, int oa, const void* pb0,
                              const void* pb1, const void* gb, int ob, int F, int K, const void* X, int ldx, int M,
                              void* out, int ldo, int act, void* stream) {
  using namespace la::pp;
  if (pp_check(F, K, M, ldx, 1) || ldo < F || (act != 0 && act != 3)) return -1;
  if (!pp_fmt_ok(fmt, pa1, ga) || !pp_fmt_ok(fmt, pb1, gb)) return -1;
  Args a = pp_args(pa0, pa1, ga, oa + F, K, X, ldx, M, 1, out, ldo, 0, 1);
  a.n_tiles = (F + BN / 2 - 1) / (BN / 2);
  a.real_tiles = a.m_tiles * a.n_tiles;
  a.glu = Glu{(const uint8_t*)pb0, (const uint8_t*)pb1, (const uint8_t*)gb, oa, ob, F, act};
  const int grid = (a.real_tiles + 7) / 8 * 8;
  hipStream_t st = (hipStream_t)stream;
  switch (fmt) {
    case FMT_Q4_K: hipLaunchKernelGGL((gemm_pp_kernel<FMT_Q4_K, true>), dim3(grid), dim3(NT), 0, st, a); break;
    case FMT_Q6_K: hipLaunchKernelGGL((gemm_pp_kernel<FMT_Q6_K, true>), dim3(grid), dim3(NT), 0, st, a); break;
    case FMT_BF16: hipLaunchKernelGGL((gemm_pp_kernel<FMT_BF16, true>), dim3(grid), dim3(NT), 0, st, a); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}
