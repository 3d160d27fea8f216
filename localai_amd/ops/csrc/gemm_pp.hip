// Prefill GEMM (M >= ~1024 rows): out[m][n] = sum_k X[m,k] * W[n,k], W in its GGUF quantisation
// (Q4_K, Q6_K) or bf16.  SURVEY §2.8 K6: the reference reaches this through ggml's mmq / dequant +
// hipBLAS GemmEx inside llama_decode (backend/cpp/llama/grpc-server.cpp:1910); here it is one
// hand-written CDNA4 kernel that never materialises a bf16 copy of the weight.
//
// Design (MI355X, cdna_hip_programming.md §5 "The 256^2 8-phase template", T1-T5):
//   * 256 x 256 output tile, BK = 64, 8 waves (512 threads) = 2 per SIMD, one workgroup per CU;
//     wave (wr, wc) = (wave >> 2, wave & 3) owns rows [128 wr, +128) x cols [64 wc, +64);
//   * v_mfma_f32_16x16x32_bf16 with SWAPPED operands (A-slot = W fragment, B-slot = X
//     fragment), so each lane's 4 accumulators are 4 consecutive output COLUMNS of one row and
//     the epilogue stores 8 / 16 bytes per lane with no LDS transpose;
//   * each K-tile is 4 phases (one 64 x 32 quadrant x K = 64 = 16 MFMAs per wave); the two wave
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
//     read: 32 weights / thread / K-tile, ~2.8 VALU each, hidden behind the other group's
//     MFMAs;
//   * counted vmcnt, raw s_barrier, all LDS in one array, s_setprio(1) around the MFMA clusters;
//   * XCD-aware tile order (each XCD takes a contiguous run, M fastest: the 32 workgroups of an
//     XCD share one weight panel in its L2), split-K into fp32 slabs, GLU (gate|up) epilogue.
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

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int ABUF = BM * BK * 2;              // 32 KiB bf16 X image per K-tile
constexpr int BBUF = BN * BK * 2;              // 32 KiB bf16 W image per K-tile
constexpr int LDS_BYTES = 3 * ABUF + 2 * BBUF;  // 160 KiB: X ring of 3, W images of 2

LA_DEV int swz(int r) { return (r >> 1) & 7; }

LA_DEV void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
template <int N>
LA_DEV void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
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
    r.q = ld_x4(s.p0, s.o0 + 32 * ks);
    r.s = ld_x2(s.gsc, s.os + 128 * ks);
  }
  LA_DEV static void wait_reg(Raw& r) {  // pins the registers at the wait (see raw_wait)
    asm volatile("" : "+v"(r.q), "+v"(r.s));
  }
  template <int HALF>
  LA_DEV static void deq(const Raw& r, int, bf16x8& c0, bf16x8& c1) {
    const float D = h2f((HALF ? r.s.y : r.s.x) & 0xFFFFu), O = h2f((HALF ? r.s.y : r.s.x) >> 16);
    if constexpr (HALF == 0) {
      c0 = deq8(nib_lo(r.q.x), nib_lo(r.q.y), D, O);
      c1 = deq8(nib_lo(r.q.z), nib_lo(r.q.w), D, O);
    } else {
      c0 = deq8(nib_hi(r.q.x), nib_hi(r.q.y), D, O);
      c1 = deq8(nib_hi(r.q.z), nib_hi(r.q.w), D, O);
    }
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
    r.ql = ld_x4(s.p0, s.o0 + 32 * ks);
    r.qh = ld_x4(s.p1, s.o1 + 16 * (ks & ~1));
    r.s = ld_x2(s.gsc, s.os + 128 * ks);
  }
  LA_DEV static void wait_reg(Raw& r) { asm volatile("" : "+v"(r.ql), "+v"(r.qh), "+v"(r.s)); }
  template <int HALF>
  LA_DEV static void deq(const Raw& r, int ks, bf16x8& c0, bf16x8& c1) {
    // this thread's 16-k scale group is h; the caller passes it folded into ks's high bit
    const int h = ks >> 30, sh = 2 * (ks & 1) + 4 * HALF;
    const uint32_t sv = HALF ? r.s.y : r.s.x;
    const float S = h2f(h ? (sv >> 16) : (sv & 0xFFFFu)), O = -32.0f * S;
    uint32_t q[4];
    const uint32_t l[4] = {r.ql.x, r.ql.y, r.ql.z, r.ql.w};
    const uint32_t hb[4] = {r.qh.x, r.qh.y, r.qh.z, r.qh.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t nb = HALF ? nib_hi(l[j]) : nib_lo(l[j]);
      asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q[j]) : "v"((hb[j] >> sh) << 4), "s"(0x30303030u), "v"(nb));
    }
    c0 = deq8(q[0], q[1], S, O);
    c1 = deq8(q[2], q[3], S, O);
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

template <int FMT, bool GLU>
LA_DEV void tile_run(uint8_t* __restrict__ lds, const Args& a, int tile) {
  using F = Fmt<FMT>;
  constexpr bool Q = FMT != FMT_BF16;
  constexpr int R = F::R;
  const int mt = tile % a.m_tiles;
  const int rest = tile / a.m_tiles;
  const int nt = rest % a.n_tiles;
  const int split = rest / a.n_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int m0 = mt * BM;
  const int KT = a.K >> 6;
  const int ks0 = split * a.per_split;
  const int nk = min(KT, ks0 + a.per_split) - ks0;  // even (host guarantees)
  if (nk <= 0) return;

  uint8_t* const Abase = lds;
  uint8_t* const Bbase = lds + 3 * ABUF;

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
    uint8_t* dst = Abase + (t % 3) * ABUF + 32 * wave * 128;
    const bf16* xk = a.X + F::xk(ks0 + t);
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j) glds16(xk + xoff[j], dst + j * 1024);
  };

  // ---- W: bf16 weights by DMA (wave w stages tile columns [32 w, +32)); quantised weights by
  // register loads (thread -> column c, k-half h) + dequant into the LDS image
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
    hh = tid >> 8;
    const int t8 = tid & 255;
    cw = ((t8 & 7) << 1) | ((t8 >> 3) & 1) | (t8 & 0xF0);  // lanes 0..7 -> swz 0..7: conflict-free writes
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
      uint8_t* dst = Bbase + (t & 1) * BBUF + 32 * wave * 128;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(wsrc[j] + 64 * (ks0 + t), dst + j * 1024);
    }
  };
  const int wb_off0 = cw * 128 + 16 * ((2 * hh) ^ swz(cw));
  const int wb_off1 = cw * 128 + 16 * ((2 * hh + 1) ^ swz(cw));
  const int wb_off4 = cw * 128 + 16 * ((4 + 2 * hh) ^ swz(cw));
  const int wb_off5 = cw * 128 + 16 * ((5 + 2 * hh) ^ swz(cw));
  auto dequant = [&](auto& raw, int t, auto HALF_) {
    if constexpr (Q) {
      constexpr int HALF = decltype(HALF_)::value;
      bf16x8 c0, c1;
      F::template deq<HALF>(raw, (ks0 + t) | (hh << 30), c0, c1);
      uint8_t* img = Bbase + (t & 1) * BBUF;
      *(bf16x8*)(img + (HALF ? wb_off4 : wb_off0)) = c0;
      *(bf16x8*)(img + (HALF ? wb_off5 : wb_off1)) = c1;
    }
  };

  // ---- fragments: lane (i = lane & 15, g = lane >> 4) reads row 16 blk + i, chunk 4 s + g
  const int fi = lane & 15, fg = lane >> 4;
  const int fo0 = fi * 128 + 16 * ((0 + fg) ^ swz(fi));
  const int fo1 = fi * 128 + 16 * ((4 + fg) ^ swz(fi));

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xf[4][2], wf0[2][2], wf1[2][2];
  auto read_x = [&](int t, int mh) {
    const uint8_t* A = Abase + (t % 3) * ABUF + 2048 * (8 * wr + 4 * mh);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      xf[rb][0] = *(const bf16x8*)(A + 2048 * rb + fo0);
      xf[rb][1] = *(const bf16x8*)(A + 2048 * rb + fo1);
    }
  };
  auto read_w = [&](int t, int nh, bf16x8 (&wf)[2][2]) {
    const uint8_t* B = Bbase + (t & 1) * BBUF + 2048 * (4 * wc + 2 * nh);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      wf[cb][0] = *(const bf16x8*)(B + 2048 * cb + fo0);
      wf[cb][1] = *(const bf16x8*)(B + 2048 * cb + fo1);
    }
  };
  auto mfma = [&](int mh, int nh, const bf16x8 (&wf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc[4 * mh + rb][2 * nh + cb] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][s], xf[rb][s], acc[4 * mh + rb][2 * nh + cb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto mfma_section = [&](int mh, int nh, const bf16x8 (&wf)[2][2]) {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma(mh, nh, wf);
    bar();
  };

  typename F::Raw raw0{}, raw1{};
  // ---- prologue: raw(0), X(0), raw(1), X(1)  [bf16: X(0), W(0), X(1)]
  if constexpr (Q) {
    F::load(raw0, src, ks0 + 0);
    issue_x(0, 0);
    issue_x(0, 2);
    if (nk > 1) F::load(raw1, src, ks0 + 1);
    if (nk > 1) {
      issue_x(1, 0);
      issue_x(1, 2);
    }
    vmwait<0>();  // prologue: simply drain (once per tile)
    F::wait_reg(raw0);
    F::wait_reg(raw1);
    dequant(raw0, 0, std::integral_constant<int, 0>{});
    dequant(raw0, 0, std::integral_constant<int, 1>{});
  } else {
    issue_x(0, 0);
    issue_x(0, 2);
    issue_wb(0);
    if (nk > 1) {
      issue_x(1, 0);
      issue_x(1, 2);
    }
    vmwait<0>();
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  if (wr == 1) bar();  // G1 runs one barrier behind G0

  // ---- main loop: two K-tiles per iteration (named raw register sets)
  auto ktile = [&](int t, auto& rcur, auto& rnext) {
    // rcur holds raw(t+1) (loaded during tile t-1), rnext receives raw(t+2)
    const bool more1 = t + 1 < nk, more2 = t + 2 < nk;
    // phase 0: quadrant (m0, n0); stage raw(t+2)
    read_x(t, 0);
    read_w(t, 0, wf0);
    if constexpr (Q) {
      if (more2) F::load(rnext, src, ks0 + t + 2);
    }
    mfma_section(0, 0, wf0);
    // phase 1: quadrant (m0, n1); X(t+2) pieces 0, 1  [bf16: W(t+1) first]
    read_w(t, 1, wf1);
    if constexpr (!Q) {
      if (more1) issue_wb(t + 1);
    }
    if (more2) issue_x(t + 2, 0);
    mfma_section(0, 1, wf1);
    // phase 2: quadrant (m1, n1); X(t+2) pieces 2, 3; dequant W(t+1) low half
    read_x(t, 1);
    if (more2) issue_x(t + 2, 2);
    if constexpr (Q) {
      if (more1) {
        if (more2) vmwait<R + 8>();
        else vmwait<4>();
        F::wait_reg(rcur);
        dequant(rcur, t + 1, std::integral_constant<int, 0>{});
      }
    }
    mfma_section(1, 1, wf1);
    // phase 3: quadrant (m1, n0); dequant W(t+1) high half; retire X(t+1) [+ W(t+1)]
    read_w(t, 0, wf0);
    if constexpr (Q) {
      if (more1) dequant(rcur, t + 1, std::integral_constant<int, 1>{});
    }
    if (more1) {
      if constexpr (Q) {
        if (more2) vmwait<R + 4>();
        else vmwait<0>();
      } else {
        if (more2) vmwait<4>();
        else vmwait<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    mfma_section(1, 0, wf0);
  };
  for (int t = 0; t < nk; t += 2) {
    ktile(t, raw1, raw0);
    ktile(t + 1, raw0, raw1);
  }
  if (wr == 0) bar();  // re-align the groups: every wave is past its last LDS read

  // ---- epilogue.  acc[mi][ni][e] = out[m0 + 128 wr + 16 mi + fi][64 wc + 16 ni + 4 fg + e]
  const int mrow = m0 + 128 * wr + fi;
  if constexpr (GLU) {
    // up waves (wc 2, 3) park their accumulators; gate waves (wc 0, 1) combine and store
    float* park = (float*)lds;
    const int pw = 2 * wr + (wc & 1);
    if (wc >= 2) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) *(f32x4*)(park + ((pw * 32 + mi * 4 + ni) * 64 + lane) * 4) = acc[mi][ni];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (wc < 2) {
      const int jb = nt * (BN / 2) + 64 * wc + 4 * fg;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int m = mrow + 16 * mi;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const f32x4 u = *(const f32x4*)(park + ((pw * 32 + mi * 4 + ni) * 64 + lane) * 4);
          const f32x4 gv = acc[mi][ni];
          const int j = jb + 16 * ni;
          bf16x4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = (bf16)((a.glu.act == 0 ? silu(gv[e]) : gelu_tanh(gv[e])) * u[e]);
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
    const int nb = nt * BN + 64 * wc + 4 * fg;
    float* o = a.out ? a.out + (size_t)split * a.slab : nullptr;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = mrow + 16 * mi;
      if (m >= a.M) continue;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = nb + 16 * ni;
        const f32x4 v = acc[mi][ni];
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
  if (M < 1 || N < 1 || K < 128 || (K & 127) || splits < 1 || ldx < K || (ldx & 7)) return -1;
  if ((long)M * ldx >= (1L << 31)) return -1;
  const int KT = K / 64;
  if (KT % splits || (KT / splits) & 1) return -1;  // equal, even K-tile counts per split
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
