// Quantised GEMM with a SHARED dequantised weight image ("bs" = B shared), for decode batches
// (M = 65..256) and prefill chunks (M up to 8192), on v_mfma_f32_32x32x16_bf16:
//   out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]  (fp32 split-K slabs, or bf16 [M][N] at S = 1)
//   GLU form:      out[m][j] = act(x Wg[j]^T) * (x Wu[j]^T), bf16 [M][F]
// W stays in its GGUF quantisation (Q4_K, Q6_K, Q8_0) or bf16.  SURVEY §2.8 K6: the reference
// reaches this through ggml's mmq / dequant + BLAS inside llama_decode
// (backend/cpp/llama/grpc-server.cpp:1910).
//
// Structure (one 256-thread workgroup per CU, ONE wave per SIMD):
//   * the workgroup tile is (4 * RM) rows x (128 * CBW) columns; wave w owns rows
//     [w*RM, (w+1)*RM) and computes them against ALL the tile's columns;
//   * wave w dequantises only the columns [32*CBW*w, 32*CBW*(w+1)) of each 64-deep K-step, ONCE,
//     into a bf16 B-fragment image in LDS that all four waves read (ds_read_b128, conflict-free
//     1 KiB fragments).  So every weight is dequantised once per workgroup (not once per wave as
//     in gemm_q32.hip, where each wave owned its columns and re-read every X row from LDS);
//   * X rows arrive by full-line 16-B global loads (8 rows x 128 B per wave instruction, never
//     fragment-shaped), three K-steps ahead in registers, and are transposed through a PRIVATE
//     per-wave LDS image (XOR-swizzled, conflict-free for both the ds_write_b128 and the
//     A-fragment ds_read_b128): no other wave touches it, so it needs no barrier;
//   * raw weight bytes and scale records are register loads three K-steps ahead;
//   * ONE s_barrier per K-step, after the third of its four MFMA sub-steps: by then every wave
//     has written its part of the NEXT step's B image, and the fourth sub-step's MFMAs cover the
//     first fragment reads of the next step (three B images rotate, so a wave that runs ahead
//     never overwrites an image a slower wave still reads).
//   * K permutation: MFMA lane half h of sub-step s holds physical k = run(h) + 8 s .. + 8, where
//     run(h) is the h-th 32-k run of the K-step (contiguous for Q4_K / Q8_0 / bf16, 64 apart for
//     Q6_K); A and B use the same map, so the dot product is unchanged.
//   * operands swapped (A = W fragment, B = X fragment): each lane's accumulators hold runs of 4
//     consecutive output columns, so the epilogue stores 16-B (fp32) / 8-B (bf16) vectors straight
//     from registers, and the GLU epilogue pairs gate and up accumulators in the same lane.
#include <type_traits>

#include "qweight.h"

namespace la {

typedef float bsf32x16 __attribute__((ext_vector_type(16)));

LA_DEV const uint8_t* bs_scale_base(const uint8_t* gsc, int n, int K) {
  // record (n, ks) of the blocked plane [ceil(N/16)][K/64][16][8 B] (la_gemm_scales) = base + 128 ks
  return gsc + ((size_t)(n >> 4) * (K >> 6) * 16 + (n & 15)) * 8;
}

// ---------------------------------------------------------------- per-format writer traits
// A writer lane (column c = lane & 31 of its 32-column block, half hh = lane >> 5) produces four
// 8-weight pieces p = 0..3 per K-step; piece p lands in B-fragment slot (sub-step S(p), run R(p)).
template <int FMT> struct BsF;

// Q4_K: 32 code bytes per column per K-step (byte i: k = i low nibble [run 0], k = 32 + i high
// nibble [run 1]); lane hh dequantises bytes [16hh, 16hh + 16): pieces (p>>1) = byte octet,
// (p&1) = nibble/run.
template <> struct BsF<FMT_Q4_K> {
  static constexpr int RUN = 32;
  LA_DEV static int xk(int ks) { return 64 * ks; }
  struct Raw {
    u32x4 q;
    u32x2 s;
  };
  struct Ptr {
    const uint8_t* q;
    const uint8_t* s;
  };
  LA_DEV static Ptr ptr(const QW& w, int n, int hh) {
    return Ptr{w.p0 + (size_t)n * (w.K >> 1) + 16 * hh, bs_scale_base(w.p2, n, w.K)};
  }
  LA_DEV static void load(Raw& r, const Ptr& p, int ks) {
    r.q = *(const u32x4*)(p.q + 32 * ks);
    r.s = *(const u32x2*)(p.s + 128 * ks);
  }
  LA_DEV static int S(int p, int hh) { return 2 * hh + (p >> 1); }
  LA_DEV static int R(int p, int) { return p & 1; }
  template <int P>
  LA_DEV static bf16x8 deq(const Raw& r, int) {
    constexpr int o = P >> 1, run = P & 1;
    const uint32_t w0 = o ? r.q.z : r.q.x, w1 = o ? r.q.w : r.q.y;
    uint32_t a, b;
    if constexpr (run == 0) {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(a) : "v"(w0));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(b) : "v"(w1));
    } else {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(a) : "v"(w0 >> 4));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(b) : "v"(w1 >> 4));
    }
    const uint32_t sr = run ? r.s.y : r.s.x;  // f16 d*sc, f16 -dmin*m of this run's sub-block
    const float D = h2f(sr & 0xFFFFu), Mn = h2f(sr >> 16);
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = (bf16)fmaf(D, (float)((a >> (8 * j)) & 0xFFu), Mn);
      v[j + 4] = (bf16)fmaf(D, (float)((b >> (8 * j)) & 0xFFu), Mn);
    }
    return v;
  }
};

// Q6_K: K-step ks = (super-block sb, 128-half hh_, part) covers run 0 = k [128hh_ + 32part, +32)
// (ql low nibbles, qh bits 2part) and run 1 = the same + 64 (ql high nibbles, qh bits 4 + 2part);
// 32 ql bytes + 32 qh bytes per column per K-step; lane hh takes bytes [16hh, 16hh + 16) of both.
template <> struct BsF<FMT_Q6_K> {
  static constexpr int RUN = 64;
  LA_DEV static int xk(int ks) { return 256 * (ks >> 2) + 128 * ((ks >> 1) & 1) + 32 * (ks & 1); }
  struct Raw {
    u32x4 l, h;
    u32x2 s;
    int sh;
  };
  struct Ptr {
    const uint8_t* l;
    const uint8_t* h;
    const uint8_t* s;
  };
  LA_DEV static Ptr ptr(const QW& w, int n, int hh) {
    return Ptr{w.p0 + (size_t)n * (w.K >> 1) + 16 * hh, w.p1 + (size_t)n * (w.K >> 2) + 16 * hh,
               bs_scale_base(w.p2, n, w.K)};
  }
  LA_DEV static void load(Raw& r, const Ptr& p, int ks) {
    r.l = *(const u32x4*)(p.l + 32 * ks);
    r.h = *(const u32x4*)(p.h + 16 * (ks & ~1));
    r.s = *(const u32x2*)(p.s + 128 * ks);
    r.sh = 2 * (ks & 1);
  }
  LA_DEV static int S(int p, int hh) { return 2 * hh + (p >> 1); }
  LA_DEV static int R(int p, int) { return p & 1; }
  template <int P>
  LA_DEV static bf16x8 deq(const Raw& r, int hh) {
    constexpr int o = P >> 1, run = P & 1;
    const uint32_t l0 = o ? r.l.z : r.l.x, l1 = o ? r.l.w : r.l.y;
    const uint32_t h0 = o ? r.h.z : r.h.x, h1 = o ? r.h.w : r.h.y;
    const int sh = r.sh + 4 * run;
    uint32_t n0, n1, q0, q1;
    if constexpr (run == 0) {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n0) : "v"(l0));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n1) : "v"(l1));
    } else {
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n0) : "v"(l0 >> 4));
      asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(n1) : "v"(l1 >> 4));
    }
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q0) : "v"((h0 >> sh) << 4), "s"(0x30303030u), "v"(n0));
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q1) : "v"((h1 >> sh) << 4), "s"(0x30303030u), "v"(n1));
    const uint32_t sr = run ? r.s.y : r.s.x;  // f16 d*sc of the 16-k groups g0, g1 of this run
    const float Sc = h2f(hh ? (sr >> 16) : (sr & 0xFFFFu)), O = -32.0f * Sc;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = (bf16)fmaf(Sc, (float)((q0 >> (8 * j)) & 0xFFu), O);
      v[j + 4] = (bf16)fmaf(Sc, (float)((q1 >> (8 * j)) & 0xFFu), O);
    }
    return v;
  }
};

// Q8_0: 64 code bytes per column per K-step = two 32-blocks (runs); lane hh takes run hh.
template <> struct BsF<FMT_Q8_0> {
  static constexpr int RUN = 32;
  LA_DEV static int xk(int ks) { return 64 * ks; }
  struct Raw {
    u32x4 a, b;
    uint32_t s;
  };
  struct Ptr {
    const uint8_t* q;
    const uint8_t* s;
  };
  LA_DEV static Ptr ptr(const QW& w, int n, int hh) {
    return Ptr{w.p0 + (size_t)n * w.K + 32 * hh, bs_scale_base(w.p2, n, w.K)};
  }
  LA_DEV static void load(Raw& r, const Ptr& p, int ks) {
    r.a = *(const u32x4*)(p.q + 64 * ks);
    r.b = *(const u32x4*)(p.q + 64 * ks + 16);
    r.s = *(const uint32_t*)(p.s + 128 * ks);
  }
  LA_DEV static int S(int p, int) { return p; }
  LA_DEV static int R(int, int hh) { return hh; }
  template <int P>
  LA_DEV static bf16x8 deq(const Raw& r, int hh) {
    const u32x4& Q = P < 2 ? r.a : r.b;
    const uint32_t w0 = (P & 1) ? Q.z : Q.x, w1 = (P & 1) ? Q.w : Q.y;
    uint32_t lo, hi;  // int8 -> q + 128 as an unsigned byte
    asm("v_xor_b32 %0, 0x80808080, %1" : "=v"(lo) : "v"(w0));
    asm("v_xor_b32 %0, 0x80808080, %1" : "=v"(hi) : "v"(w1));
    const float d = h2f(hh ? (r.s >> 16) : (r.s & 0xFFFFu)), o = -128.0f * d;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = (bf16)fmaf(d, (float)((lo >> (8 * j)) & 0xFFu), o);
      v[j + 4] = (bf16)fmaf(d, (float)((hi >> (8 * j)) & 0xFFu), o);
    }
    return v;
  }
};

// bf16 weights: lane hh copies run hh (32 weights = 64 B) of its column.
template <> struct BsF<FMT_BF16> {
  static constexpr int RUN = 32;
  LA_DEV static int xk(int ks) { return 64 * ks; }
  struct Raw {
    u32x4 v[4];
  };
  struct Ptr {
    const uint8_t* q;
  };
  LA_DEV static Ptr ptr(const QW& w, int n, int hh) { return Ptr{w.p0 + ((size_t)n * w.K + 32 * hh) * 2}; }
  LA_DEV static void load(Raw& r, const Ptr& p, int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = *(const u32x4*)(p.q + 128 * ks + 16 * i);
  }
  LA_DEV static int S(int p, int) { return p; }
  LA_DEV static int R(int, int hh) { return hh; }
  template <int P>
  LA_DEV static bf16x8 deq(const Raw& r, int) {
    return __builtin_bit_cast(bf16x8, r.v[P]);
  }
};

// ---------------------------------------------------------------- geometry
template <int RM_, int CBW_, int D_ = 3>
struct BsCfg {
  static constexpr int D = D_;                   // register ring depth (K-steps of loads in flight)
  static constexpr int RM = RM_;                 // rows per wave
  static constexpr int CBW = CBW_;               // 32-column blocks each wave dequantises
  static constexpr int MB = RM / 32;             // 32-row blocks per wave
  static constexpr int NCB = 4 * CBW;            // 32-column blocks per tile
  static constexpr int BM = 4 * RM, BN = 32 * NCB;
  static constexpr int XL = RM / 8;              // X load instructions per wave per K-step
  static constexpr int BIMG = 4 * NCB * 1024;    // one K-step's B image
  static constexpr int XIMG = RM * 128;          // one wave's X image of one K-step
  static constexpr int LDS = 3 * BIMG + 4 * 2 * XIMG;
  static_assert(RM % 32 == 0 && LDS <= 163840, "bs geometry");
};

struct BsGlu {
  QW up;
  int oa, ob, F, act;
};

// Grouped MoE rows (bsmoe_kernel): `order` points at the expert's first grouped pair; pair p is
// token p / topk's slot p % topk, weighted by wts[p].
struct BsMoe {
  const int* order;
  int topk;
  const float* wts;
};

LA_DEV float bs_gelu_tanh(float x) { return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))); }

// Epilogue straight from the accumulators: lane (m = c32, hh) of block (cb, mb) holds columns
// n = 32cb + 8g + 4hh + e (g = reg >> 2, e = reg & 3) of row 32mb + c32 of the wave's rows.
// MODE 3 (grouped MoE down projection): row m is pair mo.order[m]; its routing-weighted fp32 row
// goes to slab (split * topk + slot), row token.
template <class C, int MODE>
LA_DEV void bs_epilogue(const bsf32x16 (&acc)[C::NCB][C::MB], const QW& w, int mt, int nt, int split, int M,
                        float* __restrict__ out, bf16* __restrict__ outb, int ldo, long slab, const BsGlu& glu,
                        const BsMoe& mo) {
  constexpr int RM = C::RM, MB = C::MB, NCB = C::NCB;
  const int lane = threadIdx.x & 63, c32 = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mrow0 = mt * C::BM + wave * RM + c32;
  if constexpr (MODE == 1) {
    const int j0 = nt * (C::BN / 2);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = mrow0 + 32 * mb;
      if (m >= M) continue;
#pragma unroll
      for (int cb = 0; cb < NCB / 2; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int j = j0 + 32 * cb + 8 * g + 4 * hh;
          bf16x4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gv = acc[cb][mb][4 * g + e], uv = acc[cb + NCB / 2][mb][4 * g + e];
            hv[e] = (bf16)((glu.act == 0 ? silu(gv) : bs_gelu_tanh(gv)) * uv);
          }
          if (j < glu.F) *(bf16x4*)(outb + (size_t)m * ldo + j) = hv;  // F % 4 == 0
        }
    }
  } else if constexpr (MODE == 3) {
    const int n0 = nt * C::BN;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = mrow0 + 32 * mb;
      if (m >= M) continue;
      const int pair = mo.order[m], tok = pair / mo.topk, slot = pair - tok * mo.topk;
      const float sc = mo.wts[pair];
      float* o = out + (size_t)(split * mo.topk + slot) * slab + (size_t)tok * ldo;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + 32 * cb + 8 * g + 4 * hh;
          const f32x4 v{sc * acc[cb][mb][4 * g], sc * acc[cb][mb][4 * g + 1], sc * acc[cb][mb][4 * g + 2],
                        sc * acc[cb][mb][4 * g + 3]};
          if (n < w.N) *(f32x4*)(o + n) = v;  // N % 4 == 0
        }
    }
  } else {
    const int n0 = nt * C::BN;
    constexpr bool BFO = MODE == 2;  // bf16 [M][ldo] output, else fp32 slab `split`
    float* o = BFO ? nullptr : out + (size_t)split * slab;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = mrow0 + 32 * mb;
      if (m >= M) continue;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + 32 * cb + 8 * g + 4 * hh;
          const f32x4 v{acc[cb][mb][4 * g], acc[cb][mb][4 * g + 1], acc[cb][mb][4 * g + 2], acc[cb][mb][4 * g + 3]};
          if (n < w.N) {  // N % 4 == 0
            if constexpr (BFO) {
              bf16x4 bv;
              bv[0] = (bf16)v[0];
              bv[1] = (bf16)v[1];
              bv[2] = (bf16)v[2];
              bv[3] = (bf16)v[3];
              *(bf16x4*)(outb + (size_t)m * ldo + n) = bv;
            } else {
              *(f32x4*)(o + (size_t)m * ldo + n) = v;
            }
          }
        }
    }
  }
}

// One (M tile, N tile, K split) of a plain (MODE 0 fp32 slabs / 2 bf16), GLU (MODE 1) or grouped
// MoE down (MODE 3) GEMM.  GATHER: logical row m reads X row mo.order[m] / mo.topk (the token of a
// grouped MoE pair).
template <int FMT, class C, int MODE, int ABL = 0, int GATHER = 0>
LA_DEV void bs_tile(uint8_t* __restrict__ lds, const QW& w, int mt, int nt, int split, const bf16* __restrict__ X,
                    int ldx, int M, int per_split, float* __restrict__ out, bf16* __restrict__ outb, int ldo,
                    long slab, const BsGlu& glu, const BsMoe& mo = BsMoe{}) {
  using F = BsF<FMT>;
  constexpr int RM = C::RM, CBW = C::CBW, MB = C::MB, NCB = C::NCB, XL = C::XL;
  constexpr int BIMG = C::BIMG, XIMG = C::XIMG;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KS = w.K >> 6;
  const int k0 = split * per_split;
  const int nk = min(KS, k0 + per_split) - k0;
  if (nk <= 0) return;
  const int kl = k0 + nk - 1;  // last K-step of this split (load indices clamp here)

  const int c32 = lane & 31, hh = lane >> 5;

  // ---- writer columns: this wave dequantises col-blocks cb = wave*CBW + i
  typename F::Ptr wp[CBW];
#pragma unroll
  for (int i = 0; i < CBW; ++i) {
    const int cb = wave * CBW + i;
    if constexpr (MODE == 1) {
      const bool up = cb >= NCB / 2;
      const int j = nt * (C::BN / 2) + (up ? cb - NCB / 2 : cb) * 32 + c32;
      const QW& q = up ? glu.up : w;
      wp[i] = F::ptr(q, (up ? glu.ob : glu.oa) + min(j, glu.F - 1), hh);
    } else {
      wp[i] = F::ptr(w, min(nt * C::BN + cb * 32 + c32, w.N - 1), hh);
    }
  }
  // ---- X rows of this wave: load instruction i covers rows 8i .. 8i+7, lane -> (row, 16-B chunk)
  const bf16* xp[XL];
  uint32_t xw[XL];  // ds_write offsets inside a wave X image
#pragma unroll
  for (int i = 0; i < XL; ++i) {
    const int r = 8 * i + (lane >> 3), c = lane & 7;
    int m = min(mt * C::BM + wave * RM + r, M - 1);
    if constexpr (GATHER) m = mo.order[m] / mo.topk;
    xp[i] = X + (size_t)m * ldx + (c < 4 ? 8 * c : F::RUN + 8 * (c - 4));
    xw[i] = (uint32_t)(r * 8 + (c ^ ((r >> 1) & 7))) * 16;
  }
  uint32_t xr_off[MB][4];  // A-fragment ds_read offsets (row 32mb + c32, chunk 4hh + s)
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = 32 * mb + c32;
      xr_off[mb][s] = (uint32_t)(r * 8 + ((4 * hh + s) ^ ((r >> 1) & 7))) * 16;
    }

  uint8_t* bimg = lds;                                  // [3][4 s][NCB][64 lanes][16 B]
  uint8_t* ximg = lds + 3 * BIMG + wave * 2 * XIMG;     // this wave's [2][RM][8][16 B]

  // register rings (three K-steps deep)
  constexpr int D = C::D;
  typename F::Raw wr[D][CBW];
  u32x4 xr[D][XL];
  auto load_w = [&](auto P_, int t) {
    constexpr int P = decltype(P_)::value;
    const int ks = min(k0 + t, kl);
    if constexpr (ABL & 8) return;  // probe: no weight loads
#pragma unroll
    for (int i = 0; i < CBW; ++i) F::load(wr[P][i], wp[i], ks);
  };
  // X rows [i0, i1) of the load instructions of K-step t into register set P
  auto load_x = [&](auto P_, int t, int i0, int i1) {
    constexpr int P = decltype(P_)::value;
    const int xk = F::xk(min(k0 + t, kl));
    if constexpr (ABL & 4) return;  // probe: no X loads
#pragma unroll
    for (int i = 0; i < XL; ++i)
      if (i >= i0 && i < i1) {
        // X bypasses the CU's L1 (nt): it is never re-read by this CU, and a 32 KB-per-step stream
        // through the 32 KB L1 would evict the weight lines that the next three K-steps re-read
        if constexpr (ABL & 2048) xr[P][i] = *(const u32x4*)(xp[i] + xk);
        else xr[P][i] = __builtin_nontemporal_load((const u32x4*)(xp[i] + xk));
      }
  };
  // keep each sub-step's loads, LDS traffic and dequant beside that sub-step's MFMAs: without
  // the fence the compiler hoists the whole step's global loads into one burst at its start,
  // and four lock-stepped waves' bursts then queue behind each other in the CU's memory pipe
  auto fence = [&]() {
    if constexpr (!(ABL & 1024)) __builtin_amdgcn_sched_barrier(0);
  };
  // dequantise piece p of every column block of K-step (in register set P) into B image `img`
  auto deq_piece = [&](auto P_, auto p_, uint8_t* img) {
    constexpr int P = decltype(P_)::value, p = decltype(p_)::value;
#pragma unroll
    for (int i = 0; i < CBW; ++i) {
      const int cb = wave * CBW + i;
      bf16x8 v;
      if constexpr (ABL & 2) v = __builtin_bit_cast(bf16x8, u32x4{wr[P][i].q.x, wr[P][i].q.y, wr[P][i].q.z, wr[P][i].s.x});
      else v = F::template deq<p>(wr[P][i], hh);
      const int s = F::S(p, hh), run = F::R(p, hh);
      *(bf16x8*)(img + ((s * NCB + cb) * 64 + c32 + 32 * run) * 16) = v;
    }
  };
  auto write_x = [&](auto P_, int i, uint8_t* img) {
    constexpr int P = decltype(P_)::value;
    if constexpr (ABL & 32) return;  // probe: no X image writes
    *(u32x4*)(img + xw[i]) = xr[P][i];
  };

  bsf32x16 acc[NCB][MB];
#pragma unroll
  for (int a = 0; a < NCB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // ---- prologue: K-steps 0, 1, 2 in flight; step 0's X image and B image written
  using I4 = std::integral_constant<int, 4>;
  load_w(I0{}, 0);
  load_x(I0{}, 0, 0, XL);
  load_w(I1{}, 1);
  load_x(I1{}, 1, 0, XL);
  if constexpr (D > 2) {
    load_w(I2{}, 2);
    load_x(I2{}, 2, 0, XL);
  }
  if constexpr (D > 3) {
    load_w(I3{}, 3);
    load_x(I3{}, 3, 0, XL);
  }
#pragma unroll
  for (int i = 0; i < XL; ++i) write_x(I0{}, i, ximg);
  deq_piece(I0{}, I0{}, bimg);
  deq_piece(I0{}, I1{}, bimg);
  deq_piece(I0{}, I2{}, bimg);
  deq_piece(I0{}, I3{}, bimg);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  bf16x8 bf[2][NCB];  // B fragments: [sub-step parity][col block]
  bf16x8 af[2][MB];   // A fragments: [sub-step parity][row block]
  auto read_b = [&](bf16x8 (&dst)[NCB], const uint8_t* img, int s) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      if constexpr (ABL & 64) asm volatile("; probe: no B read" : "+v"(dst[cb]));
      else dst[cb] = *(const bf16x8*)(img + ((s * NCB + cb) * 64 + lane) * 16);
    }
  };
  auto read_a = [&](bf16x8 (&dst)[MB], const uint8_t* img, auto s_) {
    constexpr int s = decltype(s_)::value;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      if constexpr (ABL & 128) asm volatile("; probe: no A read" : "+v"(dst[mb]));
      else dst[mb] = *(const bf16x8*)(img + xr_off[mb][s]);
    }
  };
  auto mfmas = [&](const bf16x8 (&a)[MB], const bf16x8 (&b)[NCB]) {
    if constexpr (LA_SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        if constexpr (ABL & 1) asm volatile("; probe: no MFMA" ::"v"(a[mb]), "v"(b[cb]));
        else acc[cb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[cb], a[mb], acc[cb][mb], 0, 0, 0);
    if constexpr (LA_SETPRIO) __builtin_amdgcn_s_setprio(0);
  };
  read_b(bf[0], bimg, 0);
  read_a(af[0], ximg, I0{});

  // One K-step t: register sets P = t % 3 (compile time), images by t (run time).  Fragments of
  // sub-step s + 1 are read while sub-step s's MFMAs run; the next step's first fragments are read
  // after the barrier, under the fourth sub-step's MFMAs.
  auto step = [&](auto P_, int t) {
    constexpr int P = decltype(P_)::value;
    using NX = std::integral_constant<int, (P + 1) % D>;
    const int ib = t % 3;
    const uint8_t* bcur = bimg + ib * BIMG;
    uint8_t* bnxt = bimg + ((ib + 1) % 3) * BIMG;
    const uint8_t* xcur = ximg + (t & 1) * XIMG;
    uint8_t* xnxt = ximg + ((t + 1) & 1) * XIMG;
    // operands of step t + D go into the register sets step t has finished with, a quarter of
    // the X rows per sub-step
    auto sub = [&](auto s_) {
      constexpr int s = decltype(s_)::value;
      read_a(af[(s + 1) & 1], xcur, std::integral_constant<int, s + 1>{});
      read_b(bf[(s + 1) & 1], bcur, s + 1);
      fence();  // the next sub-step's fragment reads issue BEFORE this sub-step's MFMAs
      if constexpr (s == 0) load_w(P_, t + D);
      load_x(P_, t + D, s * XL / 4, (s + 1) * XL / 4);
      // this sub-step's share of the next step's work: dequant pieces + X image writes
      if constexpr (s == 0) {
        deq_piece(NX{}, I0{}, bnxt);
        deq_piece(NX{}, I1{}, bnxt);
      } else if constexpr (s == 1) {
        deq_piece(NX{}, I2{}, bnxt);
      } else {
        deq_piece(NX{}, I3{}, bnxt);
      }
#pragma unroll
      for (int i = s * XL / 4; i < (s + 1) * XL / 4; ++i) write_x(NX{}, i, xnxt);
      mfmas(af[s & 1], bf[s & 1]);
      fence();
    };
    sub(I0{});
    sub(I1{});
    sub(I2{});
    // every wave's share of the next B image is written and its reads of image t-2 are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(ABL & 16)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 3 * XL / 4; i < XL; ++i) write_x(NX{}, i, xnxt);
    load_x(P_, t + D, 3 * XL / 4, XL);
    read_a(af[0], xnxt, I0{});
    read_b(bf[0], bnxt, 0);
    fence();
    mfmas(af[1], bf[1]);
    fence();
  };

  int t = 0;
  for (; t + D <= nk; t += D) {
    step(I0{}, t);
    step(I1{}, t + 1);
    if constexpr (D > 2) step(I2{}, t + 2);
    if constexpr (D > 3) step(I3{}, t + 3);
  }
  if (t < nk) step(I0{}, t);
  if constexpr (D > 2)
    if (t + 1 < nk) step(I1{}, t + 1);
  if constexpr (D > 3)
    if (t + 2 < nk) step(I2{}, t + 2);

  bs_epilogue<C, MODE>(acc, w, mt, nt, split, M, out, outb, ldo, slab, glu, mo);
}

// The same tile with X in the BLOCKED layout Xb[ceil(M/32)][K/8][32 rows][8] bf16 (16-B chunk
// (row r, k-chunk c) at ((r/32 * K/8 + c) * 32 + r%32) * 16 bytes): an A fragment (32 rows x 8 k
// per lane half) is then two 512-B contiguous runs, so every X load is a full-line load straight
// into the fragment registers -- no private LDS transpose (its ds_write pass was most of the LDS
// write traffic), and X loads need no LDS space at all.  The producer kernels write this layout.
template <int FMT, class C, int MODE, int ABL = 0>
LA_DEV void bs_tile_xb(uint8_t* __restrict__ lds, const QW& w, int mt, int nt, int split, const bf16* __restrict__ Xb,
                       int M, int per_split, float* __restrict__ out, bf16* __restrict__ outb, int ldo, long slab,
                       const BsGlu& glu) {
  using F = BsF<FMT>;
  constexpr int RM = C::RM, CBW = C::CBW, MB = C::MB, NCB = C::NCB, BIMG = C::BIMG, D = C::D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KS = w.K >> 6;
  const int k0 = split * per_split;
  const int nk = min(KS, k0 + per_split) - k0;
  if (nk <= 0) return;
  const int kl = k0 + nk - 1;
  const int c32 = lane & 31, hh = lane >> 5;

  typename F::Ptr wp[CBW];
#pragma unroll
  for (int i = 0; i < CBW; ++i) {
    const int cb = wave * CBW + i;
    if constexpr (MODE == 1) {
      const bool up = cb >= NCB / 2;
      const int j = nt * (C::BN / 2) + (up ? cb - NCB / 2 : cb) * 32 + c32;
      const QW& q = up ? glu.up : w;
      wp[i] = F::ptr(q, (up ? glu.ob : glu.oa) + min(j, glu.F - 1), hh);
    } else {
      const int n = min(nt * C::BN + cb * 32 + c32, w.N - 1);
      wp[i] = F::ptr(w, n, hh);
      if constexpr ((ABL & 16384) && FMT == FMT_Q4_K) {
        // probe: codes repacked [N/32][K/64][32 cols][32 B] (one K-step of 32 columns = 1 KiB)
        wp[i].q = w.p0 + ((size_t)(n >> 5) * (w.K >> 6) * 32 + (n & 31)) * 32 + 16 * hh;
      }
    }
  }
  // A-fragment pointers: row block mb of this wave (clamped into the allocated blocks), lane row
  // c32, run hh; + 8 * (chunk of K-step ks, sub-step s) * 32 elements
  const int nmb = (M + 31) >> 5;
  const bf16* xp[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int b = min((mt * C::BM + wave * RM) / 32 + mb, nmb - 1);
    xp[mb] = Xb + ((size_t)b * (w.K >> 3) * 32 + (size_t)(F::RUN / 8) * hh * 32 + c32) * 8;
  }
  uint8_t* bimg = lds;  // [3][4 s][NCB][64 lanes][16 B]

  typename F::Raw wr[D][CBW];
  bf16x8 xr[D][MB][4];  // A fragments of D K-steps
  auto load_w = [&](auto P_, int t) {
    constexpr int P = decltype(P_)::value;
    const int ks = min(k0 + t, kl);
    if constexpr (ABL & 8) return;
#pragma unroll
    for (int i = 0; i < CBW; ++i) {
      if constexpr ((ABL & 16384) && FMT == FMT_Q4_K) {
        wr[P][i].q = *(const u32x4*)(wp[i].q + 1024 * ks);
        wr[P][i].s = *(const u32x2*)(wp[i].s + 128 * ks);
      } else {
        F::load(wr[P][i], wp[i], ks);
      }
    }
  };
  auto load_x = [&](auto P_, int t, auto s_) {
    constexpr int P = decltype(P_)::value, s = decltype(s_)::value;
    const int c0 = F::xk(min(k0 + t, kl)) >> 3;  // first 8-k chunk of run 0
    if constexpr (ABL & 4) return;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) xr[P][mb][s] = *(const bf16x8*)(xp[mb] + (size_t)(c0 + s) * 256);
  };
  auto fence = [&]() {
    if constexpr (!(ABL & 1024)) __builtin_amdgcn_sched_barrier(0);
  };
  auto deq_piece = [&](auto P_, auto p_, uint8_t* img) {
    constexpr int P = decltype(P_)::value, p = decltype(p_)::value;
#pragma unroll
    for (int i = 0; i < CBW; ++i) {
      const int cb = wave * CBW + i;
      const bf16x8 v = F::template deq<p>(wr[P][i], hh);
      const int s = F::S(p, hh), run = F::R(p, hh);
      *(bf16x8*)(img + ((s * NCB + cb) * 64 + c32 + 32 * run) * 16) = v;
    }
  };

  bsf32x16 acc[NCB][MB];
#pragma unroll
  for (int a = 0; a < NCB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  auto load_x_all = [&](auto P_, int t) {
    load_x(P_, t, I0{});
    load_x(P_, t, I1{});
    load_x(P_, t, I2{});
    load_x(P_, t, I3{});
  };
  load_w(I0{}, 0);
  load_x_all(I0{}, 0);
  load_w(I1{}, 1);
  load_x_all(I1{}, 1);
  if constexpr (D > 2) {
    load_w(I2{}, 2);
    load_x_all(I2{}, 2);
  }
  if constexpr (D > 3) {
    load_w(I3{}, 3);
    load_x_all(I3{}, 3);
  }
  deq_piece(I0{}, I0{}, bimg);
  deq_piece(I0{}, I1{}, bimg);
  deq_piece(I0{}, I2{}, bimg);
  deq_piece(I0{}, I3{}, bimg);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  bf16x8 bf[2][NCB];
  auto read_b = [&](bf16x8 (&dst)[NCB], const uint8_t* img, int s) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) dst[cb] = *(const bf16x8*)(img + ((s * NCB + cb) * 64 + lane) * 16);
  };
  auto mfmas = [&](auto P_, auto s_, const bf16x8 (&b)[NCB]) {
    constexpr int P = decltype(P_)::value, s = decltype(s_)::value;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        acc[cb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[cb], xr[P][mb][s], acc[cb][mb], 0, 0, 0);
      }
  };
  read_b(bf[0], bimg, 0);

  auto step = [&](auto P_, int t) {
    constexpr int P = decltype(P_)::value;
    using NX = std::integral_constant<int, (P + 1) % D>;
    const int ib = t % 3;
    const uint8_t* bcur = bimg + ib * BIMG;
    uint8_t* bnxt = bimg + ((ib + 1) % 3) * BIMG;
    auto sub = [&](auto s_) {
      constexpr int s = decltype(s_)::value;
      read_b(bf[(s + 1) & 1], bcur, s + 1);
      fence();  // the next sub-step's fragment reads issue BEFORE this sub-step's MFMAs
      if constexpr (s == 0) load_w(P_, t + D);
      if constexpr (s == 0) {
        deq_piece(NX{}, I0{}, bnxt);
        deq_piece(NX{}, I1{}, bnxt);
      } else if constexpr (s == 1) {
        deq_piece(NX{}, I2{}, bnxt);
      } else {
        deq_piece(NX{}, I3{}, bnxt);
      }
      mfmas(P_, s_, bf[s & 1]);
      load_x(P_, t + D, s_);  // this sub-step's A fragments are consumed: refill for step t + D
      fence();
    };
    sub(I0{});
    sub(I1{});
    sub(I2{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(ABL & 16)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_b(bf[0], bnxt, 0);
    fence();
    mfmas(P_, I3{}, bf[1]);
    load_x(P_, t + D, I3{});
    fence();
  };

  int t = 0;
  for (; t + D <= nk; t += D) {
    step(I0{}, t);
    step(I1{}, t + 1);
    if constexpr (D > 2) step(I2{}, t + 2);
    if constexpr (D > 3) step(I3{}, t + 3);
  }
  if (t < nk) step(I0{}, t);
  if constexpr (D > 2)
    if (t + 1 < nk) step(I1{}, t + 1);
  if constexpr (D > 3)
    if (t + 2 < nk) step(I2{}, t + 2);
  bs_epilogue<C, MODE>(acc, w, mt, nt, split, M, out, outb, ldo, slab, glu, BsMoe{});
}

// Tile id -> (n tile fastest, then m tile, then split).  Blocks are dealt round-robin over the 8
// XCDs; each XCD takes a contiguous run of tile ids (bijective for any grid), so the 32 CUs of an
// XCD sweep the n tiles of ONE m tile together (its X rows stay in that XCD's L2) and the XCDs
// walk the weight in step (its bytes are shared through the Infinity Cache).
LA_DEV int bs_tile_id(int real) {
  const int b = blockIdx.x, x = b & 7, q = real >> 3, r = real & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

template <int FMT, class C, int MODE>
__global__ __launch_bounds__(256, 1) void bsgemm_kernel(QW w, const bf16* __restrict__ X, int ldx, int M,
                                                         int per_split, int m_tiles, int n_tiles, int real,
                                                         float* __restrict__ out, bf16* __restrict__ outb, int ldo,
                                                         long slab) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[C::LDS];
  if ((int)blockIdx.x >= real) return;
  const int tile = bs_tile_id(real);
  const int nt = tile % n_tiles, r = tile / n_tiles, mt = r % m_tiles, split = r / m_tiles;
  bs_tile<FMT, C, MODE>(lds, w, mt, nt, split, X, ldx, M, per_split, out, outb, ldo, slab, BsGlu{});
}

template <int ABL>
__global__ __launch_bounds__(256, 1) void bsgemm_probe_kernel(QW w, const bf16* __restrict__ X, int ldx, int M,
                                                               int m_tiles, int n_tiles, int real,
                                                               bf16* __restrict__ outb) {
  using C = BsCfg<64, (ABL & 512) ? 2 : 1, (ABL & 512) ? 2 : (ABL & 256) ? 4 : 3>;
  constexpr int AB = ABL & ~(256 | 512);
  __shared__ __attribute__((aligned(1024))) uint8_t lds[C::LDS];
  if ((int)blockIdx.x >= real) return;
  const int tile = bs_tile_id(real);
  if constexpr (ABL & 8192)
    bs_tile_xb<FMT_Q4_K, C, 2, (AB & ~8192)>(lds, w, tile / n_tiles, tile % n_tiles, 0, X, M, w.K >> 6, nullptr, outb,
                                             w.N, 0, BsGlu{});
  else
    bs_tile<FMT_Q4_K, C, 2, AB>(lds, w, tile / n_tiles, tile % n_tiles, 0, X, ldx, M, w.K >> 6, nullptr, outb, w.N,
                                0, BsGlu{});
}

// Two weights of one fused output (Q4_K q|k beside a Q6_K v): segment B's tiles follow A's.
template <int FA, int FB, class C, int MODE>
__global__ __launch_bounds__(256, 1) void bsgemm2_kernel(QW wa, QW wb, int col_b, const bf16* __restrict__ X, int ldx,
                                                          int M, int per_split, int m_tiles, int nta, int ntb,
                                                          int tiles_a, int real, float* __restrict__ out,
                                                          bf16* __restrict__ outb, int ldo, long slab) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[C::LDS];
  if ((int)blockIdx.x >= real) return;
  int tile = bs_tile_id(real);
  if (tile < tiles_a) {
    const int nt = tile % nta, r = tile / nta;
    bs_tile<FA, C, MODE>(lds, wa, r % m_tiles, nt, r / m_tiles, X, ldx, M, per_split, out, outb, ldo, slab, BsGlu{});
  } else {
    tile -= tiles_a;
    const int nt = tile % ntb, r = tile / ntb;
    bs_tile<FB, C, MODE>(lds, wb, r % m_tiles, nt, r / m_tiles, X, ldx, M, per_split, out ? out + col_b : nullptr,
                      outb ? outb + col_b : nullptr, ldo, slab, BsGlu{});
  }
}

template <int FMT, class C>
__global__ __launch_bounds__(256, 1) void bsgemm_glu_kernel(QW wg, BsGlu glu, const bf16* __restrict__ X, int ldx,
                                                             int M, int m_tiles, int n_tiles, int real,
                                                             bf16* __restrict__ outb, int ldo) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[C::LDS];
  if ((int)blockIdx.x >= real) return;
  const int tile = bs_tile_id(real);
  const int nt = tile % n_tiles, mt = tile / n_tiles;
  bs_tile<FMT, C, 1>(lds, wg, mt, nt, 0, X, ldx, M, wg.K >> 6, nullptr, outb, ldo, 0, glu);
}

// Grouped MoE GEMM: every local expert's routed rows in ONE launch, no host read of the grouping.
// The grid covers cmax = ceil(P / BM) + E row chunks (P = T * topk pairs), enough for any routing:
// sum_e ceil(M_e / BM) <= P / BM + E.  Tile id -> (n tile fastest, row chunk, split); a workgroup
// finds the expert of its chunk with a wave-wide prefix sum over the per-expert chunk counts (read
// from off[], identical in every wave) and exits when the chunk is past the last expert's rows.
//   MODE 1: gate|up of the expert (gate rows [0, F), up rows [F, 2F) of one weight), GLU fused, X
//           rows gathered from the tokens -> bf16 h rows in grouped order (row off[e] + m)
//   MODE 3: down projection of the grouped h rows -> routing-weighted fp32 rows scattered to slab
//           (split * topk + slot), row token
template <int FMT, class C, int MODE>
__global__ __launch_bounds__(256, 1) void bsmoe_kernel(const QW* __restrict__ qws, const int* __restrict__ order,
                                                        const int* __restrict__ off, int E, int topk,
                                                        const bf16* __restrict__ X, int ldx, int cmax, int n_tiles,
                                                        int per_split, int real, const float* __restrict__ wts,
                                                        float* __restrict__ out, bf16* __restrict__ outb, int ldo,
                                                        long slab, int F, int act) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[C::LDS];
  if ((int)blockIdx.x >= real) return;
  const int tile = bs_tile_id(real);
  const int nt = tile % n_tiles, r = tile / n_tiles, c = r % cmax, split = r / cmax;
  const int lane = threadIdx.x & 63;
  int e = -1, cl = 0, base = 0;
  for (int e0 = 0; e0 < E; e0 += 64) {
    const int ei = e0 + lane;
    const int cnt = ei < E ? (off[ei + 1] - off[ei] + C::BM - 1) / C::BM : 0;
    int inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(inc, d);
      if (lane >= d) inc += v;
    }
    const unsigned long long hit = __ballot(cnt > 0 && c >= base + inc - cnt && c < base + inc);
    if (hit) {
      const int l = __ffsll((long long)hit) - 1;
      e = e0 + l;
      cl = c - base - (__shfl(inc, l) - __shfl(cnt, l));
      break;
    }
    base += __shfl(inc, 63);
  }
  e = __builtin_amdgcn_readfirstlane(e);
  cl = __builtin_amdgcn_readfirstlane(cl);
  if (e < 0) return;
  const int o0 = off[e], Me = off[e + 1] - o0;
  QW w = qws[e];
  const BsMoe mo{order + o0, topk, wts};
  if constexpr (MODE == 1) {
    const BsGlu glu{w, 0, F, F, act};
    w.N = F;
    bs_tile<FMT, C, 1, 0, 1>(lds, w, cl, nt, 0, X, ldx, Me, w.K >> 6, nullptr, outb + (size_t)o0 * ldo, ldo, 0, glu,
                             mo);
  } else {
    bs_tile<FMT, C, 3>(lds, w, cl, nt, split, X + (size_t)o0 * ldx, ldx, Me, per_split, out, nullptr, ldo, slab,
                       BsGlu{}, mo);
  }
}

// variant ids (ops/__init__.py BS_TILES): tile, rows per wave, column blocks per wave, ring depth
//   0: 256 x 128 (RM 64, CBW 1, D 3)   1: 128 x 128 (RM 32, CBW 1, D 3; two workgroups per CU)
//   2: 256 x 256 (RM 64, CBW 2, D 2)   3: 256 x 128 (RM 64, CBW 1, D 4)
template <class Fn>
static int bs_var(int var, Fn&& fn) {
  switch (var) {
    case 0: fn(BsCfg<64, 1>{}); break;
    case 1: fn(BsCfg<32, 1>{}); break;
    case 2: fn(BsCfg<64, 2, 2>{}); break;
    case 3: fn(BsCfg<64, 1, 4>{}); break;
    default: return -1;
  }
  return 0;
}

template <int FMT>
static int bs_launch(int var, const QW& w, const bf16* X, int ldx, int M, int splits, float* out, bf16* outb, int ldo,
                     long slab, hipStream_t st) {
  const int KS = w.K >> 6, per = (KS + splits - 1) / splits;
  return bs_var(var, [&](auto c) {
    using C = decltype(c);
    const int m_tiles = (M + C::BM - 1) / C::BM, n_tiles = (w.N + C::BN - 1) / C::BN;
    const int real = m_tiles * n_tiles * splits;
    if (outb)
      hipLaunchKernelGGL((bsgemm_kernel<FMT, C, 2>), dim3(real), dim3(256), 0, st, w, X, ldx, M, per, m_tiles, n_tiles,
                         real, out, outb, ldo, slab);
    else
      hipLaunchKernelGGL((bsgemm_kernel<FMT, C, 0>), dim3(real), dim3(256), 0, st, w, X, ldx, M, per, m_tiles, n_tiles,
                         real, out, outb, ldo, slab);
  });
}

template <int FA, int FB>
static int bs_launch2(int var, const QW& wa, const QW& wb, const bf16* X, int ldx, int M, int splits, float* out,
                      bf16* outb, int ldo, long slab, hipStream_t st) {
  const int KS = wa.K >> 6, per = (KS + splits - 1) / splits;
  return bs_var(var, [&](auto c) {
    using C = decltype(c);
    const int m_tiles = (M + C::BM - 1) / C::BM;
    const int nta = (wa.N + C::BN - 1) / C::BN, ntb = (wb.N + C::BN - 1) / C::BN;
    const int tiles_a = m_tiles * nta * splits, real = tiles_a + m_tiles * ntb * splits;
    if (outb)
      hipLaunchKernelGGL((bsgemm2_kernel<FA, FB, C, 2>), dim3(real), dim3(256), 0, st, wa, wb, wa.N, X, ldx, M, per,
                         m_tiles, nta, ntb, tiles_a, real, out, outb, ldo, slab);
    else
      hipLaunchKernelGGL((bsgemm2_kernel<FA, FB, C, 0>), dim3(real), dim3(256), 0, st, wa, wb, wa.N, X, ldx, M, per,
                         m_tiles, nta, ntb, tiles_a, real, out, outb, ldo, slab);
  });
}

template <int FMT>
static int bs_launch_glu(int var, const QW& wg, const BsGlu& glu, const bf16* X, int ldx, int M, bf16* outb, int ldo,
                         hipStream_t st) {
  return bs_var(var, [&](auto c) {
    using C = decltype(c);
    const int m_tiles = (M + C::BM - 1) / C::BM, n_tiles = (glu.F + C::BN / 2 - 1) / (C::BN / 2);
    const int real = m_tiles * n_tiles;
    hipLaunchKernelGGL((bsgemm_glu_kernel<FMT, C>), dim3(real), dim3(256), 0, st, wg, glu, X, ldx, M, m_tiles, n_tiles,
                       real, outb, ldo);
  });
}

template <int FMT, int MODE>
static int bsmoe_launch(int var, const QW* qws, int N, int K, int E, const int* order, const int* off, int topk,
                        const bf16* X, int ldx, int P, int splits, const float* wts, float* out, bf16* outb, int ldo,
                        long slab, int act, hipStream_t st) {
  const int KS = K >> 6, per = (KS + splits - 1) / splits;
  return bs_var(var, [&](auto c) {
    using C = decltype(c);
    const int cmax = (P + C::BM - 1) / C::BM + E;
    const int n_tiles = MODE == 1 ? (N + C::BN / 2 - 1) / (C::BN / 2) : (N + C::BN - 1) / C::BN;
    const int real = cmax * n_tiles * splits;
    hipLaunchKernelGGL((bsmoe_kernel<FMT, C, MODE>), dim3(real), dim3(256), 0, st, qws, order, off, E, topk, X, ldx,
                       cmax, n_tiles, per, real, wts, out, outb, ldo, slab, N, act);
  });
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// Operand conventions of la_qgemm32 (gemm_q32.hip): p0/p1 format planes, gsc the blocked scale
// plane (la_gemm_scales; unused for bf16 weights); out fp32 slabs [splits][M][ldo] (stride slab)
// or bf16 [M][ldo] (out_bf16, splits == 1).  ldo and ldx multiples of 8; X 16-B aligned.
static bool la_bs_fmt(int f) { return f == la::FMT_Q4_K || f == la::FMT_Q6_K || f == la::FMT_Q8_0 || f == la::FMT_BF16; }

extern "C" int la_bsgemm(int fmt, const void* p0, const void* p1, const void* gsc, int N, int K, const void* X,
                         int ldx, int M, int splits, void* out, int ldo, long slab, int out_bf16, int var,
                         void* stream) {
  using namespace la;
  if (M < 1 || N < 1 || (N & 3) || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7) || (ldo & 3)) return -1;
  if (!la_bs_fmt(fmt) || (fmt != FMT_BF16 && !gsc) || (fmt == FMT_Q6_K && !p1)) return -2;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  if ((long)M * ldx >= (1L << 31) || (long)M * ldo >= (1L << 31)) return -1;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)gsc, nullptr, N, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = out_bf16 ? nullptr : (float*)out;
  bf16* ob = out_bf16 ? (bf16*)out : nullptr;
  int rc;
  switch (fmt) {
    case FMT_Q4_K: rc = bs_launch<FMT_Q4_K>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    case FMT_Q6_K: rc = bs_launch<FMT_Q6_K>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    case FMT_Q8_0: rc = bs_launch<FMT_Q8_0>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
    default: rc = bs_launch<FMT_BF16>(var, w, x, ldx, M, splits, o, ob, ldo, slab, st); break;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Two weights (same K) side by side: columns [0, Na) from (fa, pa*), [Na, Na+Nb) from (fb, pb*).
extern "C" int la_bsgemm2(int fa, const void* pa0, const void* pa1, const void* ga, int Na, int fb, const void* pb0,
                          const void* pb1, const void* gb, int Nb, int K, const void* X, int ldx, int M, int splits,
                          void* out, int ldo, long slab, int out_bf16, int var, void* stream) {
  using namespace la;
  if (M < 1 || Na < 1 || Nb < 1 || (K & 255) || splits < 1 || ldo < Na + Nb || ldx < K || (ldx & 7) || (ldo & 3) ||
      (Na & 3) || (Nb & 3))
    return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  if ((long)M * ldx >= (1L << 31) || (long)M * ldo >= (1L << 31) || !ga || !gb) return -1;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  QW wa{(const uint8_t*)pa0, (const uint8_t*)pa1, (const uint8_t*)ga, nullptr, Na, K};
  QW wb{(const uint8_t*)pb0, (const uint8_t*)pb1, (const uint8_t*)gb, nullptr, Nb, K};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  float* o = out_bf16 ? nullptr : (float*)out;
  bf16* ob = out_bf16 ? (bf16*)out : nullptr;
  int rc;
  if (fa == FMT_Q4_K && fb == FMT_Q6_K) rc = bs_launch2<FMT_Q4_K, FMT_Q6_K>(var, wa, wb, x, ldx, M, splits, o, ob, ldo, slab, st);
  else if (fa == FMT_Q6_K && fb == FMT_Q4_K) rc = bs_launch2<FMT_Q6_K, FMT_Q4_K>(var, wa, wb, x, ldx, M, splits, o, ob, ldo, slab, st);
  else return -2;
  if (rc) return rc;
  return (int)hipGetLastError();
}

// h = act(x Wg^T) * (x Wu^T) -> bf16 [M][ldo]; gate rows oa .. oa+F of (pa*, ga), up rows ob ..
// ob+F of (pb*, gb), both of format fmt.  act: 0 SwiGLU, 3 GeGLU.
extern "C" int la_bsgemm_glu(int fmt, const void* pa0, const void* pa1, const void* ga, int oa, const void* pb0,
                             const void* pb1, const void* gb, int ob, int F, int K, const void* X, int ldx, int M,
                             void* out, int ldo, int act, int var, void* stream) {
  using namespace la;
  if (M < 1 || F < 1 || (F & 3) || (K & 255) || ldo < F || ldx < K || (ldx & 7) || (ldo & 3)) return -1;
  if (act != 0 && act != 3) return -1;
  if (!la_bs_fmt(fmt) || (fmt != FMT_BF16 && (!ga || !gb))) return -2;
  if ((long)M * ldx >= (1L << 31) || (long)M * ldo >= (1L << 31)) return -1;
  QW wg{(const uint8_t*)pa0, (const uint8_t*)pa1, (const uint8_t*)ga, nullptr, oa + F, K};
  BsGlu glu{QW{(const uint8_t*)pb0, (const uint8_t*)pb1, (const uint8_t*)gb, nullptr, ob + F, K}, oa, ob, F, act};
  hipStream_t st = (hipStream_t)stream;
  const bf16* x = (const bf16*)X;
  bf16* o = (bf16*)out;
  int rc;
  switch (fmt) {
    case FMT_Q4_K: rc = bs_launch_glu<FMT_Q4_K>(var, wg, glu, x, ldx, M, o, ldo, st); break;
    case FMT_Q6_K: rc = bs_launch_glu<FMT_Q6_K>(var, wg, glu, x, ldx, M, o, ldo, st); break;
    case FMT_Q8_0: rc = bs_launch_glu<FMT_Q8_0>(var, wg, glu, x, ldx, M, o, ldo, st); break;
    default: rc = bs_launch_glu<FMT_BF16>(var, wg, glu, x, ldx, M, o, ldo, st); break;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Grouped MoE GEMM (see bsmoe_kernel).  qws: device array of E QW descriptors {codes, aux,
// blocked scale plane, -, N, K} (MoEWeights.desc32); order / off: the pair grouping of
// la_moe_route (off[E] may be < P: pairs past it belong to no local expert); P = T * topk.
//   mode 1: X [T][ldx] tokens -> out bf16 [P][ldo]; N = F (each expert weight holds 2F rows);
//           splits must be 1; act 0 SwiGLU / 3 GeGLU
//   mode 2: X [P][ldx] grouped h rows -> out fp32 [splits * topk][T][ldo] (stride slab), rows
//           scaled by wts[pair]; rows of pairs of no local expert are left unwritten
extern "C" int la_bsmoe(int fmt, int mode, const void* qws, int N, int K, int E, const int* order, const int* off,
                        int topk, const void* X, int ldx, int T, int splits, const float* wts, void* out, int ldo,
                        long slab, int act, int var, void* stream) {
  using namespace la;
  if (T < 1 || N < 1 || (N & 3) || E < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7) || (ldo & 3) ||
      topk < 1 || !qws || !order || !off)
    return -1;
  if (mode == 1 && (splits != 1 || (act != 0 && act != 3))) return -1;
  if (mode == 2 && (!wts || slab < (long)T * ldo)) return -1;
  if (mode != 1 && mode != 2) return -1;
  if (fmt != FMT_Q4_K && fmt != FMT_Q6_K && fmt != FMT_Q8_0) return -2;
  const int P = T * topk;
  const int KS = K / 64, per = (KS + splits - 1) / splits;
  if (per * (splits - 1) >= KS) return -1;
  if ((long)P * ldx >= (1L << 31) || (long)P * ldo >= (1L << 31) || (long)(P / 32 + E) * (N / 32 + 1) * splits >= (1L << 31))
    return -1;
  hipStream_t st = (hipStream_t)stream;
  const QW* q = (const QW*)qws;
  const bf16* x = (const bf16*)X;
  float* o = mode == 2 ? (float*)out : nullptr;
  bf16* ob = mode == 1 ? (bf16*)out : nullptr;
  int rc;
#define BSMOE_F(F_)                                                                                                  \
  rc = mode == 1 ? bsmoe_launch<F_, 1>(var, q, N, K, E, order, off, topk, x, ldx, P, 1, wts, o, ob, ldo, slab, act, st) \
                 : bsmoe_launch<F_, 3>(var, q, N, K, E, order, off, topk, x, ldx, P, splits, wts, o, ob, ldo, slab, act, st);
  switch (fmt) {
    case FMT_Q4_K: BSMOE_F(FMT_Q4_K) break;
    case FMT_Q6_K: BSMOE_F(FMT_Q6_K) break;
    default: BSMOE_F(FMT_Q8_0) break;
  }
#undef BSMOE_F
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Probe (scripts/bs_bench.py --abl): Q4_K, variant 0, S = 1, bf16 out, ldx = K, ldo = N, with
// ablation bits 1 no MFMA, 2 no dequant, 4 no X loads, 8 no W loads, 16 no barrier, 32 no X image
// writes, 64 no B fragment reads, 128 no A fragment reads.
extern "C" int la_bsgemm_probe(int abl, const void* p0, const void* gsc, int N, int K, const void* X, int ldx, int M,
                               void* out, void* stream) {
  using namespace la;
  const int BN = (abl & 512) ? 256 : 128;
  QW w{(const uint8_t*)p0, nullptr, (const uint8_t*)gsc, nullptr, N, K};
  const int m_tiles = (M + 255) / 256, n_tiles = (N + BN - 1) / BN, real = m_tiles * n_tiles;
  hipStream_t st = (hipStream_t)stream;
#define BS_P(A)                                                                                          \
  case A:                                                                                                \
    hipLaunchKernelGGL((bsgemm_probe_kernel<A>), dim3(real), dim3(256), 0, st, w, (const bf16*)X, ldx, M, m_tiles, \
                       n_tiles, real, (bf16*)out);                                                       \
    break;
  switch (abl) {
    BS_P(0) BS_P(1) BS_P(2) BS_P(4) BS_P(8) BS_P(12) BS_P(16) BS_P(32) BS_P(64) BS_P(128) BS_P(192) BS_P(254)
    BS_P(6) BS_P(14) BS_P(46) BS_P(17) BS_P(256) BS_P(260) BS_P(264) BS_P(272) BS_P(1024)
    BS_P(1280) BS_P(2048) BS_P(2304) BS_P(8192) BS_P(8448) BS_P(8704) BS_P(512) BS_P(8196) BS_P(8200)
    BS_P(8208) BS_P(24576) BS_P(25088) BS_P(24580)
    default: return -1;
  }
#undef BS_P
  return (int)hipGetLastError();
}
