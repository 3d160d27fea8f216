// Batched-decode quantised GEMM, dequantising in registers (M <= a few hundred rows):
//   out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]     (fp32 split-K slabs, or bf16 [M][N] at S = 1)
//
// SURVEY §2.8 K5/K6 (ggml mmq / dequant + hipBLAS, [external]).  Third design after qgemm_mid
// (register-staged X + LDS-dequantised W, 256 x 128 tile) and qgemm_ws (warp-specialised LDS-DMA);
// profiles/decode_gemv_study.md measured both limited by the activation (X) stream and the LDS
// bytes of the dequantised W tile.  Here:
//   * tile 128 (M) x 256 (N), 8 waves = 4 column groups x 2 K-halves: wave (g, h) owns columns
//     64g..64g+63 and the k16 chunks 2h, 2h+1 of every 64-deep K-step, so it computes a 128 x 64
//     tile (8 accumulators of v_mfma_f32_32x32x16_bf16) reading only half of each X slot; the two
//     K-halves are summed through LDS once, after the loop.  X bytes per FLOP are half those of a
//     256 x 128 tile; at M = 256 the two M tiles of one N tile are placed on one XCD and share the
//     weight bytes through its L2;
//   * W never exists as bf16 in LDS: its raw 4-bit codes (a fragment-ordered copy built once at
//     load, 1 KiB per 32 columns x 64 k) and per-K-step scale records arrive by LDS-DMA and each
//     wave expands its own B fragments in registers (v_cvt_f32_ubyteN + v_fma_f32 +
//     v_cvt_pk_bf16_f32), each feeding 4 MFMAs;
//   * X also arrives by LDS-DMA, in MFMA fragment order (1 KiB per 32-row x 16-k fragment,
//     lane-linear, conflict-free ds_read_b128);
//   * one uniform software pipeline over a 6-slot LDS ring: step t issues the DMAs of step t + 4,
//     waits with a counted vmcnt for its own DMAs of step t, one s_barrier, then computes.  Two
//     waves per SIMD, so one wave's DMA issue, LDS reads and dequant VALU overlap the other's MFMAs.
// Weight numerics: w = (d * sc_j) * q - (dmin * m_j) in fp32 per 32-sub-block, rounded once to
// bf16: the same bf16 weight values as the dequantised hipBLASLt copy it replaces.
#include "qweight.h"

namespace la {

constexpr int DQ_D = 4;     // K-steps in flight
constexpr int DQ_NS = 6;    // LDS ring slots (>= D + 2: a slow wave may still read step t-1's slot)
constexpr int DQ_BM = 128;  // rows per tile
constexpr int DQ_BN = 256;  // columns per tile
// LDS slot: [X: 16 fragments x 1 KiB][W codes: 8 blocks of 32 cols x 1 KiB][W scales: 2 x 1 KiB]
constexpr int DQ_SX = 0, DQ_SQ = 16384, DQ_SS = DQ_SQ + 8 * 1024, DQ_SLOT = DQ_SS + 2 * 1024;

LA_DEV void dq_glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// 8 weights of one lane's B fragment: dword x holds e = b (low nibble) and e = b + 4 (high
// nibble) in byte b; D, Mn = scale and negated min of their 32-sub-block.
LA_DEV bf16x8 dq_expand_q4(uint32_t x, float D, float Mn) {
  // lo / hi are formed opaquely so each weight stays ONE v_cvt_f32_ubyteN (the combiner would
  // otherwise fold the masks into a per-weight shift + and)
  uint32_t lo, hi;
  asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(lo) : "v"(x));
  asm("v_and_b32 %0, 0x0f0f0f0f, %1" : "=v"(hi) : "v"(x >> 4));
  bf16x8 r;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    r[b] = (bf16)fmaf(D, (float)((lo >> (8 * b)) & 0xFFu), Mn);
    r[b + 4] = (bf16)fmaf(D, (float)((hi >> (8 * b)) & 0xFFu), Mn);
  }
  return r;
}

// qsw: [NB][K/64][64 lanes][16 B]  (NB = 8 * ceil(N/256) blocks of 32 columns): lane l = 32h + c ->
//      column 32nb + c; dword kc holds the 8 codes of k = 64t + 16kc + 8h + e (e = 0..7)
// ssw: [NB/4][K/64][4 blocks][32 cols][8 B] = f16 d, f16 dmin, u8 sc, u8 m of sub-block 2(t%4),
//      u8 sc, u8 m of sub-block 2(t%4)+1
// ABL (probe builds only, scripts/dq_probe.py): bit0 drops the MFMAs, bit1 the dequant VALU,
// bit2 the X DMAs, bit3 the W DMAs, bit4 the barrier -- results are garbage, timings the point.
template <int ABL = 0>
__global__ __launch_bounds__(512, 2) void qgemm_dq_q4k_kernel(
    const uint8_t* __restrict__ qsw, const uint8_t* __restrict__ ssw, int N, int K, const bf16* __restrict__ X,
    int ldx, int M, int nks, int n_tiles, int m_tiles, int n_real, float* __restrict__ out, bf16* __restrict__ outb,
    int ldo, long slab) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[DQ_NS * DQ_SLOT];
  // XCD-aware tile order: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of
  // tiles, M fastest, so the M tiles of one N tile (same weight bytes) sit on one L2.
  const int pid = blockIdx.x;
  const int tile = (pid & 7) * (gridDim.x >> 3) + (pid >> 3);
  if (tile >= n_real) return;  // padding blocks (grid rounded up to a multiple of 8)
  const int mt = tile % m_tiles;
  const int rest = tile / m_tiles;
  const int ntile = rest % n_tiles;
  const int split = rest / n_tiles;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cg = wave & 3, kh = wave >> 2;  // column group (64 cols), K-half (k16 chunks 2kh, 2kh+1)
  const int m0 = mt * DQ_BM;
  const int ks0 = split * nks;
  const int KS = K >> 6;
  const int nbt = ntile * 8;  // first 32-column block of the tile

  // DMA duties per K-step: X fragments f = 2*wave, 2*wave+1 (kc = f/4, mb = f%4); W codes of
  // block `wave`; waves 0, 1 also the scale records of block group `wave`.
  uint32_t xoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int f = 2 * wave + i, kc = f >> 2, mb = f & 3;
    xoff[i] = (uint32_t)min(m0 + 32 * mb + (lane & 31), M - 1) * ldx + 16 * kc + 8 * (lane >> 5);
  }
  const uint8_t* qsrc = qsw + ((size_t)(nbt + wave) * KS) * 1024 + lane * 16;
  const uint8_t* ssrc = ssw + ((size_t)((nbt >> 2) + (wave & 1)) * KS) * 1024 + lane * 16;
  auto issue = [&](int t) {  // K-step t (relative to the split) -> ring slot t % NS
    const int ks = ks0 + min(t, nks - 1);  // clamped tail: DMAs still issued (uniform vmcnt)
    uint8_t* sl = lds + (t % DQ_NS) * DQ_SLOT;
    if constexpr (!(ABL & 4)) {
      const bf16* xk = X + (size_t)ks * 64;
      dq_glds16(xk + xoff[0], sl + DQ_SX + (2 * wave) * 1024);
      dq_glds16(xk + xoff[1], sl + DQ_SX + (2 * wave + 1) * 1024);
    }
    if constexpr (!(ABL & 8)) {
      dq_glds16(qsrc + (size_t)ks * 1024, sl + DQ_SQ + wave * 1024);
      if (wave < 2) dq_glds16(ssrc + (size_t)ks * 1024, sl + DQ_SS + wave * 1024);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  auto compute = [&](int t) {
    const uint8_t* sl = lds + (t % DQ_NS) * DQ_SLOT;
    uint32_t q[2][2];
    float D[2], Mn[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nbl = 2 * cg + j;  // block inside the tile
      const u32x2 qq = *(const u32x2*)(sl + DQ_SQ + nbl * 1024 + lane * 16 + 8 * kh);
      q[j][0] = qq.x;
      q[j][1] = qq.y;
      const u32x2 sc = *(const u32x2*)(sl + DQ_SS + (nbl >> 2) * 1024 + (nbl & 3) * 256 + (lane & 31) * 8);
      const uint32_t smb = kh ? (sc.y >> 16) : (sc.y & 0xFFFFu);  // (sc, m) of sub-block kh
      D[j] = h2f(sc.x & 0xFFFFu) * (float)(smb & 0xFFu);
      Mn[j] = -h2f(sc.x >> 16) * (float)(smb >> 8);
    }
    const uint8_t* xs = sl + DQ_SX + lane * 16;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kc = 2 * kh + c;
      bf16x8 a[4], b[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a[mb] = *(const bf16x8*)(xs + (kc * 4 + mb) * 1024);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (ABL & 2) b[j] = __builtin_bit_cast(bf16x8, u32x4{q[j][c], q[j][c] ^ (uint32_t)D[j], 0u, 0u});
        else b[j] = dq_expand_q4(q[j][c], D[j], Mn[j]);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (ABL & 1) acc[mb][j][c] += (float)a[mb][j] * (float)b[j][mb];
          else acc[mb][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mb], b[j], acc[mb][j], 0, 0, 0);
        }
    }
  };

  // prologue: steps 0 .. D-1 in flight
  for (int i = 0; i < DQ_D; ++i) issue(i);
  constexpr int kX = (ABL & 4) ? 0 : 2, kW = (ABL & 8) ? 0 : 1;
  for (int t = 0; t < nks; ++t) {
    issue(t + DQ_D);
    // this wave's DMAs of step t are the oldest D groups back (waves 0, 1 issue one more each step)
    if (!(ABL & 8) && wave < 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQ_D * (kX + kW + 1)) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQ_D * (kX + kW)) : "memory");
    if constexpr (!(ABL & 16)) __builtin_amdgcn_s_barrier();  // every wave's DMAs of step t landed
    asm volatile("" ::: "memory");
    compute(t);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS
  __syncthreads();                                  // ring reads done: LDS reused for the K-half sum

  // K-half reduction: waves kh = 1 park their 128 x 64 partial in LDS, waves kh = 0 add and store.
  // Layout [cg][mb][j][i/4][lane][4 f32]: every access a lane-linear ds_*_b128.
  float* red = (float*)lds;
  if (kh == 1) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4)
          *(f32x4*)(red + ((((cg * 4 + mb) * 2 + j) * 4 + i4) * 64 + lane) * 4) =
              f32x4{acc[mb][j][4 * i4], acc[mb][j][4 * i4 + 1], acc[mb][j][4 * i4 + 2], acc[mb][j][4 * i4 + 3]};
  }
  __syncthreads();
  if (kh == 1) return;
  // acc[mb][j] reg i -> row 32mb + (i&3) + 8(i>>2) + 4(lane>>5), col 32(nbt + 2cg + j) + (lane&31)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = (nbt + 2 * cg + j) * 32 + (lane & 31);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const f32x4 o = *(const f32x4*)(red + ((((cg * 4 + mb) * 2 + j) * 4 + i4) * 64 + lane) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * i4 + r;
          const int m = m0 + 32 * mb + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          const float v = acc[mb][j][i] + o[r];
          if (m < M && n < N) {
            if (outb) outb[(size_t)m * ldo + n] = (bf16)v;
            else out[(size_t)split * slab + (size_t)m * ldo + n] = v;
          }
        }
      }
    }
  }
}

// Fragment-ordered copy of Q4_K planes (qs in ggml order [N][K/2], scm [N][K/256][16] =
// (sc0,m0,...,sc7,m7), dd [N][K/256][2] f16 (d, dmin)) -> qsw / ssw above, columns padded to a
// multiple of 256 (padding repeats row N-1).  One thread per (32-col block, K-step, lane).
__global__ void dq_swizzle_q4k_kernel(const uint8_t* __restrict__ qs, const uint8_t* __restrict__ scm,
                                      const uint16_t* __restrict__ dd, int N, int K, int NB, uint8_t* __restrict__ qsw,
                                      uint8_t* __restrict__ ssw) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int KS = K >> 6;
  const long total = (long)NB * KS * 64;
  if (gid >= total) return;
  const int lane = (int)(gid & 63);
  const long r = gid >> 6;
  const int t = (int)(r % KS);
  const int nb = (int)(r / KS);
  const int h = lane >> 5, c = lane & 31;
  const int n = min(nb * 32 + c, N - 1);
  const int sb = t >> 2, tq = t & 3;  // super-block, K-step inside it (64 k = chunk tq of ggml's 4)
  const uint8_t* q = qs + (size_t)n * (K >> 1) + sb * 128 + 32 * tq;  // ggml: byte l -> k 64tq + l (lo), +32 (hi)
  uint32_t words[4];
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    uint32_t wv = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      // e = b and e = b + 4 of k_local = 16kc + 8h + e (0..63 inside the K-step)
      const int k0 = 16 * kc + 8 * h + b, k1 = k0 + 4;
      const uint32_t v0 = (k0 < 32) ? (q[k0] & 0xFu) : (q[k0 - 32] >> 4);
      const uint32_t v1 = (k1 < 32) ? (q[k1] & 0xFu) : (q[k1 - 32] >> 4);
      wv |= (v0 | (v1 << 4)) << (8 * b);
    }
    words[kc] = wv;
  }
  *(u32x4*)(qsw + (size_t)gid * 16) = u32x4{words[0], words[1], words[2], words[3]};
  if (h == 0) {
    const uint8_t* s = scm + ((size_t)n * (K >> 8) + sb) * 16;
    const uint32_t dpair = *(const uint32_t*)(dd + ((size_t)n * (K >> 8) + sb) * 2);
    const int j0 = 2 * tq, j1 = 2 * tq + 1;
    const uint32_t scm4 = (uint32_t)s[2 * j0] | ((uint32_t)s[2 * j0 + 1] << 8) | ((uint32_t)s[2 * j1] << 16) |
                          ((uint32_t)s[2 * j1 + 1] << 24);
    *(u32x2*)(ssw + (((size_t)(nb >> 2) * KS + t) * 4 + (nb & 3)) * 256 + c * 8) = u32x2{dpair, scm4};
  }
}

template <int ABL>
static void dq_launch(const uint8_t* q, const uint8_t* sc, int N, int K, const bf16* x, int ldx, int M, int splits,
                      float* o, bf16* ob, int ldo, long slab, hipStream_t st) {
  const int per = K / 64 / splits;
  const int n_tiles = (N + DQ_BN - 1) / DQ_BN, m_tiles = (M + DQ_BM - 1) / DQ_BM;
  const int real = n_tiles * m_tiles * splits;
  const int grid = (real + 7) / 8 * 8;
  hipLaunchKernelGGL((qgemm_dq_q4k_kernel<ABL>), dim3(grid), dim3(512), 0, st, q, sc, N, K, x, ldx, M, per, n_tiles,
                     m_tiles, real, o, ob, ldo, slab);
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// qsw / ssw sizes: la_dq_plane_bytes(N, K, which) (which 0: codes, 1: scales).
extern "C" long la_dq_plane_bytes(int N, int K, int which) {
  const long nb = (long)(N + la::DQ_BN - 1) / la::DQ_BN * 8;
  return which == 0 ? nb * (K / 64) * 1024 : nb / 4 * (K / 64) * 1024;
}

extern "C" int la_dq_swizzle(int fmt, const void* p0, const void* p2, const void* p3, int N, int K, void* qsw,
                             void* ssw, void* stream) {
  using namespace la;
  if (fmt != FMT_Q4_K || N < 1 || (K & 255)) return -1;
  const int NB = (N + DQ_BN - 1) / DQ_BN * 8;
  const long total = (long)NB * (K >> 6) * 64;
  hipLaunchKernelGGL(dq_swizzle_q4k_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)p0, (const uint8_t*)p2, (const uint16_t*)p3, N, K, NB, (uint8_t*)qsw,
                     (uint8_t*)ssw);
  return (int)hipGetLastError();
}

// out: fp32 slabs [splits][M][ldo] (slab stride `slab`), or bf16 [M][ldo] when out_bf16 (splits == 1).
// wnt: kept for the ABI (one tile shape: 128 x 256).
extern "C" int la_qgemm_dq(int fmt, const void* qsw, const void* ssw, int N, int K, const void* X, int ldx, int M,
                           int splits, void* out, int ldo, long slab, int out_bf16, int wnt, void* stream) {
  using namespace la;
  (void)wnt;
  if (fmt != FMT_Q4_K) return -2;
  if (M < 1 || N < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7)) return -1;
  if (out_bf16 && splits != 1) return -1;
  if (!out_bf16 && slab < (long)M * ldo) return -1;
  if ((long)M * ldx >= (1L << 31)) return -1;  // 32-bit X offsets
  if ((K / 64) % splits) return -1;
  dq_launch<0>((const uint8_t*)qsw, (const uint8_t*)ssw, N, K, (const bf16*)X, ldx, M, splits,
               out_bf16 ? nullptr : (float*)out, out_bf16 ? (bf16*)out : nullptr, ldo, slab, (hipStream_t)stream);
  return (int)hipGetLastError();
}

// probe entry (scripts/dq_probe.py): ablation bits, fp32 slabs, ldx = K, ldo = N
extern "C" int la_qgemm_dq_probe(const void* qsw, const void* ssw, int N, int K, const void* X, int M, int splits,
                                 void* out, int abl, void* stream) {
  using namespace la;
  const uint8_t* q = (const uint8_t*)qsw;
  const uint8_t* sc = (const uint8_t*)ssw;
  const bf16* x = (const bf16*)X;
  float* o = (float*)out;
  const long slab = (long)M * N;
  hipStream_t st = (hipStream_t)stream;
#define DQ_PROBE(A) \
  case A: dq_launch<A>(q, sc, N, K, x, K, M, splits, o, nullptr, N, slab, st); break;
  switch (abl) {
    DQ_PROBE(0) DQ_PROBE(1) DQ_PROBE(2) DQ_PROBE(3) DQ_PROBE(4) DQ_PROBE(8) DQ_PROBE(12) DQ_PROBE(13) DQ_PROBE(14)
    DQ_PROBE(15) DQ_PROBE(16) DQ_PROBE(31)
    default: return -1;
  }
#undef DQ_PROBE
  return (int)hipGetLastError();
}
