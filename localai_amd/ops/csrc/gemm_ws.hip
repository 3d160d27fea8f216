// Warp-specialised Q4_K GEMM for batched decode (M <= 256 rows: the whole decode batch in one
// tile):  out[s][m][n] = sum_{k in split s} X[m,k] * W[n,k]   (fp32 split-K slabs)
//
// Same contract and numerics as qgemm_mid ([external] mmq), different
// schedule.  The ablation of qgemm_mid at M = 256 (profiles/decode_gemv_study.md §3): with
// one 512-thread workgroup per CU its time is not the MFMAs (removing them changed ~10 %);
// it is the weight stream's HBM latency -- vmcnt retires in issue order, so the L2-resident X
// chunks and the HBM weights share one prefetch distance -- plus register-staged LDS traffic,
// all serialised behind the same waves' MFMAs by one barrier per K-step.
//
// Here every byte moves by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no ds_write
// issue) and each wave has one job (896 threads = 14 waves):
//   waves 0-7   consumers: ds_read_b128 + v_mfma_f32_16x16x32_bf16 only; 4 (M) x 2 (N) waves,
//               64x64 output tile each, workgroup tile 256 x 128 x 64;
//   waves 8-9   X loaders: the 256 x 64 bf16 activation tile of K-step t+1 (32 KiB, 16 DMAs
//               per wave) into a 2-slot X ring, XOR-swizzled 16-B chunks (chunk ^ (row & 7):
//               rows of exactly 128 B, conflict-free ds_read_b128 fragments);
//   waves 10-13 W loaders + dequantisers: raw Q4_K bytes of K-step t+D (qs + scale header,
//               2 DMAs per wave) into a D-deep raw ring on their OWN vmcnt (never throttled
//               by X); the raw bytes of K-step t+1 are expanded to bf16 in registers and
//               written to a 2-slot W tile ring.
// One s_barrier per K-step separates "consumers read slot t" from "loaders fill slot t+1".
// The W loaders keep their DMAs in flight across barriers (raw s_barrier, lgkmcnt only: a
// __syncthreads would drain them -- cdna_hip_programming.md "Pipelining across barriers").
// All LDS is one __shared__ array (a second object makes hipcc wait vmcnt(0) before reads).
#include "qraw.h"

namespace la {

constexpr int WS_BM = 256, WS_BN = 128, WS_BK = 64;
constexpr int WS_CW = 8, WS_XW = 2, WS_WW = 4;        // consumer / X-loader / W-loader waves
constexpr int WS_T = 64 * (WS_CW + WS_XW + WS_WW);
constexpr int WS_D = 5;                               // raw-W ring depth (K-steps in flight)
constexpr int WS_WLDS = WS_BK + 16;                   // bf16 per W-tile row (160 B: conflict-free)
constexpr int WS_XBYTES = WS_BM * WS_BK * 2;          // one X slot: 32 KiB
constexpr int WS_WBYTES = WS_BN * WS_WLDS * 2;        // one bf16 W slot: 20 KiB
constexpr int WS_RAWW = 2048;                         // raw bytes per W wave per K-step (qs 1 KiB + hdr 1 KiB)
constexpr int WS_RBYTES = WS_RAWW * WS_WW;            // one raw slot: 8 KiB
constexpr int WS_LDS_BYTES = 2 * WS_XBYTES + 2 * WS_WBYTES + WS_D * WS_RBYTES;  // 144 KiB
constexpr int WS_UNROLL = 2 * WS_D;                   // loop unroll: ring slot indices compile-time

LA_DEV void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

__global__ __launch_bounds__(WS_T) void qgemm_ws_q4k_kernel(QW w, const bf16* __restrict__ X, int ldx, int M,
                                                           int nks, float* __restrict__ out, int ldo, long slab) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[WS_LDS_BYTES];
  uint8_t* const xslot = lds;                                   // 2 x 32 KiB
  uint8_t* const wslot = lds + 2 * WS_XBYTES;                   // 2 x 20 KiB
  uint8_t* const rslot = lds + 2 * WS_XBYTES + 2 * WS_WBYTES;   // D x 8 KiB
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int N = w.N;
  const int n0 = blockIdx.x * WS_BN, m0 = blockIdx.z * WS_BM;
  const int ks0 = blockIdx.y * nks;  // host: equal splits
  const int last = ks0 + nks - 1;

  if (wave < WS_CW) {
    // ------------------------------------------------------------------ consumers
    const int wm = wave >> 1, wn = wave & 1;
    const int r = lane & 15, g = lane >> 4;
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int xsw = r & 7;  // rows of this wave's A fragments: wm*64 + 16i + r  ==> row & 7 == r & 7
    __syncthreads();        // prologue: slot 0 filled
    for (int t = 0; t < nks; ++t) {
      const uint8_t* xs = xslot + (t & 1) * WS_XBYTES;
      const bf16* ws = (const bf16*)(wslot + (t & 1) * WS_WBYTES);
#pragma unroll
      for (int kk = 0; kk < WS_BK; kk += 32) {
        bf16x8 a[4], b[4];
        const int p = ((kk >> 3) + g) ^ xsw;  // physical 16-B chunk of logical chunk kk/8 + g
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = *(const bf16x8*)(xs + (wm * 64 + i * 16 + r) * 128 + p * 16);
          b[i] = *(const bf16x8*)(ws + (wn * 64 + i * 16 + r) * WS_WLDS + kk + 8 * g);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
      }
      __syncthreads();
    }
    float* o = out + (size_t)blockIdx.y * slab;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = n0 + wn * 64 + nt * 16 + r;
      if (n >= N) continue;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * 64 + mt * 16 + 4 * g + i;
          if (m < M) o[(size_t)m * ldo + n] = acc[mt][nt][i];
        }
      }
    }
  } else if (wave < WS_CW + WS_XW) {
    // ------------------------------------------------------------------ X loaders
    // DMA j of this wave covers tile rows 8j'..8j'+7 (j' = 16 xw + j): lane l -> row
    // 8j' + l/8, physical chunk l%8, which holds logical chunk (l%8) ^ (row & 7).
    const int xw = wave - WS_CW;
    const int lrow = lane >> 3, lp = lane & 7;
    uint32_t goff[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = 8 * (16 * xw + j) + lrow;
      goff[j] = (uint32_t)min(m0 + row, M - 1) * ldx + 8 * (lp ^ (row & 7));  // rows >= M: never stored
    }
    auto fill = [&](int ks, int slot) {
      const bf16* xk = X + (size_t)ks * WS_BK;
      uint8_t* dst = xslot + slot * WS_XBYTES + (16 * xw) * 1024;
#pragma unroll
      for (int j = 0; j < 16; ++j) glds16(xk + goff[j], dst + j * 1024);
    };
    fill(ks0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nks; ++t) {
      fill(min(ks0 + t + 1, last), (t + 1) & 1);  // the slot consumers read at step t-1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();                            // publishes slot t+1
    }
  } else {
    // ------------------------------------------------------------------ W loaders / dequant
    // wave ww owns tile columns 32ww .. 32ww+31.  Its part of a raw slot: [32 cols][32 B] qs,
    // then [32 cols][16 B] scale header (lanes 32-63 write a duplicate copy).
    const int ww = wave - WS_CW - WS_XW;
    const int ncol = min(n0 + 32 * ww + (lane >> 1), N - 1);  // clamped rows: garbage, never stored
    const int hcol = min(n0 + 32 * ww + (lane & 31), N - 1);
    const uint32_t qs_off = (uint32_t)ncol * (w.K >> 1) + 16 * (lane & 1);
    const uint32_t hd_off = (uint32_t)hcol * (w.K >> 8) * 16;
    auto issue = [&](int ks, int slot) {
      uint8_t* dst = rslot + slot * WS_RBYTES + ww * WS_RAWW;
      glds16(w.p0 + 32 * ks + qs_off, dst);
      glds16(w.p1 + 16 * (ks >> 2) + hd_off, dst + 1024);
    };
    // lane expands units u = lane + 64v (v = 0, 1): column c = u >> 2 (0..31), q = u & 3 ->
    // the 16 weights k = 16q .. 16q+15 of the K-step
    auto expand = [&](int ks, int rs, int buf) {
      const uint8_t* src = rslot + rs * WS_RBYTES + ww * WS_RAWW;
      bf16* dst = (bf16*)(wslot + buf * WS_WBYTES);
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int u = lane + 64 * v, c = u >> 2, q = u & 3;
        MidRaw<FMT_Q4_K> raw;
        raw.qs = *(const u32x4*)(src + c * 32 + 16 * (q & 1));
        raw.hdr = *(const u32x4*)(src + 1024 + c * 16);
        typename MidRaw<FMT_Q4_K>::Addr ad;
        ad.half = q >> 1;
        bf16x8 d[2];
        raw.deq(ad, ks, d);
        bf16* o = dst + (32 * ww + c) * WS_WLDS + 16 * q;
        *(bf16x8*)o = d[0];
        *(bf16x8*)(o + 8) = d[1];
      }
    };
    // prologue: raw K-steps 0 .. D-1 in flight; K-step 0 expanded into W slot 0
#pragma unroll
    for (int i = 0; i < WS_D; ++i) issue(min(ks0 + i, last), i);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (WS_D - 1)) : "memory");
    expand(ks0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // step t: raw slot t % D (K-step t, expanded at step t-1) refills with K-step t + D; then
    // K-step t+1 (raw slot (t+1) % D) is expanded into W slot (t+1)&1 once its DMAs landed
    for (int t0 = 0; t0 < nks; t0 += WS_UNROLL) {
#pragma unroll
      for (int i = 0; i < WS_UNROLL; ++i) {
        const int t = t0 + i;
        if (t < nks) {
          issue(min(ks0 + t + WS_D, last), i % WS_D);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (WS_D - 1)) : "memory");  // K-step t+1 landed
          expand(min(ks0 + t + 1, last), (i + 1) % WS_D, (t + 1) & 1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS
  }
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
// Q4_K only; splits must divide K/64 into equal parts.
extern "C" int la_qgemm_ws(int fmt, const void* p0, const void* p1, const void* p2, const void* p3, int N, int K,
                           const void* X, int ldx, int M, int splits, void* out, int ldo, long slab, void* stream) {
  using namespace la;
  if (fmt != FMT_Q4_K) return -2;
  if (M < 1 || (K & 255) || splits < 1 || ldo < N || ldx < K || (ldx & 7) || slab < (long)M * ldo) return -1;
  if ((long)N * K >= (1L << 31) || (long)M * ldx >= (1L << 31)) return -1;  // 32-bit staging offsets
  const int total = K / WS_BK, per = total / splits;
  if (per * splits != total) return -1;
  QW w{(const uint8_t*)p0, (const uint8_t*)p1, (const uint8_t*)p2, (const uint8_t*)p3, N, K};
  dim3 grid((N + WS_BN - 1) / WS_BN, splits, (M + WS_BM - 1) / WS_BM);
  hipLaunchKernelGGL(qgemm_ws_q4k_kernel, grid, dim3(WS_T), 0, (hipStream_t)stream, w, (const bf16*)X, ldx, M, per,
                     (float*)out, ldo, slab);
  return (int)hipGetLastError();
}
