// One-shot all-reduce over peer-mapped IPC buffers, for the latency-bound tensor-parallel decode
// messages (SURVEY §2.9 "Planned TP collective shapes", §2.11: "custom one-shot / two-shot
// all-reduce kernels over peer-mapped IPC buffers for latency-critical decode messages").
//
// On an 8-GPU MI355X node every GPU has a direct xGMI link to each of its 7 peers, so a
// one-shot read-reduce (every rank reads every peer's chunk directly) uses all links at once,
// where a ring would move each byte over one link per step; a 16 KiB decode row is two orders of
// magnitude below the size where bandwidth matters, so the cost is one flag round trip.
//
// Buffers: every rank owns one hipMalloc'd region, exported with hipIpcGetMemHandle and opened by
// the other ranks (parallel/custom_ar.py):
//   [flags  : AR_MAXB blocks x AR_MAXR ranks int32]   epochs written by the PEERS
//   [counter: AR_MAXB int32]                          this rank's per-block call count
//   [err    : int32]                                  set when a wait timed out
//   [data   : 2 slots x AR_MAXB x 4 KiB]              this rank's input, by epoch parity
// Block b always owns elements [1024 b, 1024 b + 1024) and the 4 KiB at 4096 b of a slot, whatever
// the message size or element type, so every block is an independent channel (its own flag row,
// counter and data bytes) and calls of different sizes can follow each other freely.
// Protocol, per block b (one chunk of the message), call epoch e (= ++counter[b]), slot e & 1:
//   1. copy the chunk of the local input into the own data slot;
//   2. release (system scope), then store e into flag[b][rank] of every PEER buffer;
//   3. wait until flag[b][q] >= e for every peer q in the own buffer (bounded spin: a dead peer
//      sets err and the block proceeds instead of hanging the GPU), then acquire (system scope);
//   4. out[chunk] = sum over ranks 0..R-1 in rank order (fp32), so every rank gets the same bits.
// Two data slots suffice without a closing barrier: a peer signals call n+1 only after its call n
// kernel (all of its reads of slot n & 1) has completed, and this rank rewrites that slot at call
// n+2, after it has seen those signals.  Each block touches only its own chunk, flag row and
// counter, so there is no grid-wide synchronisation and the kernel replays inside a hipGraph.
#include "common.h"

namespace la {

constexpr int AR_MAXB = 256;  // blocks (chunks) per call
constexpr int AR_MAXR = 8;    // ranks
constexpr int AR_T = 256;
constexpr long AR_FLAGS = 0, AR_COUNTER = AR_MAXB * AR_MAXR * 4, AR_ERR = AR_COUNTER + AR_MAXB * 4;
constexpr long AR_DATA = 16384;  // data area offset (header rounded up)
constexpr long AR_CHUNK = 1024;  // elements per block
constexpr long AR_SLOT = AR_MAXB * AR_CHUNK * 4;  // bytes per parity slot (1 MiB)

struct ARArgs {
  const void* in;
  void* out;
  long n;          // elements
  int bf16;        // element type: 1 bf16, 0 fp32
  int rank, world;
  uint8_t* bufs[AR_MAXR];
  long spin_limit;
};

LA_DEV int ar_load_flag(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

__global__ __launch_bounds__(AR_T) void allreduce_oneshot_kernel(ARArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const long e0 = (long)b * AR_CHUNK;
  const long e1 = min(a.n, e0 + AR_CHUNK);
  uint8_t* own = a.bufs[a.rank];
  int* counter = (int*)(own + AR_COUNTER) + b;
  const int ep = *counter + 1;
  const long slot = AR_DATA + (long)(ep & 1) * AR_SLOT + (long)b * AR_CHUNK * 4;  // this block's 4 KiB
  const int esz = a.bf16 ? 2 : 4;

  // 1. local chunk -> own data slot (16-byte vectors; e0 and e1 - e0 are multiples of 8 elements
  //    except possibly the message tail, handled element-wise)
  {
    const uint8_t* src = (const uint8_t*)a.in + e0 * esz;
    uint8_t* dst = own + slot;
    const long bytes = (e1 - e0) * esz, v16 = bytes >> 4;
    for (long i = tid; i < v16; i += AR_T) ((u32x4*)dst)[i] = ((const u32x4*)src)[i];
    for (long i = (v16 << 4) + tid; i < bytes; i += AR_T) dst[i] = src[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's stores have left it
  __syncthreads();
  // 2. publish: the chunk reaches memory before the flag (system-scope release by the signalling lanes)
  if (tid < a.world && tid != a.rank) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* peer_flag = (int*)(a.bufs[tid] + AR_FLAGS) + b * AR_MAXR + a.rank;
    __hip_atomic_store(peer_flag, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every peer's chunk b of this epoch (bounded)
  if (tid < a.world && tid != a.rank) {
    const int* f = (const int*)(own + AR_FLAGS) + b * AR_MAXR + tid;
    long spins = 0;
    while (ar_load_flag(f) < ep) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > a.spin_limit) {
        // every rank's error word: the group drops the custom path together whichever rank timed out
        for (int r = 0; r < a.world; ++r)
          __hip_atomic_store((int*)(a.bufs[r] + AR_ERR), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' data, not stale lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 4. reduce in rank order (identical bits on every rank)
  for (long i = e0 + tid * 8; i < e1; i += AR_T * 8) {
    const int cnt = (int)min(8L, e1 - i);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      const uint8_t* src = a.bufs[r] + slot + (i - e0) * esz;
      if (a.bf16) {
        if (cnt == 8) {
          const bf16x8 v = *(const bf16x8*)src;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
        } else {
          for (int j = 0; j < cnt; ++j) acc[j] += (float)((const bf16*)src)[j];
        }
      } else {
        if (cnt == 8) {
          const f32x4 v0 = *(const f32x4*)src, v1 = *(const f32x4*)(src + 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] += v0[j];
            acc[j + 4] += v1[j];
          }
        } else {
          for (int j = 0; j < cnt; ++j) acc[j] += ((const float*)src)[j];
        }
      }
    }
    if (a.bf16) {
      bf16* o = (bf16*)a.out + i;
      for (int j = 0; j < cnt; ++j) o[j] = (bf16)acc[j];
    } else {
      float* o = (float*)a.out + i;
      for (int j = 0; j < cnt; ++j) o[j] = acc[j];
    }
  }
  if (tid == 0) *counter = ep;
}

// ----------------------------------------------------------------------------- fused AR + add + norm
// The decode layer boundary of a tensor-parallel group in ONE launch: split-K slab sum of the local
// row-parallel partial (bf16 into the one-shot data slot), the one-shot exchange, the rank-ordered
// sum, + bias, + residual (fp32, updated in place), and RMSNorm / LayerNorm into the next layer's
// bf16 input -- where the unfused path runs reduce -> all-reduce -> add_norm (three launches,
// SURVEY §2.11).  One workgroup per row; row t owns the channels [t*nch, (t+1)*nch) (nch = D/1024
// rounded up) of the one-shot region, element e of the row in channel e/1024 at its own parity
// slot, so rows are independent channels and calls interleave freely with one-shot calls.
constexpr int ARN_IT = 4;  // 8-element groups per thread: D <= 256 x 8 x 4 = 8192

struct ARNArgs {
  const void* p;        // local partial: S fp32 slabs [S][M][D] (S >= 1) or one bf16 matrix (S == 0)
  long slab;
  int S;
  int D, rank, world;
  uint8_t* bufs[AR_MAXR];
  long spin_limit;
  float* residual;      // [M][D] fp32, += sum (+ bias)
  const float* bias;    // [D] or null: added once, after the sum
  const float* w;       // norm weight [D]
  const float* nb;      // LayerNorm bias [D] or null
  bf16* out;            // [M][D]
  float eps;
  int mode;             // 0 RMSNorm, 1 LayerNorm
};

__global__ __launch_bounds__(AR_T) void allreduce_add_norm_kernel(ARNArgs a) {
  __shared__ float red[AR_T / 64];
  const int t = blockIdx.x, tid = threadIdx.x, D = a.D;
  const int nch = (D + (int)AR_CHUNK - 1) / (int)AR_CHUNK, b0 = t * nch;
  uint8_t* own = a.bufs[a.rank];
  const int* counters = (const int*)(own + AR_COUNTER);
  // this thread's element groups: e = 8 (tid + AR_T k)
  float v[ARN_IT][8];
  long off[ARN_IT];  // byte offset of the group inside a slot region (channel base + within)
  int par[ARN_IT];
  // 1. local row (slab sum in fp32, rounded to bf16 as the wire format) -> own data slots
#pragma unroll
  for (int k = 0; k < ARN_IT; ++k) {
    const int e = 8 * (tid + AR_T * k);
    off[k] = 0;
    par[k] = 0;
    if (e >= D) continue;
    const int ch = e / (int)AR_CHUNK;
    par[k] = (counters[b0 + ch] + 1) & 1;
    off[k] = (long)(b0 + ch) * AR_CHUNK * 4 + (long)(e - ch * (int)AR_CHUNK) * 2;
    bf16x8 o;
    if (a.S == 0) {
      o = *(const bf16x8*)((const bf16*)a.p + (long)t * D + e);
    } else {
      const float* src = (const float*)a.p + (long)t * D + e;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < a.S; s0 += 4) {
        f32x4 lo[4], hi[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // clamped, all in flight before the adds
          const float* q = src + (long)min(s0 + i, a.S - 1) * a.slab;
          lo[i] = *(const f32x4*)q;
          hi[i] = *(const f32x4*)(q + 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float m = (s0 + i < a.S) ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] = fmaf(m, lo[i][j], acc[j]);
            acc[j + 4] = fmaf(m, hi[i][j], acc[j + 4]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)acc[j];
    }
    *(bf16x8*)(own + AR_DATA + (long)par[k] * AR_SLOT + off[k]) = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 2./3. per channel c (thread c * 8 + q): signal peer q, then wait for peer q's epoch
  const int c = tid >> 3, q = tid & 7;
  const bool fl = c < nch && q < a.world && q != a.rank;
  const int ep_c = (c < nch) ? counters[b0 + c] + 1 : 0;
  if (fl) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* pf = (int*)(a.bufs[q] + AR_FLAGS) + (b0 + c) * AR_MAXR + a.rank;
    __hip_atomic_store(pf, ep_c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (fl) {
    const int* f = (const int*)(own + AR_FLAGS) + (b0 + c) * AR_MAXR + q;
    long spins = 0;
    while (ar_load_flag(f) < ep_c) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > a.spin_limit) {
        for (int r = 0; r < a.world; ++r)
          __hip_atomic_store((int*)(a.bufs[r] + AR_ERR), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 4. rank-ordered sum (identical bits everywhere) + bias + residual; row statistics
  float* rrow = a.residual + (long)t * D;
  float s1 = 0.f;
#pragma unroll
  for (int k = 0; k < ARN_IT; ++k) {
    const int e = 8 * (tid + AR_T * k);
    if (e >= D) continue;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      const bf16x8 x = *(const bf16x8*)(a.bufs[r] + AR_DATA + (long)par[k] * AR_SLOT + off[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)x[j];
    }
    const f32x4 r0 = *(const f32x4*)(rrow + e), r1 = *(const f32x4*)(rrow + e + 4);
    f32x4 b0v = {0.f, 0.f, 0.f, 0.f}, b1v = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
      b0v = *(const f32x4*)(a.bias + e);
      b1v = *(const f32x4*)(a.bias + e + 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[k][j] = r0[j] + (acc[j] + b0v[j]);
      v[k][j + 4] = r1[j] + (acc[j + 4] + b1v[j]);
    }
    *(f32x4*)(rrow + e) = f32x4{v[k][0], v[k][1], v[k][2], v[k][3]};
    *(f32x4*)(rrow + e + 4) = f32x4{v[k][4], v[k][5], v[k][6], v[k][7]};
#pragma unroll
    for (int j = 0; j < 8; ++j) s1 += a.mode == 0 ? v[k][j] * v[k][j] : v[k][j];
  }
  float mean = 0.f, rstd;
  if (a.mode == 0) {
    rstd = rsqrtf(block_sum<AR_T>(s1, red) / (float)D + a.eps);
  } else {
    mean = block_sum<AR_T>(s1, red) / (float)D;
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < ARN_IT; ++k) {
      const int e = 8 * (tid + AR_T * k);
      if (e >= D) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) s2 += (v[k][j] - mean) * (v[k][j] - mean);
    }
    rstd = rsqrtf(block_sum<AR_T>(s2, red) / (float)D + a.eps);
  }
  // 5. the next layer's normed input
#pragma unroll
  for (int k = 0; k < ARN_IT; ++k) {
    const int e = 8 * (tid + AR_T * k);
    if (e >= D) continue;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float y = (v[k][j] - mean) * rstd * a.w[e + j];
      if (a.nb) y += a.nb[e + j];
      o[j] = (bf16)y;
    }
    *(bf16x8*)(a.out + (long)t * D + e) = o;
  }
  // 6. this row's channels advance one epoch
  if (tid < nch) ((int*)(own + AR_COUNTER))[b0 + tid] = counters[b0 + tid] + 1;
}

// ----------------------------------------------------------------------------- two-shot// ----------------------------------------------------------------------------- two-shot
// Reduce-scatter + all-gather over the same kind of peer-mapped region, for messages past the
// one-shot's 256 K elements (decode rows of a wide TP batch: 256 x 4096 fp32 = 4 MiB; prefill
// chunks up to 4 M elements).  One-shot makes every rank read all R copies of the message (R x n
// bytes per rank); two-shot reads ~2n: rank r reduces only its 1/R sub-range of each 1024-element
// block (reading that sub-range from every rank), stores the sum in its own result slot, and then
// every rank gathers the R reduced sub-ranges.  Same per-block channels, epochs and parity slots
// as the one-shot; a second flag row per block orders phase 2 after phase 1 on every rank.
//   region: [flags1 | flags2 : AR2_MAXB x AR_MAXR int32] [counter : AR2_MAXB] [err]
//           [data : 2 parity slots x 16 MiB] [result : 2 parity slots x 16 MiB]
// Slot reuse is safe for the reason given above: a peer signals epoch e+1 only after its epoch-e
// kernel (every read of this rank's epoch-e slots) has finished.  Every element is reduced once,
// by its owner, in rank order (fp32), so all ranks hold identical bits.
constexpr int AR2_MAXB = 4096;
constexpr int AR2_GRID = 128;  // persistent workgroups (see allreduce_twoshot_kernel)
constexpr long AR2_F1 = 0, AR2_F2 = (long)AR2_MAXB * AR_MAXR * 4, AR2_CNT = 2 * AR2_F2,
               AR2_ERR = AR2_CNT + AR2_MAXB * 4;
constexpr long AR2_DATA = 524288;                 // header rounded up (512 KiB)
constexpr long AR2_SLOT = (long)AR2_MAXB * AR_CHUNK * 4;  // 16 MiB per parity slot
static_assert(AR2_ERR + 64 <= AR2_DATA, "two-shot header");

LA_DEV void ar_signal(uint8_t* const* bufs, int world, int rank, long flags_off, int b, int ep, int tid) {
  if (tid < world && tid != rank) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* f = (int*)(bufs[tid] + flags_off) + b * AR_MAXR + rank;
    __hip_atomic_store(f, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

LA_DEV void ar_wait(uint8_t* own, uint8_t* const* bufs, int world, int rank, long flags_off, long err_off, int b,
                    int ep, int tid, long spin_limit) {
  if (tid < world && tid != rank) {
    const int* f = (const int*)(own + flags_off) + b * AR_MAXR + tid;
    long spins = 0;
    while (ar_load_flag(f) < ep) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > spin_limit) {
        for (int r = 0; r < world; ++r)  // every rank's error word (see the one-shot wait)
          __hip_atomic_store((int*)(bufs[r] + err_off), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// One chunk (1024 elements) of the two-shot protocol, run by one workgroup.
LA_DEV void ar2_chunk(const ARArgs& a, int b) {
  const int tid = threadIdx.x, R = a.world;
  const long e0 = (long)b * AR_CHUNK;
  const long e1 = min(a.n, e0 + AR_CHUNK);
  uint8_t* own = a.bufs[a.rank];
  int* counter = (int*)(own + AR2_CNT) + b;
  const int ep = *counter + 1;
  const long boff = (long)b * AR_CHUNK * 4;                        // this block's bytes in a slot
  const long dslot = AR2_DATA + (long)(ep & 1) * AR2_SLOT + boff;   // inputs
  const long rslot = AR2_DATA + (long)(2 + (ep & 1)) * AR2_SLOT + boff;  // reduced sub-ranges
  const int esz = a.bf16 ? 2 : 4;
  // 1. local chunk -> own data slot
  {
    const uint8_t* src = (const uint8_t*)a.in + e0 * esz;
    uint8_t* dst = own + dslot;
    const long bytes = (e1 - e0) * esz, v16 = bytes >> 4;
    for (long i = tid; i < v16; i += AR_T) ((u32x4*)dst)[i] = ((const u32x4*)src)[i];
    for (long i = (v16 << 4) + tid; i < bytes; i += AR_T) dst[i] = src[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_signal(a.bufs, R, a.rank, AR2_F1, b, ep, tid);
  ar_wait(own, a.bufs, R, a.rank, AR2_F1, AR2_ERR, b, ep, tid, a.spin_limit);
  // 2. reduce-scatter: this rank's sub-range of the block (multiples of 8 elements)
  const long sub = ((AR_CHUNK / R) + 7) & ~7L;
  const long s0 = min(e1, e0 + (long)a.rank * sub), s1 = min(e1, s0 + sub);
  for (long i = s0 + tid * 8; i < s1; i += AR_T * 8) {
    const int cnt = (int)min(8L, s1 - i);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < R; ++r) {
      const uint8_t* src = a.bufs[r] + dslot + (i - e0) * esz;
      if (a.bf16) {
        if (cnt == 8) {
          const bf16x8 v = *(const bf16x8*)src;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
        } else {
          for (int j = 0; j < cnt; ++j) acc[j] += (float)((const bf16*)src)[j];
        }
      } else {
        if (cnt == 8) {
          const f32x4 v0 = *(const f32x4*)src, v1 = *(const f32x4*)(src + 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] += v0[j];
            acc[j + 4] += v1[j];
          }
        } else {
          for (int j = 0; j < cnt; ++j) acc[j] += ((const float*)src)[j];
        }
      }
    }
    uint8_t* dst = own + rslot + (i - e0) * esz;
    if (a.bf16) {
      for (int j = 0; j < cnt; ++j) ((bf16*)dst)[j] = (bf16)acc[j];
    } else {
      for (int j = 0; j < cnt; ++j) ((float*)dst)[j] = acc[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ar_signal(a.bufs, R, a.rank, AR2_F2, b, ep, tid);
  ar_wait(own, a.bufs, R, a.rank, AR2_F2, AR2_ERR, b, ep, tid, a.spin_limit);
  // 3. all-gather: every rank's reduced sub-range, from its result slot, into out
  {
    const long bytes = (e1 - e0) * esz, v16 = bytes >> 4;
    const long subb = sub * esz;  // a sub-range is a multiple of 16 bytes
    for (long i = tid; i < v16; i += AR_T) {
      const int q = (int)min((long)R - 1, (i << 4) / subb);
      ((u32x4*)((uint8_t*)a.out + e0 * esz))[i] = ((const u32x4*)(a.bufs[q] + rslot))[i];
    }
    for (long i = (v16 << 4) + tid; i < bytes; i += AR_T) {
      const int q = (int)min((long)R - 1, i / subb);
      ((uint8_t*)a.out + e0 * esz)[i] = (a.bufs[q] + rslot)[i];
    }
  }
  if (tid == 0) *counter = ep;
  __syncthreads();  // the next chunk of this workgroup reuses the same LDS-free, register-only path
}

// Persistent grid of at most AR2_GRID workgroups, each walking chunks g, g + G, ... in order: the
// waits of chunk c only ever target the peers' workgroup that walks the same chunk sequence.  The
// protocol needs every rank's grid resident at once: on separate GPUs a 128-workgroup grid always
// is; when R ranks SHARE one device (tests, rehearsals) the caller caps the grid at AR2_GRID / R
// (max_grid) so the R grids -- beside a GEMM on another stream -- still fit the CUs' wave slots,
// and every wait is bounded by spin_limit (error word set, RCCL from then on) if they do not.
__global__ __launch_bounds__(AR_T) void allreduce_twoshot_kernel(ARArgs a, int nb) {
  for (int c = blockIdx.x; c < nb; c += gridDim.x) ar2_chunk(a, c);
}

}  // namespace la

// C ABI ---------------------------------------------------------------------------
extern "C" long la_ar2_buffer_bytes() { return la::AR2_DATA + 4 * la::AR2_SLOT; }
extern "C" long la_ar2_max_elems() { return (long)la::AR2_MAXB * la::AR_CHUNK; }
extern "C" long la_ar2_err_offset() { return la::AR2_ERR; }

extern "C" int la_allreduce_twoshot(const void* in, void* out, long n, int bf16, int rank, int world,
                                    const void* const* bufs, long spin_limit, void* stream, int max_grid) {
  using namespace la;
  if (world < 1 || world > AR_MAXR || rank < 0 || rank >= world || n < 1) return -1;
  if (n > (long)AR2_MAXB * AR_CHUNK) return -2;
  ARArgs a{};
  a.in = in;
  a.out = out;
  a.n = n;
  a.bf16 = bf16;
  a.rank = rank;
  a.world = world;
  a.spin_limit = spin_limit;
  for (int r = 0; r < world; ++r) {
    if (!bufs[r]) return -1;
    a.bufs[r] = (uint8_t*)bufs[r];
  }
  const int nb = (int)((n + AR_CHUNK - 1) / AR_CHUNK);
  const int cap = (max_grid > 0 && max_grid < AR2_GRID) ? max_grid : AR2_GRID;
  hipLaunchKernelGGL(allreduce_twoshot_kernel, dim3(nb < cap ? nb : cap), dim3(AR_T), 0, (hipStream_t)stream, a,
                     nb);
  return (int)hipGetLastError();
}
// Fused decode layer boundary (allreduce_add_norm_kernel): M rows of D (D % 8 == 0, D <= 8192,
// M * ceil(D / 1024) <= 256 channels) on the one-shot region `bufs`.
extern "C" int la_allreduce_add_norm(const void* p, long slab, int S, int M, int D, int rank, int world,
                                     const void* const* bufs, long spin_limit, void* residual, const void* bias,
                                     const void* w, const void* nb, void* out, float eps, int mode, void* stream) {
  using namespace la;
  if (world < 1 || world > AR_MAXR || rank < 0 || rank >= world || M < 1 || D < 8 || (D & 7) ||
      D > AR_T * 8 * ARN_IT || S < 0 || S > 64 || (S > 0 && slab < (long)M * D) || !p || !residual || !w || !out ||
      (mode != 0 && mode != 1))
    return -1;
  const int nch = (D + (int)AR_CHUNK - 1) / (int)AR_CHUNK;
  if ((long)M * nch > AR_MAXB) return -2;
  ARNArgs a{};
  a.p = p;
  a.slab = slab;
  a.S = S;
  a.D = D;
  a.rank = rank;
  a.world = world;
  a.spin_limit = spin_limit;
  for (int r = 0; r < world; ++r) {
    if (!bufs[r]) return -1;
    a.bufs[r] = (uint8_t*)bufs[r];
  }
  a.residual = (float*)residual;
  a.bias = (const float*)bias;
  a.w = (const float*)w;
  a.nb = (const float*)nb;
  a.out = (bf16*)out;
  a.eps = eps;
  a.mode = mode;
  hipLaunchKernelGGL(allreduce_add_norm_kernel, dim3(M), dim3(AR_T), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" long la_ar_buffer_bytes() { return la::AR_DATA + 2 * la::AR_SLOT; }
extern "C" long la_ar_max_elems() { return la::AR_MAXB * la::AR_CHUNK; }
extern "C" long la_ar_err_offset() { return la::AR_ERR; }

// bufs: world device pointers (own + opened peers) of regions of la_ar_buffer_bytes() bytes.
extern "C" int la_allreduce_oneshot(const void* in, void* out, long n, int bf16, int rank, int world,
                                    const void* const* bufs, long spin_limit, void* stream) {
  using namespace la;
  if (world < 1 || world > AR_MAXR || rank < 0 || rank >= world || n < 1) return -1;
  if (n > AR_MAXB * AR_CHUNK) return -2;
  ARArgs a{};
  a.in = in;
  a.out = out;
  a.n = n;
  a.bf16 = bf16;
  a.rank = rank;
  a.world = world;
  a.spin_limit = spin_limit;
  for (int r = 0; r < world; ++r) {
    if (!bufs[r]) return -1;
    a.bufs[r] = (uint8_t*)bufs[r];
  }
  const int nb = (int)((n + AR_CHUNK - 1) / AR_CHUNK);
  hipLaunchKernelGGL(allreduce_oneshot_kernel, dim3(nb), dim3(AR_T), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
