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

// ----------------------------------------------------------------------------- two-shot
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
