// On-device sampling: the whole llama.cpp sampler chain runs on the GPU,
// one workgroup per sequence, and only the chosen token ids (4 B/row) go back to the host
// instead of the 513 KB logits row the reference copies every step.
//
// Chain semantics follow llama.cpp @ d5cb868 common/sampling.cpp [external] as driven by
// LocalAI's grpc-server.cpp (params_parse / parse_options):
//   logit_bias -> penalties (repeat/frequency/presence over last-n)   [la_penalties]
//   mirostat == 0 : top_k -> tail-free(z) -> typical(p) -> top_p -> min_p -> temperature -> dist
//   mirostat == 2 : temperature -> mirostat_v2(tau, eta)  (mu state kept on device)
//   temperature <= 0 : greedy argmax
// Philox4x32-10 keyed by (seed, per-row counter) supplies the uniform draw.
#include "common.h"

namespace la {

struct SampleRow {
  float temp, top_p, min_p, typical_p, tfs_z, tau, eta;
  int top_k, mirostat, pad;
  unsigned long long seed, counter;
};

constexpr int SMP_T = 1024;
constexpr int SMP_BATCH = 8;  // float4 loads in flight per thread in the argmax scan
constexpr int CAP = 1024;

LA_DEV uint32_t fkey(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

LA_DEV void philox(uint64_t seed, uint64_t ctr, uint32_t out[4]) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x9E3779B9u, c3 = 0x85EBCA6Bu;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct SmpShared {
  float cval[CAP];
  int cidx[CAP];
  float fred[SMP_T / 64];
  int ired[SMP_T / 64];
  unsigned hist[256];
  float scan[SMP_T];
  int tok2[CAP];
  int count;
  int sel;
  uint32_t prefix;
  int kleft;
};

// block-wide (max, argmax) with lowest-index tie break
LA_DEV void block_argmax(float& v, int& i, SmpShared& sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { sh.fred[w] = v; sh.ired[w] = i; }
  __syncthreads();
  v = sh.fred[0]; i = sh.ired[0];
  for (int k = 1; k < SMP_T / 64; ++k)
    if (sh.fred[k] > v || (sh.fred[k] == v && sh.ired[k] < i)) { v = sh.fred[k]; i = sh.ired[k]; }
}

// f(value, index) over one logits row, every element once, increasing index per thread.
// Aligned rows stream float4s with SMP_BATCH loads in flight per thread (clamped indices,
// masked calls): each full pass over a 128k vocabulary is then 4 memory round trips per
// thread, not 125 dependent scalar loads -- the sampler makes up to ~10 such passes.
template <typename F>
LA_DEV void row_foreach(const float* row, int V, F&& f) {
  int i0 = 0;
  if ((((uintptr_t)row) & 15) == 0) {
    const int V4 = V >> 2;
    const float4* row4 = (const float4*)row;
    for (int j0 = threadIdx.x; j0 < V4; j0 += SMP_BATCH * SMP_T) {
      float4 v[SMP_BATCH];
#pragma unroll
      for (int k = 0; k < SMP_BATCH; ++k) v[k] = row4[min(j0 + k * SMP_T, V4 - 1)];
#pragma unroll
      for (int k = 0; k < SMP_BATCH; ++k) {
        const int j = j0 + k * SMP_T;
        if (j < V4) { f(v[k].x, 4 * j); f(v[k].y, 4 * j + 1); f(v[k].z, 4 * j + 2); f(v[k].w, 4 * j + 3); }
      }
    }
    i0 = V4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < V; i += SMP_T) f(row[i], i);
}

// f(value, index) over row[lo, hi) in order (one thread's contiguous chunk), 8 loads in flight;
// f returns false to stop early.
template <typename F>
LA_DEV void chunk_foreach(const float* row, int lo, int hi, F&& f) {
  for (int i0 = lo; i0 < hi; i0 += 8) {
    float r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = row[min(i0 + k, hi - 1)];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i0 + k < hi && !f(r[k], i0 + k)) return;
  }
}

// exclusive prefix sum over the block (thread order); total -> *tot
LA_DEV float block_excl_scan(float v, SmpShared& sh, float* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) sh.fred[w] = x;
  __syncthreads();
  float base = 0.f, t = 0.f;
#pragma unroll
  for (int k = 0; k < SMP_T / 64; ++k) {
    const float c = sh.fred[k];
    if (k < w) base += c;
    t += c;
  }
  __syncthreads();
  *tot = t;
  return base + x - v;
}

// k-th largest key (1-based) among row keys via 4-pass 8-bit radix select
LA_DEV uint32_t radix_kth(const float* row, int V, int k, SmpShared& sh) {
  uint32_t prefix = 0, mask = 0;
  int kleft = k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += SMP_T) sh.hist[i] = 0;
    __syncthreads();
    row_foreach(row, V, [&](float v, int) {
      const uint32_t key = fkey(v);
      if ((key & mask) == prefix) atomicAdd(&sh.hist[(key >> shift) & 255u], 1u);
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      // digit search from 255 down, one wave: lane l owns digits 255-4l .. 252-4l, a lane
      // prefix scan gives each lane the count above its digits, and the first lane whose
      // running count reaches kleft walks its 4 digits (same answer as a serial scan that
      // stops at digit 0)
      const int l = threadIdx.x;
      int c4[4], own = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) { c4[q] = (int)sh.hist[255 - 4 * l - q]; own += c4[q]; }
      int inc = own;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (l >= o) inc += y;
      }
      const unsigned long long hit = __ballot(inc >= kleft);
      const int L = hit ? (__ffsll((long long)hit) - 1) : 63;
      if (l == L) {
        int acc = inc - own, d = 255 - 4 * l;
#pragma unroll
        for (int q = 0; q < 4; ++q, --d) {
          if (d == 0 || acc + c4[q] >= kleft) break;
          acc += c4[q];
        }
        sh.kleft = kleft - acc;
        sh.prefix = prefix | ((uint32_t)d << shift);
      }
    }
    __syncthreads();
    prefix = sh.prefix;
    kleft = sh.kleft;
    mask |= 255u << shift;
    __syncthreads();
  }
  return prefix;
}

// bitonic sort of sh.cval/cidx[0..n) descending by value (n padded to pow2 with -inf)
LA_DEV void block_sort_desc(SmpShared& sh, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = n + threadIdx.x; i < P; i += SMP_T) { sh.cval[i] = -INFINITY; sh.cidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += SMP_T) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool desc = ((i & k) == 0);
          const float a = sh.cval[i], b = sh.cval[ixj];
          const bool a_first = (a > b) || (a == b && sh.cidx[i] < sh.cidx[ixj]);
          if (desc ? !a_first : a_first) {
            sh.cval[i] = b; sh.cval[ixj] = a;
            const int t = sh.cidx[i]; sh.cidx[i] = sh.cidx[ixj]; sh.cidx[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(SMP_T) void sample_kernel(const float* __restrict__ logits, long ld, int V,
                                                       const SampleRow* __restrict__ params, float* __restrict__ mu,
                                                       int* __restrict__ out_tok, float* __restrict__ out_p) {
  __shared__ SmpShared sh;
  const int b = blockIdx.x;
  const float* row = logits + (long)b * ld;
  const SampleRow P = params[b];

  // max / argmax: 16-byte loads when the row is aligned, SMP_BATCH of them issued before the
  // first compare (clamped indices, never branched on, so they all stay in flight): a 128k
  // vocabulary is 4 HBM round trips per thread instead of 16 -- the greedy path is one
  // workgroup per row, so this loop IS its latency.  Clamped duplicates re-read element
  // V4-1 with its own index, which cannot change the (value, lowest index) result.
  float mv = -INFINITY;
  int mi = 0x7fffffff;
  int i0 = 0;
  if ((((uintptr_t)row) & 15) == 0) {
    const int V4 = V >> 2;
    const float4* row4 = (const float4*)row;
    for (int j0 = threadIdx.x; j0 < V4; j0 += SMP_BATCH * SMP_T) {
      float4 v[SMP_BATCH];
#pragma unroll
      for (int k = 0; k < SMP_BATCH; ++k) v[k] = row4[min(j0 + k * SMP_T, V4 - 1)];
#pragma unroll
      for (int k = 0; k < SMP_BATCH; ++k) {
        const int j = min(j0 + k * SMP_T, V4 - 1);
        if (v[k].x > mv) { mv = v[k].x; mi = 4 * j; }
        if (v[k].y > mv) { mv = v[k].y; mi = 4 * j + 1; }
        if (v[k].z > mv) { mv = v[k].z; mi = 4 * j + 2; }
        if (v[k].w > mv) { mv = v[k].w; mi = 4 * j + 3; }
      }
    }
    i0 = V4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < V; i += SMP_T) {
    const float v = row[i];
    if (v > mv) { mv = v; mi = i; }
  }
  block_argmax(mv, mi, sh);
  if (P.temp <= 0.f) {
    if (threadIdx.x == 0) { out_tok[b] = mi; if (out_p) out_p[b] = 1.f; }
    return;
  }
  uint32_t rnd[4];
  philox(P.seed, P.counter, rnd);
  const float u01 = ((rnd[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);

  if (P.mirostat == 2) {
    // temperature, then keep p >= 2^-mu (prefix of the sorted list), renormalise, sample
    const float invT = 1.f / P.temp;
    float z = 0.f;
    row_foreach(row, V, [&](float v, int) { z += __expf((v - mv) * invT); });
    z = block_sum<SMP_T>(z, sh.fred);
    const float m = mu[b];
    const float thr = exp2f(-m) * z;  // unnormalised mass threshold
    // contiguous chunk per thread (row is L2-resident by now) for an ordered prefix scan
    const int C = (V + SMP_T - 1) / SMP_T;
    const int lo = threadIdx.x * C, hi = min(V, lo + C);
    float part = 0.f;
    chunk_foreach(row, lo, hi, [&](float v, int i) {
      const float e = __expf((v - mv) * invT);
      if (e >= thr || i == mi) part += e;
      return true;
    });
    if (threadIdx.x == 0) sh.sel = mi;
    float zk;
    float acc = block_excl_scan(part, sh, &zk);
    const float target = u01 * zk;
    if (target >= acc && target < acc + part) {
      chunk_foreach(row, lo, hi, [&](float v, int i) {
        const float e = __expf((v - mv) * invT);
        if (!(e >= thr || i == mi)) return true;
        acc += e;
        if (target < acc) { sh.sel = i; return false; }
        return true;
      });
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int s = sh.sel;
      const float ps = __expf((row[s] - mv) * invT) / zk;
      out_tok[b] = s;
      if (out_p) out_p[b] = ps;
      mu[b] = m - P.eta * (-log2f(ps) - P.tau);
    }
    return;
  }

  // ---------------- standard chain
  int k = P.top_k;
  if (k <= 0 || k > V) k = V;
  // threshold for top-k, and candidate prefilter by min_p (valid: min_p is relative to the max)
  uint32_t key_k = 0;
  if (k < V) key_k = radix_kth(row, V, k, sh);
  // Z over the top-k set (top_p normalisation in llama.cpp is over the post-top-k list)
  float zk = 0.f;
  int cnt = 0;
  float thr = -INFINITY;
  if (P.min_p > 0.f && P.min_p <= 1.f) thr = mv + logf(P.min_p);
  // Z over the top-k set, and the candidate count (if > CAP the threshold rises to the
  // CAP-th largest) in one pass
  row_foreach(row, V, [&](float v, int) {
    if (k == V || fkey(v) >= key_k) {
      zk += __expf(v - mv);
      if (v >= thr) ++cnt;
    }
  });
  zk = block_sum<SMP_T>(zk, sh.fred);
  cnt = (int)block_sum<SMP_T>((float)cnt, sh.fred);
  uint32_t key_c = 0;
  bool capped = false;
  if (cnt > CAP) { key_c = radix_kth(row, V, CAP, sh); capped = true; }
  if (threadIdx.x == 0) sh.count = 0;
  __syncthreads();
  row_foreach(row, V, [&](float v, int i) {
    const uint32_t kk = fkey(v);
    if ((k == V || kk >= key_k) && v >= thr && (!capped || kk >= key_c)) {
      const int slot = atomicAdd(&sh.count, 1);
      if (slot < CAP) { sh.cval[slot] = v; sh.cidx[slot] = i; }
    }
  });
  __syncthreads();
  int n = min(sh.count, CAP);
  block_sort_desc(sh, n);
  if (n > k) n = k;

  if (threadIdx.x == 0) {
    // tail-free sampling
    if (P.tfs_z < 1.f && n > 2) {
      float z = 0.f;
      for (int i = 0; i < n; ++i) z += __expf(sh.cval[i] - mv);
      // second derivatives of the sorted probabilities
      float sum2 = 0.f;
      for (int i = 0; i < n - 2; ++i) {
        const float p0 = __expf(sh.cval[i] - mv) / z, p1 = __expf(sh.cval[i + 1] - mv) / z,
                    p2 = __expf(sh.cval[i + 2] - mv) / z;
        sum2 += fabsf((p0 - p1) - (p1 - p2));
      }
      int last = n;
      if (sum2 > 0.f) {
        float cum = 0.f;
        for (int i = 0; i < n - 2; ++i) {
          const float p0 = __expf(sh.cval[i] - mv) / z, p1 = __expf(sh.cval[i + 1] - mv) / z,
                      p2 = __expf(sh.cval[i + 2] - mv) / z;
          cum += fabsf((p0 - p1) - (p1 - p2)) / sum2;
          if (cum > P.tfs_z) { last = i + 1; break; }
        }
      }
      n = max(1, last);
    }
    sh.count = n;
  }
  __syncthreads();
  n = sh.count;

  // locally typical sampling: re-sort by |surprise - entropy| ascending, keep until mass >= p
  if (P.typical_p < 1.f && n > 1) {
    if (threadIdx.x == 0) {
      float z = 0.f, H = 0.f;
      for (int i = 0; i < n; ++i) z += __expf(sh.cval[i] - mv);
      for (int i = 0; i < n; ++i) { const float p = __expf(sh.cval[i] - mv) / z; H -= p * logf(p); }
      sh.fred[0] = z; sh.fred[1] = H;
    }
    __syncthreads();
    const float z = sh.fred[0], H = sh.fred[1];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += SMP_T) {
      const float p = __expf(sh.cval[i] - mv) / z;
      sh.scan[i] = sh.cval[i];   // logit of slot i
      sh.tok2[i] = sh.cidx[i];   // token of slot i
      sh.cval[i] = -fabsf(-logf(p) - H);
      sh.cidx[i] = i;
    }
    __syncthreads();
    block_sort_desc(sh, n);
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int last = n;
      for (int i = 0; i < n; ++i) {
        cum += __expf(sh.scan[sh.cidx[i]] - mv) / z;
        if (cum >= P.typical_p) { last = i + 1; break; }
      }
      for (int i = 0; i < last; ++i) {
        const int slot = sh.cidx[i];
        sh.cval[i] = sh.scan[slot];
        sh.cidx[i] = sh.tok2[slot];
      }
      sh.count = last;
    }
    __syncthreads();
    n = sh.count;
    block_sort_desc(sh, n);  // back to logit order for top_p
    if (threadIdx.x == 0) {
      float z2 = 0.f;
      for (int i = 0; i < n; ++i) z2 += __expf(sh.cval[i] - mv);
      sh.fred[0] = z2;
    }
    __syncthreads();
    zk = sh.fred[0];
  } else if (P.tfs_z < 1.f) {
    // tail-free renormalises over its kept prefix
    if (threadIdx.x == 0) {
      float z2 = 0.f;
      for (int i = 0; i < n; ++i) z2 += __expf(sh.cval[i] - mv);
      sh.fred[0] = z2;
    }
    __syncthreads();
    zk = sh.fred[0];
  }

  if (threadIdx.x == 0) {
    // top_p over the current list (normalised by zk), then min_p (already prefiltered), then temperature
    if (P.top_p < 1.f) {
      float cum = 0.f;
      int last = n;
      for (int i = 0; i < n; ++i) {
        cum += __expf(sh.cval[i] - mv) / zk;
        if (cum >= P.top_p) { last = i + 1; break; }
      }
      n = last;
    }
    const float invT = 1.f / P.temp;
    const float m0 = sh.cval[0];
    float z = 0.f;
    for (int i = 0; i < n; ++i) z += __expf((sh.cval[i] - m0) * invT);
    const float target = u01 * z;
    float acc = 0.f;
    int sel = n - 1;
    for (int i = 0; i < n; ++i) {
      acc += __expf((sh.cval[i] - m0) * invT);
      if (target < acc) { sel = i; break; }
    }
    out_tok[b] = sh.cidx[sel];
    if (out_p) out_p[b] = __expf((sh.cval[sel] - m0) * invT) / z;
  }
}

// grammar-constrained rows: tokens outside the row's allowed-token mask (slot of the engine's
// device mask pool, one byte per token; slot < 0 = unconstrained row) get -inf before the
// sampler, so the in-graph sample is already grammar-valid.  grid (chunks, rows); unconstrained
// rows exit at once.
__global__ __launch_bounds__(256) void grammar_mask_kernel(float* __restrict__ logits, long ld, int V,
                                                           const int* __restrict__ slot,
                                                           const unsigned char* __restrict__ pool, long pool_ld) {
  const int row = blockIdx.y;
  const int s = slot[row];
  if (s < 0) return;
  const unsigned char* m = pool + (long)s * pool_ld;
  float* l = logits + (long)row * ld;
  for (int v = blockIdx.x * 256 + threadIdx.x; v < V; v += gridDim.x * 256)
    if (!m[v]) l[v] = -INFINITY;
}

// grammar rows across a multi-step run: after each in-graph sample, a row's mask slot follows the
// transition table the host has learned (next[slot][token], -2 = not learned yet).  An unknown
// transition parks the row at -3 (no mask; the host keeps its tokens up to that point and drops
// the rest of the run for that row).  Rows at -1 (unconstrained) and -3 are left alone.
__global__ __launch_bounds__(256) void grammar_advance_kernel(const int* __restrict__ tok, int* __restrict__ slot,
                                                              const short* __restrict__ next, int V, int B) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int s = slot[b];
  if (s < 0) return;
  const int t = tok[b];
  const int ns = (t >= 0 && t < V) ? (int)next[(long)s * V + t] : -2;
  slot[b] = ns >= 0 ? ns : -3;
}

// penalties over the last-n window (llama_sampler_penalties): every distinct token t in the
// window gets  l = l>0 ? l/rp : l*rp ;  l -= count*freq + (count>0)*presence
__global__ __launch_bounds__(256) void penalties_kernel(float* __restrict__ logits, long ld,
                                                        const int* __restrict__ hist, int hist_ld,
                                                        const int* __restrict__ hist_len,
                                                        const float* __restrict__ pen /* [B][3] */, int nl_token,
                                                        const int* __restrict__ penalize_nl, int col0 = 0,
                                                        int ncols = 0x7fffffff) {
  const int b = blockIdx.x;
  const int L = hist_len[b];
  const float rp = pen[3 * b], fp = pen[3 * b + 1], pp = pen[3 * b + 2];
  if (L <= 0 || (rp == 1.f && fp == 0.f && pp == 0.f)) return;
  const int* h = hist + (long)b * hist_ld;
  float* row = logits + (long)b * ld;
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const int t = h[i];
    if (t < 0) continue;
    bool first = true;
    int cnt = 0;
    for (int j = 0; j < L; ++j) {
      if (h[j] == t) {
        if (j < i) { first = false; break; }
        ++cnt;
      }
    }
    if (!first) continue;
    if (t == nl_token && penalize_nl && !penalize_nl[b]) continue;
    if (t < col0 || t - col0 >= ncols) continue;  // another rank's column
    float l = row[t - col0];
    if (rp != 1.f) l = (l > 0.f) ? l / rp : l * rp;
    l -= (float)cnt * fp + (cnt > 0 ? pp : 0.f);
    row[t - col0] = l;
  }
}

// In-graph penalty window: append each row's sampled token to its ring of the last pcap[b]
// tokens (order is irrelevant to the penalties, which count occurrences) and refresh the
// window length the penalties kernel reads.
__global__ void pen_push_kernel(const int* __restrict__ next, int B, int* __restrict__ hist, int hist_ld,
                                int* __restrict__ cnt, int* __restrict__ len, const int* __restrict__ cap) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int c = cnt[b], k = cap[b];
  if (k <= 0) return;
  hist[(long)b * hist_ld + c % k] = next[b];
  cnt[b] = c + 1;
  len[b] = min(c + 1, k);
}

// ---------------------------------------------------------------- tensor-parallel sampling
// Vocabulary-parallel logits: rank r holds columns [base, base + Vs) of every row.  Nothing here
// gathers a full row; the ranks exchange per-row candidates / statistics through small fp32
// buffers in which every rank writes only its own slot (the others are zero), so ONE sum
// all-reduce -- the graph-replayable custom all-reduce -- is the exchange.

// ascending sort of sh.cval/cidx[0..n) by token index (bitonic, pads at the end)
LA_DEV void block_sort_idx(SmpShared& sh, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = n + threadIdx.x; i < P; i += SMP_T) { sh.cval[i] = -INFINITY; sh.cidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += SMP_T) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool asc = ((i & k) == 0);
          const bool swap = asc ? (sh.cidx[i] > sh.cidx[ixj]) : (sh.cidx[i] < sh.cidx[ixj]);
          if (swap) {
            const float a = sh.cval[i]; sh.cval[i] = sh.cval[ixj]; sh.cval[ixj] = a;
            const int t = sh.cidx[i]; sh.cidx[i] = sh.cidx[ixj]; sh.cidx[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Standard-chain candidates: the C largest logits of this rank's columns (ties: highest value,
// then lowest id), written in increasing id order as (value, global id) pairs to out[b][C][2];
// unused entries (-inf, 0).  Every rank's C >= top_k candidates together hold the global top-k,
// and the chain after top-k (tail-free, typical, top-p, min-p, temperature, draw) sees only those.
__global__ __launch_bounds__(SMP_T) void tp_topc_kernel(const float* __restrict__ logits, long ld, int Vs, int C,
                                                        int base, float* __restrict__ out) {
  __shared__ SmpShared sh;
  const int b = blockIdx.x;
  const float* row = logits + (long)b * ld;
  float* o = out + (long)b * C * 2;
  uint32_t key_c = 0;
  if (C < Vs) key_c = radix_kth(row, Vs, C, sh);
  if (threadIdx.x == 0) sh.count = 0;
  __syncthreads();
  row_foreach(row, Vs, [&](float v, int i) {
    if (C >= Vs || fkey(v) >= key_c) {
      const int slot = atomicAdd(&sh.count, 1);
      if (slot < CAP) { sh.cval[slot] = v; sh.cidx[slot] = i; }
    }
  });
  __syncthreads();
  int n = min(sh.count, CAP);
  __syncthreads();
  if (n > C) {  // ties at the C-th value: keep the lowest ids
    block_sort_desc(sh, n);
    n = C;
  }
  block_sort_idx(sh, n);
  for (int j = threadIdx.x; j < C; j += SMP_T) {
    o[2 * j] = j < n ? sh.cval[j] : -INFINITY;
    o[2 * j + 1] = j < n ? (float)(base + sh.cidx[j]) : 0.f;
  }
}

// Mirostat 2 over vocabulary shards, four phases with a sum-exchange between each (x1, x2, x3:
// [world][B][.] buffers, this rank's slot written): the same arithmetic as sample_kernel's
// mirostat branch (temperature, keep e >= 2^-mu * Z or the argmax, renormalise, draw with the
// row's Philox uniform, mu update), with the sums taken per rank and combined in rank order.
// Rows without mirostat 2 are skipped by every phase.
LA_DEV bool tp_miro_row(const SampleRow& P) { return P.mirostat == 2 && P.temp > 0.f; }

// phase 1: local max, its (lowest) global id and Z_r = sum exp((v - m_r) / T)
__global__ __launch_bounds__(SMP_T) void tp_miro1_kernel(const float* __restrict__ logits, long ld, int Vs,
                                                         int base, const SampleRow* __restrict__ params,
                                                         float* __restrict__ x1) {
  __shared__ SmpShared sh;
  const int b = blockIdx.x;
  const SampleRow P = params[b];
  if (!tp_miro_row(P)) return;
  const float* row = logits + (long)b * ld;
  float mv = -INFINITY;
  int mi = 0x7fffffff;
  row_foreach(row, Vs, [&](float v, int i) {
    if (v > mv || (v == mv && i < mi)) { mv = v; mi = i; }
  });
  block_argmax(mv, mi, sh);
  const float invT = 1.f / P.temp;
  float z = 0.f;
  row_foreach(row, Vs, [&](float v, int) { z += __expf((v - mv) * invT); });
  z = block_sum<SMP_T>(z, sh.fred);
  if (threadIdx.x == 0) {
    x1[3 * b] = mv;
    x1[3 * b + 1] = (float)(base + mi);
    x1[3 * b + 2] = z;
  }
}

struct TpMiro {
  float M, g, Z, thr, invT;
};

LA_DEV TpMiro tp_miro_global(const float* X1, int world, int B, int b, float temp, float mu) {
  TpMiro t;
  t.invT = 1.f / temp;
  t.M = -INFINITY;
  t.g = 3.0e38f;
  for (int r = 0; r < world; ++r) {
    const float m = X1[((long)r * B + b) * 3], id = X1[((long)r * B + b) * 3 + 1];
    if (m > t.M || (m == t.M && id < t.g)) { t.M = m; t.g = id; }
  }
  t.Z = 0.f;
  for (int r = 0; r < world; ++r) {
    const float* x = X1 + ((long)r * B + b) * 3;
    if (x[0] > -INFINITY) t.Z += x[2] * __expf((x[0] - t.M) * t.invT);
  }
  t.thr = exp2f(-mu) * t.Z;
  return t;
}

// phase 2: W_r = sum over this rank's kept tokens of e = exp((v - M) / T)
__global__ __launch_bounds__(SMP_T) void tp_miro2_kernel(const float* __restrict__ logits, long ld, int Vs,
                                                         int base, const SampleRow* __restrict__ params,
                                                         const float* __restrict__ mu, const float* __restrict__ X1,
                                                         int world, int B, float* __restrict__ x2) {
  __shared__ SmpShared sh;
  const int b = blockIdx.x;
  const SampleRow P = params[b];
  if (!tp_miro_row(P)) return;
  const TpMiro t = tp_miro_global(X1, world, B, b, P.temp, mu[b]);
  const float* row = logits + (long)b * ld;
  const int gl = (int)t.g - base;  // the global argmax's local index (outside [0, Vs) elsewhere)
  float w = 0.f;
  row_foreach(row, Vs, [&](float v, int i) {
    const float e = __expf((v - t.M) * t.invT);
    if (e >= t.thr || i == gl) w += e;
  });
  w = block_sum<SMP_T>(w, sh.fred);
  if (threadIdx.x == 0) x2[b] = w;
}

// phase 3: the rank whose kept mass holds the draw picks the token by an ordered scan
__global__ __launch_bounds__(SMP_T) void tp_miro3_kernel(const float* __restrict__ logits, long ld, int Vs,
                                                         int base, const SampleRow* __restrict__ params,
                                                         const float* __restrict__ mu, const float* __restrict__ X1,
                                                         const float* __restrict__ X2, int world, int rank, int B,
                                                         float* __restrict__ x3) {
  __shared__ SmpShared sh;
  const int b = blockIdx.x;
  const SampleRow P = params[b];
  if (!tp_miro_row(P)) return;
  const TpMiro t = tp_miro_global(X1, world, B, b, P.temp, mu[b]);
  float zk = 0.f;
  for (int r = 0; r < world; ++r) zk += X2[(long)r * B + b];
  uint32_t rnd[4];
  philox(P.seed, P.counter, rnd);
  const float u01 = ((rnd[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float target = u01 * zk;
  int rs = -1, last = -1;
  float acc0 = 0.f, run = 0.f;
  for (int r = 0; r < world; ++r) {
    const float w = X2[(long)r * B + b];
    if (w > 0.f) last = r;
    if (rs < 0 && w > 0.f && target < run + w) { rs = r; acc0 = run; }
    run += w;
  }
  if (rs < 0) {  // rounding put the draw past the last mass: the last rank with mass takes it
    rs = last;
    acc0 = 0.f;
    for (int r = 0; r < last; ++r) acc0 += X2[(long)r * B + b];
  }
  if (rs != rank) return;
  const float* row = logits + (long)b * ld;
  const int gl = (int)t.g - base;
  const int C = (Vs + SMP_T - 1) / SMP_T;
  const int lo = threadIdx.x * C, hi = min(Vs, lo + C);
  float part = 0.f;
  int lastk = -1;
  chunk_foreach(row, lo, hi, [&](float v, int i) {
    const float e = __expf((v - t.M) * t.invT);
    if (e >= t.thr || i == gl) { part += e; lastk = i; }
    return true;
  });
  if (threadIdx.x == 0) {
    sh.sel = -1;
    sh.count = -1;
  }
  float tot;
  float acc = acc0 + block_excl_scan(part, sh, &tot);  // (synchronises: the inits above are visible)
  if (target >= acc && target < acc + part) {
    chunk_foreach(row, lo, hi, [&](float v, int i) {
      const float e = __expf((v - t.M) * t.invT);
      if (!(e >= t.thr || i == gl)) return true;
      acc += e;
      if (target < acc) { sh.sel = i; return false; }
      return true;
    });
  }
  __syncthreads();
  // no thread claimed it (rounding): the rank's last kept token
  int lk = lastk;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lk = max(lk, __shfl_xor(lk, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(&sh.count, lk);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int s = sh.sel >= 0 ? sh.sel : sh.count;
    if (s >= 0) {
      x3[2 * b] = (float)(base + s + 1);
      x3[2 * b + 1] = __expf((row[s] - t.M) * t.invT);
    }
  }
}

// phase 4: every rank takes the picked token, its probability and the mu update
__global__ void tp_miro4_kernel(const SampleRow* __restrict__ params, float* __restrict__ mu,
                                const float* __restrict__ X2, const float* __restrict__ X3, int world, int B,
                                int* __restrict__ out_tok) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const SampleRow P = params[b];
  if (!tp_miro_row(P)) return;
  float zk = 0.f, id = 0.f, es = 0.f;
  for (int r = 0; r < world; ++r) {
    zk += X2[(long)r * B + b];
    id += X3[((long)r * B + b) * 2];
    es += X3[((long)r * B + b) * 2 + 1];
  }
  const int tok = (int)id - 1;
  out_tok[b] = tok;
  if (tok >= 0 && zk > 0.f && es > 0.f) mu[b] = mu[b] - P.eta * (-log2f(es / zk) - P.tau);
}

}  // namespace la

extern "C" int la_pen_push(const int* next, int B, int* hist, int hist_ld, int* cnt, int* len, const int* cap,
                           void* stream) {
  hipLaunchKernelGGL(la::pen_push_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, next, B, hist,
                     hist_ld, cnt, len, cap);
  return (int)hipGetLastError();
}

extern "C" int la_sample(const float* logits, long ld, int B, int V, const void* params, float* mu, int* out_tok,
                         float* out_p, void* stream) {
  hipLaunchKernelGGL(la::sample_kernel, dim3(B), dim3(la::SMP_T), 0, (hipStream_t)stream, logits, ld, V,
                     (const la::SampleRow*)params, mu, out_tok, out_p);
  return (int)hipGetLastError();
}

extern "C" int la_grammar_mask(float* logits, long ld, int B, int V, const int* slot, const unsigned char* pool,
                               long pool_ld, void* stream) {
  hipLaunchKernelGGL(la::grammar_mask_kernel, dim3(32, B), dim3(256), 0, (hipStream_t)stream, logits, ld, V, slot,
                     pool, pool_ld);
  return (int)hipGetLastError();
}

extern "C" int la_grammar_advance(const int* tok, int* slot, const short* next, int V, int B, void* stream) {
  hipLaunchKernelGGL(la::grammar_advance_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, tok, slot,
                     next, V, B);
  return (int)hipGetLastError();
}

extern "C" int la_penalties(float* logits, long ld, int B, const int* hist, int hist_ld, const int* hist_len,
                            const float* pen, int nl_token, const int* penalize_nl, void* stream) {
  hipLaunchKernelGGL(la::penalties_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ld, hist, hist_ld,
                     hist_len, pen, nl_token, penalize_nl, 0, 0x7fffffff);
  return (int)hipGetLastError();
}

extern "C" int la_sample_row_bytes() { return (int)sizeof(la::SampleRow); }

// Penalties on a vocabulary shard: history tokens outside [col0, col0 + ncols) are skipped and the
// rest index logits[t - col0] (tensor-parallel rows hold only their columns).
extern "C" int la_penalties_cols(float* logits, long ld, int B, const int* hist, int hist_ld, const int* hist_len,
                                 const float* pen, int nl_token, const int* penalize_nl, int col0, int ncols,
                                 void* stream) {
  hipLaunchKernelGGL(la::penalties_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ld, hist, hist_ld,
                     hist_len, pen, nl_token, penalize_nl, col0, ncols);
  return (int)hipGetLastError();
}

extern "C" int la_tp_topc(const float* logits, long ld, int B, int Vs, int C, int base, float* out, void* stream) {
  if (C < 1 || C > 1024 || Vs < 1) return -1;
  hipLaunchKernelGGL(la::tp_topc_kernel, dim3(B), dim3(la::SMP_T), 0, (hipStream_t)stream, logits, ld, Vs, C, base,
                     out);
  return (int)hipGetLastError();
}

// phase 1..4 of the vocabulary-parallel mirostat 2 sampler (see tp_miro*_kernel); x1/x2/x3 are the
// exchange buffers [world][B][3 | 1 | 2] after their all-reduce (phase p writes its own slot of
// the next one: own1 / own2 / own3 = this rank's slot).
extern "C" int la_tp_mirostat(int phase, const float* logits, long ld, int B, int Vs, int base, int world, int rank,
                              const void* params, float* mu, const float* x1, const float* x2, const float* x3,
                              float* own, int* out_tok, void* stream) {
  using namespace la;
  hipStream_t st = (hipStream_t)stream;
  const SampleRow* P = (const SampleRow*)params;
  switch (phase) {
    case 1: hipLaunchKernelGGL(tp_miro1_kernel, dim3(B), dim3(SMP_T), 0, st, logits, ld, Vs, base, P, own); break;
    case 2:
      hipLaunchKernelGGL(tp_miro2_kernel, dim3(B), dim3(SMP_T), 0, st, logits, ld, Vs, base, P, mu, x1, world, B, own);
      break;
    case 3:
      hipLaunchKernelGGL(tp_miro3_kernel, dim3(B), dim3(SMP_T), 0, st, logits, ld, Vs, base, P, mu, x1, x2, world,
                         rank, B, own);
      break;
    case 4:
      hipLaunchKernelGGL(tp_miro4_kernel, dim3((B + 255) / 256), dim3(256), 0, st, P, mu, x2, x3, world, B, out_tok);
      break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
