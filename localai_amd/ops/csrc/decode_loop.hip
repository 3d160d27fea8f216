// Device-resident multi-step decode (no host round trip between decode steps).
//
// The reference's llama.cpp server loop copies logits to the host, samples there and
// rebuilds the batch every token.  Here one captured hipGraph = forward + logit bias +
// sampler + `advance`, and the graph is replayed K times back to back: `advance` feeds the
// sampled token back as the next input, bumps positions / sequence lengths, computes the next
// KV slot from the (pre-reserved) block table, bumps each row's Philox counter and records the
// token in a [K, B] history the host reads once per K steps.
#include "common.h"

namespace la {

struct SampleRowHdr {  // must match sampling.hip SampleRow
  float temp, top_p, min_p, typical_p, tfs_z, tau, eta;
  int top_k, mirostat, pad;
  unsigned long long seed, counter;
};

// logits[row, col] += val for the first *count entries (ignore_eos bans, logit_bias).
__global__ void __launch_bounds__(256) logit_bias_kernel(float* __restrict__ logits, long ld,
                                                         const int* __restrict__ rows, const int* __restrict__ cols,
                                                         const float* __restrict__ vals, const int* __restrict__ count,
                                                         int cap) {
  const int n = min(*count, cap);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&logits[(long)rows[i] * ld + cols[i]], vals[i]);  // entries may repeat a (row, col)
}

// One workgroup: rows are independent; thread 0 bumps the step counter after all rows read it.
__global__ void __launch_bounds__(1024) decode_advance_kernel(
    const int* __restrict__ next_tok, int* __restrict__ tok, int* __restrict__ pos, int* __restrict__ lens,
    int* __restrict__ slots, const int* __restrict__ bt, int bt_ld, int BS, int B, int* __restrict__ hist,
    int hist_cap, int* __restrict__ step, SampleRowHdr* __restrict__ prm) {
  const int s = *step;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int t = next_tok[b];
    if (s < hist_cap) hist[(long)s * B + b] = t;
    if (slots[b] < 0) continue;  // padding row: stays parked on (pos 0, no KV write)
    tok[b] = t;
    const int p = pos[b] + 1;
    pos[b] = p;
    lens[b] = p + 1;
    slots[b] = bt[(long)b * bt_ld + p / BS] * BS + (p % BS);
    prm[b].counter += 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) *step = s + 1;
}

}  // namespace la

extern "C" int la_logit_bias(float* logits, long ld, const int* rows, const int* cols, const float* vals,
                             const int* count, int cap, void* stream) {
  if (cap <= 0) return 0;
  const int grid = min((cap + 255) / 256, 256);
  hipLaunchKernelGGL(la::logit_bias_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, logits, ld, rows, cols,
                     vals, count, cap);
  return (int)hipGetLastError();
}

extern "C" int la_decode_advance(const int* next_tok, int* tok, int* pos, int* lens, int* slots, const int* bt,
                                 int bt_ld, int BS, int B, int* hist, int hist_cap, int* step, void* prm,
                                 void* stream) {
  hipLaunchKernelGGL(la::decode_advance_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, next_tok, tok, pos,
                     lens, slots, bt, bt_ld, BS, B, hist, hist_cap, step, (la::SampleRowHdr*)prm);
  return (int)hipGetLastError();
}
