// Mamba (selective state-space) decode step, gfx950.
//
// One recurrent step per sequence and layer, between the library GEMVs of in_proj / x_proj /
// dt_proj / out_proj (models/mamba.py):
//   la_mamba_conv_step : rolls the depthwise causal-conv window by one token, convolves, adds the
//                        bias and applies SiLU  ->  x [B, I]
//   la_mamba_ssm_step  : softplus(dt), h = exp(dt * A) * h + dt * B * x, y = <h, C> + D * x,
//                        y *= SiLU(z)            ->  y [B, I]   (state h updated in place)
// Both are memory-trivial (a few KB per sequence per layer); one lane per (sequence, channel),
// 64-wide waves over the channel axis, every operand read once with unit stride across lanes.
// Reference behaviour: the `mamba` Python backend (backend/python/mamba/backend.py) running
// mamba_ssm's selective_state_update; numerics are checked against transformers' Mamba slow
// path and models/mamba.py's PyTorch step (tests/test_mamba.py).
#include <hip/hip_runtime.h>

namespace la {

__device__ __forceinline__ float silu(float v) { return v / (1.0f + __expf(-v)); }
__device__ __forceinline__ float softplus(float v) { return v > 20.0f ? v : log1pf(__expf(v)); }

// conv_state [B, I, K] (fp32, oldest first); xz [B, 2I] fp32 (x = first half); w [I, K]; bias [I] or null.
__global__ void __launch_bounds__(256) mamba_conv_step_kernel(float* __restrict__ conv_state,
                                                              const float* __restrict__ xz, long xz_ld,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ x_out, int B, int I, int K) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * I) return;
  const int b = (int)(idx / I), i = (int)(idx % I);
  float* st = conv_state + idx * K;
  const float* wi = w + (long)i * K;
  float acc = bias ? bias[i] : 0.0f;
  for (int k = 0; k < K - 1; ++k) {
    const float v = st[k + 1];
    st[k] = v;
    acc += v * wi[k];
  }
  const float xn = xz[(long)b * xz_ld + i];
  st[K - 1] = xn;
  acc += xn * wi[K - 1];
  x_out[idx] = silu(acc);
}

// ssm_state [B, I, N] fp32; x [B, I]; dt [B, I] (dt_proj output incl. bias, pre-softplus);
// bc [B, ld_bc] with B at offset off_b and C at off_c (N each); A [I, N] = -exp(A_log); D [I];
// z = xz[:, I:2I]; y [B, I].
__global__ void __launch_bounds__(256) mamba_ssm_step_kernel(float* __restrict__ ssm_state,
                                                             const float* __restrict__ x,
                                                             const float* __restrict__ dt_in,
                                                             const float* __restrict__ bc, long bc_ld, int off_b,
                                                             int off_c, const float* __restrict__ A,
                                                             const float* __restrict__ Dv,
                                                             const float* __restrict__ xz, long xz_ld,
                                                             float* __restrict__ y, int B, int I, int N) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * I) return;
  const int b = (int)(idx / I), i = (int)(idx % I);
  const float dt = softplus(dt_in[idx]);
  const float xv = x[idx];
  const float* Bm = bc + (long)b * bc_ld + off_b;
  const float* Cm = bc + (long)b * bc_ld + off_c;
  const float* Ai = A + (long)i * N;
  float* h = ssm_state + idx * N;
  float acc = 0.0f;
  for (int n = 0; n < N; ++n) {
    const float hn = __expf(dt * Ai[n]) * h[n] + dt * Bm[n] * xv;
    h[n] = hn;
    acc += hn * Cm[n];
  }
  acc += Dv[i] * xv;
  y[idx] = acc * silu(xz[(long)b * xz_ld + I + i]);
}

}  // namespace la

extern "C" int la_mamba_conv_step(float* conv_state, const float* xz, long xz_ld, const float* w, const float* bias,
                                  float* x_out, int B, int I, int K, void* stream) {
  if (B <= 0 || I <= 0 || K <= 0 || K > 64) return (int)hipErrorInvalidValue;
  const long n = (long)B * I;
  hipLaunchKernelGGL(la::mamba_conv_step_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, conv_state, xz, xz_ld, w, bias, x_out, B, I, K);
  return (int)hipGetLastError();
}

extern "C" int la_mamba_ssm_step(float* ssm_state, const float* x, const float* dt, const float* bc, long bc_ld,
                                 int off_b, int off_c, const float* A, const float* Dv, const float* xz, long xz_ld,
                                 float* y, int B, int I, int N, void* stream) {
  if (B <= 0 || I <= 0 || N <= 0 || N > 256) return (int)hipErrorInvalidValue;
  const long n = (long)B * I;
  hipLaunchKernelGGL(la::mamba_ssm_step_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ssm_state, x, dt, bc, bc_ld, off_b, off_c, A, Dv, xz, xz_ld, y, B, I, N);
  return (int)hipGetLastError();
}
