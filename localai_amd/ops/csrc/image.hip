// LLaVA / CLIP image preprocessing on the device (the reference does it on the CPU
// in llama.cpp's clip.cpp / our former PIL path): resize (PIL's separable BICUBIC resample,
// bit-exact: same coefficient tables, same 22-bit fixed-point accumulation, same uint8 rounding
// of the horizontal pass), letterbox / centre-crop placement on a canvas, mean/std normalisation
// and the split into S x S tiles of the vision tower's input -- two launches per resized image
// instead of a host resize + crop + paste + normalise + copy per tile.
//
// Pass 1 (la_img_resample_h): uint8 HWC [H][W][3] -> uint8 [H][OW][3], each output column a
//   weighted sum of ksize source columns (int32 coefficients precomputed on the host exactly as
//   PIL's precompute_coeffs + normalize_coeffs_8bpc).
// Pass 2 (la_img_resample_v_tiles): uint8 [H][OW][3] -> fp32 tiles [t0 + tile][3][S][S]: canvas
//   pixel (cy, cx) shows resized pixel (cy - oy, cx - ox) (oy / ox < 0 crops, > 0 letterboxes) or
//   the fill colour outside it; each value is resampled vertically (same fixed point), then
//   (v / 255 - mean[c]) / std[c].
#include "common.h"

namespace la {

constexpr int IMG_PREC = 22;  // PIL PRECISION_BITS = 32 - 8 - 2

LA_DEV uint8_t img_clip8(int ss) {
  const int v = ss >> IMG_PREC;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ __launch_bounds__(256) void img_resample_h_kernel(const uint8_t* __restrict__ src, int H, int W,
                                                             uint8_t* __restrict__ dst, int OW,
                                                             const int* __restrict__ bounds,
                                                             const int* __restrict__ coef, int ksize) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // one output pixel (all 3 channels)
  if (i >= (long)H * OW) return;
  const int y = (int)(i / OW), x = (int)(i % OW);
  const int xmin = bounds[2 * x], xn = bounds[2 * x + 1];
  const int* k = coef + (long)x * ksize;
  const uint8_t* row = src + ((long)y * W + xmin) * 3;
  int s0 = 1 << (IMG_PREC - 1), s1 = s0, s2 = s0;
  for (int j = 0; j < xn; ++j) {
    const int w = k[j];
    s0 += row[3 * j] * w;
    s1 += row[3 * j + 1] * w;
    s2 += row[3 * j + 2] * w;
  }
  uint8_t* o = dst + i * 3;
  o[0] = img_clip8(s0);
  o[1] = img_clip8(s1);
  o[2] = img_clip8(s2);
}

struct ImgPlace {
  int OH, OW;         // resized image
  int CH, CW;         // canvas
  int oy, ox;         // resized image origin on the canvas
  int S, t0;          // tile side, first tile index
  float mean[3], inv_std[3];
  int fill[3];        // uint8 fill colour outside the image
};

__global__ __launch_bounds__(256) void img_resample_v_tiles_kernel(const uint8_t* __restrict__ src,
                                                                   const int* __restrict__ bounds,
                                                                   const int* __restrict__ coef, int ksize,
                                                                   ImgPlace P, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // one canvas pixel
  if (i >= (long)P.CH * P.CW) return;
  const int cy = (int)(i / P.CW), cx = (int)(i % P.CW);
  const int y = cy - P.oy, x = cx - P.ox;
  int v[3];
  if (y >= 0 && y < P.OH && x >= 0 && x < P.OW) {
    const int ymin = bounds[2 * y], yn = bounds[2 * y + 1];
    const int* k = coef + (long)y * ksize;
    int s0 = 1 << (IMG_PREC - 1), s1 = s0, s2 = s0;
    for (int j = 0; j < yn; ++j) {
      const uint8_t* p = src + ((long)(ymin + j) * P.OW + x) * 3;
      const int w = k[j];
      s0 += p[0] * w;
      s1 += p[1] * w;
      s2 += p[2] * w;
    }
    v[0] = img_clip8(s0);
    v[1] = img_clip8(s1);
    v[2] = img_clip8(s2);
  } else {
    v[0] = P.fill[0];
    v[1] = P.fill[1];
    v[2] = P.fill[2];
  }
  const int tiles_x = P.CW / P.S;
  const int t = P.t0 + (cy / P.S) * tiles_x + cx / P.S;
  const int ty = cy % P.S, tx = cx % P.S;
  const long plane = (long)P.S * P.S;
  float* o = out + (long)t * 3 * plane + (long)ty * P.S + tx;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c * plane] = ((float)v[c] * (1.0f / 255.0f) - P.mean[c]) * P.inv_std[c];
}

}  // namespace la

extern "C" int la_img_resample_h(const void* src, int H, int W, void* dst, int OW, const int* bounds, const int* coef,
                                 int ksize, void* stream) {
  if (H < 1 || W < 1 || OW < 1 || ksize < 1) return -1;
  const long n = (long)H * OW;
  hipLaunchKernelGGL(la::img_resample_h_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)src, H, W, (uint8_t*)dst, OW, bounds, coef, ksize);
  return (int)hipGetLastError();
}

extern "C" int la_img_resample_v_tiles(const void* src, int OH, int OW, const int* bounds, const int* coef, int ksize,
                                       int CH, int CW, int oy, int ox, int S, int t0, const float* mean,
                                       const float* std_, const int* fill, void* out, void* stream) {
  if (OH < 1 || OW < 1 || S < 1 || CH % S || CW % S || ksize < 1) return -1;
  la::ImgPlace P{OH, OW, CH, CW, oy, ox, S, t0, {mean[0], mean[1], mean[2]},
                 {1.f / std_[0], 1.f / std_[1], 1.f / std_[2]}, {fill[0], fill[1], fill[2]}};
  const long n = (long)CH * CW;
  hipLaunchKernelGGL(la::img_resample_v_tiles_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const uint8_t*)src, bounds, coef, ksize, P, (float*)out);
  return (int)hipGetLastError();
}
