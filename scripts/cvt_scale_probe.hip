// Semantics probe: does v_cvt_scalef32_pk_bf16_fp8 apply its f32 scale as a full multiply or
// only as a power of two?  Inputs: fp8 e4m3 bytes 0x00..0x0F (= b * 2^-9 exactly).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void probe(const float* scales, uint32_t* out, int ns) {
  int i = threadIdx.x;
  if (i >= ns * 8) return;
  float s = scales[i / 8];
  uint32_t src = (uint32_t)((2 * (i % 8)) | ((2 * (i % 8) + 1) << 8)) | (0x0F0E0000u);
  uint32_t r;
  asm volatile("v_cvt_scalef32_pk_bf16_fp8 %0, %1, %2" : "=v"(r) : "v"(src), "v"(s));
  out[i] = r;
}

static float bf(uint32_t h) { uint32_t u = h << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
  const int ns = 4;
  float hs[ns] = {512.0f, 512.0f * 1.37f, 512.0f * 0.0123f, 3.0f};
  float* ds; uint32_t* dout;
  hipMalloc(&ds, sizeof(hs)); hipMalloc(&dout, ns * 8 * 4);
  hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, ds, dout, ns);
  uint32_t h[ns * 8];
  hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < ns * 8; ++i) {
    int b0 = 2 * (i % 8), b1 = b0 + 1;
    float s = hs[i / 8];
    printf("scale %-10g b=%2d -> %-12g (exact %-12g)  b=%2d -> %-12g (exact %-12g)\n", s, b0, bf(h[i] & 0xFFFF),
           b0 * s / 512.0f, b1, bf(h[i] >> 16), b1 * s / 512.0f);
  }
  return 0;
}
