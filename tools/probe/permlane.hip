// Verify v_permlane16/32_swap semantics (cross-row column reduction building block).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const float* in, float* out) {
  const int l = threadIdx.x;
  float v = in[l];
  // variant A: builtin with two distinct copies
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  out[64 + l] = x;
  out[128 + l] = y;
  float s = x + y;
  float p = s, q = s;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p), "+v"(q));
  out[l] = p + q;
}
int main() {
  float h[64], r[192]; float *d, *o;
  for (int i = 0; i < 64; ++i) h[i] = (float)(1 << (i % 16)) + 100000.f * (i / 16);
  hipMalloc(&d, 256); hipMalloc(&o, 768);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(r, o, 768, hipMemcpyDeviceToHost);
  int ok = 1;
  for (int l = 0; l < 64; ++l) {
    float want = h[l % 16] + h[l % 16 + 16] + h[l % 16 + 32] + h[l % 16 + 48];
    if (r[l] != want) ok = 0;
  }
  printf("sum over rows %s; lane0 %.0f want %.0f; a0[0]=%.0f a0[32]=%.0f a1[0]=%.0f a1[32]=%.0f\n",
         ok ? "OK" : "WRONG", r[0], h[0] + h[16] + h[32] + h[48], r[64], r[96], r[128], r[160]);
  return ok ? 0 : 1;
}
