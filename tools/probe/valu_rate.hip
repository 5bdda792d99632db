// valu_rate.hip -- issue rate of independent VALU ops on gfx950 at the step kernel's
// occupancy (one 1024-thread block per CU = 4 waves per SIMD) and at 1 / 2 waves per SIMD.
// hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void k_rate(float* out, int iters, float s) {
  f2 a[8];
  float b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = (f2){threadIdx.x * 1e-3f + i, i * 0.5f}; b[i] = a[i].x; }
  const f2 m = {s, s * 0.5f}, c = {0.25f, 0.125f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (KIND == 0) a[i] = __builtin_elementwise_fma(a[i], m, c);   // v_pk_fma_f32
        else if constexpr (KIND == 1) b[i] = fmaf(b[i], s, 0.25f);               // v_fma_f32
        else if constexpr (KIND == 3) {                                          // v_fma_f64
          double d = (double)b[i];
          d = fma(d, (double)s, 0.25);
          b[i] = (float)d;
        } else if constexpr (KIND == 4) {                                        // v_pk_fma_f16
          uint32_t u = __builtin_bit_cast(uint32_t, b[i]), r2;
          asm volatile("v_pk_fma_f16 %0, %1, %2, %3" : "=v"(r2) : "v"(u), "v"(0x3c003c00u), "v"(u));
          b[i] = __builtin_bit_cast(float, r2);
        } else if constexpr (KIND == 5) {                                        // v_dot2_f32_bf16
          const uint32_t u = __builtin_bit_cast(uint32_t, a[i].y);
          float r2;
          asm volatile("v_dot2_f32_bf16 %0, %1, %2, %3" : "=v"(r2) : "v"(u), "v"(0x3f803f80u), "v"(b[i]));
          b[i] = r2;
        } else if constexpr (KIND == 6) {                                        // cvt f32 -> bf16 x2
          uint32_t r2;
          asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r2) : "v"(b[i]), "v"(a[i].x));
          b[i] = __builtin_bit_cast(float, r2 ^ 0x00010001u);
        } else {                                                                  // pk_mul clamp
          f2 r2;
          asm volatile("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(r2) : "v"(a[i]), "v"(m));
          a[i] = r2;
        }
      }
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += a[i].x + a[i].y + b[i];
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  float* out;
  hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  const char* names[7] = {"v_pk_fma_f32", "v_fma_f32", "v_pk_mul_f32 clamp", "f64 fma+cvt",
                          "v_pk_fma_f16", "v_dot2_f32_bf16", "v_cvt_pk_bf16_f32"};
  for (int kind = 0; kind < 7; ++kind) {
    for (int thr : {256, 512, 1024}) {
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_rate<0>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else if (kind == 1) hipLaunchKernelGGL(k_rate<1>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else if (kind == 2) hipLaunchKernelGGL(k_rate<2>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else if (kind == 3) hipLaunchKernelGGL(k_rate<3>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else if (kind == 4) hipLaunchKernelGGL(k_rate<4>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else if (kind == 5) hipLaunchKernelGGL(k_rate<5>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
        else hipLaunchKernelGGL(k_rate<6>, dim3(256), dim3(thr), 0, 0, out, iters, 0.999f);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double winst = (double)iters * 16 * 8 * (thr / 64);   // wave-instructions per CU
      const double ns_per = ms * 1e6 / (winst / 4);                  // per SIMD
      printf("%-20s waves/SIMD %d: %.3f ms, %.3f ns per wave-instr per SIMD (%.2f cyc @2.4GHz)\n",
             names[kind], thr / 256, ms, ns_per, ns_per * 2.4);
    }
  }
  return 0;
}
