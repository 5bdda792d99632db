// Calibration of the gfx950 FP32 FLOP counters against kernels of known instruction
// counts (one kernel per instruction form, 1024 waves x N instructions each):
//   rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS
//             SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32
//             SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU -- ./flops_cal
// hipcc --offload-arch=gfx950 -O3 flops_cal.hip -o flops_cal
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int N = 1000;

__global__ __launch_bounds__(256) void cal_fma(float* out) {
  float a = threadIdx.x, b = 1.0001f, c = 0.5f;
  for (int i = 0; i < N; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void cal_pk_fma(float* out) {
  f2 a = {(float)threadIdx.x, 1.f}, b = {1.0001f, 1.0002f}, c = {0.5f, 0.25f};
  for (int i = 0; i < N; ++i)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  out[blockIdx.x * 256 + threadIdx.x] = a.x + a.y;
}
__global__ __launch_bounds__(256) void cal_add(float* out) {
  float a = threadIdx.x, b = 1.0001f;
  for (int i = 0; i < N; ++i) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void cal_pk_add(float* out) {
  f2 a = {(float)threadIdx.x, 1.f}, b = {1.0001f, 1.0002f};
  for (int i = 0; i < N; ++i) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  out[blockIdx.x * 256 + threadIdx.x] = a.x + a.y;
}
__global__ __launch_bounds__(256) void cal_mul(float* out) {
  float a = threadIdx.x, b = 1.0001f;
  for (int i = 0; i < N; ++i) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void cal_exp(float* out) {
  float a = threadIdx.x * 1e-3f;
  for (int i = 0; i < N; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(a));
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void cal_max(float* out) {
  float a = threadIdx.x, b = 1.0001f;
  for (int i = 0; i < N; ++i) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void cal_mfma(float* out) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 0.5f;
  for (int i = 0; i < N; ++i)
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
  float* d;
  if (hipMalloc(&d, 256 * 256 * sizeof(float)) != hipSuccess) return 1;
  const dim3 g(256), b(256);   // 1024 waves per kernel
  hipLaunchKernelGGL(cal_fma, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_pk_fma, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_add, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_pk_add, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_mul, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_exp, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_max, g, b, 0, 0, d);
  hipLaunchKernelGGL(cal_mfma, g, b, 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("waves per kernel 1024, instructions per wave %d\n", N);
  hipFree(d);
  return 0;
}
