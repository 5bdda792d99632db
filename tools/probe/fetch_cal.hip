// Calibration of the gfx950 FETCH_SIZE / WRITE_SIZE counters against kernels of known byte
// counts, one kernel per access width / scope / stride (MI355X_MICROARCH.md: FETCH_SIZE reads
// exactly half of a 16 B/lane streaming read; other widths uncalibrated).  Each kernel touches
// a 64 MiB buffer exactly once:
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_cal ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_cal
// hipcc --offload-arch=gfx950 -O3 fetch_cal.hip -o fetch_cal
// tools/traffic_cal.py turns the two passes into bytes-per-counted-byte factors per pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr size_t BYTES = (size_t)64 << 20;
constexpr int NT = 256;
typedef float v4 __attribute__((ext_vector_type(4)));

// reads: the sum goes to one dword per thread (written to a separate small buffer)
__global__ __launch_bounds__(NT) void rd_x4(const float4* __restrict__ in, float* out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  const float4 v = in[i];
  if (v.x == -1.2345f) out[threadIdx.x] = v.y + v.z + v.w;
}
__global__ __launch_bounds__(NT) void rd_x2(const float2* __restrict__ in, float* out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  const float2 v = in[i];
  if (v.x == -1.2345f) out[threadIdx.x] = v.y;
}
__global__ __launch_bounds__(NT) void rd_x1(const float* __restrict__ in, float* out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  const float v = in[i];
  if (v == -1.2345f) out[threadIdx.x] = v;
}
// system-scope dword loads (L2 bypassed), as the block-pair exchange polls read
__global__ __launch_bounds__(NT) void rd_x1_sys(const float* __restrict__ in, float* out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  float v;
  asm volatile("global_load_dword %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(in + i));
  if (v == -1.2345f) out[threadIdx.x] = v;
}
__global__ __launch_bounds__(NT) void rd_x4_sys(const float4* __restrict__ in, float* out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  v4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(in + i));
  if (v.x == -1.2345f) out[threadIdx.x] = v.y + v.z + v.w;
}
// one dword per 64 B / 128 B line: whole lines move for 1/16 or 1/32 of their bytes
__global__ __launch_bounds__(NT) void rd_x1_s64(const float* __restrict__ in, float* out) {
  const size_t i = ((size_t)blockIdx.x * NT + threadIdx.x) * 16;
  const float v = in[i];
  if (v == -1.2345f) out[threadIdx.x] = v;
}
__global__ __launch_bounds__(NT) void rd_x1_s128(const float* __restrict__ in, float* out) {
  const size_t i = ((size_t)blockIdx.x * NT + threadIdx.x) * 32;
  const float v = in[i];
  if (v == -1.2345f) out[threadIdx.x] = v;
}
// writes
__global__ __launch_bounds__(NT) void wr_x4(float4* __restrict__ o) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  o[i] = make_float4(i, 1.f, 2.f, 3.f);
}
__global__ __launch_bounds__(NT) void wr_x1(float* __restrict__ o) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  o[i] = (float)i;
}
__global__ __launch_bounds__(NT) void wr_x1_sys(float* __restrict__ o) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  const float v = (float)i;
  asm volatile("global_store_dword %0, %1, off sc0 sc1" : : "v"(o + i), "v"(v) : "memory");
}
__global__ __launch_bounds__(NT) void wr_x4_sys(float4* __restrict__ o) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  const v4 v = {(float)i, 1.f, 2.f, 3.f};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(o + i), "v"(v) : "memory");
}
// one dword per 64 B line (partial-line writes, as a strided partial-gradient store)
__global__ __launch_bounds__(NT) void wr_x1_s64(float* __restrict__ o) {
  const size_t i = ((size_t)blockIdx.x * NT + threadIdx.x) * 16;
  o[i] = (float)i;
}

int main() {
  float *in, *o, *sink;
  if (hipMalloc(&in, BYTES) != hipSuccess || hipMalloc(&o, BYTES) != hipSuccess ||
      hipMalloc(&sink, 4096) != hipSuccess)
    return 1;
  if (hipMemset(in, 0, BYTES) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 2;
  const size_t n4 = BYTES / 16, n2 = BYTES / 8, n1 = BYTES / 4;
  hipLaunchKernelGGL(rd_x4, dim3(n4 / NT), dim3(NT), 0, 0, (const float4*)in, sink);
  hipLaunchKernelGGL(rd_x2, dim3(n2 / NT), dim3(NT), 0, 0, (const float2*)in, sink);
  hipLaunchKernelGGL(rd_x1, dim3(n1 / NT), dim3(NT), 0, 0, in, sink);
  hipLaunchKernelGGL(rd_x1_sys, dim3(n1 / NT), dim3(NT), 0, 0, in, sink);
  hipLaunchKernelGGL(rd_x4_sys, dim3(n4 / NT), dim3(NT), 0, 0, (const float4*)in, sink);
  hipLaunchKernelGGL(rd_x1_s64, dim3(n1 / 16 / NT), dim3(NT), 0, 0, in, sink);
  hipLaunchKernelGGL(rd_x1_s128, dim3(n1 / 32 / NT), dim3(NT), 0, 0, in, sink);
  hipLaunchKernelGGL(wr_x4, dim3(n4 / NT), dim3(NT), 0, 0, (float4*)o);
  hipLaunchKernelGGL(wr_x1, dim3(n1 / NT), dim3(NT), 0, 0, o);
  hipLaunchKernelGGL(wr_x1_sys, dim3(n1 / NT), dim3(NT), 0, 0, o);
  hipLaunchKernelGGL(wr_x4_sys, dim3(n4 / NT), dim3(NT), 0, 0, (float4*)o);
  hipLaunchKernelGGL(wr_x1_s64, dim3(n1 / 16 / NT), dim3(NT), 0, 0, o);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  printf("bytes per kernel %zu (strided kernels: every 64 B / 128 B line touched once)\n", BYTES);
  hipFree(in);
  hipFree(o);
  hipFree(sink);
  return 0;
}
