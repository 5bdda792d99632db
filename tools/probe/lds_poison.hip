// Diagnostic helper: fill the LDS of every CU with a value (exposes kernels that read LDS
// they never wrote).  hipcc --offload-arch=gfx950 -O3 -fPIC -shared lds_poison.hip -o liblds_poison.so
#include <hip/hip_runtime.h>
__global__ __launch_bounds__(1024) void k_poison(float v, int words) {
  extern __shared__ float s[];
  for (int i = threadIdx.x; i < words; i += 1024) s[i] = v;
  __syncthreads();
  if (s[threadIdx.x] == 12345.f) s[0] = 1.f;   // keep the stores
}
extern "C" int lds_poison(float v, void* stream) {
  const int bytes = 160 * 1024;
  hipFuncSetAttribute((const void*)k_poison, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  hipLaunchKernelGGL(k_poison, dim3(2048), dim3(1024), bytes, (hipStream_t)stream, v, bytes / 4);
  return (int)hipGetLastError();
}
