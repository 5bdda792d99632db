// Occupancy probe (not shipped): how many workgroups of a given size / dynamic LDS run on one
// CU at once.  Each block spins ~5 us; wave 0 records its start time and CU placement.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int V>
__global__ void spin(unsigned long long* st, int lds_words) {
  extern __shared__ float lds[];
  if constexpr (V == 64) asm volatile("v_mov_b32 v63, 0" ::: "v63");
  if constexpr (V == 72) asm volatile("v_mov_b32 v71, 0" ::: "v71");
  if constexpr (V == 80) asm volatile("v_mov_b32 v79, 0" ::: "v79");
  if constexpr (V == 96) asm volatile("v_mov_b32 v95, 0" ::: "v95");
  if constexpr (V == 128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
  for (int i = threadIdx.x; i < lds_words; i += blockDim.x) lds[i] = (float)i;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 2] = t0;
    st[blockIdx.x * 2 + 1] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                             ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < 500) {}   // 5 us at 100 MHz
  if (lds_words && lds[(threadIdx.x * 7) % lds_words] < -1.f) st[0] = 0;   // keep the LDS live
}

template <int V>
int run(unsigned long long* d, int nb, int thr, int kbv) {
  hipFuncSetAttribute((const void*)spin<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipMemset(d, 0, nb * 16);
  hipLaunchKernelGGL(spin<V>, dim3(nb), dim3(thr), kbv * 1024, 0, d, kbv * 256);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<unsigned long long> h(nb * 2);
  hipMemcpy(h.data(), d, nb * 16, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < nb; ++b) t0 = std::min(t0, h[2 * b]);
  std::vector<int> first(8 * 8 * 2 * 16, 0);
  int nfirst = 0;
  for (int b = 0; b < nb; ++b) {
    if ((h[2 * b] - t0) * 0.01 > 2.0) continue;
    const unsigned hw = (unsigned)h[2 * b + 1], xcc = (unsigned)(h[2 * b + 1] >> 32) & 0xf;
    const int key = (((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16) + ((hw >> 8) & 0xf);
    first[key]++;
    ++nfirst;
  }
  int mx = 0, ncu = 0;
  for (int v : first) { mx = std::max(mx, v); ncu += v > 0; }
  printf("vgprs %3d threads %4d lds %3d KB: %d blocks in the first 2 us on %d CUs, max %d per CU\n",
         V, thr, kbv, nfirst, ncu, mx);
  return 0;
}

int main() {
  const int nb = 256 * 8;
  unsigned long long* d;
  hipMalloc(&d, nb * 16);
  int rc = 0;
  rc |= run<0>(d, nb, 512, 35);
  rc |= run<64>(d, nb, 512, 35);
  rc |= run<72>(d, nb, 512, 35);
  rc |= run<80>(d, nb, 512, 35);
  rc |= run<96>(d, nb, 512, 35);
  rc |= run<128>(d, nb, 512, 35);
  rc |= run<72>(d, nb, 512, 0);
  rc |= run<72>(d, nb, 256, 0);
  rc |= run<128>(d, nb, 256, 0);
  return rc;
}
