// Microbenchmark: latency of a data exchange between the two blocks of a commit pair
// placed on the same XCD (blockIdx = (c/8)*16 + h*8 + c%8), 1024 threads + 144 KiB LDS per
// block (one block per CU), with the L2 dirtied by unrelated stores first.  Each exchange:
// write 16 KiB, release fence, flag store; spin on the partner's flag (bounded), acquire,
// read the partner's 16 KiB and verify.  hipcc --offload-arch=gfx950 -O3 xchg.hip -o xchg
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int NEX = 6, WORDS = 4096;

__global__ __launch_bounds__(1024) void k_pair(float* xbuf, unsigned* flags, float* dirty,
                                               unsigned long long* stamps, int* errs, int B,
                                               int mode) {
  extern __shared__ float lds[];
  const int blk = blockIdx.x;
  const int c = (blk / 16) * 8 + (blk % 8), h = (blk / 8) & 1;
  if (c >= B) return;
  const int t = threadIdx.x;
  for (int i = t; i < 36 * 1024; i += 1024) lds[i] = (float)i;
  // dirty the L2 with unrelated stores (like the step kernel's outputs)
  for (int i = t; i < 64 * 1024; i += 1024) dirty[(size_t)blk * 64 * 1024 + i] = (float)(i + blk);
  __syncthreads();
  unsigned* myf = flags + 2 * c + h;
  unsigned* pf = flags + 2 * c + (1 - h);
  float* mine = xbuf + ((size_t)c * 2 + h) * WORDS;
  const float* theirs = xbuf + ((size_t)c * 2 + 1 - h) * WORDS;
  __shared__ unsigned long long st[NEX + 1];
  __shared__ int bad;
  if (t == 0) { bad = 0; st[0] = __builtin_amdgcn_s_memrealtime(); }
  for (int e = 1; e <= NEX; ++e) {
    for (int i = t; i < WORDS; i += 1024) mine[i] = (float)(e * 100000 + h * 10000 + i) + lds[i];
    __syncthreads();
    if (t == 0) {
      if (mode == 0) {
        __threadfence();                                            // agent-scope release
        __hip_atomic_store(myf, (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_store(myf, (unsigned)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(pf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)e) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { bad = 1000; break; }   // 200 ms
      }
    }
    __syncthreads();
    int lb = 0;
    for (int i = t; i < WORDS; i += 1024) {
      const float want = (float)(e * 100000 + (1 - h) * 10000 + i) + lds[i];
      lb += theirs[i] != want;
    }
    if (lb) atomicAdd(&bad, lb);
    __syncthreads();
    if (t == 0) st[e] = __builtin_amdgcn_s_memrealtime();
  }
  if (t == 0) {
    for (int e = 0; e <= NEX; ++e) stamps[(size_t)blk * (NEX + 1) + e] = st[e];
    errs[blk] = bad;
  }
}

int main() {
  const int B = 100, G = (B + 7) / 8 * 16;
  float *xbuf, *dirty;
  unsigned* flags;
  unsigned long long* stamps;
  int* errs;
  hipMalloc(&xbuf, (size_t)B * 2 * WORDS * 4);
  hipMalloc(&dirty, (size_t)G * 64 * 1024 * 4);
  hipMalloc(&flags, (size_t)B * 2 * 4);
  hipMalloc(&stamps, (size_t)G * (NEX + 1) * 8);
  hipMalloc(&errs, (size_t)G * 4);
  hipFuncSetAttribute((const void*)k_pair, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);
  unsigned long long* hs = (unsigned long long*)malloc((size_t)G * (NEX + 1) * 8);
  int* he = (int*)malloc(G * 4);
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(flags, 0, (size_t)B * 2 * 4);
      hipMemset(errs, 0, (size_t)G * 4);
      hipEvent_t a, b;
      hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_pair, dim3(G), dim3(1024), 144 * 1024, 0, xbuf, flags, dirty, stamps,
                         errs, B, mode);
      hipEventRecord(b);
      if (hipEventSynchronize(b) != hipSuccess) { printf("kernel failed\n"); return 1; }
      float ms; hipEventElapsedTime(&ms, a, b);
      hipMemcpy(hs, stamps, (size_t)G * (NEX + 1) * 8, hipMemcpyDeviceToHost);
      hipMemcpy(he, errs, (size_t)G * 4, hipMemcpyDeviceToHost);
      double sum = 0; int n = 0, bad = 0;
      for (int blk = 0; blk < G; ++blk) {
        const int c = (blk / 16) * 8 + (blk % 8);
        if (c >= B) continue;
        bad += he[blk];
        for (int e = 1; e <= NEX; ++e) { sum += (double)(hs[blk * (NEX + 1) + e] - hs[blk * (NEX + 1) + e - 1]); ++n; }
      }
      printf("mode %d rep %d: kernel %.1f us, mean exchange %.2f us, errors %d\n", mode, rep,
             ms * 1e3, sum / n * 0.01, bad);
    }
  }
  return 0;
}
