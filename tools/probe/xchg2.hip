// Microbenchmark: exchange latency between the two blocks of a commit pair WITHOUT an
// L2 writeback fence: data stored write-through (system-scope relaxed atomic stores ->
// global_store sc0 sc1), s_waitcnt vmcnt(0) + barrier, flag store sc0 sc1; the reader
// spins on an sc0 sc1 load, then reads the partner's words with sc0 sc1 loads (L2 miss).
// mode 4: mode 3 at agent scope (sc1 stores / loads: the L2 of the XCD, not memory).
// mode 0: agent release fence (buffer_wbl2) + agent acquire, for comparison.
// xcd 0: partner on the same XCD (blk, blk+8); 1: different XCD (blk, blk+1).
// hipcc --offload-arch=gfx950 -O3 xchg2.hip -o xchg2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int NEX = 6;

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_pair(float* xbuf, unsigned* flags, float* dirty,
                                               unsigned long long* stamps, int* errs, int B,
                                               int mode, int xcd, int words) {
  extern __shared__ float lds[];
  const int blk = blockIdx.x;
  int c, h;
  if (xcd == 0) { c = (blk / 16) * 8 + (blk % 8); h = (blk / 8) & 1; }
  else { c = blk >> 1; h = blk & 1; }
  if (c >= B) return;
  const int t = threadIdx.x;
  for (int i = t; i < 36 * 1024; i += 1024) lds[i] = (float)i;
  for (int i = t; i < 64 * 1024; i += 1024) dirty[(size_t)blk * 64 * 1024 + i] = (float)(i + blk);
  __syncthreads();
  unsigned* myf = flags + 2 * c + h;
  unsigned* pf = flags + 2 * c + (1 - h);
    __shared__ unsigned long long st[NEX + 1];
  __shared__ int bad;
  if (t == 0) { bad = 0; st[0] = __builtin_amdgcn_s_memrealtime(); }
  __syncthreads();
  if (mode == 3 || mode == 4) {
    // mode 3: mode 2 with two (value, tag) pairs per 16-byte write-through store / load
    // (global_store_dwordx4 / global_load_dwordx4 sc0 sc1): half the round trips
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    u4* xb = reinterpret_cast<u4*>(xbuf);
    const int nv = (words + 1) / 2;
    for (int e = 1; e <= NEX; ++e) {
      u4* mine = xb + (((size_t)c * 2 + h) * 2 + (e & 1)) * nv;
      const u4* theirs = xb + (((size_t)c * 2 + 1 - h) * 2 + (e & 1)) * nv;
      for (int i = t; i < nv; i += 1024) {
        const float v0 = (float)(e * 100000 + h * 10000 + 2 * i) + lds[2 * i];
        const float v1 = (float)(e * 100000 + h * 10000 + 2 * i + 1) + lds[2 * i + 1];
        const u4 w = {__float_as_uint(v0), (unsigned)e, __float_as_uint(v1), (unsigned)e};
        if (mode == 3)
          asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(mine + i), "v"(w) : "memory");
        else
          asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(mine + i), "v"(w) : "memory");
      }
      int lb = 0;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (int i = t; i < nv; i += 1024) {
        u4 w;
        do {
          if (mode == 3)
            asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(w) : "v"(theirs + i) : "memory");
          else
            asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(w) : "v"(theirs + i) : "memory");
        } while ((w.y != (unsigned)e || w.w != (unsigned)e) &&
                 __builtin_amdgcn_s_memrealtime() - t0 < 20000000ull);
        const float want0 = (float)(e * 100000 + (1 - h) * 10000 + 2 * i) + lds[2 * i];
        const float want1 = (float)(e * 100000 + (1 - h) * 10000 + 2 * i + 1) + lds[2 * i + 1];
        lb += w.y != (unsigned)e || w.w != (unsigned)e || __uint_as_float(w.x) != want0 ||
              __uint_as_float(w.z) != want1;
      }
      if (lb) atomicAdd(&bad, lb);
      __syncthreads();
      if (t == 0) st[e] = __builtin_amdgcn_s_memrealtime();
    }
  } else if (mode == 2) {
    unsigned long long* xb = reinterpret_cast<unsigned long long*>(xbuf);
    for (int e = 1; e <= NEX; ++e) {
      // double-buffered by parity (the partner may still poll round e-1's buffer)
      unsigned long long* mine = xb + (((size_t)c * 2 + h) * 2 + (e & 1)) * words;
      const unsigned long long* theirs = xb + (((size_t)c * 2 + 1 - h) * 2 + (e & 1)) * words;
      for (int i = t; i < words; i += 1024) {
        const float v = (float)(e * 100000 + h * 10000 + i) + lds[i];
        const unsigned long long w = ((unsigned long long)(unsigned)e << 32) | __float_as_uint(v);
        __hip_atomic_store(mine + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      int lb = 0;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (int i = t; i < words; i += 1024) {
        unsigned long long w;
        do {
          w = __hip_atomic_load(theirs + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } while ((unsigned)(w >> 32) != (unsigned)e &&
                 __builtin_amdgcn_s_memrealtime() - t0 < 20000000ull);
        const float want = (float)(e * 100000 + (1 - h) * 10000 + i) + lds[i];
        lb += (unsigned)(w >> 32) != (unsigned)e || __uint_as_float((unsigned)w) != want;
      }
      if (lb) atomicAdd(&bad, lb);
      __syncthreads();
      if (t == 0) st[e] = __builtin_amdgcn_s_memrealtime();
    }
  } else
  for (int e = 1; e <= NEX; ++e) {
    // double-buffered by exchange parity: the partner may still read exchange e-1
    float* mine = xbuf + (((size_t)c * 2 + h) * 2 + (e & 1)) * words;
    const float* theirs = xbuf + (((size_t)c * 2 + 1 - h) * 2 + (e & 1)) * words;
    for (int i = t; i < words; i += 1024) {
      const float v = (float)(e * 100000 + h * 10000 + i) + lds[i];
      if (mode == 0) mine[i] = v; else st_wt(mine + i, v);
    }
    if (mode != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      if (mode == 0) {
        __threadfence();
        __hip_atomic_store(myf, (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_store(myf, (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      if (mode == 0) {
        while (__hip_atomic_load(pf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)e) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { bad = 1000; break; }
        }
      } else {
        while (__hip_atomic_load(pf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < (unsigned)e) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { bad = 1000; break; }
        }
      }
    }
    __syncthreads();
    int lb = 0;
    for (int i = t; i < words; i += 1024) {
      const float want = (float)(e * 100000 + (1 - h) * 10000 + i) + lds[i];
      const float got = mode == 0 ? theirs[i] : ld_wt(theirs + i);
      lb += got != want;
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
  const int B = 100, G = (B + 7) / 8 * 16, WMAX = 4096;
  float *xbuf, *dirty;
  unsigned* flags;
  unsigned long long* stamps;
  int* errs;
  hipMalloc(&xbuf, (size_t)B * 4 * WMAX * 8);
  hipMemset(xbuf, 0, (size_t)B * 4 * WMAX * 8);
  hipMalloc(&dirty, (size_t)G * 64 * 1024 * 4);
  hipMalloc(&flags, (size_t)B * 2 * 4);
  hipMalloc(&stamps, (size_t)G * (NEX + 1) * 8);
  hipMalloc(&errs, (size_t)G * 4);
  hipFuncSetAttribute((const void*)k_pair, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);
  unsigned long long* hs = (unsigned long long*)malloc((size_t)G * (NEX + 1) * 8);
  int* he = (int*)malloc(G * 4);
  const int wl[3] = {256, 1480, 4096};
  for (int mode = 3; mode < 5; ++mode)
    for (int xcd = 0; xcd < 2; ++xcd)
      for (int wi = 0; wi < 3; ++wi) {
        const int words = wl[wi];
        const int grid = xcd == 0 ? G : 2 * B;
        double best = 1e30; int badall = 0;
        for (int rep = 0; rep < 3; ++rep) {
          hipMemset(flags, 0, (size_t)B * 2 * 4);
          hipMemset(errs, 0, (size_t)G * 4);
          hipLaunchKernelGGL(k_pair, dim3(grid), dim3(1024), 144 * 1024, 0, xbuf, flags, dirty,
                             stamps, errs, B, mode, xcd, words);
          if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
          hipMemcpy(hs, stamps, (size_t)grid * (NEX + 1) * 8, hipMemcpyDeviceToHost);
          hipMemcpy(he, errs, (size_t)grid * 4, hipMemcpyDeviceToHost);
          double sum = 0; int n = 0;
          for (int blk = 0; blk < grid; ++blk) {
            const int c = xcd == 0 ? (blk / 16) * 8 + (blk % 8) : blk >> 1;
            if (c >= B) continue;
            badall += he[blk];
            for (int e = 2; e <= NEX; ++e) { sum += (double)(hs[blk * (NEX + 1) + e] - hs[blk * (NEX + 1) + e - 1]); ++n; }
          }
          if (sum / n < best) best = sum / n;
        }
        printf("mode %d xcd %d words %5d: mean exchange %.2f us, errors %d\n", mode, xcd, words,
               best * 0.01, badall);
      }
  return 0;
}
