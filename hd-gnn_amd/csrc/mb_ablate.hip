// Ablations of the pair-tile loop structure (MODE 0, Nc=74, KK=5, SMAX=5) to find
// where the time goes.  FLAGS: 1 = skip row reduction, 2 = skip column reduction,
// 4 = skip barrier/LDS epilogue.
#include "hdgnn.hip"
namespace {
template <int FLAGS>
__global__ __launch_bounds__(1024) void mb(int N, int iters, float* out) {
  constexpr int SMAX = 5, KK = 5, NP16 = 80, LD = HS;
  __shared__ __attribute__((aligned(16))) float A[NP16 * HS], Bv[NP16 * HS], R[NP16 * HS],
      C[NP16 * HS], dl[HS];
  __shared__ float cred[4][4 * NP16 * KK];
  __shared__ uint32_t bits[NP16 * 3];
  const int t = threadIdx.x;
  for (int e = t; e < NP16 * HS; e += 1024) {
    const float v = (float)((e * 2654435761u) % 1000) * 1e-3f - 0.5f;
    A[e] = (e / HS) < N ? v : -INFINITY;
    Bv[e] = (e / HS) < N ? -0.5f * v : -INFINITY;
  }
  for (int e = t; e < NP16 * 3; e += 1024) bits[e] = e * 2654435761u;
  if (t < HS) dl[t] = 0.1f * t;
  __syncthreads();
  const int g = t >> 8, tg = t & 255, k0 = g * KK;
  const int tj = tg & 15, ti = tg >> 4, lane = t & 63, wv = tg >> 6;
  const int S = (N + 15) >> 4;
  for (int it = 0; it < iters; ++it) {
    float cacc[SMAX][KK];
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
#pragma unroll
      for (int k = 0; k < KK; ++k) cacc[c][k] = 0.f;
    for (int s = 0; s < S; ++s) {
      const int i = ti + 16 * s;
      const bool iv = i < N;
      float a[KK], racc[KK];
#pragma unroll
      for (int k = 0; k < KK; ++k) { a[k] = A[i * LD + k0 + k]; racc[k] = 0.f; }
      uint32_t wrow[3];
      const int ib = iv ? i : 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) wrow[q] = iv ? bits[ib * 3 + q] : 0u;
#pragma unroll
      for (int c = 0; c < SMAX; ++c) {
        const int j = tj + 16 * c;
        const float af = (float)((wrow[c >> 1] >> (tj + 16 * (c & 1))) & 1u);
#pragma unroll
        for (int k = 0; k < KK; ++k) {
          const float z = a[k] + fmaf(af, dl[k0 + k], Bv[j * LD + k0 + k]);
          const float e = reluf(z);
          racc[k] += e;
          cacc[c][k] += e;
        }
      }
#pragma unroll
      for (int k = 0; k < KK; ++k) {
        const float r = (FLAGS & 1) ? racc[k] : row16_sum(racc[k]);
        if (tj == 0 && iv) R[i * LD + k0 + k] = r;
      }
    }
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
#pragma unroll
      for (int k = 0; k < KK; ++k) {
        const float v = (FLAGS & 2) ? cacc[c][k] : xrow_sum4(cacc[c][k]);
        if (lane < 16) cred[g][(wv * NP16 + tj + 16 * c) * KK + k] = v;
      }
    if (!(FLAGS & 4)) {
      __syncthreads();
      for (int e = tg; e < NP16 * KK; e += 256) {
        const int j = e / KK, k = e - j * KK;
        const float v = cred[g][e] + cred[g][e + NP16 * KK] + cred[g][e + 2 * NP16 * KK] + cred[g][e + 3 * NP16 * KK];
        if (j < N) C[j * LD + k0 + k] = v;
      }
      __syncthreads();
    }
  }
  if (t == 0) out[blockIdx.x] = R[7] + C[11] + cred[0][5];
}
}  // namespace
template <class K>
float time_kernel(K k, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  k(blocks, 1); hipDeviceSynchronize();
  hipEventRecord(a); k(blocks, iters); hipEventRecord(b); hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / iters;
}
#define RUN(F) printf("  flags %d: %8.2f us  (1 block: %8.2f us)\n", F, \
  time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb<F>, dim3(nb), dim3(1024), 0, 0, 74, it, out); }, 100, 50), \
  time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb<F>, dim3(nb), dim3(1024), 0, 0, 74, it, out); }, 1, 50));
int main() {
  float* out; hipMalloc(&out, 4096 * 4);
  printf("pair-tile ablations, Nc=74 (us per call):\n");
  RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(7)
  return 0;
}
