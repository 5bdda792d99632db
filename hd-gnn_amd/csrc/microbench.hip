// microbench.hip -- isolate the building blocks of k_commit_mid on MI355X.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include microbench.hip -o microbench
// Each kernel runs one block per "commit" (100 blocks, 1024 threads) and repeats the
// building block ITERS times on LDS data, so per-call time = kernel time / ITERS.
#include "hdgnn.hip"

namespace {

template <int MODE, int ABL = 0>
__global__ __launch_bounds__(1024) void mb_tile(int N, int iters, float* out, int rmul = 1) {
  constexpr int SMAXC = 5, NC16 = 80;
  __shared__ __attribute__((aligned(16))) float A[NC16 * HS], B[NC16 * HS], R[NC16 * HS],
      C[NC16 * HS], wr[NC16 * HS], wc[NC16 * HS], dl[HS], ys[HS];
  __shared__ __attribute__((aligned(16))) float cred[4 * tile_cred_words<SMAXC, 5>()];
  __shared__ uint32_t bits[NC16 * 3];
  __shared__ float gam[NC16 * NC16];
  const int t = threadIdx.x;
  for (int e = t; e < NC16 * HS; e += 1024) {
    const int p = e / HS;
    const float v = (float)((e * 2654435761u) % 1000) * 1e-3f - 0.5f;
    A[e] = p < N ? v : -INFINITY;
    B[e] = p < N ? -v * 0.5f : -INFINITY;
    wr[e] = v;
    wc[e] = 0.3f * v;
  }
  for (int e = t; e < NC16 * NC16; e += 1024) gam[e] = (float)(e % 13) * 1e-3f;
  for (int e = t; e < NC16 * 3; e += 1024) bits[e] = e * 2654435761u;
  if (t < HS) dl[t] = 0.1f * t;
  __syncthreads();
  const int g = t >> 8, tg = t & 255;
  for (int it = 0; it < iters; ++it)
    pair_tile<5, SMAXC, MODE, HS, ABL>(N, tg, A, B, g * 5, dl, bits, 3, wr, wc, gam, NC16, R, C, ys,
                                  cred + g * tile_cred_words<SMAXC, 5>(), rmul, 0);
  if (t == 0) out[blockIdx.x] = R[7] + C[11] + ys[3];
}

}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <class K>
float time_kernel(K k, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k(blocks, 1);   // warm
  hipDeviceSynchronize();
  hipEventRecord(a);
  k(blocks, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / iters;   // us per building-block call
}

int main() {
  float* out;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  const int B = 100, IT = 50;
  printf("pair_tile Nc=74 (per call, 100 blocks x 1024 thr):\n");
  printf("  MODE0 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<0>, dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE1 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<1>, dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE2 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<2>, dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE0 no y    %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<0, 1>), dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE0 no rowr %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<0, 2>), dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE0 neither %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<0, 3>), dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE1 no y    %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<1, 1>), dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("  MODE2 no y    %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<2, 1>), dim3(nb), dim3(1024), 0, 0, 74, it, out); }, B, IT));
  printf("half rows (split mode, rmul = 2):\n");
  printf("  MODE0 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<0>, dim3(nb), dim3(1024), 0, 0, 74, it, out, 2); }, B, IT));
  printf("  MODE1 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<1>, dim3(nb), dim3(1024), 0, 0, 74, it, out, 2); }, B, IT));
  printf("  MODE2 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<2>, dim3(nb), dim3(1024), 0, 0, 74, it, out, 2); }, B, IT));
  printf("  MODE0 neither %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL((mb_tile<0, 3>), dim3(nb), dim3(1024), 0, 0, 74, it, out, 2); }, B, IT));
  printf("  N=16 MODE0 (one row block, fixed cost) %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<0>, dim3(nb), dim3(1024), 0, 0, 16, it, out, 1); }, B, IT));
  printf("  N=16 MODE1 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<1>, dim3(nb), dim3(1024), 0, 0, 16, it, out, 1); }, B, IT));
  printf("  N=16 MODE2 %8.2f us\n", time_kernel([&](int nb, int it) { hipLaunchKernelGGL(mb_tile<2>, dim3(nb), dim3(1024), 0, 0, 16, it, out, 1); }, B, IT));
  CK(hipDeviceSynchronize());
  return 0;
}
