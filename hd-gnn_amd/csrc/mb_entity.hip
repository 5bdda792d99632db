// mb_entity.hip -- ablations of the sorted-x entity forward (entity_fwd, phase E1).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include mb_entity.hip -o mb_entity
// One block per "commit" (100 blocks x 1024 threads), Ne = 200, x in 0..9, a ~ 5 %.
#include "hdgnn.hip"

namespace {

template <int ABL>
__global__ __launch_bounds__(1024) void mb_e1(int Ne, int iters, float* out, float* EG,
                                              uint16_t* rq) {
  __shared__ float Ws[2128];
  __shared__ float xs[256], xu[256], Ps[256 * HS];
  __shared__ int cum[260], offr[260], offc[260];
  __shared__ double pxd[260];
  __shared__ __attribute__((aligned(16))) float lr[256 * 16], lc[256 * 16];   // x-lists
  const int t = threadIdx.x, b = blockIdx.x;
  for (int i = t; i < 2128; i += 1024) Ws[i] = 0.01f * (float)((i * 2654435761u) % 200) - 1.f;
  for (int i = t; i < Ne; i += 1024) xs[i] = (float)((i * 7 + b) % 10);
  __syncthreads();
  if (t < 256) xu[t] = t < 10 ? (float)t : INFINITY;   // entity_fwd: +inf past nd
  if (t <= 10) { cum[t] = t * Ne / 10; pxd[t] = 0.0; }
  if (t == 0) {              // ~5 % density: degree 8..12 per row and column
    int ar = 0, ac = 0;
    for (int i = 0; i < Ne; ++i) {
      offr[i] = ar; offc[i] = ac;
      const int dr = 8 + (i * 3 + b) % 5, dc = 8 + (i * 7 + b) % 5;
      for (int n = 0; n < dr; ++n) lr[ar++] = xs[(i + 1 + 17 * n) % Ne];
      for (int n = 0; n < dc; ++n) lc[ac++] = xs[(i + 3 + 13 * n) % Ne];
      while (ar & 3) lr[ar++] = __builtin_nanf("");
      while (ac & 3) lc[ac++] = __builtin_nanf("");
    }
    offr[Ne] = ar; offc[Ne] = ac;
  }
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    entity_fwd<ABL>(t, Ws, xs, xu, cum, pxd, 10, offr, offc, lr, lc, 0, Ne, Ps,
                    EG + (size_t)b * Ne * HS, rq + (size_t)b * Ne * HS);
    __syncthreads();
  }
  if (t == 0) out[b] = Ps[7] + Ps[300];
}

}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int ABL>
float run(float* out, float* EG, uint16_t* rq, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(mb_e1<ABL>, dim3(blocks), dim3(1024), 0, 0, 200, 1, out, EG, rq);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL(mb_e1<ABL>, dim3(blocks), dim3(1024), 0, 0, 200, iters, out, EG, rq);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / iters;
}

int main() {
  float *out, *EG;
  uint16_t* rq;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMalloc(&EG, 100 * 256 * HS * sizeof(float)));
  CK(hipMalloc(&rq, 100 * 256 * HS * sizeof(uint16_t)));
  const int B = 100, IT = 20;
  printf("entity_fwd Ne=200 (us per call, %d blocks x 1024 thr)\n", B);
  printf("  full              %8.2f\n", run<0>(out, EG, rq, B, IT));
  printf("  no search         %8.2f\n", run<1>(out, EG, rq, B, IT));
  printf("  no dense          %8.2f\n", run<2>(out, EG, rq, B, IT));
  printf("  no row bits       %8.2f\n", run<4>(out, EG, rq, B, IT));
  printf("  no col bits       %8.2f\n", run<8>(out, EG, rq, B, IT));
  printf("  no bits           %8.2f\n", run<12>(out, EG, rq, B, IT));
  printf("  search only       %8.2f\n", run<14>(out, EG, rq, B, IT));
  printf("  nothing           %8.2f\n", run<15>(out, EG, rq, B, IT));
  printf("  1 block full      %8.2f\n", run<0>(out, EG, rq, 1, IT));
  CK(hipDeviceSynchronize());
  return 0;
}
