// Timing probe (not shipped): kw_ee_fwd on synthetic glide-shaped inputs (B=100, Ne=200,
// Nc=74, n uniform in [Ne/2, 3Ne/2] clipped to Ne as hdgnn/synth.py draws it), per-wave
// s_memrealtime stamps at the phase boundaries (100 MHz clock).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DHDG_EE_PROBE -Iinclude
//          -Ihd-gnn_amd/csrc tools/probe/eefwd_probe.hip hd-gnn_amd/csrc/hdgnn.hip -o ...
#include "../../hd-gnn_amd/csrc/wide.hip"
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  using namespace hdg;
  const int B = 100, Ne = 200, Nc = 74, WE = (Ne + 31) / 32;
  const int aligned_only = argc > 1 ? atoi(argv[1]) : 0;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<uint32_t> ab((size_t)B * Ne * WE, 0u);
  std::vector<int32_t> hid((size_t)B * Ne), nl(B);
  std::vector<float> rho((size_t)B * Ne * H), gam((size_t)B * Ne * H), D(1024);
  for (int b = 0; b < B; ++b) {
    int n = Ne / 2 + (int)(rng() % (Ne + 1));
    nl[b] = aligned_only ? Ne : std::min(n, Ne);
    for (int i = 0; i < Ne; ++i) {
      for (int j = 0; j < Ne; ++j)
        if (i != j && (rng() % 100) < 5) ab[((size_t)b * Ne + i) * WE + j / 32] |= 1u << (j & 31);
      const int id = (int)(rng() % (Nc + Nc / 4 + 1));
      hid[(size_t)b * Ne + i] = (i < nl[b] && id < Nc && rng() % 5) ? id : -1;
    }
  }
  for (auto& v : rho) v = 0.5f * U(rng);
  for (auto& v : gam) v = 0.5f * U(rng);
  for (auto& v : D) v = 0.3f * U(rng);
  const int tiles = ee_fwd_tiles(Ne);
  uint32_t* dab; int32_t *dhid, *dnl; float *drho, *dgam, *dD; unsigned long long *dnc, *dst;
  const size_t nst = (size_t)B * tiles * NWP * 8;
  CK(hipMalloc(&dab, ab.size() * 4)); CK(hipMalloc(&dhid, hid.size() * 4)); CK(hipMalloc(&dnl, B * 4));
  CK(hipMalloc(&drho, rho.size() * 4)); CK(hipMalloc(&dgam, gam.size() * 4)); CK(hipMalloc(&dD, 4096));
  CK(hipMalloc(&dnc, (size_t)B * tiles * 2 * Nc * 8)); CK(hipMalloc(&dst, nst * 8));
  CK(hipMemcpy(dab, ab.data(), ab.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhid, hid.data(), hid.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dnl, nl.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drho, rho.data(), rho.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dgam, gam.data(), gam.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dD, D.data(), 4096, hipMemcpyHostToDevice));
  CK(hipMemset(dst, 0, nst * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ee_stamps), &dst, sizeof(dst)));
  CK(hipFuncSetAttribute((const void*)kw_ee_fwd<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e9f;
  for (int r = 0; r < 30; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kw_ee_fwd<1>, dim3(tiles, B), dim3(NTP), ee_fwd_lds(Ne, Nc), 0, dab, dhid,
                       dnl, (const float*)nullptr, Off{}, dD, Ne, Nc, drho, dgam, dnc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> st(nst);
  CK(hipMemcpy(st.data(), dst, nst * 8, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, tend = 0;
  for (size_t w = 0; w < nst / 8; ++w) if (st[w * 8]) { t0 = std::min(t0, st[w * 8]); tend = std::max(tend, std::max(st[w * 8 + 5], st[w * 8 + 0])); }
  printf("aligned_only=%d best event %.2f us, stamp span %.2f us\n", aligned_only, best * 1e3, (tend - t0) * 0.01);
  // per phase: median / max durations over waves that ran the loop; start-time spread
  const char* nm[5] = {"stage+barrier", "setup+rh", "loop", "bins", "write"};
  std::vector<double> d[5], start, endv;
  for (size_t w = 0; w < nst / 8; ++w) {
    const unsigned long long* s = &st[w * 8];
    if (!s[0]) continue;
    start.push_back((s[0] - t0) * 0.01);
    if (!s[5]) continue;            // early-exit tile
    endv.push_back((s[5] - t0) * 0.01);
    if (!s[2]) continue;
    for (int k = 0; k < 5; ++k) d[k].push_back((s[k + 1] - s[k]) * 0.01);
  }
  auto q = [](std::vector<double> v, double f) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
  printf("waves %zu started, %zu full; start p50 %.2f p90 %.2f max %.2f us; end p50 %.2f max %.2f us\n",
         start.size(), d[0].size(), q(start, .5), q(start, .9), q(start, 1.), q(endv, .5), q(endv, 1.));
  for (int k = 0; k < 5; ++k)
    printf("  %-14s p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", nm[k], q(d[k], .1), q(d[k], .5), q(d[k], .9), q(d[k], 1.));
  // residency: wave 0 of each block -> (xcc, se, cu); blocks per CU that start in the first
  // microsecond, and the start-time histogram (1 us bins)
  std::vector<int> hist(40, 0);
  std::vector<int> first(8 * 16 * 16 * 2, 0), total(8 * 16 * 16 * 2, 0);
  for (size_t blk = 0; blk < nst / 8 / NWP; ++blk) {
    const unsigned long long* s = &st[blk * NWP * 8];
    if (!s[0]) continue;
    const double ts = (s[0] - t0) * 0.01;
    hist[std::min(39, (int)ts)]++;
    const unsigned hw = (unsigned)s[6], xcc = (unsigned)s[7] & 0xf;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    const int key = ((xcc * 8 + se) * 2 + sh) * 16 + cu;
    total[key]++;
    if (ts < 1.0) first[key]++;
  }
  printf("block start histogram (1 us bins):");
  for (int i = 0; i < 40; ++i) if (hist[i]) printf(" [%d]=%d", i, hist[i]);
  printf("\n");
  int mx[8] = {0}, ncu = 0;
  for (size_t k = 0; k < first.size(); ++k) if (total[k]) { ++ncu; mx[std::min(7, first[k])]++; }
  printf("CUs used %d; CUs by blocks started in the first us:", ncu);
  for (int i = 0; i < 8; ++i) if (mx[i]) printf(" %d:%d", i, mx[i]);
  printf("\n");
  return 0;
}
