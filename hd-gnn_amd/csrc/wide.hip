// wide.hip -- general path of the HD-GNN training step: any Ne / Nc (<= 4096 / 2048) and
// all four model variants (model_1..model_4.py), built from many 256-thread blocks per
// commit with the commit state in HBM.  The fused path (hdgnn.hip) covers model_2 at the
// benchmark shapes; this path covers everything else (model_4's entity-edge stage, the
// model_1 / model_3 wirings, the stress shapes Ne=1024 / Nc=512) and doubles as a
// cross-check of the fused kernel.
//
// One training step, as a sequence of launches on the caller's stream (x' = x for
// model_1 / model_3, ENT = model_2/4 entity stage, EE = model_4 entity-edge stage):
//   kw_derive       derived weight products (M = V2 U1e, offsets, differences)
//   kw_ent_fwd      ENT: P_i  = sum_j relu(z_ij) + relu(z_ji)     (mlp_entity_B1 + agg)
//                   EE : R1_i = sum_j relu(z'_ij), C1_i = sum_j relu(z'_ji)
//   node_fwd_tile   ENT: E_bar, h, o, x'          EE: R, C, rho, gam (classifier operands),
//                   in kw_ent_fwd's blocks after their tile's pair sums
//   kw_ee_fwd       EE : entity-edge classifier + softmax on every relation the index file
//                   maps, aggregated into n_c[2:4] (marshalling_B2 of B_2's edge part)
//   kw_cross_fwd    n_c = [K_s x', K_t x', n_c[2:4]]; hunk first-layer alpha, beta
//   kw_hunk_fwd     G_p = sum_q relu(a_p + b_q + y d) (row pass), H_q (column pass),
//                   sigma / tau (classifier first layer on eff = S_p + T_q)
//   kw_hunk_cls     classifier + softmax-CE per hunk pair, gamma = dL/dz1
//   -- backward --
//   kw_hunk_clsb    Dsig / Dtau (row / column pass), dG / dH, classifier + V2 grads
//   kw_hunk_mlpb    Dalpha / Dbeta, V1 / c1 grads
//   kw_dn           dn_c (gradient of the cross-graph aggregate)
//   kw_node_bwd     ENT: dx', E3 and W5 grads, rho = dP
//   kw_ent_bwd      ENT: first-layer grads of mlp_entity_B1
//   kw_ee_clsb      EE : classifier backward, one column pass: dgam + classifier grads,
//                   per-tile partial rows of drho (wave sums over the tile's columns)
//   kw_ee_nodeb     EE : dR, dC -> phi, psi; classifier U1e, Q2, q2 grads
//   kw_ee_firstb    EE : first-layer grads of mlp_entityedge_B1 (shared w1_1)
//   kw_grad_reduce  fixed-order sum of every per-block partial row -> flat gradient
//
// Determinism: no floating-point atomics anywhere.  Per-block partial gradient rows are
// summed in a fixed order; row/column sums over pairs are recomputed by a row pass and a
// column pass instead of being scattered.  The one scatter (relation -> hunk bins of
// kw_ee_fwd) accumulates in 2^-32 fixed point with integer atomics, order-independent.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "hdgnn.h"
#include "hdgnn_internal.h"

namespace hdg {
namespace {

constexpr int H = HS;
constexpr int HP = H + 1;   // padded LDS rows (odd stride: conflict-free column access)
constexpr int TN = 64;      // nodes per tile, one per lane
constexpr int NT = 256;     // threads per block
constexpr int NW = NT / 64;
constexpr double FIX = 4294967296.0;   // 2^32 fixed-point scale of the hunk bins

__device__ __forceinline__ float relu(float v) { return fmaxf(v, 0.f); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave time stamps of one kernel (timing builds only: -DHDG_WSTAMP=<kernel id>, read by
// tools/wstamp.py through hdg_wstamp_set): 8 s_memrealtime slots (100 MHz) per wave,
// [block (x fastest)][wave][slot], lane 0 of the wave storing.
#ifdef HDG_WSTAMP
__device__ unsigned long long* g_wst;
#define WSTAMP(kid, k)                                                                      \
  do {                                                                                      \
    if constexpr (HDG_WSTAMP == (kid)) {                                                    \
      if ((threadIdx.x & 63) == 0 && g_wst)                                                 \
        g_wst[(((size_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) *  \
                   (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] =                    \
            __builtin_amdgcn_s_memrealtime();                                               \
    }                                                                                       \
  } while (0)
#else
#define WSTAMP(kid, k) do {} while (0)
#endif
#ifndef HDG_ABL_QJ    // ablation builds only: kw_first_bwd's neighbour rows read from the own
#define HDG_ABL_QJ 0  // row (cache-hot, wrong sums)
#endif
#ifndef HDG_ABL_DX    // ablation builds only: kw_node_bwd's count-phase loads (1 counts, 2 dn)
#define HDG_ABL_DX 0
#endif
#ifndef HDG_ABL_XJ    // ablation builds only: neighbour x reads at conflict-free addresses
#define HDG_ABL_XJ 0  // (wrong sums; for timing the LDS gathers of the walks)
#endif


template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}
// v_permlane32_swap / v_permlane16_swap (VALU, no LDS): swap32 trades x's lanes 32-63 for
// y's lanes 0-31, swap16 x's rows 1, 3 for y's rows 0, 2 (inline asm: the ROCm 7.2
// builtins mis-assign the two results; two wait states after a VALU write of the operands)
__device__ __forceinline__ void swap32(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void swap16(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}

// wave sum by a VALU butterfly (permlane swaps across the 32- / 16-lane halves, DPP inside
// a row): every lane ends with the same total (each level adds the same two partial
// sums in every lane, and fp32 addition commutes)
__device__ __forceinline__ float wsum(float v) {
  float x = v, y = v;
  swap32(x, y);
  v = x + y;
  x = v;
  y = v;
  swap16(x, y);
  v = x + y;
  v += dppf<0x128>(v);   // row_ror:8        lane ^ 8
  v += dppf<0x141>(v);   // row_half_mirror  7 - lane (per 8)
  v += dppf<0x4E>(v);    // quad_perm        lane ^ 2
  v += dppf<0xB1>(v);    // quad_perm        lane ^ 1
  return v;
}
// sum over a 16-lane DPP row; every lane of the row receives the total
__device__ __forceinline__ float row_total16(float v) {
  v += dppf<0x128>(v);
  v += dppf<0x141>(v);
  v += dppf<0x4E>(v);
  v += dppf<0xB1>(v);
  return v;
}

// Sums of the 20 values v[k] over the 64 lanes of a wave by a transposed butterfly (one
// exchange per pair of values and level instead of six per value), all in the VALU:
// permlane swaps across the 32- and 16-lane halves, then DPP inside a 16-lane row
// (row_ror:8 = lane ^ 8, row_half_mirror = 7 - lane within 8, quad_perm for ^2, ^1);
// a lane keeps the first or second half of the values by its lane bit.  store(k, total)
// runs on one lane per value; cnt tracks how many real values a lane's block holds.
template <class F>
__device__ __forceinline__ void wave_sums20(const float (&v)[20], const int lane, F store) {
  float w1[10], w2[5], w3[3], w4[2];
  int base = 0, cnt;
#pragma unroll
  for (int i = 0; i < 10; ++i) {                          // 20 -> 10 | 10 (lane bit 5)
    float x = v[i], y = v[i + 10];
    swap32(x, y);
    w1[i] = x + y;
  }
  base += (lane & 32) ? 10 : 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {                           // 10 -> 5 | 5 (lane bit 4)
    float x = w1[i], y = w1[i + 5];
    swap16(x, y);
    w2[i] = x + y;
  }
  base += (lane & 16) ? 5 : 0;
  bool up = lane & 8;                                     // 5 -> 3 | 2
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float a = w2[i], b = i + 3 < 5 ? w2[i + 3] : 0.f;
    w3[i] = (up ? b : a) + dppf<0x128>(up ? a : b);
  }
  base += up ? 3 : 0;
  cnt = up ? 2 : 3;
  up = lane & 4;                                          // 3 -> 2 | 1  (2 -> 2 | 0)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float a = w3[i], b = i + 2 < 3 ? w3[i + 2] : 0.f;
    w4[i] = (up ? b : a) + dppf<0x141>(up ? a : b);
  }
  base += up ? 2 : 0;
  cnt = up ? cnt - 2 : (cnt < 2 ? cnt : 2);
  up = lane & 2;                                          // 2 -> 1 | 1
  float w5 = (up ? w4[1] : w4[0]) + dppf<0x4E>(up ? w4[0] : w4[1]);
  base += up ? 1 : 0;
  cnt = up ? cnt - 1 : (cnt < 1 ? cnt : 1);
  w5 += dppf<0xB1>(w5);
  if (!(lane & 1) && cnt >= 1) store(base, w5);
}

// Sums of the 20 values v[k] over each 32-lane half of a wave (lanes 0-31 and 32-63 kept
// apart) by the same transposed butterfly: a permlane16 swap across the half's two DPP
// rows, then DPP inside a row (row_ror:8, row_half_mirror, quad_perm ^2, ^1).
// store(half, k, total) runs on one lane per half and value.
template <class F>
__device__ __forceinline__ void half_sums20(const float (&v)[20], const int lane, F store) {
  float w1[10], w2[5], w3[3], w4[2];
#pragma unroll
  for (int i = 0; i < 10; ++i) {                          // 20 -> 10 | 10 (lane bit 4)
    float x = v[i], y = v[i + 10];
    swap16(x, y);
    w1[i] = x + y;
  }
  int base = (lane & 16) ? 10 : 0, cnt;
  bool up = lane & 8;                                     // 10 -> 5 | 5
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const float a = w1[i], b = w1[i + 5];
    w2[i] = (up ? b : a) + dppf<0x128>(up ? a : b);
  }
  base += up ? 5 : 0;
  up = lane & 4;                                          // 5 -> 3 | 2
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float a = w2[i], b = i + 3 < 5 ? w2[i + 3] : 0.f;
    w3[i] = (up ? b : a) + dppf<0x141>(up ? a : b);
  }
  base += up ? 3 : 0;
  cnt = up ? 2 : 3;
  up = lane & 2;                                          // 3 -> 2 | 1  (2 -> 2 | 0)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float a = w3[i], b = i + 2 < 3 ? w3[i + 2] : 0.f;
    w4[i] = (up ? b : a) + dppf<0x4E>(up ? a : b);
  }
  base += up ? 2 : 0;
  cnt = up ? cnt - 2 : (cnt < 2 ? cnt : 2);
  up = lane & 1;                                          // 2 -> 1 | 1
  const float w5 = (up ? w4[1] : w4[0]) + dppf<0xB1>(up ? w4[0] : w4[1]);
  base += up ? 1 : 0;
  cnt = up ? cnt - 1 : (cnt < 1 ? cnt : 1);
  if (cnt >= 1) store(lane >> 5, base, w5);
}

// Sums of the 20 values v[k] over each 16-lane DPP row (a quarter of the wave) by the same
// transposed butterfly inside the row (row_ror:8, row_half_mirror, quad_perm ^2, ^1); a
// lane ends with 0-2 of its quarter's totals: store(slot, k, total), slot 0 / 1, on one
// lane per quarter and value (the same lane and slot for every call)
// One level of a transposed butterfly on five pairs (a_i, b_i) without selects: lanes in
// the DPP banks of LO get a_i + a_i(partner), lanes in HI b_i + b_i(partner), as two DPP
// adds into one register whose bank masks split the lanes (a lane kept by the mask is
// written by exactly one of the two).  CTRL: row_ror:8 (partner lane ^ 8; LO = banks 0, 1)
// or row_half_mirror (partner 7 - lane within 8; LO = banks 0, 2).  Same sums, same bits
// as keep + dpp(send) with two selects per pair; one s_nop for the block (its inputs'
// VALU writes precede it, the block writes only its outputs).
#define HDG_XLEVEL5(CTRL, LO, HI)                                                          \
  asm volatile("s_nop 1\n\t"                                                             \
               "v_add_f32_dpp %0, %5, %5 " CTRL " row_mask:0xf bank_mask:" LO "\n\t"        \
               "v_add_f32_dpp %0, %10, %10 " CTRL " row_mask:0xf bank_mask:" HI "\n\t"      \
               "v_add_f32_dpp %1, %6, %6 " CTRL " row_mask:0xf bank_mask:" LO "\n\t"        \
               "v_add_f32_dpp %1, %11, %11 " CTRL " row_mask:0xf bank_mask:" HI "\n\t"      \
               "v_add_f32_dpp %2, %7, %7 " CTRL " row_mask:0xf bank_mask:" LO "\n\t"        \
               "v_add_f32_dpp %2, %12, %12 " CTRL " row_mask:0xf bank_mask:" HI "\n\t"      \
               "v_add_f32_dpp %3, %8, %8 " CTRL " row_mask:0xf bank_mask:" LO "\n\t"        \
               "v_add_f32_dpp %3, %13, %13 " CTRL " row_mask:0xf bank_mask:" HI "\n\t"      \
               "v_add_f32_dpp %4, %9, %9 " CTRL " row_mask:0xf bank_mask:" LO "\n\t"        \
               "v_add_f32_dpp %4, %14, %14 " CTRL " row_mask:0xf bank_mask:" HI               \
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4])               \
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(b[0]), "v"(b[1]),  \
                 "v"(b[2]), "v"(b[3]), "v"(b[4]))
__device__ __forceinline__ void xlevel5_ror8(const float* a, const float* b, float* o) {
  HDG_XLEVEL5("row_ror:8", "0x3", "0xc");
}
__device__ __forceinline__ void xlevel5_hmirror(const float* a, const float* b, float* o) {
  HDG_XLEVEL5("row_half_mirror", "0x5", "0xa");
}
#undef HDG_XLEVEL5

template <class F>
__device__ __forceinline__ void quarter_sums20(const float (&v)[20], const int lane, F store) {
  float w1[10], w2[5], w3[3], w4[2];
  bool up = lane & 8;                                     // 20 -> 10 | 10
  xlevel5_ror8(v, v + 10, w1);                            // pairs (v[i], v[i + 10]), i < 5
  xlevel5_ror8(v + 5, v + 15, w1 + 5);                    //   and i = 5..9
  int base = up ? 10 : 0;
  up = lane & 4;                                          // 10 -> 5 | 5
  xlevel5_hmirror(w1, w1 + 5, w2);
  base += up ? 5 : 0;
  up = lane & 2;                                          // 5 -> 3 | 2
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float a = w2[i], b = i + 3 < 5 ? w2[i + 3] : 0.f;
    w3[i] = (up ? b : a) + dppf<0x4E>(up ? a : b);
  }
  base += up ? 3 : 0;
  int cnt = up ? 2 : 3;
  up = lane & 1;                                          // 3 -> 2 | 1  (2 -> 2 | 0)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float a = w3[i], b = i + 2 < 3 ? w3[i + 2] : 0.f;
    w4[i] = (up ? b : a) + dppf<0xB1>(up ? a : b);
  }
  base += up ? 2 : 0;
  cnt = up ? cnt - 2 : (cnt < 2 ? cnt : 2);
  if (cnt >= 1) store(0, base, w4[0]);
  if (cnt >= 2) store(1, base + 1, w4[1]);
}

__device__ __forceinline__ unsigned long long qfix(float v) {
  return (unsigned long long)__double2ll_rn((double)v * FIX);
}

// derived weights (kw_derive), float offsets into the D buffer
enum : int {
  D_M = 0,                 // [20][20] V2 . U1e  (hunk MLP second layer into the classifier)
  D_S0 = 400,              // sigma offset  (Nc-1) c2 U1e + U1[0] + d1
  D_T0 = 420,              // tau offset    (Nc-1) c2 U1e
  D_EPS = 440,             // U1[1] - U1[0]
  D_CV = 460,              // U2[:,1] - U2[:,0]
  D_DLT = 480,             // V1[9] - V1[8]
  D_EED = 500,             // EE classifier P1[1] - P1[0]
  D_EEC = 520,             // EE classifier U2'[:,1] - U2'[:,0]
  D_EECQ = 544,            // -log2(e) (U2'[:,1] - U2'[:,0])    (kw_ee_clsb: e = 2^delta')
  D_EEBQ = 564,            // -log2(e) (b2'[1] - b2'[0])
  D_AUX = 568,             // [7] train steps: lpara, lmap, |theta1|, |theta2|,
                           //     sqrt(1-b2^t)/(1-b1^t), b1^(t+1), b2^(t+1)  (kw_reduce_adam)
  D_WORDS = 576
};

// Prepared batch of the general path, per commit (words): cross-graph counts as in the
// fused layout, then the sorted-x tables of the entity stages (k_prep_counts, kw_prep_sort):
//   ks, kt [Nc][Ne] u16   ncst [Nc][2] f32   xsrt [NE4] x ascending   perm [NE4] node of slot
//   xu [NE4] distinct values   cum [NE4+4] #nodes with x < xu[q]   pxd [NE4+4] f64 sums
//   meta[4] = {nd}
// followed, after all B commits, by a^T [B][Ne][WE] and y^T [B][Nc][WC] (kw_prep_T).
struct GenPrep {
  int ks, kt, ncst, xsrt, perm, xu, cum, pxd, meta, words;
};

__host__ __device__ inline GenPrep gen_prep(int Ne, int Nc) {
  GenPrep G;
  const int NE4 = (Ne + 3) & ~3;
  const int kw = ((Nc * Ne + 1) / 2 + 3) & ~3;
  int o = 0;
  G.ks = o;   o += kw;
  G.kt = o;   o += kw;
  G.ncst = o; o += (2 * Nc + 3) & ~3;
  G.xsrt = o; o += NE4;
  G.perm = o; o += NE4;
  G.xu = o;   o += NE4;
  G.cum = o;  o += NE4 + 4;
  G.pxd = o;  o += 2 * (NE4 + 4);     // every offset above is a multiple of 4: 8-B aligned
  G.meta = o; o += 4;
  G.words = (o + 63) & ~63;
  return G;
}

// neighbour id lists (kw_prep_lists), past the per-commit words, aT and yT: counts u32
// [2][B][Ne] (side 0: row bits of a, 1: column bits), ids u16 [2][B][Ne][LS] -- the j != i
// with a_ij = 1 (side 0) / a_ji = 1 (side 1) ascending, padded to a multiple of 4 with the
// sentinel Ne.  Offsets in 4-byte words from the prep base.
__host__ __device__ inline int list_stride(int Ne) { return (Ne + 3) & ~3; }
struct ListLayout {
  size_t cnt, ids, end;
};
__host__ __device__ inline ListLayout list_layout(int B, int Ne, int Nc) {
  const size_t WE = (Ne + 31) / 32, WC = (Nc + 31) / 32;
  ListLayout L;
  L.cnt = ((size_t)B * gen_prep(Ne, Nc).words + (size_t)B * Ne * WE + (size_t)B * Nc * WC + 3) &
          ~(size_t)3;
  L.ids = L.cnt + ((2 * (size_t)B * Ne + 3) & ~(size_t)3);
  L.end = L.ids + (size_t)B * Ne * list_stride(Ne);     // 2 sides x LS/2 words
  return L;
}

// label id lists (kw_prep_lists on y, the sorted hunk passes' walks): counts u32 [2][B][Nc]
// (side 0: row p of y, 1: column q), ids u16 [2][B][Nc][LSc] ascending, padded to a
// multiple of 4 with the sentinel Nc; after the entity lists (model_2 / model_4) or yT
__host__ __device__ inline ListLayout ylist_layout(int B, int Ne, int Nc, bool ent) {
  const ListLayout L = list_layout(B, Ne, Nc);
  ListLayout Y;
  Y.cnt = ((ent ? L.end : L.cnt) + 3) & ~(size_t)3;
  Y.ids = Y.cnt + ((2 * (size_t)B * Nc + 3) & ~(size_t)3);
  Y.end = Y.ids + (size_t)B * Nc * list_stride(Nc);
  return Y;
}

// model_4, after everything above (kw_prep_order; the entity-edge kernels' dispatch orders):
//   the commits by decreasing relation rows, u32 [B4] (B4 = B rounded up to 4; kw_ee_clsb),
//   the (commit, 32-row tile) pairs b * te + T by decreasing work, u32 [te B] (kw_ee_fwd)
constexpr int EE_ORDER_MAX = 12288;   // te B: kw_prep_order's LDS rank table; blockIdx order beyond

// per-block partial gradient rows: segment s holds n consecutive parameters starting at
// flat index p0, laid out [n][rows] at part + off
constexpr int MAXSEG = 16;
struct Seg {
  int p0, n, rows;
  long long off;
};
struct Segs {
  Seg s[MAXSEG];
  int count;
};
enum : int {
  SG_CLS = 0,   // H2_W2 .. H2_B2 (42)                 kw_hunk_cls
  SG_CE,        // CE sum, correct count (slots NP, NP+1) kw_hunk_cls
  SG_CLSB_H2,   // H2_W1 .. H2_B1 (460)                kw_hunk_clsb (2 passes)
  SG_CLSB_H1,   // H1_W2 .. H1_B2 (420)                kw_hunk_clsb (2 passes)
  SG_MLPB,      // H1_W1 .. H1_B1 (220)                kw_hunk_mlpb (2 passes)
  SG_E3,        // E3_W1 .. E3_B2 (461)                kw_node_bwd
  SG_E1W5,      // E1_W5 .. E1_B5 (420)                kw_node_bwd
  SG_E1W1,      // E1_W1 .. E1_B1 (100)                kw_ent_bwd
  SG_ECW1A,     // EC_W1 rows 0, 1 (40)                kw_ee_clsb column pass
  SG_ECB1,      // EC_B1 .. EC_B2 (62)                 kw_ee_clsb column pass
  SG_ECW1E,     // EC_W1 rows 2..21 (400)              kw_ee_nodeb
  SG_EEW2,      // EE_W2 .. EE_B2 (420)                kw_ee_nodeb
  SG_EEW11,     // EE_W11 .. EE_B1 (80)                kw_ee_firstb
  SG_COUNT
};

__device__ __forceinline__ void put(float* part, const Seg& s, int q, int row, float v) {
  part[s.off + (long long)q * s.rows + row] = v;
}

// copy n floats of the parameter vector (or any global array) into LDS (no barrier)
__device__ __forceinline__ void stage_w(float* dst, const float* src, int n) {
  for (int e = threadIdx.x; e < n; e += blockDim.x) dst[e] = src[e];
}

// ---------------------------------------------------------------------------------
// block helpers
// ---------------------------------------------------------------------------------
// Block sum of nv per-thread values (each wave xor-reduces, then a fixed 4-way sum);
// result in out[0..nv) of LDS.  red: [NW][nv].
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const float s = wsum(v[q]);
    if (lane == 0) red[w * NV + q] = s;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NV; q += NT)
    out[q] = ((red[q] + red[NV + q]) + red[2 * NV + q]) + red[3 * NV + q];
  __syncthreads();
}

// ---------------------------------------------------------------------------------
// kw_derive: weight products every phase reads (1 block)
// ---------------------------------------------------------------------------------
// With bpow (a training step that ends in kw_reduce_adam) also the step's loss terms and
// Adam factors from the pre-update parameters (D_AUX; k_adam_tf's formulas), so that no
// block of the final reduce + Adam kernel depends on another.
__device__ __forceinline__ void derive_body(const float* __restrict__ W, const Off& o, int Nc,
                                            float* __restrict__ D,
                                            const float* __restrict__ bpow) {
  const int t = threadIdx.x;
  if (bpow) {
    __shared__ float red[NW * 3];
    __shared__ float tot[3];
    const int np = o.NP, TH1 = np - 4, TH2 = np - 2;
    float v[3] = {0.f, 0.f, 0.f};
    for (int p = t; p < np; p += NT) {
      const float w = W[p];
      v[0] = fmaf(w, w, v[0]);
      if (p >= TH1 && p < TH1 + 2) v[1] = fmaf(w, w, v[1]);
      if (p >= TH2 && p < TH2 + 2) v[2] = fmaf(w, w, v[2]);
    }
    block_sum<3>(v, red, tot);
    if (t == 0) {
      const float n1 = sqrtf(tot[1]), n2 = sqrtf(tot[2]);
      const float b1p = bpow[0], b2p = bpow[1];
      D[D_AUX + 0] = 0.0005f * tot[0];
      D[D_AUX + 1] = 0.01f * (n2 + n1);
      D[D_AUX + 2] = n1;
      D[D_AUX + 3] = n2;
      D[D_AUX + 4] = sqrtf(1.f - b2p) / (1.f - b1p);
      D[D_AUX + 5] = b1p * 0.9f;
      D[D_AUX + 6] = b2p * 0.999f;
    }
  }
  const float Nc1 = (float)(Nc - 1);
  for (int e = t; e < H * H; e += NT) {           // M[l][k] = sum_m V2[l][m] U1e[m][k]
    const int l = e / H, k = e - l * H;
    float acc = 0.f;
    for (int m = 0; m < H; ++m)
      acc = fmaf(W[o.H1_W2 + l * H + m], W[o.H2_W1 + (2 + m) * H + k], acc);
    D[D_M + e] = acc;
  }
  if (t < H) {
    float cu = 0.f;
    for (int m = 0; m < H; ++m) cu = fmaf(W[o.H1_B2 + m], W[o.H2_W1 + (2 + m) * H + t], cu);
    cu *= Nc1;
    D[D_T0 + t] = cu;
    D[D_S0 + t] = cu + (W[o.H2_W1 + t] + W[o.H2_B1 + t]);
    D[D_EPS + t] = W[o.H2_W1 + H + t] - W[o.H2_W1 + t];
    D[D_CV + t] = W[o.H2_W2 + 2 * t + 1] - W[o.H2_W2 + 2 * t];
    D[D_DLT + t] = W[o.H1_W1 + 9 * H + t] - W[o.H1_W1 + 8 * H + t];
    if (o.EC_W1 >= 0) {
      D[D_EED + t] = W[o.EC_W1 + H + t] - W[o.EC_W1 + t];
      D[D_EEC + t] = W[o.EC_W2 + 2 * t + 1] - W[o.EC_W2 + 2 * t];
      D[D_EECQ + t] = -1.4426950408889634f * D[D_EEC + t];
      if (t == 0) D[D_EEBQ] = -1.4426950408889634f * (W[o.EC_B2 + 1] - W[o.EC_B2]);
    }
  }
}

__global__ __launch_bounds__(NT) void kw_derive(const float* __restrict__ W, Off o, int Nc,
                                                float* __restrict__ D,
                                                const float* __restrict__ bpow) {
  derive_body(W, o, Nc, D, bpow);
}

// The m-range of the other index a wave sweeps, split around this tile's own nodes
// [t0, t0 + 64) so the self pair (m == node) is masked only where it can occur.
template <class F>
__device__ __forceinline__ void sweep(int N, int t0, F f) {
  const int w = uni(threadIdx.x >> 6);
  const int lo = (N * w) / NW, hi = (N * (w + 1)) / NW;
  const int a = lo < t0 ? lo : t0, e1 = hi < t0 ? hi : t0;
  const int t1 = t0 + TN;
  const int b0 = lo > t0 ? lo : t0, b1 = hi < t1 ? hi : t1;
  const int c0 = lo > t1 ? lo : t1;
  for (int m = a; m < e1; ++m) f(m, false);
  for (int m = b0; m < b1; ++m) f(m, true);
  for (int m = c0; m < hi; ++m) f(m, false);
}

__device__ __forceinline__ float bitf(const uint32_t* row, int m) {
  return ((row[m >> 5] >> (m & 31)) & 1u) ? 1.f : 0.f;
}

// ---- 8-wave pass helpers (hunk and entity-edge classifier passes) ----
constexpr int NTP = 512;
constexpr int NWP = NTP / 64;
constexpr int CHM = 128;
constexpr int H2 = H / 2;
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 relu2(f2 v) { return __builtin_elementwise_max(v, (f2){0.f, 0.f}); }
// [z > 0] on both halves in one op: clamp(z * 2^126, 0, 1) (exact for normal z; -0, NaN -> 0)
__device__ __forceinline__ f2 step2(f2 z) {
  f2 r;
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(z), "v"((f2){0x1p126f, 0x1p126f}));
  return r;
}
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// ln x for x in [1, 2] (the two-class CE's log(1 + e^-|d|) and log(e0 + e1)): v_log_f32
// (log2, ~1 ulp, no denormal range to guard) times ln 2 -- 2 VALU ops where logf expands to
// a denormal-scaled, split-constant sequence of ~11
__device__ __forceinline__ float ln_1to2(float x) { return __builtin_amdgcn_logf(x) * 0.693147182f; }
// [x + c > 0] for a packed pair in ONE op where only the step of the sum is used (not the
// sum): clamp(fma(x, 2^64, c 2^64)).  The fma rounds the exact (x + c) 2^64 once, so the
// result is 0 for x + c <= 0 (-0, NaN: 0) and 1 for every x + c >= 2^-64; it differs from
// step2(fl(x + c)) only for 0 < x + c < 2^-64.  cs = c 2^64 (exact and finite for |c| <
// 2^63; -inf masks the pair).
#ifndef HDG_STEPF
#define HDG_STEPF 1
#endif
constexpr float STEP_S = 0x1p64f;
__device__ __forceinline__ f2 stepf2(f2 x, f2 cs) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 clamp"
      : "=v"(r) : "v"(x), "s"((f2){STEP_S, STEP_S}), "v"(cs));
  return r;
}
__device__ __forceinline__ f2 ld2(const float* p) { return (f2){p[0], p[1]}; }

// rows [c0, c1) of a [N][H] array -> LDS (float4 copies; rows are 80 B, 16-B aligned)
__device__ __forceinline__ void stage_rows(float* dst, const float* src, int c0, int c1) {
  const float4* s4 = reinterpret_cast<const float4*>(src + (size_t)c0 * H);
  float4* d4 = reinterpret_cast<float4*>(dst);
  for (int e = threadIdx.x; e < (c1 - c0) * (H / 4); e += blockDim.x) d4[e] = s4[e];
}

// sum the NWP waves' packed accumulators of the 64 lane-nodes -> res[64][HP]
__device__ __forceinline__ void combine8(const f2 (&acc)[H2], float* buf, float* res) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    buf[(w * TN + lane) * HP + 2 * kk] = acc[kk].x;
    buf[(w * TN + lane) * HP + 2 * kk + 1] = acc[kk].y;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H;
    float s = buf[n * HP + k];
#pragma unroll
    for (int q = 1; q < NWP; ++q) s += buf[(q * TN + n) * HP + k];
    res[n * HP + k] = s;
  }
  __syncthreads();
}

template <int NV>
__device__ __forceinline__ void block_sum8(float (&v)[NV], float* red, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const float s = wsum(v[q]);
    if (lane == 0) red[w * NV + q] = s;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NV; q += NTP) {
    float s = red[q];
    for (int u = 1; u < NWP; ++u) s += red[u * NV + q];
    out[q] = s;
  }
  __syncthreads();
}

#ifndef HDG_WPRIO   // wave priority by progress through the wave's share: kw_hunk_fwd and
#define HDG_WPRIO 1  // kw_hunk_mlpb (stress, dense form: 35.0 -> 33.8 and 54.3 -> 52.1 us; in
#endif               // kw_hunk_clsb it cost 66.7 -> 73.5 us, in kw_hunk_cls nothing)
// priority 3 / 2 / 1 / 0 from the start / first quarter / half / three quarters of a wave's
// share (the issue arbiter then favours waves that are behind; all values wave-uniform)
__device__ __forceinline__ void share_prio(int m, int lo, int hi) {
  if constexpr (HDG_WPRIO) {
    const int d = m - lo, n = hi - lo;
    if (d == 0) __builtin_amdgcn_s_setprio(3);
    else if (d == n >> 2) __builtin_amdgcn_s_setprio(2);
    else if (d == n >> 1) __builtin_amdgcn_s_setprio(1);
    else if (d == (3 * n) >> 2) __builtin_amdgcn_s_setprio(0);
  }
}
__device__ __forceinline__ void prio0() {
  if constexpr (HDG_WPRIO) __builtin_amdgcn_s_setprio(0);
}
#ifndef HDG_EPRIO   // experiment: the same in kw_ee_fwd's relation loop / kw_ee_clsb's trips
#define HDG_EPRIO 0
#endif
__device__ __forceinline__ void trip_prio_e(int it, int n) {
  if constexpr (HDG_EPRIO) {
    if (it == 0) __builtin_amdgcn_s_setprio(3);
    else if (it == n >> 2) __builtin_amdgcn_s_setprio(2);
    else if (it == n >> 1) __builtin_amdgcn_s_setprio(1);
    else if (it == (3 * n) >> 2) __builtin_amdgcn_s_setprio(0);
  }
}
__device__ __forceinline__ void prio0_e() {
  if constexpr (HDG_EPRIO) __builtin_amdgcn_s_setprio(0);
}

// the wave's share [lo, hi) of chunk [c0, c1)
__device__ __forceinline__ void wave_share(int c0, int c1, int& lo, int& hi) {
  const int w = uni(threadIdx.x >> 6), len = c1 - c0;
  lo = c0 + (len * w) / NWP;
  hi = c0 + (len * (w + 1)) / NWP;
}


// ---------------------------------------------------------------------------------
// Sorted-x entity sums.  For hidden unit k the a = 0 pre-activation of pair (i, j) is
// affine in the scalar x_j, so {j : z_ij > 0} is a prefix or a suffix of the x-sorted
// order: a binary search over the nd distinct values finds it, and the f64 prefix sums
// give its relu sum (count * offset + slope * sum x).  The a = 1 pairs add
// relu(z + d) - relu(z) over the set bits of the node's row (a) / column (a^T), and the
// diagonal is removed once per side.  O(Ne H (log nd + deg)) per commit instead of
// O(Ne^2 H).  Rounding contract (fp contract off): E1 row form z0 = fl(u_i + fl(x_j w1)),
// EE z0 = fma(x_j, w, U_i); the searches, corrections and backward masks share it.
// Thread map: wave g of the block owns hidden units [5g, 5g+5), lane = node of the tile.
// ---------------------------------------------------------------------------------
constexpr int KPW = H / NW;   // hidden units per wave

struct SortTabs {
  const float* xu;
  const int* cum;
  const double* pxd;
  int nd;
  const float* xs;    // the commit's x staged in LDS (stage_tabs with xg)
};

__device__ __forceinline__ SortTabs sort_tabs(const uint32_t* prep, const GenPrep& GP, int b) {
  const uint32_t* pp = prep + (size_t)b * GP.words;
  SortTabs T;
  T.xu = reinterpret_cast<const float*>(pp + GP.xu);
  T.cum = reinterpret_cast<const int*>(pp + GP.cum);
  T.pxd = reinterpret_cast<const double*>(pp + GP.pxd);
  T.nd = (int)pp[GP.meta];
  T.xs = nullptr;
  return T;
}

// the commit's sorted tables copied into LDS (dynamic, sort_lds_bytes); all threads
__device__ __forceinline__ SortTabs stage_tabs(const uint32_t* prep, const GenPrep& GP, int b,
                                               int Ne, void* lds, const float* xg = nullptr) {
  const SortTabs G = sort_tabs(prep, GP, b);
  const int NE4 = (Ne + 3) & ~3;
  double* pxd = reinterpret_cast<double*>(lds);
  int* cum = reinterpret_cast<int*>(pxd + NE4 + 4);
  float* xu = reinterpret_cast<float*>(cum + NE4 + 4);
  float* xs = xu + NE4;
  for (int e = threadIdx.x; e <= G.nd; e += blockDim.x) {
    pxd[e] = G.pxd[e];
    cum[e] = G.cum[e];
    if (e < G.nd) xu[e] = G.xu[e];
  }
  if (xg) {  // the neighbour walks read x_j from LDS, not one dependent HBM load each;
             // xs[Ne] = NaN for the lists' sentinel (a clamped fma turns it into 0)
    for (int e = threadIdx.x; e < Ne; e += blockDim.x) xs[e] = xg[e];
    if (threadIdx.x == 0) xs[Ne] = __builtin_nanf("");
  }
  __syncthreads();
  SortTabs T;
  T.xu = xu;
  T.cum = cum;
  T.pxd = pxd;
  T.nd = G.nd;
  T.xs = xg ? xs : nullptr;
  return T;
}

__host__ __device__ inline size_t sort_lds_bytes(int Ne) {
  const size_t NE4 = (Ne + 3) & ~3;
  return (NE4 + 4) * 8 + (NE4 + 4) * 4 + (2 * NE4 + 4) * 4;   // pxd, cum, xu, x (+ sentinel)
}

__device__ __forceinline__ int top_pow2(int n) { return 1 << (31 - __builtin_clz((unsigned)n)); }

// boundary q of the set {distinct values v : pred(v)} when pred is monotone: with
// inc = pred increasing in v the set is [q, nd) (suffix), otherwise [0, q) (prefix);
// NB independent searches in lockstep (search n: pred(n, v), increasing when inc[n]): one
// LDS round trip per level for all of them instead of one per level and search
template <int NB, class P>
__device__ __forceinline__ void set_bounds(const SortTabs& T, const bool (&inc)[NB],
                                           int (&q)[NB], P pred) {
#pragma unroll
  for (int n = 0; n < NB; ++n) q[n] = 0;
  for (int s = top_pow2(T.nd); s > 0; s >>= 1) {
    float xv[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int m = q[n] + s - 1;
      xv[n] = T.xu[m < T.nd ? m : T.nd - 1];
    }
#pragma unroll
    for (int n = 0; n < NB; ++n)
      if (q[n] + s - 1 < T.nd && pred(n, xv[n]) != inc[n]) q[n] += s;
  }
}

// walk node i's neighbour id list (list_layout; side 0: a_ij = 1, 1: a_ji = 1) four ids per
// 8-byte load: f(j) for each id of a group, the sentinel Ne included (callers make it a
// zero term).  One independent group of loads per trip instead of a bit walk whose trip
// count is the set bits of every word.
// part / nparts: this caller's share of the list's 4-id groups (contiguous, in order).
template <int LB = 4, class F>
__device__ __forceinline__ void for_list(const uint32_t* prep, int side, int b, int i, int Ne,
                                         int Nc, F f, int part = 0, int nparts = 1) {
  const int B = gridDim.y, LS = list_stride(Ne);
  const ListLayout L = list_layout(B, Ne, Nc);
  const size_t r = ((size_t)side * B + b) * Ne + i;
  const int ng = ((int)prep[L.cnt + r] + 3) >> 2;
  const uint2* ids = reinterpret_cast<const uint2*>(
      reinterpret_cast<const uint16_t*>(prep + L.ids) + r * LS);
  const int g1 = (ng * (part + 1)) / nparts;
  // LB groups' loads issued together before any is used (clamped to the list, so always in
  // bounds): one HBM round trip per LB groups instead of one per group -- the walk is
  // latency-bound, the trip count being the longest list of the wave's lanes
  for (int g0 = (ng * part) / nparts; g0 < g1; g0 += LB) {
    uint2 q[LB];
#pragma unroll
    for (int u = 0; u < LB; ++u) q[u] = ids[g0 + u < g1 ? g0 + u : g0];
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      if (g0 + u < g1) {
        f((int)(q[u].x & 0xffffu));
        f((int)(q[u].x >> 16));
        f((int)(q[u].y & 0xffffu));
        f((int)(q[u].y >> 16));
      }
    }
  }
}

// a = 1 correction of one neighbour as ONE clamped fma per hidden unit (the fused path's
// entity_fwd form): z0 = A x_j + B is affine in x_j, and
//   relu(z0 + d) - relu(z0) = d clamp((s z0 + t) / d, 0, 1),  (s, t) = (1, d) for d >= 0,
//   (-1, 0) for d < 0,
// so the correction sum is d * sum_j clamp(x_j ca + cb, 0, 1) with ca = s A / d,
// cb = (s B + t) / d; |d| < 2^-100 counts as d = 0 (below the sum's rounding)
struct ClampCoef {
  float ca, cb;
};
__device__ __forceinline__ ClampCoef clamp_coef(const float A, const float B, const float d) {
  const float sg = d >= 0.f ? 1.f : -1.f, tg = d >= 0.f ? d : 0.f;
  const float rd = fabsf(d) >= 0x1p-100f ? 1.f / d : 0.f;
  return {sg * A * rd, fmaf(sg, B, tg) * rd};
}
__device__ __forceinline__ f2 clamp_fma2(const float x, const f2 a, const f2 b) {
  f2 xx;
  xx.x = x;
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(r) : "v"(xx), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float clamp_fma1(const float x, const float a, const float b) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(x), "v"(a), "v"(b));
  return r;
}

// MODE 0 (E1, model_2.py:161-188): P_i = sum_{j!=i} relu(z_ij) + relu(z_ji)
// MODE 1 (EE, model_4.py:206-243): R1_i = sum_{j!=i} relu(z'_ij), C1_i = sum relu(z'_ji)
// HALVES = 2 (8 waves): waves g + 4 hw; the halves hw split each node's neighbour lists (hw 1
// hands its sums over through LDS, `hand`), hw 0 also does the dense part and the stores
template <int MODE, int HALVES>
__device__ __forceinline__ void ent_fwd_sorted(const float* __restrict__ x,
                                               const uint32_t* __restrict__ abits,
                                               const uint32_t* __restrict__ aT,
                                               const uint32_t* __restrict__ prep,
                                               const float* __restrict__ W, const Off& o, int Ne,
                                               int Nc, float* __restrict__ out0,
                                               float* __restrict__ out1, float* hand) {
#pragma clang fp contract(off)
  const GenPrep GP = gen_prep(Ne, Nc);
  const int b = blockIdx.y, t0 = blockIdx.x * TN;
  const int lane = threadIdx.x & 63, g = uni((threadIdx.x >> 6) & 3);
  const int hw = HALVES == 2 ? uni(threadIdx.x >> 8) : 0;
  const int i0 = t0 + lane;
  extern __shared__ __attribute__((aligned(16))) double tabs_lds[];
  const SortTabs T = stage_tabs(prep, GP, b, Ne, tabs_lds, x + (size_t)b * Ne);
  if (HALVES == 1 && i0 >= Ne) return;   // no barriers below (HALVES = 2: one, lanes clamped)
  const bool live = i0 < Ne;
  const int i = live ? i0 : Ne - 1;
  const float* xb = T.xs;
  const float xi = xb[i];
  float u[KPW], v[KPW], s1[KPW], s2[KPW], c0[KPW], wa[KPW], wb[KPW], dd[KPW];
  double dense[KPW], dense2[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const int k = g * KPW + kk;
    if constexpr (MODE == 0) {
      const float w0 = W[o.E1_W1 + k], w1 = W[o.E1_W1 + H + k], w2 = W[o.E1_W1 + 2 * H + k];
      c0[kk] = w2 + W[o.E1_B1 + k];
      dd[kk] = W[o.E1_W1 + 3 * H + k] - w2;
      wa[kk] = w0;
      wb[kk] = w1;
      u[kk] = fmaf(xi, w0, c0[kk]);
      v[kk] = xi * w1;
    } else {
      const float w = W[o.EE_W11 + k], w20 = W[o.EE_W12 + k];
      dd[kk] = W[o.EE_W12 + H + k] - w20;
      wa[kk] = w;
      u[kk] = fmaf(xi, w, w20 + W[o.EE_B1 + k]);
    }
    s1[kk] = 0.f;
    s2[kk] = 0.f;
  }
  // the set boundaries of every unit (and both pair orders in MODE 0) searched in lockstep
  constexpr int NS = MODE == 0 ? 2 * KPW : KPW;
  bool sinc[NS];
  int sb[NS];
  if (!hw) {
#pragma unroll
  for (int n = 0; n < NS; ++n) sinc[n] = (MODE == 0 && n < KPW ? wb[n] : wa[n % KPW]) >= 0.f;
  set_bounds<NS>(T, sinc, sb, [&](int n, float xq) {
    if constexpr (MODE == 0) {
      if (n < KPW) return (u[n] + xq * wb[n]) > 0.f;
      const int kk = n - KPW;
      return (fmaf(xq, wa[kk], c0[kk]) + v[kk]) > 0.f;
    } else {
      return fmaf(xq, wa[n], u[n]) > 0.f;
    }
  });
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    if constexpr (MODE == 0) {
      const float w0 = wa[kk], w1 = wb[kk], uu = u[kk], vv = v[kk], cc = c0[kk];
      const int br = sb[kk], bc = sb[KPW + kk];
      const int rlo = w1 >= 0.f ? br : 0, rhi = w1 >= 0.f ? T.nd : br;
      const int clo = w0 >= 0.f ? bc : 0, chi = w0 >= 0.f ? T.nd : bc;
      double acc = (double)(T.cum[rhi] - T.cum[rlo]) * (double)uu +
                   (double)w1 * (T.pxd[rhi] - T.pxd[rlo]);
      acc += (double)(T.cum[chi] - T.cum[clo]) * ((double)vv + (double)cc) +
             (double)w0 * (T.pxd[chi] - T.pxd[clo]);
      acc -= 2.0 * (double)relu(uu + vv);
      dense[kk] = acc;
    } else {
      const float w = wa[kk], uu = u[kk];
      const int br = sb[kk];
      const int lo = w >= 0.f ? br : 0, hi = w >= 0.f ? T.nd : br;
      const double acc = (double)(T.cum[hi] - T.cum[lo]) * (double)uu +
                         (double)w * (T.pxd[hi] - T.pxd[lo]) - (double)relu(fmaf(xi, w, uu));
      dense[kk] = acc;
      dense2[kk] = acc;
    }
  }
  }   // (hw 0)
  WSTAMP(7, 1);
  // a = 1 corrections: row bits (pairs (i, j)), column bits (pairs (j, i)), one clamped
  // packed fma per two hidden units and neighbour (clamp_coef); KPW = 5: two packed
  // pairs + one scalar unit
  static_assert(KPW == 5, "packed correction layout");
  {
    f2 ra[2], rb2[2], ca[2], cb[2];
    float rat, rbt, cat, cbt;
    ClampCoef q[KPW], qc[KPW];
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      // row form z0 = u + x_j w1 (MODE 0) / x_j w + u (MODE 1); column form
      // z0 = x_j w0 + c0 + v (MODE 0) / x_j w + u (MODE 1)
      q[kk] = clamp_coef(MODE == 0 ? wb[kk] : wa[kk], u[kk], dd[kk]);
      qc[kk] = clamp_coef(wa[kk], MODE == 0 ? c0[kk] + v[kk] : u[kk], dd[kk]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ra[h] = (f2){q[2 * h].ca, q[2 * h + 1].ca};
      rb2[h] = (f2){q[2 * h].cb, q[2 * h + 1].cb};
      ca[h] = (f2){qc[2 * h].ca, qc[2 * h + 1].ca};
      cb[h] = (f2){qc[2 * h].cb, qc[2 * h + 1].cb};
    }
    rat = q[4].ca; rbt = q[4].cb; cat = qc[4].ca; cbt = qc[4].cb;
    f2 sr[2] = {(f2){0.f, 0.f}, (f2){0.f, 0.f}}, sc[2] = {sr[0], sr[1]};
    float srt = 0.f, sct = 0.f;
    for_list<2>(prep, 0, b, i, Ne, Nc, [&](int j) {   // xb[Ne] = NaN: clamps to 0
      const float xj = HDG_ABL_XJ ? xb[lane + (j & 1)] : xb[j];
      sr[0] += clamp_fma2(xj, ra[0], rb2[0]);
      sr[1] += clamp_fma2(xj, ra[1], rb2[1]);
      srt += clamp_fma1(xj, rat, rbt);
    }, hw, HALVES);
    for_list<2>(prep, 1, b, i, Ne, Nc, [&](int j) {
      const float xj = HDG_ABL_XJ ? xb[lane + (j & 1)] : xb[j];
      sc[0] += clamp_fma2(xj, ca[0], cb[0]);
      sc[1] += clamp_fma2(xj, ca[1], cb[1]);
      sct += clamp_fma1(xj, cat, cbt);
    }, hw, HALVES);
    if constexpr (HALVES == 2) {                  // hw 1's sums, added in a fixed order
      float* hd = hand + g * 10 * TN + lane;
      if (hw) {
        hd[0 * TN] = sr[0].x; hd[1 * TN] = sr[0].y; hd[2 * TN] = sr[1].x; hd[3 * TN] = sr[1].y;
        hd[4 * TN] = srt;
        hd[5 * TN] = sc[0].x; hd[6 * TN] = sc[0].y; hd[7 * TN] = sc[1].x; hd[8 * TN] = sc[1].y;
        hd[9 * TN] = sct;
      }
      __syncthreads();
      if (hw) return;                             // no barriers below
      sr[0] += (f2){hd[0 * TN], hd[1 * TN]};
      sr[1] += (f2){hd[2 * TN], hd[3 * TN]};
      srt += hd[4 * TN];
      sc[0] += (f2){hd[5 * TN], hd[6 * TN]};
      sc[1] += (f2){hd[7 * TN], hd[8 * TN]};
      sct += hd[9 * TN];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      s1[2 * h] = sr[h].x * dd[2 * h];
      s1[2 * h + 1] = sr[h].y * dd[2 * h + 1];
      s2[2 * h] = sc[h].x * dd[2 * h];
      s2[2 * h + 1] = sc[h].y * dd[2 * h + 1];
    }
    s1[4] = srt * dd[4];
    s2[4] = sct * dd[4];
  }
  if (!live) return;
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const size_t gi = ((size_t)b * Ne + i) * H + g * KPW + kk;
    if constexpr (MODE == 0) {
      out0[gi] = (float)dense[kk] + (s1[kk] + s2[kk]);
    } else {
      out0[gi] = (float)dense[kk] + s1[kk];
      out1[gi] = (float)dense2[kk] + s2[kk];
    }
  }
}


// ---------------------------------------------------------------------------------
// node_fwd_tile (kw_ent_fwd's tail, one 64-node tile)
//   ENT (model_2.py:181-205): E_bar = P W5 + 2(Ne-1) b5; h = relu([x, E_bar] W1' + b1');
//        o = h w2' + b2'; x' = relu(o)
//   EE  (model_4.py:232-243, 282-304): R = R1 Q2 + (Ne-1) q2, C = C1 Q2 + (Ne-1) q2;
//        classifier first-layer operands rho = R U1e' + U1'[0] + b1', gam = C U1e'
// ---------------------------------------------------------------------------------
// 64 x 20 row-block products on MFMA: f(n, k, c) with c = sum_m As[n][m] Wm[m][k] for the
// tile's 64 rows (As [64][HP] in LDS, Wm [H][H] row-major in LDS); 4 x 2 16x16 tiles over
// the block's waves; columns >= H read the zero word kz with stride 0 and are not passed on
// (Wm element (m, k) at Wm[m * SM + k * SK]: SM = H, SK = 1 row-major, SM = 1, SK = H for
// the transposed weight)
template <int SM = H, int SK = 1, class F>
__device__ __forceinline__ void rows_x_w(const float* As, const float* Wm, const float* kz,
                                         F f) {
  const int lane = threadIdx.x & 63;
  for (int tile = threadIdx.x >> 6; tile < 8; tile += blockDim.x >> 6) {   // wave-uniform
    const int n0 = (tile >> 1) * 16, kc = (tile & 1) * 16 + (lane & 15);
    const bool cv = kc < H;
    const f4v c = mfma_tile16_p(As + (n0 + (lane & 15)) * HP, 1, cv ? Wm + kc * SK : kz,
                                cv ? SM : 0, H, lane);
    if (cv)
#pragma unroll
      for (int j = 0; j < 4; ++j) f(n0 + 4 * (lane >> 4) + j, kc, c[j]);
  }
}

struct NodeFwdOut {
  float *Eb, *hE, *ov, *xp, *Rn, *Cn, *rho, *gmm;
};

// the tile's 64 nodes (t0 = blockIdx.x * TN, commit blockIdx.y): ENT (ent_part) or EE
__device__ __forceinline__ void node_fwd_tile(const float* __restrict__ x,
                                              const float* __restrict__ W, const Off& o, int Ne,
                                              bool ent_part, const float* __restrict__ P,
                                              const float* __restrict__ R1,
                                              const float* __restrict__ C1, const NodeFwdOut& no) {
  float *Eb = no.Eb, *hE = no.hE, *ov = no.ov, *xp = no.xp;
  float *Rn = no.Rn, *Cn = no.Cn, *rho = no.rho, *gmm = no.gmm;
  __shared__ float A[TN * HP], Bs[TN * HP], Cs[TN * HP], Ds[TN * HP];
  __shared__ float Wl[896];                       // the block's weights, staged once
  __shared__ float kz[1];                         // 0.f: stride-0 operand of padding tiles
  const int b = blockIdx.y, t0 = blockIdx.x * TN, t = threadIdx.x;
  const int nn = Ne - t0 < TN ? Ne - t0 : TN;
  const size_t base = ((size_t)b * Ne + t0) * H;
  const float Ne1 = (float)(Ne - 1);
  if (t == 0) kz[0] = 0.f;
  // rows n >= nn of the LDS tiles are never stored (MFMA rows are independent)
  if (ent_part) {
    const float *W5 = Wl, *B5 = Wl + 400, *W1e = Wl + 420, *B1e = Wl + 840, *W2e = Wl + 860;
    stage_w(Wl, W + o.E1_W5, 420);                // W5 | b5
    stage_w(Wl + 420, W + o.E3_W1, 461);          // W1' | b1' | w2' | b2'
    for (int e = t; e < nn * H; e += blockDim.x) A[(e / H) * HP + e % H] = P[base + e];
    __syncthreads();
    rows_x_w(A, W5, kz, [&](int n, int k, float c) {   // E_bar = P W5 + 2 (Ne-1) b5
      const float v = c + (2.f * Ne1) * B5[k];
      Bs[n * HP + k] = v;
      if (n < nn) Eb[base + n * H + k] = v;
    });
    __syncthreads();
    rows_x_w(Bs, W1e + H, kz, [&](int n, int k, float c) {   // h = relu(x W1'[0] + E_bar W1'[1:] + b1')
      const float xv = n < nn ? x[(size_t)b * Ne + t0 + n] : 0.f;
      const float v = relu(fmaf(xv, W1e[k], c) + B1e[k]);
      Cs[n * HP + k] = v;
      if (n < nn) hE[base + n * H + k] = v;
    });
    __syncthreads();
    for (int n = t; n < nn; n += blockDim.x) {
      float acc = Wl[880];
      for (int k = 0; k < H; ++k) acc = fmaf(Cs[n * HP + k], W2e[k], acc);
      ov[(size_t)b * Ne + t0 + n] = acc;
      xp[(size_t)b * Ne + t0 + n] = relu(acc);
    }
    return;
  }
  const float *Q2 = Wl, *q2 = Wl + 400, *P1 = Wl + 420, *p1b = Wl + 860;
  stage_w(Wl, W + o.EE_W2, 420);                  // Q2 | q2
  stage_w(Wl + 420, W + o.EC_W1, 460);            // U1' (22 x 20) | b1'
  for (int e = t; e < nn * H; e += blockDim.x) {
    A[(e / H) * HP + e % H] = R1[base + e];
    Bs[(e / H) * HP + e % H] = C1[base + e];
  }
  __syncthreads();
  rows_x_w(A, Q2, kz, [&](int n, int k, float c) {      // R = R1 Q2 + (Ne-1) q2
    const float v = c + Ne1 * q2[k];
    Cs[n * HP + k] = v;
    if (n < nn) Rn[base + n * H + k] = v;
  });
  rows_x_w(Bs, Q2, kz, [&](int n, int k, float c) {     // C = C1 Q2 + (Ne-1) q2
    const float v = c + Ne1 * q2[k];
    Ds[n * HP + k] = v;
    if (n < nn) Cn[base + n * H + k] = v;
  });
  __syncthreads();
  rows_x_w(Cs, P1 + 2 * H, kz, [&](int n, int k, float c) {   // rho = R U1'[2:] + U1'[0] + b1'
    if (n < nn) rho[base + n * H + k] = c + (P1[k] + p1b[k]);
  });
  rows_x_w(Ds, P1 + 2 * H, kz, [&](int n, int k, float c) {   // gam = C U1'[2:]
    if (n < nn) gmm[base + n * H + k] = c;
  });
}


// grid (te (+1), B, 1 + EE): z = 0 the entity stage (variants 2 / 4), else the EE stage.
// D != NULL: one more x column whose block (te, 0, 0) runs kw_derive's work (no kernel of
// its own; nothing here reads D).  HALVES = 2: 8 waves, the neighbour walks split over two
// wave halves and node_fwd_tile's 8 MFMA tiles one per wave, while the grid fits 2 blocks
// per CU (ent_fwd_halves); HALVES = 1: 4 waves
template <int HALVES>
__global__ __launch_bounds__(256 * HALVES) __attribute__((amdgpu_waves_per_eu(4))) void kw_ent_fwd(const float* __restrict__ x,
                                                 const uint32_t* __restrict__ abits,
                                                 const uint32_t* __restrict__ aT,
                                                 const uint32_t* __restrict__ prep,
                                                 const float* __restrict__ W, Off o, int Ne,
                                                 int Nc, int ent, float* __restrict__ P,
                                                 float* __restrict__ R1, float* __restrict__ C1,
                                                 float* __restrict__ D,
                                                 const float* __restrict__ bpow, NodeFwdOut no) {
  if (D && blockIdx.x == gridDim.x - 1) {       // block-uniform
    if (blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < NT) derive_body(W, o, Nc, D, bpow);
    return;
  }
  __shared__ float hand[HALVES == 2 ? NW * 10 * TN : 1];   // hw 1's walk sums [g][10][lane]
  WSTAMP(7, 0);
  const bool ent_part = blockIdx.z == 0 && ent;
  if (ent_part)
    ent_fwd_sorted<0, HALVES>(x, abits, aT, prep, W, o, Ne, Nc, P, nullptr, hand);
  else
    ent_fwd_sorted<1, HALVES>(x, abits, aT, prep, W, o, Ne, Nc, R1, C1, hand);
  // the per-node products on the tile (node_fwd_tile): its inputs are this block's outputs
  // (global writes made visible to the block by the barrier)
  WSTAMP(7, 2);
  __syncthreads();
  WSTAMP(7, 3);
  node_fwd_tile(x, W, o, Ne, ent_part, P, R1, C1, no);
  WSTAMP(7, 4);
}

// ---------------------------------------------------------------------------------
// kw_ee_fwd  grid (ceil(Ne / TF), B), 8 waves
//   model_4: e'_ij = softmax(U2'^T relu(P1'^T [1-a, a, eff_ij] + p1) + p2) replaces the
//   one-hot E_edge in B_2 (model_4.py:95-97), and marshalling_B2 bins B_2 by the index
//   file's hunk maps: n_c[2+m] += e'_r[m] for c in {hid[i'], hid[j']} of every relation
//   r < n(n-1) on the n-grid (utils2.py:121-137).  Relations outside that range feed
//   nothing, so only they are evaluated.  The two-class softmax is a sigmoid of the logit
//   difference: e = exp(-delta) = 2^delta' (prescaled D_EECQ / D_EEBQ), p1 = 1 / (1 + e),
//   p0 = e p1; the weight constants are wave-uniform scalar loads.
//   A block takes TF = 32 index rows i'; each half of a wave holds all 32 (one per lane) and
//   walks its own sixteenth of the j' range, so a 200-row commit fills 7 blocks (224 lane
//   rows) instead of 4 x 64.  Relation r -> entity pair (i, j) on the Ne-grid is advanced
//   incrementally.  kappa = rho_i + (gam_j + a d): rho_i in registers (reloaded when the
//   lane's row changes), gam and gam + d LDS tables (Ne <= EE_TAB_LDS_MAX; else read from
//   HBM, the same sums).  Source bins: per-lane sums;
//   target bins: one 32-lane sum per half-wave and step into tsum[j'], binned after the
//   loop.  Both go to the block's LDS bins in 2^-32 fixed point (integer adds: order-free),
//   which leave as one partial row per tile.
// ---------------------------------------------------------------------------------
constexpr int TF = 32;                // index rows per kw_ee_fwd block
#ifndef HDG_EEF_WAVES
#define HDG_EEF_WAVES 16              // kw_ee_fwd's waves per block in table modes 2 / 0
#endif
constexpr int EE_TAB_LDS_MAX = 400;   // Ne up to which gam, gam + d sit in LDS
__host__ __device__ inline int ee_fwd_tiles(int Ne) { return (Ne + TF - 1) / TF; }
// table modes: 1 gam and gam + d in LDS (Ne <= EE_TAB_LDS_MAX), 2 gam alone in LDS (+ a d
// by one fma per unit pair; while it fits), 0 gam rows from HBM / L2
__host__ __device__ inline size_t ee_fwd_head(int Ne, int Nc) {
  return (size_t)((2 * Nc + 1) & ~1) * 8 + (size_t)((2 * Ne + 3) & ~3) * 4;
}
constexpr size_t EE_FWD_LDS_CAP = 160 * 1024;
__host__ __device__ inline int ee_fwd_mode(int Ne, int Nc) {
  if (Ne <= EE_TAB_LDS_MAX) return 1;
  return ee_fwd_head(Ne, Nc) + (size_t)Ne * H * 4 <= EE_FWD_LDS_CAP ? 2 : 0;
}
__host__ __device__ inline size_t ee_fwd_lds(int Ne, int Nc) {
  const int m = ee_fwd_mode(Ne, Nc);
  return ee_fwd_head(Ne, Nc) + (m == 1 ? (size_t)2 * Ne * H * 4 : m == 2 ? (size_t)Ne * H * 4 : 0);
}

#ifdef HDG_EE_PROBE   // timing probe builds only (tools/probe/eefwd_probe.hip)
__device__ unsigned long long* g_ee_stamps;
#define EE_STAMP(k) const unsigned long long ee_ts##k = __builtin_amdgcn_s_memrealtime()
#define EE_FLUSH()                                                                         \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0) {                                                         \
      unsigned long long* w_ = g_ee_stamps +                                               \
          ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * NWP + (threadIdx.x >> 6)) * 8;  \
      w_[0] = ee_ts0; w_[1] = ee_ts1; w_[2] = ee_ts2; w_[3] = ee_ts3; w_[4] = ee_ts4;      \
      w_[5] = __builtin_amdgcn_s_memrealtime();                                            \
      w_[6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));                                   \
      w_[7] = __builtin_amdgcn_s_getreg(20 | (31 << 11));                                  \
    }                                                                                      \
  } while (0)
#else
#define EE_STAMP(k) do {} while (0)
#define EE_FLUSH() do {} while (0)
#endif

// NWF waves per block: 8 with the LDS tables of mode 1 (3 blocks per CU), 16 in modes 2 / 0,
// whose one block per CU (the 80 KiB gam table at Ne = 1024) otherwise ran 8 waves per CU
template <int TM, int NWF>   // table mode (ee_fwd_mode), waves per block
__global__ __launch_bounds__(64 * NWF) void kw_ee_fwd(const uint32_t* __restrict__ abits,
                                                 const int32_t* __restrict__ hidg,
                                                 const int32_t* __restrict__ nleng,
                                                 const float* __restrict__ W, Off o,
                                                 const float* __restrict__ D, int Ne, int Nc,
                                                 const float* __restrict__ rho,
                                                 const float* __restrict__ gmm,
                                                 unsigned long long* __restrict__ ncpart,
                                                 int snake, const uint32_t* __restrict__ sorder) {
#pragma clang fp contract(off)
  constexpr int NTF = 64 * NWF;
  (void)W;
  (void)o;
  extern __shared__ __attribute__((aligned(16))) unsigned long long bins[];   // [Nc][2] | ...
  float* tsum = reinterpret_cast<float*>(bins + ((2 * Nc + 1) & ~1));         // [Ne][2]
  float* gl = tsum + ((2 * Ne + 3) & ~3);                                     // gam [Ne][H]
  float* gdl = gl + Ne * H;                                                   // gam + d
  EE_STAMP(0);
  WSTAMP(5, 0);
  int b = blockIdx.y, tile = blockIdx.x;
  if (snake > 0) {   // (b, tile) by the dispatch order (the note above kw_ee_clsb)
    const int te = gridDim.x, total = te * gridDim.y, i = blockIdx.y * te + blockIdx.x;
    const int r = i / snake, q = i - r * snake;
    const int len = total - r * snake < snake ? total - r * snake : snake;
    const int sg = (int)sorder[r * snake + ((r & 1) ? len - 1 - q : q)];   // (kw_prep_order)
    b = sg >= 0 && sg < total ? sg / te : 0;
    tile = sg >= 0 && sg < total ? sg - b * te : 0;
  }
  const int t0 = tile * TF;
  const int t = threadIdx.x, lane = t & 63, wv = uni(t >> 6), half = lane >> 5;
  unsigned long long* outp = ncpart + ((size_t)b * gridDim.x + tile) * 2 * Nc;
  const float* rb = rho + (size_t)b * Ne * H;
  const float* gb = gmm + (size_t)b * Ne * H;
  // the gam table (Ne H <= 4 NTF float4 for Ne <= EE_TAB_LDS_MAX) is fetched in one batch of
  // float4 loads before the commit's length is known: one memory round trip for the stage
  // instead of one per loop trip, and none waiting on nleng
  constexpr int GQ = (EE_TAB_LDS_MAX * H / 4 + NTF - 1) / NTF;
  const int nq = Ne * H / 4;                       // H % 4 == 0: whole float4 per row
  constexpr bool LDS = TM == 1;
  float4 gv[LDS ? GQ : 1];
  if constexpr (LDS) {
#pragma unroll
    for (int u = 0; u < GQ; ++u) {
      const int q = t + u * NTF;
      gv[u] = q < nq ? reinterpret_cast<const float4*>(gb)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // the hunk ids the bins take after the loop (the lane's row i', the thread's first target
  // column), fetched with the same batch
  const int32_t* hb = hidg + (size_t)b * Ne;
  const int ipl = t0 + (lane & 31);
  const int hsv = hb[ipl < Ne ? ipl : Ne - 1];
  const int htv = hb[(t >> 1) < Ne ? (t >> 1) : Ne - 1];
  int n = nleng[b];
  n = n < 0 ? 0 : (n > Ne ? Ne : n);
  for (int c = t; c < 2 * Nc; c += NTF) bins[c] = 0ull;
  if (n < 2 || t0 >= n) {         // block-uniform: this tile holds no index row
    for (int c = t; c < 2 * Nc; c += NTF) outp[c] = 0ull;
    return;
  }
  for (int e = t; e < 2 * n; e += NTF) tsum[e] = 0.f;
  if constexpr (TM == 2) {        // gam alone: the commit's rows, float4 copies
    for (int q = t; q < nq; q += NTF)
      reinterpret_cast<float4*>(gl)[q] = reinterpret_cast<const float4*>(gb)[q];
  }
  if constexpr (LDS) {
#pragma unroll
    for (int u = 0; u < GQ; ++u) {
      const int q = t + u * NTF;
      if (q < nq) {
        const float4 d = *reinterpret_cast<const float4*>(D + D_EED + (4 * q) % H);
        reinterpret_cast<float4*>(gl)[q] = gv[u];
        reinterpret_cast<float4*>(gdl)[q] =
            make_float4(gv[u].x + d.x, gv[u].y + d.y, gv[u].z + d.z, gv[u].w + d.w);
      }
    }
  }
  __syncthreads();
  EE_STAMP(1);
  WSTAMP(5, 1);
  const int WE = (Ne + 31) >> 5;
  const int ip = t0 + (lane & 31);
  const bool live = ip < n;
  const int ipc = live ? ip : 0;
  const int part = 2 * wv + half, NPART = 2 * NWF;
  const int jlo = (n * part) / NPART, jhi = (n * (part + 1)) / NPART;
  const int trips = (n + NPART - 1) / NPART;   // >= every part's length: both halves step
  const int r0 = ipc * (n - 1) + jlo - (jlo > ipc ? 1 : 0);
  int ei = r0 / (Ne - 1), ejj = r0 - ei * (Ne - 1);
  // rho_i in registers, loaded from HBM / L2 when the lane's entity row changes (every
  // Ne - 1 relations, about once per lane at glide): per relation only the gam row is read
  // from LDS, and rho is not staged at all
  f2 rh[H2];
  const float* rsrc = rb;
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) rh[kk] = ld2(rsrc + (ei < Ne ? ei : Ne - 1) * H + 2 * kk);
  int cur = ei;
  const float bq = D[D_EEBQ];
  // the classifier's prescaled weight differences in VGPRs for the whole loop (as scalar
  // operands they were refetched through the scalar cache every relation, and the wait for
  // them joined the wait for the gam rows)
  f2 cq[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    cq[kk] = ld2(D + D_EECQ + 2 * kk);
    asm volatile("" : "+v"(cq[kk].x), "+v"(cq[kk].y));
  }
  float s0 = 0.f, s1 = 0.f;
  // class-bit words: the lane's relations walk the a-bit rows in order, so the word index
  // ei * WE + (j >> 5) grows by at most one per relation; the next word is prefetched
  // when the current one is taken, so the load's latency is never on the relation chain
  const uint32_t* ab = abits + (size_t)b * Ne * WE;
  const int wlast = Ne * WE - 1;
  int widx = (ei < Ne ? ei : Ne - 1) * WE + ((ejj + (ejj >= ei ? 1 : 0)) >> 5);
  widx = widx < wlast ? widx : wlast;
  uint32_t wcur = ab[widx], wnxt = ab[widx + 1 < wlast ? widx + 1 : wlast];
  EE_STAMP(2);
  WSTAMP(5, 2);
  for (int it = 0; it < trips; ++it) {
    trip_prio_e(it, trips);
    const int jp = jlo + it;
    const bool valid = live && jp < jhi && jp != ip;
    float p0 = 0.f, p1 = 0.f;
    if (valid) {
      const int ej = ejj + (ejj >= ei ? 1 : 0);
      if (ei != cur) {
#pragma unroll
        for (int kk = 0; kk < H2; ++kk) rh[kk] = ld2(rsrc + ei * H + 2 * kk);
        cur = ei;
      }
      const int nidx = ei * WE + (ej >> 5);
      if (nidx != widx) {
        wcur = nidx == widx + 1 ? wnxt : ab[nidx];
        widx = nidx;
        wnxt = ab[nidx + 1 < wlast ? nidx + 1 : wlast];
      }
      const bool a1 = (wcur >> (ej & 31)) & 1u;
      f2 dz = {bq, 0.f}, dzb = {0.f, 0.f};   // two chains: the fma latency overlaps
      if constexpr (LDS) {
        const float4* g4 = reinterpret_cast<const float4*>((a1 ? gdl : gl) + ej * H);
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {   // kappa = rho_i + (gam_j + a d), as kw_ee_clsb
          const float4 g = g4[v];
          const f2 ka = relu2(rh[2 * v] + (f2){g.x, g.y});
          const f2 kb = relu2(rh[2 * v + 1] + (f2){g.z, g.w});
          dz = fma2(ka, cq[2 * v], dz);
          dzb = fma2(kb, cq[2 * v + 1], dzb);
        }
      } else {   // kappa = rho_i + fma(a, d, gam_j): the same bits as gam + d for a = 1
        const float af = a1 ? 1.f : 0.f;
        const f2 a2 = {af, af};
        const float4* g4 = reinterpret_cast<const float4*>((TM == 2 ? gl : gb) + (size_t)ej * H);
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {
          const float4 g = g4[v];
          const f2 ka = relu2(rh[2 * v] + fma2(a2, ld2(D + D_EED + 4 * v), (f2){g.x, g.y}));
          const f2 kb = relu2(rh[2 * v + 1] + fma2(a2, ld2(D + D_EED + 4 * v + 2), (f2){g.z, g.w}));
          dz = fma2(ka, cq[2 * v], dz);
          dzb = fma2(kb, cq[2 * v + 1], dzb);
        }
      }
      dz += dzb;
      const float e = __builtin_amdgcn_exp2f(fminf(dz.x + dz.y, 64.f));
      p1 = __builtin_amdgcn_rcpf(1.f + e);
      p0 = e * p1;
      if (++ejj == Ne - 1) { ejj = 0; ++ei; }
    }
    s0 += p0;
    s1 += p1;
    // 32-lane sums of (p0, p1) per half: one permlane16 swap, then a 16-lane DPP reduction;
    // DPP row q of the wave ends with half q >> 1's sum of p_(q & 1)
    float x = p0, y = p1;
    swap16(x, y);
    const float v = row_total16(x + y);
    if ((lane & 15) == 0 && jp < jhi) tsum[2 * jp + ((lane >> 4) & 1)] = v;
  }
  prio0_e();
  EE_STAMP(3);
  WSTAMP(5, 3);
  if (live) {                          // source bins: the lane's row i'
    const int hs = hsv;
    if (hs >= 0 && hs < Nc) {
      atomicAdd(&bins[2 * hs], qfix(s0));
      atomicAdd(&bins[2 * hs + 1], qfix(s1));
    }
  }
  __syncthreads();
  for (int e = t; e < 2 * n; e += NTF) {   // target bins: column j' of the tile's rows
    const int ht = e == t ? htv : hb[e >> 1];
    if (ht >= 0 && ht < Nc) atomicAdd(&bins[2 * ht + (e & 1)], qfix(tsum[e]));
  }
  __syncthreads();
  // per-tile partial bins, summed in tile order by kw_cross_fwd / k_commit_step (no global
  // atomics: the L2s of the 8 XCDs are not coherent for device-scope atomics)
  EE_STAMP(4);
  WSTAMP(5, 4);
  for (int c = t; c < 2 * Nc; c += NTF) outp[c] = bins[c];
  EE_FLUSH();
}

// ---------------------------------------------------------------------------------
// kw_cross_fwd  grid (ceil(Nc/4), B), one wave per hunk c
//   marshalling_B2 (model_2.py:146-158): n_c = [K_s x', K_t x', class part] with the
//   class part = static relation counts (ncst) or the EE aggregate; then the hunk MLP
//   first layer split per node (model_2.py:257-260):
//     alpha_c = n_c V1[0:4] + V1[8] + c1,   beta_c = n_c V1[4:8]
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void kw_cross_fwd(
    const uint32_t* __restrict__ prep, const float* __restrict__ xv, const float* __restrict__ W,
    Off o, int Ne, int Nc, const unsigned long long* __restrict__ ncpart, int nt,
    float* __restrict__ nvec, float* __restrict__ alpha, float* __restrict__ beta) {
  const GenPrep PL = gen_prep(Ne, Nc);
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int c = blockIdx.x * NW + uni(threadIdx.x >> 6);
  if (c >= Nc) return;   // wave-uniform; no block barrier below
  const uint32_t* pp = prep + (size_t)b * PL.words;
  const uint16_t* ks = reinterpret_cast<const uint16_t*>(pp + PL.ks) + (size_t)c * Ne;
  const uint16_t* kt = reinterpret_cast<const uint16_t*>(pp + PL.kt) + (size_t)c * Ne;
  const float* xb = xv + (size_t)b * Ne;
  float a0 = 0.f, a1 = 0.f;
  if ((Ne & 3) == 0) {   // rows 8-byte aligned: 4 nodes per lane and load, 4 trips in flight
    constexpr int U = 4;
    for (int I0 = 4 * lane; I0 < Ne; I0 += 256 * U) {
      uint2 vs[U], vt[U];
      float4 xx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int I = I0 + 256 * u < Ne ? I0 + 256 * u : I0;   // clamped load, value unused
        vs[u] = *reinterpret_cast<const uint2*>(ks + I);
        vt[u] = *reinterpret_cast<const uint2*>(kt + I);
        xx[u] = *reinterpret_cast<const float4*>(xb + I);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (I0 + 256 * u >= Ne) break;
        const float x4[4] = {xx[u].x, xx[u].y, xx[u].z, xx[u].w};
        const uint32_t s4[4] = {vs[u].x & 0xffffu, vs[u].x >> 16, vs[u].y & 0xffffu, vs[u].y >> 16};
        const uint32_t t4[4] = {vt[u].x & 0xffffu, vt[u].x >> 16, vt[u].y & 0xffffu, vt[u].y >> 16};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a0 = fmaf((float)s4[q], x4[q], a0);
          a1 = fmaf((float)t4[q], x4[q], a1);
        }
      }
    }
  } else {
    for (int I = lane; I < Ne; I += 64) {
      const float xi = xb[I];
      a0 = fmaf((float)ks[I], xi, a0);
      a1 = fmaf((float)kt[I], xi, a1);
    }
  }
  float nv[4];
  nv[0] = wsum(a0);
  nv[1] = wsum(a1);
  if (ncpart) {                    // EE aggregate: sum of the kw_ee_fwd tile partials
    unsigned long long a2 = 0ull, a3 = 0ull;
    for (int tl = 0; tl < nt; ++tl) {
      const unsigned long long* pr = ncpart + ((size_t)b * nt + tl) * 2 * Nc;
      a2 += pr[2 * c];
      a3 += pr[2 * c + 1];
    }
    nv[2] = (float)((double)a2 * (1.0 / FIX));
    nv[3] = (float)((double)a3 * (1.0 / FIX));
  } else {
    const float* ncst = reinterpret_cast<const float*>(pp + PL.ncst);
    nv[2] = ncst[2 * c];
    nv[3] = ncst[2 * c + 1];
  }
  if (lane < 4) nvec[((size_t)b * Nc + c) * 4 + lane] = nv[lane];
  if (lane < H) {
    const int k = lane;
    float al = W[o.H1_W1 + 8 * H + k] + W[o.H1_B1 + k], be = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      al = fmaf(nv[m], W[o.H1_W1 + m * H + k], al);
      be = fmaf(nv[m], W[o.H1_W1 + (4 + m) * H + k], be);
    }
    alpha[((size_t)b * Nc + c) * H + k] = al;
    beta[((size_t)b * Nc + c) * H + k] = be;
  }
}

// ---------------------------------------------------------------------------------
// Hunk pair passes (tile of 64 hunks = lanes, 8 waves split the swept index m).  The
// swept side's node vectors are staged in LDS in chunks of CHM rows and read as
// broadcast float4; hidden units run as packed fp32 pairs.  The self pair (n, n) is not
// a relation: it is accumulated like any other and subtracted once with the identical
// expression.
// ---------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------
// kw_hunk_fwd  grid (tc, B, 2): z = 0 row pass (G), 1 column pass (H)
//   mlp_hunk_B2 first layer relu sums (model_2.py:257-275):
//     G_p = sum_{q!=p} relu(alpha_p + beta_q + y_pq delta),  H_q = sum_{p!=q} (same)
//   epilogue: sigma_p = G_p M + s0, tau_q = H_q M + t0 (classifier first layer, 304-318)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(NTP) void kw_hunk_fwd(const uint32_t* __restrict__ ybits,
                                                   const uint32_t* __restrict__ yT,
                                                   const float* __restrict__ D, int Nc,
                                                   const float* __restrict__ alpha,
                                                   const float* __restrict__ beta,
                                                   float* __restrict__ G, float* __restrict__ Hh,
                                                   float* __restrict__ sig, float* __restrict__ tau) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float os_[CHM * H];
  __shared__ float buf[NWP * TN * HP];
  __shared__ float res[TN * HP];
  __shared__ float Ml[H * H];
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN;
  const int lane = threadIdx.x & 63;
  const int nd = t0 + lane, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  stage_w(Ml, D + D_M, H * H);                    // visible after the first chunk barrier
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H;
  const float* oth = (z ? alpha : beta) + (size_t)b * Nc * H;
  const uint32_t* brow = (z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC;
  f2 ow[H2], dl[H2], acc[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    ow[kk] = ld2(own + ncl * H + 2 * kk);
    dl[kk] = ld2(D + D_DLT + 2 * kk);
    acc[kk] = (f2){0.f, 0.f};
  }
  for (int c0 = 0; c0 < Nc; c0 += CHM) {
    const int c1 = c0 + CHM < Nc ? c0 + CHM : Nc;
    __syncthreads();
    stage_rows(os_, oth, c0, c1);
    __syncthreads();
    int lo, hi;
    wave_share(c0, c1, lo, hi);
    int wi = -1;
    uint32_t word = 0;
    for (int m = lo; m < hi; ++m) {
      share_prio(m, lo, hi);
      if ((m >> 5) != wi) { wi = m >> 5; word = brow[wi]; }
      const float yf = ((word >> (m & 31)) & 1u) ? 1.f : 0.f;
      const f2 y2 = {yf, yf};
      const float4* o4 = reinterpret_cast<const float4*>(os_ + (m - c0) * H);
#pragma unroll
      for (int v = 0; v < H / 4; ++v) {   // relu(z) summed as z [z > 0]: step + packed fma
        const float4 q = o4[v];          // (no packed max on gfx950)
        const f2 za = fma2(y2, dl[2 * v], ow[2 * v] + (f2){q.x, q.y});
        const f2 zb = fma2(y2, dl[2 * v + 1], ow[2 * v + 1] + (f2){q.z, q.w});
        acc[2 * v] = fma2(za, step2(za), acc[2 * v]);
        acc[2 * v + 1] = fma2(zb, step2(zb), acc[2 * v + 1]);
      }
    }
    prio0();
  }
  if ((threadIdx.x >> 6) == 0) {   // remove the self pair once
    const float yf = bitf(brow, ncl);
    const f2 y2 = {yf, yf};
#pragma unroll
    for (int kk = 0; kk < H2; ++kk) {
      const f2 zs = fma2(y2, dl[kk], ow[kk] + ld2(oth + ncl * H + 2 * kk));
      acc[kk] -= zs * step2(zs);      // the loop's form: the same value leaves
    }
  }
  combine8(acc, buf, res);
  float* gout = (z ? Hh : G) + (size_t)b * Nc * H;
  float* sout = (z ? tau : sig) + (size_t)b * Nc * H;
  const float* off = D + (z ? D_T0 : D_S0);
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H;
    if (t0 + n >= Nc) continue;
    float sacc = 0.f;
    for (int l = 0; l < H; ++l) sacc = fmaf(res[n * HP + l], Ml[l * H + k], sacc);
    gout[(t0 + n) * H + k] = res[n * HP + k];
    sout[(t0 + n) * H + k] = sacc + off[k];
  }
}

// ---------------------------------------------------------------------------------
// kw_hunk_cls  grid (tc, B, CLS_SPLIT): lane = hunk column q, grid z and then the 8 waves
//   split the rows p
//   mlp_hunkedge_B2 (model_2.py:304-324) + softmax CE (115-118):
//     kappa_pq = relu(sigma_p + tau_q + y_pq eps), z = kappa U2 + d2, CE = lse(z) - z_y
//   TRAIN: gamma_pq = 10 / (B Pc) (p1 - y) = dL/dz1 (= -dL/dz0), parked for the backward;
//   partial rows of dU2, dd2 and the CE sum
// ---------------------------------------------------------------------------------
constexpr int CLS_SPLIT = 2;   // kw_hunk_cls row ranges per column tile (grid z)
template <bool TRAIN>
__global__ __launch_bounds__(NTP) void kw_hunk_cls(
    const uint32_t* __restrict__ yT, const float* __restrict__ W, Off o,
    const float* __restrict__ D, int Nc, const float* __restrict__ sig,
    const float* __restrict__ tau, float* __restrict__ probs, float* __restrict__ logits,
    float* __restrict__ gam, float ce_scale, float* __restrict__ part, Segs sg,
    const int gam_out) {
#pragma clang fp contract(off)
  // gam_out = 0: gamma is not stored -- kw_hunk_clsb rebuilds it from the stored p1
  // (probs) and y, the same float ops on the same bits
  // sigma rows | 4 pad words | sigma + eps (the y = 1 rows): a lane's row is picked by its
  // y bit, and the pad puts the two tables' rows on different banks (the b128 reads of a
  // wave hit two addresses, else 2-way conflicts: the tables are 2560 words apart)
  __shared__ __attribute__((aligned(16))) float sst[2 * CHM * H + 4];
  float* ss = sst;
  float* se = sst + CHM * H + 4;
  __shared__ float red[NWP * 23];
  __shared__ float tot[23];
  const int b = blockIdx.y, t0 = blockIdx.x * TN, tc = gridDim.x;
  const int lane = threadIdx.x & 63;
  const int q = t0 + lane;
  const bool live = q < Nc;
  const int qc = live ? q : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const int Pc = Nc * (Nc - 1);
  const float* sgb = sig + (size_t)b * Nc * H;
  const uint32_t* ycol = yT + ((size_t)b * Nc + qc) * WC;   // bit p: y_pq (p != q)
  // kappa = (sigma_p + y eps) + tau_q: the y = 1 rows from a second staged table (picked
  // by address, no per-pair fma); U2 and b2 are wave-uniform scalar loads in the loop
  f2 tq[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) tq[kk] = ld2(tau + ((size_t)b * Nc + qc) * H + 2 * kk);
  const f2 bb = ld2(W + o.H2_B2);
  // the d form's classifier column c and the CE scale pinned in VGPRs: as uniform values
  // the compiler re-issued their scalar loads every pair, each with an lgkmcnt(0) wait that
  // also drained the pair's LDS reads
  f2 cvr[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    cvr[kk] = ld2(D + D_CV + 2 * kk);
    asm volatile("" : "+v"(cvr[kk]));
  }
  float ces = ce_scale;
  asm volatile("" : "+v"(ces));
  float* prb = probs ? probs + (size_t)b * 2 * Pc : nullptr;
  float* lgb = logits ? logits + (size_t)b * 2 * Pc : nullptr;
  float ce = 0.f, gs = 0.f, corr = 0.f;
  f2 za[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) za[kk] = (f2){0.f, 0.f};
  // grid z splits the rows p into gridDim.z contiguous ranges (more waves per SIMD; one
  // partial row each)
  const int r0 = (Nc * (int)blockIdx.z) / (int)gridDim.z;
  const int r1 = (Nc * ((int)blockIdx.z + 1)) / (int)gridDim.z;
  for (int c0 = r0; c0 < r1; c0 += CHM) {
    const int c1 = c0 + CHM < r1 ? c0 + CHM : r1;
    __syncthreads();
    stage_rows(ss, sgb, c0, c1);
    for (int e = threadIdx.x; e < (c1 - c0) * H; e += NTP)
      se[e] = sgb[(size_t)c0 * H + e] + D[D_EPS + e % H];
    __syncthreads();
    int lo, hi;
    wave_share(c0, c1, lo, hi);
    int wi = -1;
    uint32_t word = 0;
    for (int p = lo; p < hi; ++p) {   // y_pq from the lane's y^T row: one load per 32 rows
      if ((p >> 5) != wi) { wi = p >> 5; word = ycol[wi]; }
      const float yf = ((word >> (p & 31)) & 1u) ? 1.f : 0.f;
      const float4* s4 = reinterpret_cast<const float4*>((yf > 0.f ? se : ss) + (p - c0) * H);
      f2 kap[H2];
#pragma unroll
      for (int v = 0; v < H / 4; ++v) {
        const float4 sv = s4[v];
        kap[2 * v] = relu2((f2){sv.x, sv.y} + tq[2 * v]);
        kap[2 * v + 1] = relu2((f2){sv.z, sv.w} + tq[2 * v + 1]);
      }
      float p0, p1, cep;
      if (lgb) {   // both logits (returned; probs = softmax of them, block-uniform branch)
        f2 zz = bb;
#pragma unroll
        for (int kk = 0; kk < H2; ++kk) {
          zz = fma2((f2){kap[kk].x, kap[kk].x}, ld2(W + o.H2_W2 + 4 * kk), zz);
          zz = fma2((f2){kap[kk].y, kap[kk].y}, ld2(W + o.H2_W2 + 4 * kk + 2), zz);
        }
        const float z0 = zz.x, z1 = zz.y;
        const float mx = fmaxf(z0, z1);
        const float e0 = __expf(z0 - mx), e1 = __expf(z1 - mx);
        const float ssum = e0 + e1, inv = __builtin_amdgcn_rcpf(ssum);   // [1, 2]: 1-ulp rcp
        p0 = e0 * inv;
        p1 = e1 * inv;
        cep = (ln_1to2(ssum) + mx) - (yf > 0.f ? z1 : z0);
        if (live && q != p) {
          const int r = p * (Nc - 1) + q - (q > p ? 1 : 0);
          lgb[r] = z0;
          lgb[Pc + r] = z1;
        }
      } else {     // two classes need only d = z1 - z0 = relu(kappa) . c + (b1 - b0), as the
                   // fused kernel's M7: p1 = 1 / (1 + e^-d), CE = softplus(-+d)
        f2 dd = {bb.y - bb.x, 0.f};
#pragma unroll
        for (int kk = 0; kk < H2; ++kk) dd = fma2(kap[kk], cvr[kk], dd);
        const float d = dd.x + dd.y;
        const float ex = __expf(-fabsf(d));
        const float inv = __builtin_amdgcn_rcpf(1.f + ex);   // 1 + e in (1, 2]: 1-ulp rcp
        const float ps = ex * inv;
        p1 = d >= 0.f ? inv : ps;
        p0 = d >= 0.f ? ps : inv;
        cep = ln_1to2(1.f + ex) + relu(yf > 0.f ? -d : d);
      }
      if (live && q != p) {
        const int r = p * (Nc - 1) + q - (q > p ? 1 : 0);
        if (prb) { prb[r] = p0; prb[Pc + r] = p1; }
        ce += cep;
        corr += ((p1 > p0) == (yf > 0.f)) ? 1.f : 0.f;   // top_ACC: np.argmax, ties -> 0
        if constexpr (TRAIN) {
          const float g = ces * (p1 - yf);
          if (gam_out) gam[((size_t)b * Nc + p) * Nc + q] = g;
          gs += g;
#pragma unroll
          for (int kk = 0; kk < H2; ++kk) za[kk] = fma2(kap[kk], (f2){g, g}, za[kk]);
        }
      } else if (TRAIN && live && gam_out) {
        gam[((size_t)b * Nc + p) * Nc + q] = 0.f;   // defined diagonal, read by the passes
      }
    }
  }
  float acc[23];
  acc[0] = ce;
  acc[1] = gs;
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) { acc[2 + 2 * kk] = za[kk].x; acc[3 + 2 * kk] = za[kk].y; }
  acc[22] = corr;
  block_sum8<23>(acc, red, tot);
  const int row = (b * tc + blockIdx.x) * gridDim.z + blockIdx.z;
  if (threadIdx.x == 0) {
    put(part, sg.s[SG_CE], 0, row, tot[0]);
    put(part, sg.s[SG_CE], 1, row, tot[22]);
  }
  if constexpr (TRAIN) {
    const int t = threadIdx.x;
    if (t < H) {
      put(part, sg.s[SG_CLS], 2 * t, row, -tot[2 + t]);       // dU2[k][0]
      put(part, sg.s[SG_CLS], 2 * t + 1, row, tot[2 + t]);    // dU2[k][1]
    } else if (t < H + 2) {
      const int c = t - H;                                      // dd2
      put(part, sg.s[SG_CLS], 2 * H + c, row, c ? tot[1] : -tot[1]);
    }
  }
}

// kw_hunk_clsb's epilogue (also kw_hunk_fin2's): from the tile's per-node sums res (and
// the y-weighted sums yres, row pass), D = c (.) sums out, dG = D M^T (dH), and the partial
// rows of dU1 / dd1 / dV2 / dc2 through X = sum_n G_n (x) D_n (model_2.py:265-275, 304-321).
// LDS: res, yres, Gt [TN][HP]; X [H][H]; sumD, ysum [H]; Wl the staged M | V2 | c2 | U1e.
// Every product is a 16x16 MFMA tile on its own wave (8 waves): X (with sum_n D_n as the row
// of Gt's padding column set to 1) and dG, then dU1e and dV2 -- no serial 20- or 64-term
// LDS loops.
__device__ __forceinline__ void clsb_epilogue(
    const int z, const int b, const int t0, const int tc, const int Nc, const float* __restrict__ W,
    const Off& o, const float* __restrict__ D, const float* __restrict__ G,
    const float* __restrict__ Hh, float* __restrict__ Dsig, float* __restrict__ Dtau,
    float* __restrict__ dG, float* __restrict__ dH, float* __restrict__ part, const Segs& sg,
    float* res, float* yres, float* Gt, float* X, float* sumD, float* ysum, const float* Wl,
    const float* kzh, const int tile) {
  static_assert(NTP == 512, "clsb_epilogue maps its 16 product tiles onto 8 waves");
  const float *Ml = Wl, *V2 = Wl + H * H, *c2 = Wl + 2 * H * H, *U1e = Wl + 2 * H * H + H;
  (void)W;
  const float* gsrc = (z ? Hh : G) + (size_t)b * Nc * H;
  float* dout = (z ? Dtau : Dsig) + (size_t)b * Nc * H;
  float* gout = (z ? dH : dG) + (size_t)b * Nc * H;
  for (int e = threadIdx.x; e < TN * H; e += blockDim.x) {   // D = c (.) sums; padding rows -> 0
    const int n = e / H, k = e - n * H;
    const bool in = t0 + n < Nc;
    const float d = in ? res[n * HP + k] * D[D_CV + k] : 0.f;
    res[n * HP + k] = d;
    Gt[n * HP + k] = in ? gsrc[(t0 + n) * H + k] : 0.f;
    if (k == 0) Gt[n * HP + H] = in ? 1.f : 0.f;             // X's row H: sum_n D_n
    if (z == 0 && !in) yres[n * HP + k] = 0.f;
    if (in) dout[(t0 + n) * H + k] = d;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r16 = lane & 15;
  if (wv < 4) {   // X_blk = sum_n [G_n; 1] (x) D_n: 2 x 2 tiles, K = 64 nodes
    const int rl = (wv >> 1) * 16 + r16, kc = (wv & 1) * 16 + r16;
    const bool rv = rl <= H, cv = kc < H;
    const f4v c = mfma_tile16_p(rv ? Gt + rl : kzh, rv ? HP : 0, cv ? res + kc : kzh,
                                cv ? HP : 0, TN, lane);
    if (cv)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rr = (wv >> 1) * 16 + 4 * (lane >> 4) + j;
        if (rr < H) X[rr * H + kc] = c[j];
        else if (rr == H) sumD[kc] = c[j];
      }
    if (z == 0) {   // ysum[k] = sum_n yres[n][k]: units 5 wv .. 5 wv + 4, one wave sum each
#pragma unroll
      for (int q = 0; q < H / 4; ++q) {
        const int k = (H / 4) * wv + q;
        const float v = wsum(yres[lane * HP + k]);
        if (lane == 0) ysum[k] = v;
      }
    } else if (lane < H / 4) {
      ysum[(H / 4) * wv + lane] = 0.f;
    }
  } else {        // dG_n[l] = sum_k D_n[k] M[l][k]: 4 x 2 tiles, K = 20, two per wave
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tl = 2 * (wv - 4) + u, n0 = (tl >> 1) * 16, lc = (tl & 1) * 16 + r16;
      const bool cv = lc < H;
      const f4v c = mfma_tile16_p(res + (n0 + r16) * HP, 1, cv ? Ml + lc * H : kzh, cv ? 1 : 0,
                                  H, lane);
      if (cv)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + 4 * (lane >> 4) + j;
          if (t0 + n < Nc) gout[(t0 + n) * H + lc] = c[j];
        }
    }
  }
  __syncthreads();
  const int row = (b * tc + tile) * 2 + z;
  const float Nc1 = (float)(Nc - 1);
  const Seg& s2 = sg.s[SG_CLSB_H2];
  const Seg& s1 = sg.s[SG_CLSB_H1];
  if (wv < 4) {   // dU1e[m][k] = sum_l V2[l][m] X[l][k] + (Nc-1) c2[m] sumD[k]: 2 x 2 tiles
    const int m0 = (wv >> 1) * 16, kc = (wv & 1) * 16 + r16, mr = m0 + r16;
    const bool mv = mr < H, cv = kc < H;
    const f4v c = mfma_tile16_p(mv ? V2 + mr : kzh, mv ? H : 0, cv ? X + kc : kzh, cv ? H : 0, H,
                                lane);
    if (cv)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + 4 * (lane >> 4) + j;
        if (m < H) put(part, s2, (2 + m) * H + kc, row, fmaf(Nc1 * c2[m], sumD[kc], c[j]));
      }
  } else {        // dV2[l][m] = sum_k X[l][k] U1e[m][k]: 2 x 2 tiles
    const int tl = wv - 4, l0 = (tl >> 1) * 16, mc = (tl & 1) * 16 + r16, lr = l0 + r16;
    const bool lv = lr < H, cv = mc < H;
    const f4v c = mfma_tile16_p(lv ? X + lr * H : kzh, lv ? 1 : 0, cv ? U1e + mc * H : kzh,
                                cv ? 1 : 0, H, lane);
    if (cv)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int l = l0 + 4 * (lane >> 4) + j;
        if (l < H) put(part, s1, l * H + mc, row, c[j]);
      }
  }
  if (threadIdx.x < H) {            // dc2[m] = (Nc-1) sum_k U1e[m][k] sumD[k]
    const int m = threadIdx.x;
    float a = 0.f;
    for (int k = 0; k < H; ++k) a = fmaf(U1e[m * H + k], sumD[k], a);
    put(part, s1, H * H + m, row, Nc1 * a);
  } else if (threadIdx.x >= 64 && threadIdx.x < 64 + H) {   // dU1[0], dU1[1], dd1 (row pass)
    const int k = threadIdx.x - 64;
    const float dd1 = z == 0 ? sumD[k] : 0.f;
    const float dy1 = z == 0 ? D[D_CV + k] * ysum[k] : 0.f;
    put(part, s2, k, row, dd1 - dy1);
    put(part, s2, H + k, row, dy1);
    put(part, s2, 22 * H + k, row, dd1);
  }
}

// ---------------------------------------------------------------------------------
// kw_hunk_clsb  grid (tc, B, 2): classifier backward (model_2.py:304-321)
//   e_pqk = [kappa_pqk > 0] gamma_pq;  row pass: Dsig_p = c (.) sum_q e_pq, ysum = sum y e
//   column pass: Dtau_q = c (.) sum_p e_pq.  Epilogue: dG = Dsig M^T (dH = Dtau M^T) and
//   the partial rows of dU1 (rows 0..1 from the row pass, rows 2..21 through
//   X = sum_p G_p (x) Dsig_p + H_p (x) Dtau_p), dd1, dV2 and dc2 (model_2.py:265-275).
//   kappa = own + (other + y eps): the y = 1 rows of the swept side from a second staged
//   table (picked by address, as kw_hunk_cls), so the column pass's kappa is the forward's
//   bit for bit.  The row pass reads gamma through a transposing LDS tile (coalesced 16-byte
//   global loads, no index division).
// ---------------------------------------------------------------------------------
constexpr int GTP = CHM + 1;   // gamma tile pitch
#ifndef HDG_GAM_FROM_PROBS    // 1: training steps that write probs have kw_hunk_clsb rebuild
#define HDG_GAM_FROM_PROBS 0  // gamma from them, kw_hunk_cls storing none.  Measured at stress:
#endif                        // cls 42.0 -> 40.2 us but clsb 49.3 -> 90.6 us (scalar staging)
#ifndef HDG_CLSB_CTILE        // kw_hunk_clsb column pass: gamma staged through LDS (1) or
#define HDG_CLSB_CTILE 1      // read from global memory per swept row (0)
#endif
static_assert(CHM * TN <= TN * GTP, "the column pass's gamma tile fits the row pass's");
__global__ __launch_bounds__(NTP) __attribute__((amdgpu_waves_per_eu(4))) void kw_hunk_clsb(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ W, Off o, const float* __restrict__ D, int Nc,
    const float* __restrict__ sig, const float* __restrict__ tau, const float* __restrict__ gam,
    const float* __restrict__ G, const float* __restrict__ Hh, float* __restrict__ Dsig,
    float* __restrict__ Dtau, float* __restrict__ dG, float* __restrict__ dH,
    float* __restrict__ part, Segs sg, const float* __restrict__ probs, const float ce_scale) {
#pragma clang fp contract(off)
  // the swept rows and the gamma tile are dead once the sweep ends: combine8's buffer
  // overlays them (76 KB of LDS: two blocks per CU)
  constexpr int SWEEP_W = 2 * CHM * H + 4 + TN * GTP, BUF_W = NWP * TN * HP;
  __shared__ __attribute__((aligned(16))) float big[SWEEP_W > BUF_W ? SWEEP_W : BUF_W];
  float* os_ = big;
  float* ose = big + CHM * H + 4;                 // other + eps: the y = 1 rows (4 pad words:
  float* gt = big + 2 * CHM * H + 4;              // its rows on other banks than os_'s)
  float* buf = big;
  __shared__ float res[TN * HP], yres[TN * HP], Gt[TN * HP];
  __shared__ float X[H * H], sumD[H], ysum[H];
  __shared__ float Wl[3 * H * H + H];
  __shared__ float kzh[1];                        // 0.f: stride-0 operand of padding tiles
  if (threadIdx.x == 0) kzh[0] = 0.f;
  // Wl = M | V2 | c2 | U1e (clsb_epilogue's layout)
  stage_w(Wl, D + D_M, H * H);                    // visible after the first chunk barrier
  stage_w(Wl + H * H, W + o.H1_W2, H * H + H);    // V2 | c2
  stage_w(Wl + 2 * H * H + H, W + o.H2_W1 + 2 * H, H * H);
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN, tc = gridDim.x;
  const int lane = threadIdx.x & 63;
  const int nd = t0 + lane, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const float* own = (z ? tau : sig) + (size_t)b * Nc * H;
  const float* oth = (z ? sig : tau) + (size_t)b * Nc * H;
  const uint32_t* brow = (z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC;
  const float* gb = gam + (size_t)b * Nc * Nc;
  // probs != NULL (kw_hunk_cls stored no gamma): gamma_pq = ce_scale (p1_pq - y_pq) from the
  // stored p1 (off-diagonal layout, model_2.py:321) and the y bits, 0 on the diagonal --
  // the forward's float ops on its bits
  const size_t Pc = (size_t)Nc * (Nc - 1);
  const float* p1b = (HDG_GAM_FROM_PROBS && probs) ? probs + (size_t)b * 2 * Pc + Pc : nullptr;
  const uint32_t* ybb = ybits + (size_t)b * Nc * WC;
  auto gamma_at = [&](const int r, const int q) -> float {   // r, q < Nc
    if (!p1b) return gb[(size_t)r * Nc + q];
    if (q == r) return 0.f;
    const float p1 = p1b[(size_t)r * (Nc - 1) + q - (q > r ? 1 : 0)];
    const float yf = ((ybb[r * WC + (q >> 5)] >> (q & 31)) & 1u) ? 1.f : 0.f;
    return ce_scale * (p1 - yf);
  };
  f2 ow[H2], acc[H2], ya[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    ow[kk] = ld2(own + ncl * H + 2 * kk);
    if (HDG_STEPF) ow[kk] *= (f2){STEP_S, STEP_S};   // stepf2's c 2^64 (exact)
    acc[kk] = (f2){0.f, 0.f};
    ya[kk] = (f2){0.f, 0.f};
  }
  // gamma tile loads: thread -> (row tr + 16 i, 4 columns at tc4); rows / columns past the
  // grid read a clamped address and store 0
  const int tr = threadIdx.x >> 5, tc4 = (threadIdx.x & 31) * 4;
  const bool al4 = (Nc & 3) == 0;                 // rows 16-byte aligned: float4 loads
  WSTAMP(11, 0);
  for (int c0 = 0; c0 < Nc; c0 += CHM) {   // gamma's diagonal is 0: no self pair to remove
    const int c1 = c0 + CHM < Nc ? c0 + CHM : Nc;
    __syncthreads();
    if (c0 == 0) WSTAMP(11, 1);
    stage_rows(os_, oth, c0, c1);
    for (int e = threadIdx.x; e < (c1 - c0) * H; e += NTP)
      ose[e] = oth[(size_t)c0 * H + e] + D[D_EPS + e % H];
    if (z == 0) {
      float4 gv[TN / 16];
      const int cg = c0 + tc4;
#pragma unroll
      for (int i = 0; i < TN / 16; ++i) {
        const int r = t0 + tr + 16 * i, rc = r < Nc ? r : Nc - 1;
        const float* src = gb + (size_t)rc * Nc;
        if (!p1b && al4 && cg + 3 < c1) {
          gv[i] = *reinterpret_cast<const float4*>(src + cg);
        } else {
          gv[i].x = cg < c1 ? gamma_at(rc, cg) : 0.f;
          gv[i].y = cg + 1 < c1 ? gamma_at(rc, cg + 1) : 0.f;
          gv[i].z = cg + 2 < c1 ? gamma_at(rc, cg + 2) : 0.f;
          gv[i].w = cg + 3 < c1 ? gamma_at(rc, cg + 3) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < TN / 16; ++i) {
        const int rl = tr + 16 * i;
        const bool rin = t0 + rl < Nc;
        float* d = gt + rl * GTP + tc4;
        if (tc4 < c1 - c0) {
          d[0] = rin ? gv[i].x : 0.f;
          d[1] = rin ? gv[i].y : 0.f;
          d[2] = rin ? gv[i].z : 0.f;
          d[3] = rin ? gv[i].w : 0.f;
        }
      }
    } else if (HDG_CLSB_CTILE) {
      // column pass: the chunk's gamma rows over the tile's 64 columns, staged as they lie
      // ([m - c0][lane], pitch TN): coalesced 16-byte loads instead of one dependent global
      // load per swept row; columns past the grid 0 (their lanes' sums are not used)
      float4 gv[CHM * TN / (4 * NTP)];
      const int rr = threadIdx.x >> 4, cc4 = (threadIdx.x & 15) * 4, cg = t0 + cc4;
#pragma unroll
      for (int i = 0; i < CHM * TN / (4 * NTP); ++i) {
        const int r = c0 + rr + (NTP / 16) * i, rc = r < c1 ? r : c1 - 1;
        const float* src = gb + (size_t)rc * Nc;
        if (!p1b && al4 && cg + 3 < Nc) {
          gv[i] = *reinterpret_cast<const float4*>(src + cg);
        } else {
          gv[i].x = cg < Nc ? gamma_at(rc, cg) : 0.f;
          gv[i].y = cg + 1 < Nc ? gamma_at(rc, cg + 1) : 0.f;
          gv[i].z = cg + 2 < Nc ? gamma_at(rc, cg + 2) : 0.f;
          gv[i].w = cg + 3 < Nc ? gamma_at(rc, cg + 3) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < CHM * TN / (4 * NTP); ++i)
        *reinterpret_cast<float4*>(gt + (rr + (NTP / 16) * i) * TN + cc4) = gv[i];
    }
    __syncthreads();
    if (c0 == 0) WSTAMP(11, 2);
    int lo, hi;
    wave_share(c0, c1, lo, hi);
    // one loop per pass (block-uniform): gamma from the LDS tile (row pass) or global
    // memory (column pass) by its own load instruction, not a flat load through a selected
    // pointer; the column pass has no y-weighted sums
    auto sweep = [&](auto row_pass) {
      constexpr bool ROW = decltype(row_pass)::value;
      int wi = -1;
      uint32_t word = 0;
      for (int m = lo; m < hi; ++m) {
        if ((m >> 5) != wi) { wi = m >> 5; word = brow[wi]; }
        const bool y1 = (word >> (m & 31)) & 1u;
        const float g = ROW ? gt[lane * GTP + (m - c0)]
                            : (HDG_CLSB_CTILE ? gt[(m - c0) * TN + lane] : gamma_at(m, ncl));
        const f2 g2 = {g, g}, gy2 = y1 ? g2 : (f2){0.f, 0.f};
        // [kappa > 0] g and [kappa > 0] y g as one fma each (the products are exact)
        const float4* o4 = reinterpret_cast<const float4*>((y1 ? ose : os_) + (m - c0) * H);
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {
          const float4 q = o4[v];
          const f2 sa = HDG_STEPF ? stepf2((f2){q.x, q.y}, ow[2 * v])
                                  : step2(ow[2 * v] + (f2){q.x, q.y});
          const f2 sb = HDG_STEPF ? stepf2((f2){q.z, q.w}, ow[2 * v + 1])
                                  : step2(ow[2 * v + 1] + (f2){q.z, q.w});
          acc[2 * v] = fma2(sa, g2, acc[2 * v]);   // gamma finite, 0 on the diagonal
          acc[2 * v + 1] = fma2(sb, g2, acc[2 * v + 1]);
          if constexpr (ROW) {
            ya[2 * v] = fma2(sa, gy2, ya[2 * v]);
            ya[2 * v + 1] = fma2(sb, gy2, ya[2 * v + 1]);
          }
        }
      }
    };
    if (z == 0) sweep(std::true_type{});
    else sweep(std::false_type{});
    if (c0 == 0) WSTAMP(11, 3);
  }
  WSTAMP(11, 4);
  __syncthreads();                       // every wave is done with os_ / gt (= buf)
  combine8(acc, buf, res);
  if (z == 0) combine8(ya, buf, yres);
  WSTAMP(11, 5);
  clsb_epilogue(z, b, t0, tc, Nc, W, o, D, G, Hh, Dsig, Dtau, dG, dH, part, sg, res, yres, Gt, X,
                sumD, ysum, Wl, kzh, blockIdx.x);
  WSTAMP(11, 6);
}

// kw_hunk_mlpb's epilogue: the tile's D alpha / D beta rows out, the partial rows of dV1
// (rows 0..3 / 4..7 from the pass's node vectors, 8, 9 from the row pass) and dc1.
// res / yres: [TN][HP] LDS (padding nodes zeroed here), nt: [TN][4] LDS scratch.
__device__ __forceinline__ void mlpb_epilogue(int z, int b, int t0, int tc, int Nc,
                                              const float* __restrict__ nvec, float* res,
                                              float* yres, float* nt, float* __restrict__ Dal,
                                              float* __restrict__ Dbe, float* __restrict__ part,
                                              const Segs& sg, int tile) {
  float* dout = (z ? Dbe : Dal) + (size_t)b * Nc * H;
  for (int e = threadIdx.x; e < TN * H; e += blockDim.x) {
    const int n = e / H, k = e - n * H;
    const bool in = t0 + n < Nc;
    if (!in) { res[n * HP + k] = 0.f; yres[n * HP + k] = 0.f; }
    else dout[(t0 + n) * H + k] = res[n * HP + k];
  }
  for (int e = threadIdx.x; e < TN * 4; e += blockDim.x)
    nt[e] = (t0 + e / 4 < Nc) ? nvec[((size_t)b * Nc + t0) * 4 + e] : 0.f;
  __syncthreads();
  const int row = (b * tc + tile) * 2 + z;
  const Seg& s = sg.s[SG_MLPB];
  for (int e = threadIdx.x; e < 11 * H; e += blockDim.x) {   // rows 0..9 of V1, then c1
    const int l = e / H, k = e - l * H;
    float a = 0.f;
    if (l < 8) {
      const int m = l & 3;
      if ((l >> 2) == z)
        for (int n = 0; n < TN; ++n) a = fmaf(nt[n * 4 + m], res[n * HP + k], a);
    } else if (z == 0) {
      float sd = 0.f, sy = 0.f;
      for (int n = 0; n < TN; ++n) { sd += res[n * HP + k]; sy += yres[n * HP + k]; }
      a = l == 8 ? sd - sy : (l == 9 ? sy : sd);
    }
    put(part, s, e, row, a);
  }
}

// ---------------------------------------------------------------------------------
// kw_hunk_mlpb  grid (tc, B, 2): hunk pair MLP backward (model_2.py:257-275)
//   dz_pq = [alpha_p + beta_q + y delta > 0] (dG_p + dH_q)
//   row pass: Dalpha_p = sum_q dz, sum y dz;  column pass: Dbeta_q = sum_p dz
//   partial rows of dV1 (rows 0..3 / 4..7 / 8, 9) and dc1
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(NTP) void kw_hunk_mlpb(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ D, int Nc, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ dG, const float* __restrict__ dH,
    const float* __restrict__ nvec, float* __restrict__ Dal, float* __restrict__ Dbe,
    float* __restrict__ part, Segs sg) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float os_[CHM * H];
  __shared__ __attribute__((aligned(16))) float ws_[CHM * H];
  __shared__ float buf[NWP * TN * HP];
  __shared__ float res[TN * HP], yres[TN * HP], nt[TN * 4];
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN, tc = gridDim.x;
  const int lane = threadIdx.x & 63;
  const int nd = t0 + lane, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H;
  const float* oth = (z ? alpha : beta) + (size_t)b * Nc * H;
  const float* wown = (z ? dH : dG) + (size_t)b * Nc * H;
  const float* woth = (z ? dG : dH) + (size_t)b * Nc * H;
  const uint32_t* brow = (z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC;
  f2 ow[H2], wo[H2], dl[H2], acc[H2], ya[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    ow[kk] = ld2(own + ncl * H + 2 * kk);
    wo[kk] = ld2(wown + ncl * H + 2 * kk);
    dl[kk] = ld2(D + D_DLT + 2 * kk);
    acc[kk] = (f2){0.f, 0.f};
    ya[kk] = (f2){0.f, 0.f};
  }
  for (int c0 = 0; c0 < Nc; c0 += CHM) {
    const int c1 = c0 + CHM < Nc ? c0 + CHM : Nc;
    __syncthreads();
    stage_rows(os_, oth, c0, c1);
    stage_rows(ws_, woth, c0, c1);
    __syncthreads();
    int lo, hi;
    wave_share(c0, c1, lo, hi);
    int wi = -1;
    uint32_t word = 0;
    for (int m = lo; m < hi; ++m) {
      share_prio(m, lo, hi);
      if ((m >> 5) != wi) { wi = m >> 5; word = brow[wi]; }
      const float yf = ((word >> (m & 31)) & 1u) ? 1.f : 0.f;
      const f2 y2 = {yf, yf};
      const float4* o4 = reinterpret_cast<const float4*>(os_ + (m - c0) * H);
      const float4* w4 = reinterpret_cast<const float4*>(ws_ + (m - c0) * H);
#pragma unroll
      for (int v = 0; v < H / 4; ++v) {
        const float4 q = o4[v], r = w4[v];
        const f2 pa = fma2(y2, dl[2 * v], ow[2 * v] + (f2){q.x, q.y});
        const f2 pb = fma2(y2, dl[2 * v + 1], ow[2 * v + 1] + (f2){q.z, q.w});
        const f2 ga = wo[2 * v] + (f2){r.x, r.y}, gb2 = wo[2 * v + 1] + (f2){r.z, r.w};
        const f2 da = step2(pa) * ga;   // [p > 0] g: one packed step + multiply (g finite)
        const f2 db = step2(pb) * gb2;
        acc[2 * v] += da;
        acc[2 * v + 1] += db;
        ya[2 * v] = fma2(y2, da, ya[2 * v]);
        ya[2 * v + 1] = fma2(y2, db, ya[2 * v + 1]);
      }
    }
    prio0();
  }
  if ((threadIdx.x >> 6) == 0) {   // remove the self pair once
    const float yf = bitf(brow, ncl);
    const f2 y2 = {yf, yf};
#pragma unroll
    for (int kk = 0; kk < H2; ++kk) {
      const f2 pr = fma2(y2, dl[kk], ow[kk] + ld2(oth + ncl * H + 2 * kk));
      const f2 gg = wo[kk] + ld2(woth + ncl * H + 2 * kk);
      const f2 dz = step2(pr) * gg;   // the loop's form: the same value leaves
      acc[kk] -= dz;
      ya[kk] -= y2 * dz;
    }
  }
  combine8(acc, buf, res);
  if (z == 0) combine8(ya, buf, yres);
  mlpb_epilogue(z, b, t0, tc, Nc, nvec, res, yres, nt, Dal, Dbe, part, sg, blockIdx.x);
}

// ---------------------------------------------------------------------------------
// Sorted-threshold hunk pair sums (general path, Nc >= hunk_sorted_min()).  For hidden
// unit k the y = 0 pre-activation of pair (p, q) is z0 = fl(alpha_p + beta_q), and
// fl(a + b) > 0 exactly when b > -a, so {q : z0_pq > 0} is a suffix of the beta-sorted
// order (and {p : z0_pq > 0} of the alpha-sorted order): one binary search per node and
// unit plus f64 suffix sums replace the dense sweep (kw_hunk_fwd's relu sums,
// kw_hunk_mlpb's mask sums).  The y = 1 pairs are corrected one by one over the set bits
// of the node's label row (z1 = fl(z0 + delta), the dense kernels' expression), and the
// self pair is removed.  O(Nc H (log Nc + deg_y)) per commit instead of O(Nc^2 H).
//   side 0: beta sorted (the row pass: node p, swept q); side 1: alpha (the column pass)
// Tables per (commit, side, unit), hsort_layout: sv f32 [NcP] values ascending, sp i32 [NcP]
// node of each slot, sx f64 [NcP + 1] suffix sums of sv, sw f64 [NcP + 1] suffix sums of
// the backward weights w[sp[r]] (side 0: dH, side 1: dG; kw_hunk_wsum).
// ---------------------------------------------------------------------------------
struct HSort {
  size_t sv, sp, sx, sw;   // float offsets into the workspace
  int NcP;
};
__host__ __device__ inline size_t hsort_tab(int b, int side, int k, int len) {
  return (((size_t)b * 2 + side) * H + k) * (size_t)len;
}

// XCD-aware block map of a (T, B, 2) grid: blocks are dealt to the 8 XCDs round robin by
// linear id, so the blocks of commit b all land on XCD b % 8 (the last B % 8 commits' blocks
// in id order) -- the sorted tables one kernel writes are then read by the next from the
// same L2
__device__ __forceinline__ void xcd_commit_map(int& t, int& b, int& z) {
  const int T = gridDim.x, B = gridDim.y, Z = gridDim.z;
  const int L = blockIdx.x + T * (blockIdx.y + B * blockIdx.z);
  const int Bq = B & ~7, per = Z * T;              // commits [0, Bq): commit b on XCD b % 8
  if (L >= per * Bq) {                              // the last B % 8 commits: in id order
    const int r = L - per * Bq, rem = r % per;
    b = Bq + r / per;
    z = rem / T;
    t = rem - z * T;
    return;
  }
  const int s = L >> 3, bq = s / per, r = s - bq * per;
  b = 8 * bq + (L & 7);
  z = r / T;
  t = r - z * T;
}

// sort keys: order-preserving u32 bits of a float value
__device__ __forceinline__ uint32_t fkey(float v) {   // monotone float -> u32 (no NaN here)
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// the value of lane ^ ST (ST < 64) without the LDS crossbar where the VALU can: permlane
// swaps for 32 / 16, DPP for 8 (row_ror:8 = lane ^ 8 in a 16-lane row), 2, 1 (quad_perm);
// ds_swizzle (xor mode) for 4
template <int ST>
__device__ __forceinline__ uint32_t xlane(uint32_t v, int lane) {
  if constexpr (ST == 32 || ST == 16) {
    float x = __uint_as_float(v), y = x;
    if constexpr (ST == 32) {
      swap32(x, y);
      return __float_as_uint((lane & 32) ? x : y);
    } else {
      swap16(x, y);
      return __float_as_uint((lane & 16) ? x : y);
    }
  } else if constexpr (ST == 8) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
  } else if constexpr (ST == 4) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1F);
  } else if constexpr (ST == 2) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  } else {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  }
}
template <int ST>
__device__ __forceinline__ unsigned long long xlane64(unsigned long long v, int lane) {
  const uint32_t lo = xlane<ST>((uint32_t)v, lane), hi = xlane<ST>((uint32_t)(v >> 32), lane);
  return ((unsigned long long)hi << 32) | lo;
}

// Block-wide bitonic network: 4 waves per table, element e = 64 E w + 64 i + lane (wave w,
// register i).  Distances below 64 are lanes (xlane), below 64 E registers of the lane,
// from 64 E on partners in another wave (through LDS, two barriers per stage).  The
// sort direction of element e at merge level LEN is (e & LEN) == 0.
template <int ST, int LEN, int E>
__device__ __forceinline__ void bs_lane(unsigned long long (&k)[E], int lane, int eb) {
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const bool up = ((eb + 64 * i + lane) & LEN) == 0;
    const unsigned long long o = xlane64<ST>(k[i], lane);
    const bool keep_min = ((lane & ST) == 0) == up;
    k[i] = ((k[i] < o) == keep_min) ? k[i] : o;
  }
}
template <int ST, int LEN, int E>
__device__ __forceinline__ void bs_reg(unsigned long long (&k)[E], int lane, int eb) {
  constexpr int rs = ST >> 6;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (i & rs) continue;
    const bool up = ((eb + 64 * i + lane) & LEN) == 0;
    const unsigned long long a = k[i], c = k[i + rs];
    const bool sw = (a > c) == up;
    k[i] = sw ? c : a;
    k[i + rs] = sw ? a : c;
  }
}
template <int ST, int LEN, int E>
__device__ __forceinline__ void bs_cross(unsigned long long (&k)[E], int lane, int eb,
                                         unsigned long long* sh) {
#pragma unroll
  for (int i = 0; i < E; ++i) sh[eb + 64 * i + lane] = k[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = eb + 64 * i + lane;
    const unsigned long long o = sh[e ^ ST];
    const bool keep_min = ((e & ST) == 0) == ((e & LEN) == 0);
    k[i] = ((k[i] < o) == keep_min) ? k[i] : o;
  }
  __syncthreads();
}
template <int LEN, int ST, int E>
__device__ __forceinline__ void bs_stages(unsigned long long (&k)[E], int lane, int eb,
                                          unsigned long long* sh) {
  if constexpr (ST >= 64 * E) bs_cross<ST, LEN, E>(k, lane, eb, sh);
  else if constexpr (ST >= 64) bs_reg<ST, LEN, E>(k, lane, eb);
  else bs_lane<ST, LEN, E>(k, lane, eb);
  if constexpr (ST > 1) bs_stages<LEN, ST / 2, E>(k, lane, eb, sh);
}
template <int LEN, int E>
__device__ __forceinline__ void bs_sort(unsigned long long (&k)[E], int lane, int eb,
                                        unsigned long long* sh) {
  bs_stages<LEN, LEN / 2, E>(k, lane, eb, sh);
  if constexpr (LEN < 256 * E) bs_sort<2 * LEN, E>(k, lane, eb, sh);
}

// block-wide suffix sums over the elements e = 64 E w + 64 i + lane: out(e, sum_{r >= e} v_r)
// (each wave's chunk in registers, then the higher waves' chunk totals through LDS)
template <int E, class V, class O>
__device__ __forceinline__ void block_suffix(int lane, int w, int n, V val, O out, double* tot) {
  double sfx[E];
  double carry = 0.0;
#pragma unroll
  for (int i = E - 1; i >= 0; --i) {
    const int e = 64 * E * w + 64 * i + lane;
    double v = e < n ? val(i) : 0.0;
#pragma unroll
    for (int o2 = 1; o2 < 64; o2 <<= 1) {
      const double u = __shfl_down(v, o2);
      if (lane + o2 < 64) v += u;
    }
    v += carry;
    sfx[i] = v;
    carry = __shfl(v, 0);
  }
  if (lane == 0) tot[w] = carry;
  __syncthreads();
  double hi = 0.0;
  for (int u = NW - 1; u > w; --u) hi += tot[u];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = 64 * E * w + 64 * i + lane;
    if (e < n) out(e, sfx[i] + hi);
  }
}

// kw_hunk_sort  grid (H, B, 2), one 4-wave block per table (side, unit): the 64-bit keys
// (order-preserving value bits, node index below: ties by node, every table deterministic)
// sorted by the block-wide network, then f64 suffix sums of the values.  E = pow2(Nc) / 256
// per lane (at least 1).
template <int E>
__global__ __launch_bounds__(NT) void kw_hunk_sort(const float* __restrict__ alpha,
                                                   const float* __restrict__ beta, int Nc,
                                                   float* __restrict__ sv, int* __restrict__ sp,
                                                   double* __restrict__ sx) {
  __shared__ unsigned long long sh[256 * E];
  __shared__ double tot[NW];
  const int lane = threadIdx.x & 63, w = uni(threadIdx.x >> 6);
  int k, b, side;
  xcd_commit_map(k, b, side);
  WSTAMP(1, 0);
  const int NcP = (Nc + 3) & ~3, eb = 64 * E * w;
  const float* src = (side ? alpha : beta) + (size_t)b * Nc * H + k;
  unsigned long long key[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = eb + 64 * i + lane;
    const uint32_t kv = e < Nc ? fkey(src[(size_t)(e < Nc ? e : 0) * H]) : 0xffffffffu;
    key[i] = ((unsigned long long)kv << 32) | (uint32_t)e;
  }
  WSTAMP(1, 1);
  bs_sort<2, E>(key, lane, eb, sh);
  WSTAMP(1, 2);
  const size_t tb = hsort_tab(b, side, k, NcP), tx = hsort_tab(b, side, k, NcP + 1);
  float val[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = eb + 64 * i + lane;
    val[i] = fkey_inv((uint32_t)(key[i] >> 32));
    if (e < Nc) {
      sv[tb + e] = val[i];
      sp[tb + e] = (int)(key[i] & 0xffffffffu);
    }
  }
  if (threadIdx.x == 0) sx[tx + Nc] = 0.0;
  WSTAMP(1, 3);
  block_suffix<E>(lane, w, Nc, [&](int i) { return (double)val[i]; },
                  [&](int e, double v) { sx[tx + e] = v; }, tot);
  WSTAMP(1, 4);
}

// kw_hunk_wsum  grid (H, B, 2), one 4-wave block per table: sw[m] = sum_{r >= m} w[sp[r]][k],
// side 0: w = dH, 1: dG
template <int E>
__global__ __launch_bounds__(NT) void kw_hunk_wsum(const int* __restrict__ sp,
                                                   const float* __restrict__ dG,
                                                   const float* __restrict__ dH, int Nc,
                                                   double* __restrict__ sw) {
  __shared__ double tot[NW];
  const int lane = threadIdx.x & 63, w = uni(threadIdx.x >> 6);
  int k, b, side;
  xcd_commit_map(k, b, side);
  const int NcP = (Nc + 3) & ~3, eb = 64 * E * w;
  const float* wv = (side ? dG : dH) + (size_t)b * Nc * H + k;
  const int* pm = sp + hsort_tab(b, side, k, NcP);
  double* T = sw + hsort_tab(b, side, k, NcP + 1);
  WSTAMP(4, 0);
  int id[E];
  float v[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = eb + 64 * i + lane;
    id[i] = pm[e < Nc ? e : 0];
  }
#pragma unroll
  for (int i = 0; i < E; ++i) v[i] = wv[(size_t)id[i] * H];
  if (threadIdx.x == 0) T[Nc] = 0.0;
  WSTAMP(4, 1);
  block_suffix<E>(lane, w, Nc, [&](int i) { return (double)v[i]; },
                  [&](int e, double x) { T[e] = x; }, tot);
  WSTAMP(4, 2);
}

// E = elements per lane of the block sort: pow2(Nc) / 256, at least 1
inline int hsort_e(int Nc) {
  int e = 1;
  while (256 * e < Nc) e <<= 1;
  return e;
}

// The sorted passes stage their tables in LDS (every load of a thread issued before its
// first LDS store): the binary searches and the label walks then wait on LDS, not on one
// dependent L2 round trip per step / pair.  Two block shapes:
//   Nc <= HS_ALL_MAX: 8 waves over 128 nodes (two 64-node halves), wave w takes half w >> 2
//     and hidden units [5 (w & 3), +5); the block stages all 20 units' tables, so the four
//     unit groups of a node share its label list (L1 hits) and sigma / tau close in-block.
//   larger Nc (up to the engine's 2048): one block per (256-node tile, unit group g of 5
//     units), 4 waves, lane = node, staging only its group's tables (88 / 120 KiB at Nc =
//     2048, where all 20 units no longer fit); sigma / tau follow in kw_hunk_sig.
// The walks read the node's label id list (ylist_layout) four ids per 8-byte load, all of a
// lane's groups (up to HS_LB) in flight at once.
//   Walk rows in LDS: lane l reads the row of its own label q, so the 32 lanes of an LDS lane
// group address random rows.  Rows of 20 floats put every row start on one of 8 banks (20 q
// mod 32): 4-8-way conflicts on each 4-byte read, which made the walk LDS-bound
// (tools/wstamp.py: 30.6 of mlpb_s's 46 us at 1024x512).  Rows are staged per unit group g
// as 5 values + 1 pad (fwd) or 5 (value, weight) pairs (mlpb), node strides 26 / 42 (all
// units) or 6 / 10 (one group): 8-byte reads (64 banks, 2 per read) whose row starts take 32
// distinct bank pairs, three / five reads per label.
constexpr int HSN = 128;                  // nodes per block, all-unit shape
constexpr int HS_ALL_MAX = 512;           // largest Nc of the all-unit shape
constexpr int HS_OSF = 26, HS_OSB = 42;   // all-unit walk-row strides (floats), fwd / mlpb
constexpr int HSG = 256;                  // nodes per block, group shape
constexpr int HS_NC_MAX = 2048;
constexpr int HS_RSF = 6, HS_RSB = 10;    // group walk-row strides, fwd / mlpb
constexpr int HS_LB = 8;                  // label id groups (4 ids each) in flight per lane
constexpr int RS5 = KPW + 1;              // [node][unit] result rows of a group
__host__ __device__ inline size_t hs_lds_bytes(int Nc, int nvec) {   // nvec: 1 (fwd) / 2 (mlpb)
  const size_t NcP = (Nc + 3) & ~3;
  if (Nc <= HS_ALL_MAX) return ((size_t)H * NcP + (size_t)Nc * (nvec == 1 ? HS_OSF : HS_OSB)) * 4;
  return ((size_t)KPW * NcP + (size_t)Nc * (nvec == 1 ? HS_RSF : HS_RSB)) * 4;
}
__host__ __device__ inline int hs_tiles(int Nc) { return (Nc + HSG - 1) / HSG; }
// the all-unit shape runs for Nc <= HS_ALL_MAX unless HDG_FLAG_HUNK_GROUP asks for the group
// shape; the two differ in the order of a node's label-walk sum: the all-unit kernels walk
// the list in two halves on separate waves (dense + (half 0 + half 1)), the group kernels in
// one chain (dense + all), so their results differ by fp32 re-association
// (tests/test_general_gpu.py::test_sorted_all_unit_vs_group_shape pins it)
__host__ inline bool hs_all_shape(const hdg_shape* s) {
  return s->nc <= HS_ALL_MAX && !(s->flags & HDG_FLAG_HUNK_GROUP);
}
__host__ inline size_t hs_shape_lds_bytes(const hdg_shape* s, int nvec) {
  const size_t NcP = (s->nc + 3) & ~3;
  if (hs_all_shape(s)) return hs_lds_bytes(s->nc, nvec);
  return ((size_t)KPW * NcP + (size_t)s->nc * (nvec == 1 ? HS_RSF : HS_RSB)) * 4;
}

// copy n16 16-byte words src -> dst with every load of the thread in flight first
template <int U>
__device__ __forceinline__ void copy16(float4* __restrict__ dst, const float4* __restrict__ src,
                                       int n16) {
  for (int e0 = threadIdx.x; e0 < n16; e0 += U * blockDim.x) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x;
      v[u] = src[e < n16 ? e : e0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x;
      if (e < n16) dst[e] = v[u];
    }
  }
}

// all-unit shape: stage the 20 sorted tables sv [H][NcP], then [Nc][H] node vectors (and
// weights) into the walk-row layout, 4 float4 loads (per table) of a thread in flight
template <int NV>
__device__ __forceinline__ void hs_stage_all(int z, int b, int Nc, const float* __restrict__ sv_g,
                                             const float* __restrict__ oth,
                                             const float* __restrict__ woth, float* lds) {
  constexpr int OS = NV == 1 ? HS_OSF : HS_OSB, U = 4;
  const int NcP = (Nc + 3) & ~3;
  copy16<6>(reinterpret_cast<float4*>(lds),
            reinterpret_cast<const float4*>(sv_g + hsort_tab(b, z, 0, NcP)), H * NcP / 4);
  float* dst = lds + H * NcP;
  const int n4 = Nc * (H / 4);
  const float4* o4 = reinterpret_cast<const float4*>(oth);
  const float4* w4 = reinterpret_cast<const float4*>(woth);
  for (int e0 = threadIdx.x; e0 < n4; e0 += U * blockDim.x) {
    float4 v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x < n4 ? e0 + u * blockDim.x : e0;
      v[u] = o4[e];
      if constexpr (NV == 2) w[u] = w4[e];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x;
      if (e >= n4) continue;
      const int n = e / (H / 4), q4 = e - n * (H / 4);
      const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      float ww[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (NV == 2) {
        ww[0] = w[u].x; ww[1] = w[u].y; ww[2] = w[u].z; ww[3] = w[u].w;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = 4 * q4 + c, g = k / KPW, m = k - g * KPW;
        if constexpr (NV == 1) {
          dst[n * OS + g * 6 + m] = vv[c];
        } else {
          dst[n * OS + g * 10 + 2 * m] = vv[c];
          dst[n * OS + g * 10 + 2 * m + 1] = ww[c];
        }
      }
    }
  }
  __syncthreads();
}

// group shape: stage unit group g's sorted values sv [KPW][NcP], then its walk rows
template <int NV>
__device__ __forceinline__ void hs_stage_g(int z, int b, int g, int Nc,
                                           const float* __restrict__ sv_g,
                                           const float* __restrict__ oth,
                                           const float* __restrict__ woth, float* lds) {
  constexpr int RS = NV == 1 ? HS_RSF : HS_RSB, U = 4;
  const int NcP = (Nc + 3) & ~3;
  copy16<4>(reinterpret_cast<float4*>(lds),
            reinterpret_cast<const float4*>(sv_g + hsort_tab(b, z, g * KPW, NcP)), KPW * NcP / 4);
  float* rows = lds + KPW * NcP;
  const float* ob = oth + g * KPW;
  const float* wb = woth + g * KPW;
  for (int n0 = threadIdx.x; n0 < Nc; n0 += U * blockDim.x) {
    float v[U][KPW], w[U][KPW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * blockDim.x < Nc ? n0 + u * blockDim.x : n0;
#pragma unroll
      for (int m = 0; m < KPW; ++m) {
        v[u][m] = ob[(size_t)n * H + m];
        if constexpr (NV == 2) w[u][m] = wb[(size_t)n * H + m];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * blockDim.x;
      if (n >= Nc) continue;
#pragma unroll
      for (int m = 0; m < KPW; ++m) {
        if constexpr (NV == 1) {
          rows[n * RS + m] = v[u][m];
        } else {
          rows[n * RS + 2 * m] = v[u][m];
          rows[n * RS + 2 * m + 1] = w[u][m];
        }
      }
    }
  }
  __syncthreads();
}

// the swept side's staged row q of unit group g: o (and w for NV = 2); RS the node stride,
// GS the group stride within a node row (6 / 10 in the all-unit layout, 0 in the group one)
template <int NV, int RS, int GS>
__device__ __forceinline__ void walk_row(const float* rows, int q, int g, float (&o)[KPW],
                                         float (&w)[KPW]) {
  const float* r = rows + q * RS + g * GS;
  if constexpr (NV == 1) {
    const float2 a = *reinterpret_cast<const float2*>(r);
    const float2 c = *reinterpret_cast<const float2*>(r + 2);
    const float2 e = *reinterpret_cast<const float2*>(r + 4);
    o[0] = a.x; o[1] = a.y; o[2] = c.x; o[3] = c.y; o[4] = e.x;
  } else {
#pragma unroll
    for (int m = 0; m < KPW; ++m) {
      const float2 a = *reinterpret_cast<const float2*>(r + 2 * m);
      o[m] = a.x;
      w[m] = a.y;
    }
  }
}

// node r's label ids (ylist_layout): f(id, valid) for each, the sentinel padding invalid;
// LB groups of four ids loaded before any is used
template <int LB = HS_LB, class F>
__device__ __forceinline__ void for_ylist(const uint32_t* __restrict__ prep, const ListLayout& Y,
                                          size_t r, int Nc, F f, int part = 0, int nparts = 1) {
  const int ngt = ((int)prep[Y.cnt + r] + 3) >> 2;
  const uint2* ids = reinterpret_cast<const uint2*>(
      reinterpret_cast<const uint16_t*>(prep + Y.ids) + r * list_stride(Nc));
  const int ng = (ngt * (part + 1)) / nparts;    // this caller's share of the 4-id groups
  for (int g0 = (ngt * part) / nparts; g0 < ng; g0 += LB) {
    uint2 q[LB];
#pragma unroll
    for (int u = 0; u < LB; ++u) q[u] = ids[g0 + u < ng ? g0 + u : g0];
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      if (g0 + u < ng) {
        const int i0 = (int)(q[u].x & 0xffffu), i1 = (int)(q[u].x >> 16);
        const int i2 = (int)(q[u].y & 0xffffu), i3 = (int)(q[u].y >> 16);
        f(i0 < Nc ? i0 : Nc - 1, i0 < Nc);
        f(i1 < Nc ? i1 : Nc - 1, i1 < Nc);
        f(i2 < Nc ? i2 : Nc - 1, i2 < Nc);
        f(i3 < Nc ? i3 : Nc - 1, i3 < Nc);
      }
    }
  }
}

// the five binary searches of a lane interleaved (independent LDS chains): m[kk] = first slot
// of unit kk's ascending table (svl + kk NcP) with value > -ow[kk]
__device__ __forceinline__ void hs_search(const float* svl, int NcP, int Nc,
                                          const float (&ow)[KPW], int (&m)[KPW]) {
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) m[kk] = 0;
  for (int st = top_pow2(Nc); st > 0; st >>= 1) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int c = m[kk] + st - 1;
      if (c < Nc && !(svl[kk * NcP + c] > -ow[kk])) m[kk] += st;
    }
  }
}

// The per-lane core of the forward sorted pass: node ncl's sums over the swept side for the
// five units of group g: the dense part from the search and the f64 suffix table (dsum), the
// self pair removed, the y = 1 pairs' relu(z1) replacing relu(z0) (the sentinel ids: a zero
// term) in acc.  part / nparts: this lane's share of the label list; part 0 alone does the
// dense part and the self pair (the others' dsum and acc start at 0).  The node's sums are
// dsum + the parts' acc summed in part order.
template <int RS, int GS>
__device__ __forceinline__ void fwd_s_lane(const float* svl, const float* rows, int NcP, int Nc,
                                           int b, int z, int g, int ncl, bool ys,
                                           const float (&ow)[KPW], const float (&dl)[KPW],
                                           const double* __restrict__ sx,
                                           const uint32_t* __restrict__ prep,
                                           const ListLayout& Y, size_t yrow, float (&dsum)[KPW],
                                           float (&acc)[KPW], int part = 0, int nparts = 1) {
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    dsum[kk] = 0.f;
    acc[kk] = 0.f;
  }
  if (part == 0) {
    int m[KPW];
    hs_search(svl, NcP, Nc, ow, m);
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk)
      dsum[kk] = (float)((double)(Nc - m[kk]) * (double)ow[kk] +
                         sx[hsort_tab(b, z, g * KPW + kk, NcP + 1) + m[kk]]);
    float os[KPW], unused[KPW];
    walk_row<1, RS, GS>(rows, ncl, g, os, unused);
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const float zs = ow[kk] + os[kk];                        // the self pair, as the walk
      acc[kk] = -relu(ys ? zs + dl[kk] : zs);                  // and the dense part count it
    }
  }
  for_ylist(prep, Y, yrow, Nc, [&](int q, bool ok) {
    float oq[KPW], unused[KPW];
    walk_row<1, RS, GS>(rows, q, g, oq, unused);
    const float vm = ok ? 1.f : 0.f;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const float z0 = ow[kk] + oq[kk];
      acc[kk] += vm * (relu(z0 + dl[kk]) - relu(z0));
    }
  }, part, nparts);
}

// ... and of the backward one: Dalpha / Dbeta sums (dsum + acc) and the y-weighted sums (ya),
// parts as in fwd_s_lane
template <int RS, int GS>
__device__ __forceinline__ void mlpb_s_lane(const float* svl, const float* rows, int NcP, int Nc,
                                            int b, int z, int g, int ncl, bool ys,
                                            const float (&ow)[KPW], const float (&wo)[KPW],
                                            const float (&dl)[KPW],
                                            const double* __restrict__ sw,
                                            const uint32_t* __restrict__ prep,
                                            const ListLayout& Y, size_t yrow, float (&dsum)[KPW],
                                            float (&acc)[KPW], float (&ya)[KPW], int part = 0,
                                            int nparts = 1) {
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    dsum[kk] = 0.f;
    acc[kk] = 0.f;
    ya[kk] = 0.f;
  }
  if (part == 0) {
    int m[KPW];
    hs_search(svl, NcP, Nc, ow, m);
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk)
      dsum[kk] = (float)((double)(Nc - m[kk]) * (double)wo[kk] +
                         sw[hsort_tab(b, z, g * KPW + kk, NcP + 1) + m[kk]]);
    float os[KPW], ws[KPW];
    walk_row<2, RS, GS>(rows, ncl, g, os, ws);
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const float zs = ow[kk] + os[kk];                        // the self pair
      const float gs = wo[kk] + ws[kk];
      const bool ms = (ys ? zs + dl[kk] : zs) > 0.f;
      acc[kk] = ms ? -gs : 0.f;
      ya[kk] = (ms && ys) ? -gs : 0.f;
    }
  }
  // y = 1 pairs: the mask of z1 replaces z0's (the sentinel ids: weight 0)
  for_ylist(prep, Y, yrow, Nc, [&](int q, bool ok) {
    float oq[KPW], wq[KPW];
    walk_row<2, RS, GS>(rows, q, g, oq, wq);
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const float z0 = ow[kk] + oq[kk];
      const float gq = ok ? wo[kk] + wq[kk] : 0.f;
      const float m1 = (z0 + dl[kk]) > 0.f ? gq : 0.f;
      acc[kk] += m1 - (z0 > 0.f ? gq : 0.f);
      ya[kk] += m1;
    }
  }, part, nparts);
}

// kw_hunk_fwd_s  grid (ceil(Nc / 128), B, 2), HS_NT threads, Nc <= HS_ALL_MAX: kw_hunk_fwd's
// results (G / H, sigma / tau) from the sorted tables.  Waves 8 h + w: h the half of every
// node's label list (the walks are latency-bound and the LDS tables allow one block per
// CU: the halves give each SIMD four waves instead of two), w as the 8-wave shape (node half
// w >> 2, unit group w & 3); half 1 hands its partial sums to half 0 through res
constexpr int HS_NT = 2 * NTP;
__global__ __launch_bounds__(HS_NT) void kw_hunk_fwd_s(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ D, int Nc, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ sv, const double* __restrict__ sx,
    const uint32_t* __restrict__ prep, ListLayout Y, float* __restrict__ G,
    float* __restrict__ Hh, float* __restrict__ sig, float* __restrict__ tau) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float hs_lds[];
  __shared__ float res[HSN * HP];
  __shared__ float Ml[H * H];
  int tile, b, z;
  xcd_commit_map(tile, b, z);
  const int t0 = tile * HSN, B = gridDim.y, NcP = (Nc + 3) & ~3;
  const int lane = threadIdx.x & 63, wl = uni(threadIdx.x >> 6), w = wl & 7, lh = wl >> 3;
  const int g = w & 3, hw = w >> 2;
  const int nl = hw * TN + lane, nd = t0 + nl, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  WSTAMP(2, 0);
  stage_w(Ml, D + D_M, H * H);
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H;
  float ow[KPW], dl[KPW], dsum[KPW], acc[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    ow[kk] = own[(size_t)ncl * H + g * KPW + kk];
    dl[kk] = D[D_DLT + g * KPW + kk];
  }
  const bool ys = bitf((z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC, ncl) > 0.f;
  hs_stage_all<1>(z, b, Nc, sv, (z ? alpha : beta) + (size_t)b * Nc * H, nullptr, hs_lds);
  WSTAMP(2, 1);
  fwd_s_lane<HS_OSF, 6>(hs_lds + g * KPW * NcP, hs_lds + H * NcP, NcP, Nc, b, z, g, ncl, ys, ow,
                        dl, sx, prep, Y, ((size_t)z * B + b) * Nc + ncl, dsum, acc, lh, 2);
  WSTAMP(2, 2);
  if (lh) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) res[nl * HP + g * KPW + kk] = acc[kk];
  }
  __syncthreads();
  if (!lh) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      float* r = res + nl * HP + g * KPW + kk;
      *r = dsum[kk] + (acc[kk] + *r);
    }
  }
  __syncthreads();
  float* gout = (z ? Hh : G) + (size_t)b * Nc * H;
  float* sout = (z ? tau : sig) + (size_t)b * Nc * H;
  const float* off = D + (z ? D_T0 : D_S0);
  for (int e = threadIdx.x; e < HSN * H; e += HS_NT) {
    const int n = e / H, k = e - n * H;
    if (t0 + n >= Nc) continue;
    float sacc = 0.f;
    for (int l = 0; l < H; ++l) sacc = fmaf(res[n * HP + l], Ml[l * H + k], sacc);
    gout[(t0 + n) * H + k] = res[n * HP + k];
    sout[(t0 + n) * H + k] = sacc + off[k];
  }
  WSTAMP(2, 3);
}

// kw_hunk_fwd_g  grid (4 hs_tiles(Nc), B, 2), NT threads, Nc > HS_ALL_MAX: G (z = 0) / H
// (z = 1) of one unit group; sigma / tau follow in kw_hunk_sig
__global__ __launch_bounds__(NT) void kw_hunk_fwd_g(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ D, int Nc, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ sv, const double* __restrict__ sx,
    const uint32_t* __restrict__ prep, ListLayout Y, float* __restrict__ G,
    float* __restrict__ Hh) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float hs_lds[];
  int tg, b, z;
  xcd_commit_map(tg, b, z);
  const int g = tg & 3, t0 = (tg >> 2) * HSG, B = gridDim.y, NcP = (Nc + 3) & ~3;
  const int nd = t0 + threadIdx.x, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H + g * KPW;
  float ow[KPW], dl[KPW], dsum[KPW], acc[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    ow[kk] = own[(size_t)ncl * H + kk];
    dl[kk] = D[D_DLT + g * KPW + kk];
  }
  const bool ys = bitf((z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC, ncl) > 0.f;
  hs_stage_g<1>(z, b, g, Nc, sv, (z ? alpha : beta) + (size_t)b * Nc * H, nullptr, hs_lds);
  fwd_s_lane<HS_RSF, 0>(hs_lds, hs_lds + KPW * NcP, NcP, Nc, b, z, g, ncl, ys, ow, dl, sx, prep,
                        Y, ((size_t)z * B + b) * Nc + ncl, dsum, acc);
  if (nd < Nc) {
    float* gout = (z ? Hh : G) + ((size_t)b * Nc + nd) * H + g * KPW;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) gout[kk] = dsum[kk] + acc[kk];
  }
}

// kw_hunk_sig  grid (tc, B, 2): sigma = G M + s0 (z = 0), tau = H M + t0 (z = 1), the
// classifier first layer on kw_hunk_fwd_g's node sums (kw_hunk_fwd's epilogue)
__global__ __launch_bounds__(NT) void kw_hunk_sig(const float* __restrict__ D, int Nc,
                                                  const float* __restrict__ G,
                                                  const float* __restrict__ Hh,
                                                  float* __restrict__ sig,
                                                  float* __restrict__ tau) {
#pragma clang fp contract(off)
  __shared__ float Ml[H * H];
  __shared__ float gl[TN * HP];
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN;
  stage_w(Ml, D + D_M, H * H);
  const float* src = (z ? Hh : G) + (size_t)b * Nc * H;
  for (int e = threadIdx.x; e < TN * H; e += NT) {
    const int n = e / H, k = e - n * H;
    gl[n * HP + k] = t0 + n < Nc ? src[(size_t)(t0 + n) * H + k] : 0.f;
  }
  __syncthreads();
  float* out = (z ? tau : sig) + (size_t)b * Nc * H;
  const float* off = D + (z ? D_T0 : D_S0);
  for (int e = threadIdx.x; e < TN * H; e += NT) {
    const int n = e / H, k = e - n * H;
    if (t0 + n >= Nc) continue;
    float sacc = 0.f;
    for (int l = 0; l < H; ++l) sacc = fmaf(gl[n * HP + l], Ml[l * H + k], sacc);
    out[(size_t)(t0 + n) * H + k] = sacc + off[k];
  }
}

// kw_hunk_mlpb_s  grid (ceil(Nc / 128), B, 2), NTP threads, Nc <= HS_ALL_MAX: kw_hunk_mlpb's
// results from the sorted tables.  Row pass (z = 0, node p): D alpha_p = dG_p |S_p| +
// sum_{q in S_p} dH_q with S_p = {q : beta_q > -alpha_p}; the column pass (node q) with
// alpha's order and dG; then the y = 1 pairs' mask changes, ysum = sum y dz, and the self
// pair removed.  The epilogue (partial gradient rows) per 64-node half, as kw_hunk_mlpb's
// tiles write them.
__global__ __launch_bounds__(HS_NT) void kw_hunk_mlpb_s(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ D, int Nc, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ dG, const float* __restrict__ dH,
    const float* __restrict__ nvec, const float* __restrict__ sv, const double* __restrict__ sw,
    const uint32_t* __restrict__ prep, ListLayout Y, float* __restrict__ Dal,
    float* __restrict__ Dbe, float* __restrict__ part, Segs sg) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float hs_lds[];
  __shared__ float res[HSN * HP], yres[HSN * HP], nt[TN * 4];
  int btile, b, z;
  xcd_commit_map(btile, b, z);
  const int t0 = btile * HSN, B = gridDim.y, NcP = (Nc + 3) & ~3;
  const int tc = (Nc + TN - 1) / TN;
  const int lane = threadIdx.x & 63, wl = uni(threadIdx.x >> 6), w = wl & 7, lh = wl >> 3;
  const int g = w & 3, hw = w >> 2;                // waves 8 lh + w: as kw_hunk_fwd_s
  const int nl = hw * TN + lane, nd = t0 + nl, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H;
  const float* wown = (z ? dH : dG) + (size_t)b * Nc * H;
  WSTAMP(3, 0);
  float ow[KPW], wo[KPW], dl[KPW], dsum[KPW], acc[KPW], ya[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    ow[kk] = own[(size_t)ncl * H + g * KPW + kk];
    wo[kk] = wown[(size_t)ncl * H + g * KPW + kk];
    dl[kk] = D[D_DLT + g * KPW + kk];
  }
  const bool ys = bitf((z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC, ncl) > 0.f;
  hs_stage_all<2>(z, b, Nc, sv, (z ? alpha : beta) + (size_t)b * Nc * H,
                  (z ? dG : dH) + (size_t)b * Nc * H, hs_lds);
  WSTAMP(3, 1);
  mlpb_s_lane<HS_OSB, 10>(hs_lds + g * KPW * NcP, hs_lds + H * NcP, NcP, Nc, b, z, g, ncl, ys,
                          ow, wo, dl, sw, prep, Y, ((size_t)z * B + b) * Nc + ncl, dsum, acc, ya,
                          lh, 2);
  WSTAMP(3, 2);
  if (lh) {                                        // list half 1's partial sums -> half 0
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      res[nl * HP + g * KPW + kk] = acc[kk];
      yres[nl * HP + g * KPW + kk] = ya[kk];
    }
  }
  __syncthreads();
  if (!lh) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      float* r = res + nl * HP + g * KPW + kk;
      float* yr = yres + nl * HP + g * KPW + kk;
      *r = dsum[kk] + (acc[kk] + *r);
      *yr = ya[kk] + *yr;
    }
  }
  __syncthreads();
  for (int half = 0; half < 2; ++half) {        // kw_hunk_mlpb's rows, one per 64-node tile
    const int tile = btile * 2 + half;
    if (tile >= tc) break;                       // block-uniform
    mlpb_epilogue(z, b, tile * TN, tc, Nc, nvec, res + half * TN * HP, yres + half * TN * HP,
                  nt, Dal, Dbe, part, sg, tile);
    __syncthreads();
  }
  WSTAMP(3, 3);
}

// kw_hunk_mlpb_g  grid (4 hs_tiles(Nc), B, 2), NT threads, Nc > HS_ALL_MAX: kw_hunk_mlpb_s for
// one unit group; the epilogue of its four 64-node tiles in one pass (the group's columns of
// each tile's partial rows)
__global__ __launch_bounds__(NT) void kw_hunk_mlpb_g(
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ yT,
    const float* __restrict__ D, int Nc, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ dG, const float* __restrict__ dH,
    const float* __restrict__ nvec, const float* __restrict__ sv, const double* __restrict__ sw,
    const uint32_t* __restrict__ prep, ListLayout Y, float* __restrict__ Dal,
    float* __restrict__ Dbe, float* __restrict__ part, Segs sg) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float hs_lds[];
  __shared__ float res[HSG * RS5], yres[HSG * RS5], nt[HSG * 4];
  int tg, b, z;
  xcd_commit_map(tg, b, z);
  const int g = tg & 3, btile = tg >> 2, t0 = btile * HSG, B = gridDim.y, NcP = (Nc + 3) & ~3;
  const int tc = (Nc + TN - 1) / TN;
  const int nl = threadIdx.x, nd = t0 + nl, ncl = nd < Nc ? nd : Nc - 1;
  const int WC = (Nc + 31) >> 5;
  const float* own = (z ? beta : alpha) + (size_t)b * Nc * H + g * KPW;
  const float* wown = (z ? dH : dG) + (size_t)b * Nc * H + g * KPW;
  float ow[KPW], wo[KPW], dl[KPW], dsum[KPW], acc[KPW], ya[KPW], out[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    ow[kk] = own[(size_t)ncl * H + kk];
    wo[kk] = wown[(size_t)ncl * H + kk];
    dl[kk] = D[D_DLT + g * KPW + kk];
  }
  const bool ys = bitf((z ? yT : ybits) + ((size_t)b * Nc + ncl) * WC, ncl) > 0.f;
  hs_stage_g<2>(z, b, g, Nc, sv, (z ? alpha : beta) + (size_t)b * Nc * H,
                (z ? dG : dH) + (size_t)b * Nc * H, hs_lds);
  mlpb_s_lane<HS_RSB, 0>(hs_lds, hs_lds + KPW * NcP, NcP, Nc, b, z, g, ncl, ys, ow, wo, dl, sw,
                         prep, Y, ((size_t)z * B + b) * Nc + ncl, dsum, acc, ya);
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) out[kk] = dsum[kk] + acc[kk];
  const bool in = nd < Nc;
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    res[nl * RS5 + kk] = in ? out[kk] : 0.f;
    yres[nl * RS5 + kk] = in ? ya[kk] : 0.f;
  }
  float* dout = (z ? Dbe : Dal) + (size_t)b * Nc * H + g * KPW;
  if (in) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) dout[(size_t)nd * H + kk] = out[kk];
  }
  for (int e = threadIdx.x; e < HSG * 4; e += NT)
    nt[e] = (t0 + e / 4 < Nc) ? nvec[((size_t)b * Nc + t0) * 4 + e] : 0.f;
  __syncthreads();
  // the group's columns of mlpb_epilogue's rows 0..9 of V1 and c1, every tile of the block
  const Seg& s = sg.s[SG_MLPB];
  constexpr int NI = 11 * KPW;
  for (int e = threadIdx.x; e < (HSG / TN) * NI; e += NT) {
    const int q = e / NI, r = e - q * NI, l = r / KPW, kk = r - l * KPW;
    const int tile = btile * (HSG / TN) + q;
    if (tile >= tc) continue;
    const float* rq = res + q * TN * RS5;
    const float* yq = yres + q * TN * RS5;
    const float* nq = nt + q * TN * 4;
    float a = 0.f;
    if (l < 8) {
      const int m = l & 3;
      if ((l >> 2) == z)
        for (int n = 0; n < TN; ++n) a = fmaf(nq[n * 4 + m], rq[n * RS5 + kk], a);
    } else if (z == 0) {
      float sd = 0.f, sy = 0.f;
      for (int n = 0; n < TN; ++n) { sd += rq[n * RS5 + kk]; sy += yq[n * RS5 + kk]; }
      a = l == 8 ? sd - sy : (l == 9 ? sy : sd);
    }
    put(part, s, l * H + g * KPW + kk, (b * tc + tile) * 2 + z, a);
  }
}

// ---------------------------------------------------------------------------------
// kw_hunk_fin0/1/2: the one-sweep tiles' (kh_tile<MODE>, hdgnn.hip) block partials summed in
// a fixed order per node -- row sums over the column blocks, column sums over the row
// blocks -- the diagonal pair removed (modes 0, 1), then the epilogue of the two-pass kernel
// the mode replaces (kw_hunk_fwd / kw_hunk_mlpb / kw_hunk_clsb), unchanged.  The sum y e
// totals (modes 1, 2) go into the row pass's first tile (its epilogue only ever sums them).
// ---------------------------------------------------------------------------------
struct HTileSums {
  const float *rpart, *cpart, *ysp;
  int CC, RC;
};
// row (z = 0) / column (z = 1) sum of node nd, unit k, commit b
__device__ __forceinline__ float htile_sum(const HTileSums& hs, int z, int b, int Nc, int nd,
                                           int k) {
  const int n = z ? hs.RC : hs.CC;
  const float* p = (z ? hs.cpart : hs.rpart) + ((size_t)b * n * Nc + nd) * H + k;
  const size_t st = (size_t)Nc * H;
  float v[8];
  float a = 0.f;
  for (int q0 = 0; q0 < n; q0 += 8) {                 // eight partials' loads in flight
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = q0 + u < n ? p[(q0 + u) * st] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  return a;
}
__device__ __forceinline__ float htile_ysum(const HTileSums& hs, int b, int k) {
  const float* p = hs.ysp + (size_t)b * hs.RC * hs.CC * H + k;
  float a = 0.f;
  for (int q = 0; q < hs.RC * hs.CC; ++q) a += p[(size_t)q * H];
  return a;
}

// kw_hunk_fin0  grid (tc, B, 2): G / H (z = 0 / 1) and sigma / tau
__global__ __launch_bounds__(NTP) void kw_hunk_fin0(HTileSums hs, const float* __restrict__ D,
                                                    int Nc, const float* __restrict__ alpha,
                                                    const float* __restrict__ beta,
                                                    float* __restrict__ G, float* __restrict__ Hh,
                                                    float* __restrict__ sig,
                                                    float* __restrict__ tau) {
#pragma clang fp contract(off)
  __shared__ float res[TN * HP];
  __shared__ float Ml[H * H];
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN;
  stage_w(Ml, D + D_M, H * H);
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H, nd = t0 + n;
    float v = 0.f;
    if (nd < Nc) {
      const size_t q = ((size_t)b * Nc + nd) * H + k;
      const float zs = alpha[q] + (0.f * D[D_DLT + k] + beta[q]);   // the tile's z, y = 0
      v = htile_sum(hs, z, b, Nc, nd, k) - zs * (zs > 0.f ? 1.f : 0.f);
    }
    res[n * HP + k] = v;
  }
  __syncthreads();
  float* gout = (z ? Hh : G) + (size_t)b * Nc * H;
  float* sout = (z ? tau : sig) + (size_t)b * Nc * H;
  const float* off = D + (z ? D_T0 : D_S0);
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H;
    if (t0 + n >= Nc) continue;
    float sacc = 0.f;
    for (int l = 0; l < H; ++l) sacc = fmaf(res[n * HP + l], Ml[l * H + k], sacc);
    gout[(t0 + n) * H + k] = res[n * HP + k];
    sout[(t0 + n) * H + k] = sacc + off[k];
  }
}

// kw_hunk_fin1  grid (tc, B, 2): D alpha / D beta and kw_hunk_mlpb's partial rows
__global__ __launch_bounds__(NTP) void kw_hunk_fin1(HTileSums hs, const float* __restrict__ D,
                                                    int Nc, const float* __restrict__ alpha,
                                                    const float* __restrict__ beta,
                                                    const float* __restrict__ dG,
                                                    const float* __restrict__ dH,
                                                    const float* __restrict__ nvec,
                                                    float* __restrict__ Dal, float* __restrict__ Dbe,
                                                    float* __restrict__ part, Segs sg) {
#pragma clang fp contract(off)
  __shared__ float res[TN * HP], yres[TN * HP], nt[TN * 4];
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN, tc = gridDim.x;
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H, nd = t0 + n;
    float v = 0.f;
    if (nd < Nc) {
      const size_t q = ((size_t)b * Nc + nd) * H + k;
      const float zs = alpha[q] + (0.f * D[D_DLT + k] + beta[q]);
      const float gs = dG[q] + dH[q];
      v = htile_sum(hs, z, b, Nc, nd, k) - (zs > 0.f ? 1.f : 0.f) * gs;
    }
    res[n * HP + k] = v;
    yres[n * HP + k] = (z == 0 && blockIdx.x == 0 && n == 0) ? htile_ysum(hs, b, k) : 0.f;
  }
  __syncthreads();
  mlpb_epilogue(z, b, t0, tc, Nc, nvec, res, yres, nt, Dal, Dbe, part, sg, blockIdx.x);
}

// kw_hunk_fin2  grid (tc, B, 2): the classifier backward's sums, then kw_hunk_clsb's epilogue
__global__ __launch_bounds__(NTP) void kw_hunk_fin2(HTileSums hs, const float* __restrict__ W,
                                                    Off o, const float* __restrict__ D, int Nc,
                                                    const float* __restrict__ G,
                                                    const float* __restrict__ Hh,
                                                    float* __restrict__ Dsig,
                                                    float* __restrict__ Dtau, float* __restrict__ dG,
                                                    float* __restrict__ dH, float* __restrict__ part,
                                                    Segs sg) {
#pragma clang fp contract(off)
  __shared__ float res[TN * HP], yres[TN * HP], Gt[TN * HP];
  __shared__ float X[H * H], sumD[H], ysum[H];
  __shared__ float Wl[3 * H * H + H];
  __shared__ float kzh[1];
  if (threadIdx.x == 0) kzh[0] = 0.f;
  stage_w(Wl, D + D_M, H * H);
  stage_w(Wl + H * H, W + o.H1_W2, H * H + H);
  stage_w(Wl + 2 * H * H + H, W + o.H2_W1 + 2 * H, H * H);
  const int z = blockIdx.z, b = blockIdx.y, t0 = blockIdx.x * TN, tc = gridDim.x;
  for (int e = threadIdx.x; e < TN * H; e += NTP) {
    const int n = e / H, k = e - n * H, nd = t0 + n;
    res[n * HP + k] = nd < Nc ? htile_sum(hs, z, b, Nc, nd, k) : 0.f;
    yres[n * HP + k] = (z == 0 && blockIdx.x == 0 && n == 0) ? htile_ysum(hs, b, k) : 0.f;
  }
  __syncthreads();
  clsb_epilogue(z, b, t0, tc, Nc, W, o, D, G, Hh, Dsig, Dtau, dG, dH, part, sg, res, yres, Gt, X,
                sumD, ysum, Wl, kzh, blockIdx.x);
}

// kw_dn  grid (tc, B): dn_c[m] = sum_k V1[m][k] Dalpha_c[k] + V1[4+m][k] Dbeta_c[k]
__global__ __launch_bounds__(NT) void kw_dn(const float* __restrict__ W, Off o, int Nc,
                                            const float* __restrict__ Dal,
                                            const float* __restrict__ Dbe,
                                            float* __restrict__ dn) {
  const int b = blockIdx.y, c = blockIdx.x * TN + (threadIdx.x & 63), m = threadIdx.x >> 6;
  if (c >= Nc) return;
  const float* da = Dal + ((size_t)b * Nc + c) * H;
  const float* db = Dbe + ((size_t)b * Nc + c) * H;
  float a = 0.f;
  for (int k = 0; k < H; ++k)
    a = fmaf(W[o.H1_W1 + m * H + k], da[k], fmaf(W[o.H1_W1 + (4 + m) * H + k], db[k], a));
  dn[((size_t)b * Nc + c) * 4 + m] = a;
}

// ---------------------------------------------------------------------------------
// kw_node_bwd  grid (te, B): cross-graph + mlp2_entity_B1 backward (model_2.py:146-150,
// 190-205, 181-188): dx'_I = sum_c dn_c[0] K_s[c][I] + dn_c[1] K_t[c][I];
// do = [o > 0] dx';  dq = [h > 0] w2' do;  dE = dq W1'[1:]^T;  rho = dP = dE W5^T.
// Partial rows of dW1', db1', dw2', db2', dW5, db5.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void kw_node_bwd(
    const uint32_t* __restrict__ prep, const float* __restrict__ x, const float* __restrict__ W,
    Off o, int Ne, int Nc, const float* __restrict__ dn, const float* __restrict__ ov,
    const float* __restrict__ P, const float* __restrict__ Eb, const float* __restrict__ hE,
    float* __restrict__ rhoE, float* __restrict__ part, Segs sg, const float* __restrict__ Dal,
    const float* __restrict__ Dbe) {
  __shared__ float dxq[NW * TN], xs[TN], dov[TN];
  __shared__ float2 dnl[HS_NC_MAX];               // (dn_c[0], dn_c[1]) of the commit
  __shared__ float Pt[TN * HP], Et[TN * HP], ht[TN * HP], dq[TN * HP], dE[TN * HP];
  __shared__ float Wl[864];
  __shared__ float kzr[1];                        // 0.f: stride-0 operand of padding tiles
  const float *W1e = Wl, *W2e = Wl + 440, *W5 = Wl + 464;   // W1' (21 x 20) | b1' | w2' | b2' | W5
  if (threadIdx.x == 0) kzr[0] = 0.f;
  const GenPrep PL = gen_prep(Ne, Nc);
  const int b = blockIdx.y, t0 = blockIdx.x * TN, t = threadIdx.x, te = gridDim.x;
  const int lane = t & 63, w = t >> 6;
  const int I = t0 + lane;
  const uint32_t* pp = prep + (size_t)b * PL.words;
  WSTAMP(12, 0);
  // the tile's P / E_bar / h rows and its ov / x values are loaded first (registers), so their
  // latency hides behind the count loop instead of costing two round trips after it
  constexpr int NPE = TN * H / NT;
  static_assert(TN * H % NT == 0, "kw_node_bwd row staging");
  const size_t base = ((size_t)b * Ne + t0) * H;
  float pv[NPE], ev[NPE], hv[NPE];
#pragma unroll
  for (int it = 0; it < NPE; ++it) {
    const int e = t + it * NT, n = e / H;
    const size_t a = t0 + n < Ne ? base + e : base;           // clamped load, value dropped
    pv[it] = P[a];
    ev[it] = Eb[a];
    hv[it] = hE[a];
  }
  const int tnode = t0 + (t < TN ? t : 0) < Ne ? t0 + (t < TN ? t : 0) : Ne - 1;
  const float ovt = ov[(size_t)b * Ne + tnode], xt = x[(size_t)b * Ne + tnode];
  stage_w(Wl, W + o.E3_W1, 461);
  stage_w(Wl + 464, W + o.E1_W5, 400);
  // the commit's (dn_c[0], dn_c[1]) in LDS: the count loop's per-hunk factors are the same
  // for every lane, and as scalar loads (one s_load and lgkmcnt wait per hunk pair) they
  // cost a third of the loop (wave stamps: 16.9 -> 11.9 us without them at stress)
  if (dn) {
    const float* dnb = dn + (size_t)b * Nc * 4;
    for (int c = t; c < Nc; c += NT) dnl[c] = *reinterpret_cast<const float2*>(dnb + 4 * c);
  } else {   // dn = NULL (no entity-edge stage reads it): kw_dn's m = 0, 1 values computed
             // here, the same fma order, from the commit's Dalpha / Dbeta rows
    constexpr int DU = 2;                          // hunks per thread and round trip
    for (int c0 = t; c0 < Nc; c0 += DU * NT) {
      float4 va[DU][H / 4], vb[DU][H / 4];
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const int c = c0 + u * NT < Nc ? c0 + u * NT : c0;   // clamped load, unused
        const float4* da = reinterpret_cast<const float4*>(Dal + ((size_t)b * Nc + c) * H);
        const float4* db = reinterpret_cast<const float4*>(Dbe + ((size_t)b * Nc + c) * H);
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {
          va[u][v] = da[v];
          vb[u][v] = db[v];
        }
      }
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        if (c0 + u * NT >= Nc) break;
        const float* fa = reinterpret_cast<const float*>(va[u]);
        const float* fb = reinterpret_cast<const float*>(vb[u]);
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int k = 0; k < H; ++k) {
          a0 = fmaf(W[o.H1_W1 + k], fa[k], fmaf(W[o.H1_W1 + 4 * H + k], fb[k], a0));
          a1 = fmaf(W[o.H1_W1 + H + k], fa[k], fmaf(W[o.H1_W1 + 5 * H + k], fb[k], a1));
        }
        dnl[c0 + u * NT] = make_float2(a0, a1);
      }
    }
  }
  __syncthreads();
  WSTAMP(12, 1);
  {
    const uint16_t* ks = reinterpret_cast<const uint16_t*>(pp + PL.ks);
    const uint16_t* kt = reinterpret_cast<const uint16_t*>(pp + PL.kt);
    const int c0 = (Nc * w) / NW, c1 = (Nc * (w + 1)) / NW;
    float a = 0.f;
    if (I < Ne) {                  // NB_U hunks' counts in flight per step, same fma order
      constexpr int NB_U = 16;     // (a wave walks Nc / 4 hunks: at Nc = 512, 8 round trips)
      int c = c0;
      for (; c + NB_U <= c1; c += NB_U) {
        float vs[NB_U], vt[NB_U], d0[NB_U], d1[NB_U];
#pragma unroll
        for (int u = 0; u < NB_U; ++u) {
          if (HDG_ABL_DX & 1) {      // ablation builds only (wrong sums): no count loads
            vs[u] = (float)((c + u + I) & 3);
            vt[u] = (float)((c + u + I) & 1);
          } else {
            vs[u] = (float)ks[(size_t)(c + u) * Ne + I];
            vt[u] = (float)kt[(size_t)(c + u) * Ne + I];
          }
          if (HDG_ABL_DX & 2) {      // ... no dn loads
            d0[u] = (float)(c + u);
            d1[u] = (float)(c - u);
          } else {
            const float2 dv = dnl[c + u];
            d0[u] = dv.x;
            d1[u] = dv.y;
          }
        }
#pragma unroll
        for (int u = 0; u < NB_U; ++u) {
          a = fmaf(d0[u], vs[u], a);
          a = fmaf(d1[u], vt[u], a);
        }
      }
      for (; c + 4 <= c1; c += 4) {
        float vs[4], vt[4], d0[4], d1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          vs[u] = (float)ks[(size_t)(c + u) * Ne + I];
          vt[u] = (float)kt[(size_t)(c + u) * Ne + I];
          d0[u] = dnl[c + u].x;
          d1[u] = dnl[c + u].y;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a = fmaf(d0[u], vs[u], a);
          a = fmaf(d1[u], vt[u], a);
        }
      }
      for (; c < c1; ++c) {
        a = fmaf(dnl[c].x, (float)ks[(size_t)c * Ne + I], a);
        a = fmaf(dnl[c].y, (float)kt[(size_t)c * Ne + I], a);
      }
    }
    dxq[w * TN + lane] = a;
  }
  WSTAMP(12, 2);
#pragma unroll
  for (int it = 0; it < NPE; ++it) {
    const int e = t + it * NT, n = e / H, k = e - n * H;
    const bool in = t0 + n < Ne;
    Pt[n * HP + k] = in ? pv[it] : 0.f;
    Et[n * HP + k] = in ? ev[it] : 0.f;
    ht[n * HP + k] = in ? hv[it] : 0.f;
  }
  __syncthreads();
  if (t < TN) {
    const bool in = t0 + t < Ne;
    const float d = ((dxq[t] + dxq[TN + t]) + dxq[2 * TN + t]) + dxq[3 * TN + t];
    dov[t] = (in && ovt > 0.f) ? d : 0.f;
    xs[t] = in ? xt : 0.f;
  }
  __syncthreads();
  for (int e = t; e < TN * H; e += NT) {
    const int n = e / H, k = e - n * H;
    dq[n * HP + k] = ht[n * HP + k] > 0.f ? W2e[k] * dov[n] : 0.f;
  }
  __syncthreads();
  // dE = dq W1'[1:]^T, rho_E = dE W5^T as MFMA tiles (transposed weights: SM = 1, SK = H)
  WSTAMP(12, 3);
  rows_x_w<1, H>(dq, W1e + H, kzr, [&](int n, int m, float c) { dE[n * HP + m] = c; });
  __syncthreads();
  rows_x_w<1, H>(dE, W5, kzr, [&](int n, int l, float c) {
    if (t0 + n < Ne) rhoE[base + n * H + l] = c;
  });
  WSTAMP(12, 4);
  const int row = b * te + blockIdx.x;
  const Seg& s3 = sg.s[SG_E3];
  const Seg& s5 = sg.s[SG_E1W5];
  const float twoNe1 = 2.f * (float)(Ne - 1);
  // dW1'[l][k] = sum_n X[n][l] dq[n][k] (X = [x | E_bar], 21 rows) and dW5[l][m] =
  // sum_n P[n][l] dE[n][m] over the tile's 64 nodes as 16x16 MFMA tiles (2 x 2 each)
  for (int tile = t >> 6; tile < 8; tile += NT / 64) {      // wave-uniform
    const int which = tile >> 2, r0 = ((tile >> 1) & 1) * 16, cc = (tile & 1) * 16 + (lane & 15);
    const int rl = r0 + (lane & 15);
    const bool cv = cc < H, rv = rl < (which ? H : H + 1);
    const float* pa = kzr;
    int sa = 0;
    if (rv) {
      if (which) { pa = Pt + rl; sa = HP; }
      else if (rl == 0) { pa = xs; sa = 1; }
      else { pa = Et + rl - 1; sa = HP; }
    }
    const f4v c = mfma_tile16_p(pa, sa, cv ? (which ? dE : dq) + cc : kzr, cv ? HP : 0, TN, lane);
    if (cv)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rr = r0 + 4 * (lane >> 4) + j;
        if (rr < (which ? H : H + 1)) put(part, which ? s5 : s3, rr * H + cc, row, c[j]);
      }
  }
  for (int e = 420 + t; e < 461 + 420; e += NT) {
    float a = 0.f;
    if (e < 440) {                 // db1'
      const int k = e - 420;
      for (int n = 0; n < TN; ++n) a += dq[n * HP + k];
      put(part, s3, e, row, a);
    } else if (e < 460) {          // dw2'
      const int k = e - 440;
      for (int n = 0; n < TN; ++n) a = fmaf(ht[n * HP + k], dov[n], a);
      put(part, s3, e, row, a);
    } else if (e == 460) {         // db2'
      for (int n = 0; n < TN; ++n) a += dov[n];
      put(part, s3, e, row, a);
    } else {
      const int f = e - 461;
      if (f < 400) continue;       // dW5: MFMA tiles above
      const int m = f - 400;       // db5[m] = 2(Ne-1) sum_n dE[n][m]
      for (int n = 0; n < TN; ++n) a += dE[n * HP + m];
      a *= twoNe1;
      put(part, s5, f, row, a);
    }
  }
  WSTAMP(12, 5);
}

// ---------------------------------------------------------------------------------
// First-layer backward of the entity pair MLPs, sorted-x form.
//   E1 (model_2.py:165-170):  dz_ij = [z_ij > 0] (rho_i + rho_j)         (r = q = rho = dP)
//   EE (model_4.py:212-223):  dz'_ij = [z'_ij > 0] (phi_i + psi_j)       (r = phi, q = psi)
//   S0 = sum x_i dz, S1 = sum x_j dz, S2 = sum dz, S3 = sum a dz over all pairs.
// For node i the a = 0 set is the forward's prefix / suffix, so sum_{j in set} q_j and
// sum x_j q_j are single reads of per-k scan tables over the x-sorted order (suffix
// sums when the slope is >= 0, prefix sums otherwise; f64), built by kw_scan; the a = 1
// pairs correct the mask over the set bits of row i; the diagonal is removed.
// ---------------------------------------------------------------------------------
// kw_scan  grid (H, B, modes): tab[mode][b][k][2][Ne+1] (q sums, x q sums), f64
__global__ __launch_bounds__(NT) void kw_scan(const uint32_t* __restrict__ prep,
                                              const float* __restrict__ W, Off o, int Ne, int Nc,
                                              int mode0, const float* __restrict__ q0,
                                              const float* __restrict__ q1,
                                              double* __restrict__ tab) {
  __shared__ double c1[NT], c2[NT];
  const GenPrep GP = gen_prep(Ne, Nc);
  // the 20 unit blocks of commit b on one XCD (B % 8 == 0): the commit's rho / phi rows and
  // sorted tables are fetched into that L2 once instead of once per unit from every XCD
  int k, b, zz;
  xcd_commit_map(k, b, zz);
  const int mode = mode0 + zz, t = threadIdx.x;
  const int B = gridDim.y;
  const uint32_t* pp = prep + (size_t)b * GP.words;
  const float* xsrt = reinterpret_cast<const float*>(pp + GP.xsrt);
  const int* perm = reinterpret_cast<const int*>(pp + GP.perm);
  const float slope = mode == 0 ? W[o.E1_W1 + H + k] : W[o.EE_W11 + k];
  const bool suf = slope >= 0.f;
  const float* q = (mode == 0 ? q0 : q1) + (size_t)b * Ne * H;
  double* T = tab + (((size_t)mode * B + b) * H + k) * 2 * (Ne + 1);
  const int C = (Ne + NT - 1) / NT;
  const int p0 = t * C, p1 = p0 + C < Ne ? p0 + C : Ne;
  // C <= CR (Ne <= 1024): the thread's chunk loaded once, every load issued before the first
  // use (perm, then the gathered q and x), kept in registers for the second pass -- the
  // kernel was a chain of dependent loads per element, twice
  constexpr int CR = 4;
  const bool reg = C <= CR;
  float qv[CR], xv[CR];
  int mv[CR];
  double a1 = 0.0, a2 = 0.0;
  if (reg) {
    int pm[CR];
#pragma unroll
    for (int u = 0; u < CR; ++u) {
      const int p = p0 + u < p1 ? p0 + u : p0;           // clamped, unused past the chunk
      mv[u] = suf ? Ne - 1 - p : p;
      pm[u] = p < Ne ? perm[mv[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < CR; ++u) {
      qv[u] = q[(size_t)pm[u] * H + k];
      xv[u] = xsrt[p0 + u < Ne ? mv[u] : 0];
    }
#pragma unroll
    for (int u = 0; u < CR; ++u) {
      if (p0 + u < p1) {
        const double val = (double)qv[u];
        a1 += val;
        a2 += val * (double)xv[u];
      }
    }
  } else {
    for (int p = p0; p < p1; ++p) {            // p = position in scan order
      const int m = suf ? Ne - 1 - p : p;
      const double val = (double)q[(size_t)perm[m] * H + k];
      a1 += val;
      a2 += val * (double)xsrt[m];
    }
  }
  // exclusive scan of the per-thread chunk sums: wave shuffles, then the 4 wave totals
  const int lane = t & 63, w = t >> 6;
  double i1 = a1, i2 = a2;
#pragma unroll
  for (int o2 = 1; o2 < 64; o2 <<= 1) {
    const double u1 = __shfl_up(i1, o2), u2 = __shfl_up(i2, o2);
    if (lane >= o2) { i1 += u1; i2 += u2; }
  }
  if (lane == 63) { c1[w] = i1; c2[w] = i2; }
  __syncthreads();
  double b1 = 0.0, b2 = 0.0;
  for (int u = 0; u < w; ++u) { b1 += c1[u]; b2 += c2[u]; }
  a1 = b1 + (i1 - a1);
  a2 = b2 + (i2 - a2);
  if (t == 0) {
    T[suf ? Ne : 0] = 0.0;
    T[Ne + 1 + (suf ? Ne : 0)] = 0.0;
  }
  if (reg) {
#pragma unroll
    for (int u = 0; u < CR; ++u) {
      if (p0 + u < p1) {
        const double val = (double)qv[u];
        a1 += val;
        a2 += val * (double)xv[u];
        const int e = suf ? mv[u] : mv[u] + 1;
        T[e] = a1;
        T[Ne + 1 + e] = a2;
      }
    }
    return;
  }
  for (int p = p0; p < p1; ++p) {
    const int m = suf ? Ne - 1 - p : p;
    const double val = (double)q[(size_t)perm[m] * H + k];
    a1 += val;
    a2 += val * (double)xsrt[m];
    const int e = suf ? m : m + 1;           // suffix: sum over slots >= m; prefix: < m+1
    T[e] = a1;
    T[Ne + 1 + e] = a2;
  }
}

template <int MODE, int HALVES>
__device__ __forceinline__ void first_bwd_body(const float* __restrict__ x,
                                               const uint32_t* __restrict__ abits,
                                               const uint32_t* __restrict__ prep,
                                               const float* __restrict__ W, const Off& o, int Ne,
                                               int Nc, const float* __restrict__ ra,
                                               const float* __restrict__ rb,
                                               const double* __restrict__ tab,
                                               float* __restrict__ part, const Segs& sg,
                                               float* hand, const int tx, const int b) {
#pragma clang fp contract(off)
  const GenPrep GP = gen_prep(Ne, Nc);
  const int t0 = tx * TN, te = gridDim.x, B = gridDim.y;
  // 4 HALVES waves: wave g + 4 hw takes hidden units g; with HALVES = 2 the halves hw split
  // each lane's neighbour list (hw 1 hands its partial sums over through LDS), hw 0 also
  // does the dense part; with HALVES = 1 the 4 waves walk whole lists (no hand-off)
  const int lane = threadIdx.x & 63, g = uni((threadIdx.x >> 6) & 3);
  const int hw = HALVES == 2 ? uni(threadIdx.x >> 8) : 0;
  const int i = t0 + lane;
  const bool live = i < Ne;
  const int ic = live ? i : Ne - 1;
  extern __shared__ __attribute__((aligned(16))) double tabs_lds[];
  WSTAMP(13, 0);
  const SortTabs T = stage_tabs(prep, GP, b, Ne, tabs_lds, x + (size_t)b * Ne);
  WSTAMP(13, 1);
  const float* xb = T.xs;
  const float xi = xb[ic];
  const float* rbb = rb + (size_t)b * Ne * H;
  float S0[KPW], S1[KPW], S2[KPW], S3[KPW], u[KPW], wb[KPW], dd[KPW], ri[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const int k = g * KPW + kk;
    float slope;
    if constexpr (MODE == 0) {
      const float w2 = W[o.E1_W1 + 2 * H + k];
      slope = W[o.E1_W1 + H + k];
      dd[kk] = W[o.E1_W1 + 3 * H + k] - w2;
      u[kk] = fmaf(xi, W[o.E1_W1 + k], w2 + W[o.E1_B1 + k]);
    } else {
      const float w20 = W[o.EE_W12 + k];
      slope = W[o.EE_W11 + k];
      dd[kk] = W[o.EE_W12 + H + k] - w20;
      u[kk] = fmaf(xi, slope, w20 + W[o.EE_B1 + k]);
    }
    wb[kk] = slope;
    ri[kk] = ra[((size_t)b * Ne + ic) * H + k];
    S0[kk] = 0.f;                                 // x_i-weighted corrections only
    S1[kk] = 0.f;
    S2[kk] = 0.f;
    S3[kk] = 0.f;
  }
  if (!hw) {                                      // the dense part: hw 0
  bool sinc[KPW];
  int sb[KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) sinc[kk] = wb[kk] >= 0.f;
  set_bounds<KPW>(T, sinc, sb, [&](int n, float xq) {   // the units' searches in lockstep
    return MODE == 0 ? (u[n] + xq * wb[n]) > 0.f : fmaf(xq, wb[n], u[n]) > 0.f;
  });
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const int k = g * KPW + kk;
    const float uu = u[kk], slope = wb[kk];
    const bool inc = slope >= 0.f;
    const int br = sb[kk];
    const int lo = inc ? br : 0, hi = inc ? T.nd : br;
    const double cnt = (double)(T.cum[hi] - T.cum[lo]);
    const double sx = T.pxd[hi] - T.pxd[lo];
    const double* Tk = tab + (((size_t)MODE * B + b) * H + k) * 2 * (Ne + 1);
    const int bm = T.cum[br];
    double gs = cnt * (double)ri[kk] + Tk[bm];
    double gx = (double)ri[kk] * sx + Tk[Ne + 1 + bm];
    const float zii = MODE == 0 ? uu + xi * slope : fmaf(xi, slope, uu);
    if (zii > 0.f) {                              // remove j == i
      const double gi = (double)ri[kk] + (double)rbb[(size_t)ic * H + k];
      gs -= gi;
      gx -= (double)xi * gi;
    }
    S2[kk] = (float)gs;
    S1[kk] = (float)gx;
  }
  }
  float cs[KPW];                                  // sum of the corrections' dm
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) cs[kk] = 0.f;
  WSTAMP(13, 2);
  if (live) {   // units (0,1), (2,3) as packed pairs, unit 4 scalar; [z > 0] g as step2(z) g
    static_assert(KPW == 5, "packed correction layout");
    f2 u2[2], wb2[2], dd2[2], ri2[2], cs2[2], s12[2], s32[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u2[h] = (f2){u[2 * h], u[2 * h + 1]};
      wb2[h] = (f2){wb[2 * h], wb[2 * h + 1]};
      dd2[h] = (f2){dd[2 * h], dd[2 * h + 1]};
      ri2[h] = (f2){ri[2 * h], ri[2 * h + 1]};
      cs2[h] = (f2){0.f, 0.f};
      s12[h] = (f2){S1[2 * h], S1[2 * h + 1]};
      s32[h] = (f2){0.f, 0.f};
    }
    float cst = 0.f, s1t = S1[4], s3t = 0.f;
    // neighbour j's row of the group's 5 units and its x (the sentinel Ne reads node 0's
    // row with gg = 0: every term below vanishes)
    struct NbrRow {
      f2 q[2];
      float q4, xj;
    };
    auto ldr = [&](const int j0) -> NbrRow {
      const int j = j0 < Ne ? j0 : 0;
      const float* qj = rbb + (size_t)(HDG_ABL_QJ ? ic : j) * H + g * KPW;
      NbrRow v;
      v.q[0] = (f2){qj[0], qj[1]};
      v.q[1] = (f2){qj[2], qj[3]};
      v.q4 = qj[4];
      v.xj = HDG_ABL_XJ ? xb[lane + (j & 1)] : xb[j];
      return v;
    };
    auto use = [&](const int j0, const NbrRow& v) {
      const bool ok = j0 < Ne;
      const float vm = ok ? 1.f : 0.f;
      const float xj = v.xj;
      const f2 xx = {xj, xj};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 z0 = MODE == 0 ? u2[h] + xx * wb2[h] : fma2(xx, wb2[h], u2[h]);
        const f2 gg = (ri2[h] + v.q[h]) * vm;   // finite
        // dm and s3 from the two masks (same values as m1 - m0 and += m1); stepf2 for st1
        // is one op fewer but raises this walk to 125 VGPRs (spills at 6 waves)
        const f2 st0 = step2(z0);
        const f2 st1 = step2(z0 + dd2[h]);
        const f2 dm = (st1 - st0) * gg;
        cs2[h] += dm;
        s12[h] = fma2(xx, dm, s12[h]);
        s32[h] = fma2(st1, gg, s32[h]);
      }
      const float z0 = MODE == 0 ? u[4] + xj * wb[4] : fmaf(xj, wb[4], u[4]);
      const float z1 = z0 + dd[4];
      const float gg = ok ? ri[4] + v.q4 : 0.f;
      const float m1 = z1 > 0.f ? gg : 0.f, m0 = z0 > 0.f ? gg : 0.f;
      const float dm = m1 - m0;
      cst += dm;
      s1t = fmaf(xj, dm, s1t);
      s3t += m1;
    };
    // (one neighbour's loads then its use: 74 VGPRs, 6 waves per SIMD -- batching the row
    // loads of 4 / 8 / 16 neighbours ahead of their use measured 35.8 / 36.2 / 44.0 us
    // against 32.8 at stress, the walk wanting waves more than loads in flight)
    for_list(prep, 0, b, i, Ne, Nc, [&](int j0) { use(j0, ldr(j0)); }, hw, HALVES);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      cs[2 * h] = cs2[h].x; cs[2 * h + 1] = cs2[h].y;
      S1[2 * h] = s12[h].x; S1[2 * h + 1] = s12[h].y;
      S3[2 * h] = s32[h].x; S3[2 * h + 1] = s32[h].y;
    }
    cs[4] = cst; S1[4] = s1t; S3[4] = s3t;
  }
  WSTAMP(13, 3);
  if constexpr (HALVES == 2) {
    float* hd = hand + g * 3 * KPW * TN + lane;   // hw 1's sums, added in a fixed order
    if (hw) {
#pragma unroll
      for (int kk = 0; kk < KPW; ++kk) {
        hd[kk * TN] = cs[kk];
        hd[(KPW + kk) * TN] = S1[kk];
        hd[(2 * KPW + kk) * TN] = S3[kk];
      }
    }
    __syncthreads();
    WSTAMP(13, 4);
    if (hw) return;                               // no barriers below
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      cs[kk] += hd[kk * TN];
      S1[kk] += hd[(KPW + kk) * TN];
      S3[kk] += hd[(2 * KPW + kk) * TN];
    }
  }
  float v[4 * KPW];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const float s2 = live ? S2[kk] + cs[kk] : 0.f;
    v[kk] = live ? xi * s2 : 0.f;                  // S0 = sum_i x_i (row sum of dz)
    v[KPW + kk] = live ? S1[kk] : 0.f;
    v[2 * KPW + kk] = s2;
    v[3 * KPW + kk] = live ? S3[kk] : 0.f;
  }
  const int row = b * te + tx;
#pragma unroll
  for (int q = 0; q < 4 * KPW; ++q) v[q] = wsum(v[q]);
  if (lane == 0) {
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int k = g * KPW + kk;
      const float s0 = v[kk], s1 = v[KPW + kk], s2 = v[2 * KPW + kk], s3 = v[3 * KPW + kk];
      if constexpr (MODE == 0) {
        const Seg& s = sg.s[SG_E1W1];
        put(part, s, k, row, s0);
        put(part, s, H + k, row, s1);
        put(part, s, 2 * H + k, row, s2 - s3);
        put(part, s, 3 * H + k, row, s3);
        put(part, s, 4 * H + k, row, s2);
      } else {   // the shared w1_1 sees both slices: sum dz (x_i + x_j)
        const Seg& s = sg.s[SG_EEW11];
        put(part, s, k, row, s0 + s1);
        put(part, s, H + k, row, s2 - s3);
        put(part, s, 2 * H + k, row, s3);
        put(part, s, 3 * H + k, row, s2);
      }
    }
  }
}

// grid (te, B, stages): stage mode0 + z -- 0: E1 (ra = rb = rho_E), 1: EE (phi, psi); both
// stages of model_4's general path in one launch.  HALVES = 2 (512 threads: the neighbour
// lists split over two wave halves) while the grid fits 3 blocks per CU; HALVES = 1 (256
// threads, whole lists) beyond, where the 512-thread grid ran a second round of one block
// per CU (model_4 stress: 1,024 blocks)
template <int HALVES>
__global__ __launch_bounds__(256 * HALVES) void kw_first_bwd(const float* __restrict__ x,
                                                   const uint32_t* __restrict__ abits,
                                                   const uint32_t* __restrict__ prep,
                                                   const float* __restrict__ W, Off o, int Ne,
                                                   int Nc, int mode0, const float* __restrict__ r0,
                                                   const float* __restrict__ phi,
                                                   const float* __restrict__ psi,
                                                   const double* __restrict__ tab,
                                                   float* __restrict__ part, Segs sg) {
  __shared__ float hand[HALVES == 2 ? NW * 3 * KPW * TN : 1];   // hw 1's walk sums [g][3 KPW][lane]
  int tx, b, zz;                                   // commit b's tiles on XCD b % 8, as kw_scan's
  xcd_commit_map(tx, b, zz);                       // blocks that wrote its tables
  if (mode0 + zz == 0)
    first_bwd_body<0, HALVES>(x, abits, prep, W, o, Ne, Nc, r0, r0, tab, part, sg, hand, tx, b);
  else
    first_bwd_body<1, HALVES>(x, abits, prep, W, o, Ne, Nc, phi, psi, tab, part, sg, hand, tx, b);
}

// ---------------------------------------------------------------------------------
// kw_ee_clsb  grid (ceil(Ne/32), B), 4 waves: entity-edge classifier backward (model_4.py:286-304)
//   dz1 = p0 p1 (dp1 - dp0) = -dz0, dp_r[m] = dn[hid i'(r)][2+m] + dn[hid j'(r)][2+m]
//   (relation r -> index pair (i', j') on the n-grid, the stride quirk of utils2.py:121-137);
//   the two-class softmax as a sigmoid of the logit difference: with
//   c = U2'[:,1] - U2'[:,0], delta = (b2'[1] - b2'[0]) + sum_k relu(kappa_k) c_k,
//   e = exp(-delta) = 2^delta' (delta' from the prescaled D_EECQ / D_EEBQ), p1 = 1 / (1 + e),
//   p0 p1 = e p1^2;  g_k = [kappa_k > 0] c_k dz1 = c_k s_k: the pair loop sums
//   s_k = [kappa_k > 0] dz1 and c scales the sums once.
//   Lane = column j, the waves share the rows i (rho rows staged in LDS, broadcast reads; the
//   lane's gam row from LDS too, conflict-free [v][lane] 16-byte reads).  Per row the 64
//   lanes' s-vectors are summed across the wave: this tile's partial row of drho / c
//   (kw_ee_nodeb sums the te partials in tile order and scales by c);
//   per lane over the rows: dgam_j.  The weight constants are wave-uniform scalar loads
//   (no LDS traffic, no VGPRs).  dynamic LDS: Eq[Ne] = dn[hid q][3] - dn[hid q][2].
// ---------------------------------------------------------------------------------
// q = r / d, rem = r % d for 0 <= r < 2^24, 1 <= d < 2^12: float estimate, one select
// correction each way (the estimate is within one of q), no branches
__device__ __forceinline__ void divmod_sel(int r, int d, float inv, int& q, int& rem) {
  const int q0 = (int)((float)r * inv);
  const int r0 = r - q0 * d;
  const bool lo = r0 < 0, hi = r0 >= d;
  q = lo ? q0 - 1 : (hi ? q0 + 1 : q0);
  rem = lo ? r0 + d : (hi ? r0 - d : r0);
}

constexpr int TB = 32;   // kw_ee_clsb: columns per block (a wave's two halves take two rows)
__host__ __device__ inline int ee_bwd_tiles(int Ne) { return (Ne + TB - 1) / TB; }

// The same pair loop with two columns per lane (c and c + 16 of the tile): a wave's four
// 16-lane quarters take four rows at once, the lane adds its two columns' s-vectors
// before the row sums, and the row sums close over 16 lanes (quarter_sums20): one
// transposed butterfly per two pairs instead of one 32-lane butterfly per pair.
__device__ __forceinline__ void ee_clsb_rows_q(
    const int lo, const int hi, const int c0, const float* os_, const uint32_t* abl,
    const int Ne, const int t0, const int nrel, const int dn1, const float inv,
    const bool aligned, const float* Eq, const float4* gl, const float4* gdl,
    const float* __restrict__ D, float* rowp, f2 (&acc0)[H2], f2 (&acc1)[H2], f2 (&ag)[H2],
    float& sdl, float (&zr)[2], int (&kst)[2]) {
  const int lane = threadIdx.x & 63, qr = lane >> 4, cq = lane & 15;
  const float bq = D[D_EEBQ];
  // the classifier's prescaled weight differences read once (uniform: SGPRs); read in the
  // trip they were refetched every trip (the rowp stores may alias D for the compiler),
  // and the scalar wait drained the trip's LDS reads with them
  f2 cqs[H2];
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) cqs[kk] = ld2(D + D_EECQ + 2 * kk);
  const int trips = (hi - lo + 3) >> 2;
  const int jn0 = t0 + cq, jn1 = t0 + cq + 16;
  const bool live0 = jn0 < Ne, live1 = jn1 < Ne;
  const float Ej0 = Eq[live0 ? jn0 : Ne - 1], Ej1 = Eq[live1 ? jn1 : Ne - 1];
  int wi = -1;
  uint32_t word0 = 0, word1 = 0;
  for (int it = 0; it < trips; ++it) {
    trip_prio_e(it, trips);
    const int mr = lo + 4 * it + qr;             // the quarter's row
    const bool inr = mr < hi;
    const int m = inr ? mr : lo;                 // past the share: a staged row, d1 = 0
    if ((m >> 5) != wi) {
      wi = m >> 5;
      word0 = abl[wi * TB + cq];
      word1 = abl[wi * TB + cq + 16];
    }
    const float* orow = os_ + (m - c0) * H;
    const float4* o4 = reinterpret_cast<const float4*>(orow);
    float sv[H];
    auto column = [&](const int jn, const bool live, const float Ej, const uint32_t word,
                      const int cc, f2 (&acc)[H2], const bool first) {
      const bool a1 = (word >> (m & 31)) & 1u;
      const float af = a1 ? 1.f : 0.f;
      const f2 a2 = {af, af};
      const int r = m * (Ne - 1) + jn - (jn > m ? 1 : 0);
      const bool valid = live && inr && m != jn && r < nrel;
      float dp;
      if (aligned) {                   // n = Ne: (i', j') = (i, j)   (block-uniform branch)
        dp = Eq[m] + Ej;
      } else {
        int ip, jj;
        divmod_sel(r < nrel ? r : 0, dn1, inv, ip, jj);
        dp = Eq[ip] + Eq[jj + (jj >= ip ? 1 : 0)];
      }
      const float4* g4 = (a1 ? gdl : gl) + cc;   // gam_j + a d: the LDS table by address
      f2 pre[H2], st[H2];
#pragma unroll
      for (int v = 0; v < H / 4; ++v) {   // kappa = rho_i + (gam_j + a d), as kw_ee_fwd
        const float4 q = o4[v], g = g4[v * TB];
        pre[2 * v] = (f2){q.x, q.y} + (f2){g.x, g.y};
        pre[2 * v + 1] = (f2){q.z, q.w} + (f2){g.z, g.w};
      }
      f2 dz = {bq, 0.f}, dzb = {0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < H2; ++kk) {  // relu(kappa) = kappa [kappa > 0]
        st[kk] = step2(pre[kk]);
        if (kk & 1)
          dzb = fma2(pre[kk] * st[kk], cqs[kk], dzb);
        else
          dz = fma2(pre[kk] * st[kk], cqs[kk], dz);
      }
      dz += dzb;
      const float e = __builtin_amdgcn_exp2f(fminf(dz.x + dz.y, 64.f));
      const float p1 = __builtin_amdgcn_rcpf(1.f + e);
      const float d1 = valid ? (e * p1) * (p1 * dp) : 0.f;
      const f2 d2 = {d1, d1};
      sdl += d1;
#pragma unroll
      for (int kk = 0; kk < H2; ++kk) {
        const f2 sd = st[kk] * d2;
        acc[kk] += sd;
        ag[kk] = fma2(a2, sd, ag[kk]);
        if (first) {
          sv[2 * kk] = sd.x;
          sv[2 * kk + 1] = sd.y;
        } else {
          sv[2 * kk] += sd.x;
          sv[2 * kk + 1] += sd.y;
        }
      }
    };
    column(jn0, live0, Ej0, word0, cq, acc0, true);
    column(jn1, live1, Ej1, word1, cq + 16, acc1, false);
    // the quarter's row sums over the tile's 32 columns (drho partial, without c), and the
    // classifier's rho part of sum_j relu(kappa) dz1 = rho_i . (row sum), as ee_clsb_rows
    quarter_sums20(sv, lane, [&](int slot, int k, float x) {
      if (inr) rowp[(size_t)m * H + k] = x;
      zr[slot] = fmaf(orow[k], x, zr[slot]);
      kst[slot] = k;
    });
  }
}

// sum over the four 16-lane quarters of a wave (lanes l, l^16, l^32, l^48); every lane
// receives the total of its column lane
__device__ __forceinline__ float quarters_sum(float v) {
  float x = v, y = v;
  swap32(x, y);
  v = x + y;
  x = v;
  y = v;
  swap16(x, y);
  return x + y;
}

// Dispatch order.  A block's work is its commit's relation rows, rows_b = ceil(n_b (n_b - 1)
// / (Ne - 1)), which varies 4x over the glide commits (n 100..200); the blocks of one launch
// are all resident (3 per CU), so the kernel ends with the CU that drew the most rows (wave
// times: median 24.8 us, max 36.7 us, in blockIdx order).  With `snake` = the CU count, block
// i takes the segment (commit, tile) of rank s in the order of decreasing rows, s snaking
// over the dispatch rounds of `snake` blocks (round r = i / snake: even rounds in order, odd
// rounds reversed), so that a CU's first block (one of the heaviest) pairs with a light
// second block.  Every (commit, tile) still runs in one block, so the sums are the same bits
// in any order.  snake = 0: blockIdx order.
__device__ __forceinline__ int ee_rows(int n, int Ne) {
  n = n < 0 ? 0 : (n > Ne ? Ne : n);
  if (n < 2) return 0;
  const int r = (n * (n - 1) + Ne - 2) / (Ne - 1);
  return r < Ne ? r : Ne;
}

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3))) void kw_ee_clsb(
    const uint32_t* __restrict__ aT, const int32_t* __restrict__ hidg,
    const int32_t* __restrict__ nleng, const float* __restrict__ D, int Ne, int Nc, int snake,
    const uint32_t* __restrict__ order,
    const float* __restrict__ rho, const float* __restrict__ gmm, const float* __restrict__ dn,
    float* __restrict__ drho, float* __restrict__ dgam, float* __restrict__ part, Segs sg) {
#pragma clang fp contract(off)
  extern __shared__ float dyn[];                  // Eq[Ne] | a^T words [WE][TB]
  __shared__ __attribute__((aligned(16))) float os_[CHM * H];
  __shared__ float buf[NW * TB * HP];
  __shared__ float res[TB * HP];
  __shared__ float red[NW * 21];
  __shared__ float tot[21];
  __shared__ float cl[H];
  __shared__ float zred[NW * 4 * H];
  __shared__ float4 gl4[(H / 4) * TB];            // the columns' gam rows, [v][column]
  __shared__ float4 gdl4[(H / 4) * TB];           // gam + d
  const int te = gridDim.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int WE = (Ne + 31) >> 5;
  int b = blockIdx.y, tile = blockIdx.x;
  WSTAMP(14, 0);
  if (snake > 0) {                                 // (b, tile) by the dispatch order (above)
    const int B = gridDim.y, total = te * B, i = blockIdx.y * te + blockIdx.x;
    const int r = i / snake, q = i - r * snake;
    const int len = total - r * snake < snake ? total - r * snake : snake;
    const int s = r * snake + ((r & 1) ? len - 1 - q : q);
    const int cr = s / te;                         // commit rank, by decreasing rows
    tile = s - cr * te;
    const int ob = (int)order[cr];                 // (kw_prep_order)
    b = ob >= 0 && ob < B ? ob : 0;
  }
  const int t0 = tile * TB;
  int n = nleng[b];
  n = n < 0 ? 0 : (n > Ne ? Ne : n);
  const int nrel = n >= 2 ? n * (n - 1) : 0;
  const int dn1 = n - 1 > 0 ? n - 1 : 1;
  float* Eq = dyn;
  uint32_t* abl = reinterpret_cast<uint32_t*>(dyn + Ne);
  for (int e = t; e < Ne; e += NT) {
    const int h = hidg[(size_t)b * Ne + e];
    const float* d = dn + ((size_t)b * Nc + (h >= 0 && h < Nc ? h : 0)) * 4;
    Eq[e] = (h >= 0 && h < Nc) ? d[3] - d[2] : 0.f;
  }
  for (int e = t; e < WE * TB; e += NT) {        // a^T rows of the tile's columns: bit m = a[m][j]
    const int w = e / TB, l = e - w * TB, node = t0 + l < Ne ? t0 + l : Ne - 1;
    abl[e] = aT[((size_t)b * Ne + node) * WE + w];
  }
  if (t < H) cl[t] = D[D_EEC + t];
  for (int e = t; e < (H / 4) * TB; e += NT) {   // [v][column]: conflict-free 16-B reads
    const int v = e / TB, l = e - v * TB, node = t0 + l < Ne ? t0 + l : Ne - 1;
    const float4 g = reinterpret_cast<const float4*>(gmm + ((size_t)b * Ne + node) * H)[v];
    const float4 d = reinterpret_cast<const float4*>(D + D_EED)[v];
    gl4[e] = g;
    gdl4[e] = make_float4(g.x + d.x, g.y + d.y, g.z + d.z, g.w + d.w);
  }
  f2 acc0[H2], acc1[H2], ag[H2];        // columns c and c + 16 of the lane; a = 1 sums
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    acc0[kk] = (f2){0.f, 0.f};
    acc1[kk] = acc0[kk];
    ag[kk] = acc0[kk];
  }
  float sdl = 0.f, zr[2] = {0.f, 0.f};
  int kst[2] = {-1, -1};
  // rows holding relations r < nrel
  const int rows = nrel > 0 ? ((nrel + Ne - 2) / (Ne - 1) < Ne ? (nrel + Ne - 2) / (Ne - 1) : Ne) : 0;
  // this tile's partial rows; the rows past the relations are not written (kw_ee_nodeb reads
  // them as 0)
  float* rowp = drho + ((size_t)(b * te + tile) * Ne) * H;
  const float* rb = rho + (size_t)b * Ne * H;
  const float inv = 1.f / (float)dn1;
  const bool aligned = n == Ne;
  __syncthreads();                                 // Eq, abl, cl, gl4, gdl4
  WSTAMP(14, 1);
  for (int c0 = 0; c0 < rows; c0 += CHM) {
    const int c1 = c0 + CHM < rows ? c0 + CHM : rows;
    __syncthreads();
    stage_rows(os_, rb, c0, c1);
    __syncthreads();
    const int lo = c0 + ((c1 - c0) * uni(wv)) / NW, hi = c0 + ((c1 - c0) * (uni(wv) + 1)) / NW;
    ee_clsb_rows_q(lo, hi, c0, os_, abl, Ne, t0, nrel, dn1, inv, aligned, Eq, gl4, gdl4, D,
                   rowp, acc0, acc1, ag, sdl, zr, kst);
  }
  prio0_e();
  WSTAMP(14, 2);
  for (int e = lane; e < 4 * H; e += 64) zred[wv * 4 * H + e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 2; ++s)                      // one storing lane per (quarter, unit)
    if (kst[s] >= 0) zred[(wv * 4 + (lane >> 4)) * H + kst[s]] = zr[s];
  // column sums over the quarters (in registers), then the waves (fixed order) -> res
  {
    const int cq = lane & 15;
#pragma unroll
    for (int kk = 0; kk < H2; ++kk) {
      const float x0 = quarters_sum(acc0[kk].x), y0 = quarters_sum(acc0[kk].y);
      const float x1 = quarters_sum(acc1[kk].x), y1 = quarters_sum(acc1[kk].y);
      if (lane < 16) {
        buf[(wv * TB + cq) * HP + 2 * kk] = x0;
        buf[(wv * TB + cq) * HP + 2 * kk + 1] = y0;
      } else if (lane < 32) {
        buf[(wv * TB + 16 + cq) * HP + 2 * kk] = x1;
        buf[(wv * TB + 16 + cq) * HP + 2 * kk + 1] = y1;
      }
    }
  }
  __syncthreads();
  for (int e = t; e < TB * H; e += NT) {
    const int nn = e / H, k = e - nn * H;
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) sum += buf[(q * TB + nn) * HP + k];   // wave q's column sums
    res[nn * HP + k] = sum;
  }
  __syncthreads();
  float* dout = dgam + (size_t)b * Ne * H;
  for (int e = t; e < TB * H; e += NT) {
    const int nn = e / H, k = e - nn * H;
    if (t0 + nn < Ne) dout[(size_t)(t0 + nn) * H + k] = res[nn * HP + k] * cl[k];
  }
  float v[21];                                     // classifier partial rows
#pragma unroll
  for (int kk = 0; kk < H2; ++kk) {
    v[2 * kk] = ag[kk].x;
    v[2 * kk + 1] = ag[kk].y;
  }
  v[20] = sdl;
  block_sum<21>(v, red, tot);
  const int row = b * te + tile;
  if (t < H) {
    // sum_pairs relu(kappa_k) dz1 = sum_i rho_ik R_ik + sum_j gam_jk C_jk + d_k sum_{a=1} s_k dz1
    // (kappa = rho + gam + a d; R, C the row / column sums of s dz1)
    float sc = 0.f, zg = 0.f;
    const float* glf = reinterpret_cast<const float*>(gl4);
    for (int nn = 0; nn < TB; ++nn) {
      if (t0 + nn >= Ne) break;
      const float cs = res[nn * HP + t];
      sc += cs;
      zg = fmaf(glf[((t >> 2) * TB + nn) * 4 + (t & 3)], cs, zg);
    }
    float zw = 0.f;
    for (int q = 0; q < 4 * NW; ++q) zw += zred[q * H + t];
    const float zk = (zw + zg) + D[D_EED + t] * tot[t];
    const float sg_ = sc * cl[t];                    // sum of g over the tile
    const float a1 = tot[t] * cl[t];
    const Seg& sa = sg.s[SG_ECW1A];
    const Seg& sb = sg.s[SG_ECB1];
    put(part, sa, t, row, sg_ - a1);                 // P1[0] ([a = 0] input)
    put(part, sa, H + t, row, a1);                   // P1[1] ([a = 1] input)
    put(part, sb, t, row, sg_);                      // p1 bias
    put(part, sb, H + 2 * t, row, -zk);              // U2'[k][0]
    put(part, sb, H + 2 * t + 1, row, zk);           // U2'[k][1]
  }
  if (t == 0) {
    const Seg& sb = sg.s[SG_ECB1];
    put(part, sb, 3 * H, row, -tot[20]);
    put(part, sb, 3 * H + 1, row, tot[20]);
  }
  WSTAMP(14, 3);
}

// ---------------------------------------------------------------------------------
// kw_ee_nodeb  grid (te, B): dR = U1e' drho, dC = U1e' dgam;  phi = Q2 dR, psi = Q2 dC
// (model_4.py:232-243 backward); partial rows of dU1e' (classifier rows 2..21),
// dQ2 = sum R1 (x) dR + C1 (x) dC, dq2 = (Ne-1) sum (dR + dC)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void kw_ee_nodeb(
    const float* __restrict__ W, Off o, const float* __restrict__ D, int Ne, int np,
    const int32_t* __restrict__ nleng,
    const float* __restrict__ R1,
    const float* __restrict__ C1, const float* __restrict__ Rn, const float* __restrict__ Cn,
    const float* __restrict__ drho, const float* __restrict__ dgam, float* __restrict__ phi,
    float* __restrict__ psi, float* __restrict__ part, Segs sg) {
  __shared__ float A[TN * HP], Bq[TN * HP], R1t[TN * HP], C1t[TN * HP], Rt[TN * HP],
      Ct[TN * HP], dR[TN * HP], dC[TN * HP];
  // the weights' rows at pitch WPN = 50 words (= 18 mod 32): the 16 rows x 2 k-offsets a
  // ds_read_b32 group of the MFMA B operand reads fall on 32 distinct banks (pitch 20 put
  // rows m and m + 8 on one bank)
  constexpr int WPN = 50;
  __shared__ float Wl[2 * H * WPN];
  __shared__ float kz[1];                         // 0.f: stride-0 operand of padding tiles
  const float *U1e = Wl, *Q2 = Wl + H * WPN;      // classifier rows 2..21 | EE second layer
  if (threadIdx.x == 0) kz[0] = 0.f;
  // XCD-grouped rows: the partial-gradient stores below are 4-byte values at a stride of
  // the te*B rows, so a 64-byte line holds 16 neighbouring rows' values; dealing the rows
  // to the 8 XCDs in contiguous ranges (block L runs on XCD L % 8) lets each line's
  // partial writes merge in one L2 instead of reaching HBM from several
  const int te = gridDim.x, nrow = te * gridDim.y, lin = blockIdx.y * te + blockIdx.x;
  const int nx = nrow & ~7;
  const int lrow = lin < nx ? (lin & 7) * (nx >> 3) + (lin >> 3) : lin;
  const int b = lrow / te, tile = lrow - b * te;
  const int t0 = tile * TN, t = threadIdx.x;
  const size_t base = ((size_t)b * Ne + t0) * H;
  WSTAMP(6, 0);
  for (int e = threadIdx.x; e < H * H; e += NT) {
    const int r = e / H, c = e - r * H;
    Wl[r * WPN + c] = W[o.EC_W1 + 2 * H + e];
    Wl[H * WPN + r * WPN + c] = W[o.EE_W2 + e];
  }
  // staging: every element's loads issued before the first use (NE_IT elements per thread;
  // the np row partials of drho (kw_ee_clsb's column tiles) eight at a time, in tile order)
  constexpr int NE_IT = TN * H / NT;
  static_assert(TN * H % NT == 0, "kw_ee_nodeb staging");
  float dr[NE_IT];
#pragma unroll
  for (int it = 0; it < NE_IT; ++it) {
    const int e = t + it * NT, n = e / H, k = e - n * H;
    const bool in = t0 + n < Ne;
    dr[it] = 0.f;
    Bq[n * HP + k] = in ? dgam[base + e] : 0.f;
    R1t[n * HP + k] = in ? R1[base + e] : 0.f;
    C1t[n * HP + k] = in ? C1[base + e] : 0.f;
    Rt[n * HP + k] = in ? Rn[base + e] : 0.f;
    Ct[n * HP + k] = in ? Cn[base + e] : 0.f;
  }
  {
    const float* src = drho + ((size_t)b * np * Ne + t0) * H + t;
    const size_t sq = (size_t)Ne * H;
    // elements e < nin are in range and hold relations (kw_ee_clsb writes no row past the
    // commit's relation rows: they are 0)
    const int rl = ee_rows(nleng[b], Ne) < Ne ? ee_rows(nleng[b], Ne) : Ne;
    const int nin = rl > t0 ? (rl - t0) * H : 0;
    for (int q = 0; q < np; q += 8) {                 // 8 tiles' loads in flight, summed in order
      float v[NE_IT][8];
#pragma unroll
      for (int it = 0; it < NE_IT; ++it)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[it][u] = (q + u < np && t + it * NT < nin) ? src[(q + u) * sq + it * NT] : 0.f;
#pragma unroll
      for (int it = 0; it < NE_IT; ++it)
#pragma unroll
        for (int u = 0; u < 8; ++u) dr[it] += v[it][u];
    }
  }
  WSTAMP(6, 1);
#pragma unroll
  for (int it = 0; it < NE_IT; ++it) {
    const int e = t + it * NT, n = e / H, k = e - n * H;
    A[n * HP + k] = dr[it] * D[D_EEC + k];   // kw_ee_clsb's row partials leave c out
  }
  __syncthreads();
  WSTAMP(6, 2);
  const int lane = t & 63;
  // dR = A U1e^T, dC = Bq U1e^T, then phi = dR Q2^T, psi = dC Q2^T over the tile's 64
  // nodes as 16x16 MFMA tiles (4 node tiles x 2 column tiles per product, K = 20); columns
  // >= H read the zero word kz with stride 0 and are not stored
  for (int tile = t >> 6; tile < 16; tile += NT / 64) {     // wave-uniform
    const int which = tile >> 3, n0 = ((tile >> 1) & 3) * 16, m0 = (tile & 1) * 16;
    const int mc = m0 + (lane & 15);
    const bool cv = mc < H;
    const f4v c = mfma_tile16_p((which ? Bq : A) + (n0 + (lane & 15)) * HP, 1,
                                cv ? U1e + mc * WPN : kz, cv ? 1 : 0, H, lane);
    if (cv) {
      float* d = which ? dC : dR;
#pragma unroll
      for (int j = 0; j < 4; ++j) d[(n0 + 4 * (lane >> 4) + j) * HP + mc] = c[j];
    }
  }
  __syncthreads();
  for (int tile = t >> 6; tile < 16; tile += NT / 64) {
    const int which = tile >> 3, n0 = ((tile >> 1) & 3) * 16, l0 = (tile & 1) * 16;
    const int lc = l0 + (lane & 15);
    const bool cv = lc < H;
    const f4v c = mfma_tile16_p((which ? dC : dR) + (n0 + (lane & 15)) * HP, 1,
                                cv ? Q2 + lc * WPN : kz, cv ? 1 : 0, H, lane);
    if (cv) {
      float* d = which ? psi : phi;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 4 * (lane >> 4) + j;
        if (t0 + n < Ne) d[base + n * H + lc] = c[j];
      }
    }
  }
  WSTAMP(6, 3);
  const int row = lrow;
  const Seg& s1 = sg.s[SG_ECW1E];
  const Seg& s2 = sg.s[SG_EEW2];
  const float Ne1 = (float)(Ne - 1);
  // dU1e' = Rt^T A + Ct^T Bq and dQ2 = R1t^T dR + C1t^T dC over the tile's 64 nodes as
  // 16x16 MFMA tiles (2 x 2 per matrix, one wave per two tiles); dq2 on the VALU
  for (int tile = t >> 6; tile < 8; tile += NT / 64) {      // wave-uniform
    const int which = tile >> 2, row0 = ((tile >> 1) & 1) * 16, col0 = (tile & 1) * 16;
    const int ra = row0 + (lane & 15), cb = col0 + (lane & 15);
    const bool rv = ra < H, cv = cb < H;
    const float* a0 = which ? R1t : Rt;                     // [n][row]
    const float* b0 = which ? dR : A;                       // [n][col]
    const float* a1 = which ? C1t : Ct;
    const float* b1 = which ? dC : Bq;
    const f4v c = mfma_tile16_p(rv ? a0 + ra : kz, rv ? HP : 0, cv ? b0 + cb : kz, cv ? HP : 0,
                                TN, lane) +
                  mfma_tile16_p(rv ? a1 + ra : kz, rv ? HP : 0, cv ? b1 + cb : kz, cv ? HP : 0,
                                TN, lane);
    if (cv) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rr = row0 + 4 * (lane >> 4) + j;
        if (rr < H) put(part, which ? s2 : s1, rr * H + cb, row, c[j]);
      }
    }
  }
  if (t < H) {
    float a = 0.f;
    for (int n = 0; n < TN; ++n) a += dR[n * HP + t] + dC[n * HP + t];
    put(part, s2, 400 + t, row, a * Ne1);
  }
  WSTAMP(6, 4);
}

// ---------------------------------------------------------------------------------
// kw_grad_reduce  grid (count): one wave per parameter p = p_begin + blockIdx.x; lanes
// stride over the partial rows of p's segment in a fixed order, xor-butterfly total.
// Parameters without a segment get 0 (data-independent: map_theta*, model_3's unused
// entity-edge blocks; the trailer's fault slot: no exchanges on this path).  The correct-
// prediction count (trailer slot HDG_TR_COUNT, exact integers per row) is summed as an
// integer and written as the trailer's three 16-bit parts by that slot's wave.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void kw_grad_reduce(const float* __restrict__ part, Segs sg,
                                                     int p_begin, int np,
                                                     float* __restrict__ out) {
  const int p = p_begin + blockIdx.x, lane = threadIdx.x;
  const int pc = np + HDG_TR_COUNT;
  if (p > pc && p <= pc + 2) return;              // written by the count slot's wave
  float a = 0.f;
  unsigned long long c = 0ull;
  for (int s = 0; s < sg.count; ++s) {
    const Seg& g = sg.s[s];
    if (g.n > 0 && p >= g.p0 && p < g.p0 + g.n) {
      const float* src = part + g.off + (long long)(p - g.p0) * g.rows;
      constexpr int RU = 8;                      // rows in flight per lane (same sum order)
      for (int r0 = lane; r0 < g.rows; r0 += 64 * RU) {
        float v[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) v[u] = r0 + 64 * u < g.rows ? src[r0 + 64 * u] : 0.f;
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          if (r0 + 64 * u < g.rows) {
            if (p == pc) c += (unsigned long long)v[u];
            else a += v[u];
          }
        }
      }
      break;
    }
  }
  if (p == pc) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
    if (lane == 0) {
      float* o = out + blockIdx.x;
      o[0] = (float)(c & 0xFFFFull);
      o[1] = (float)((c >> 16) & 0xFFFFull);
      o[2] = (float)(c >> 32);
    }
    return;
  }
  a = wsum(a);
  if (lane == 0) out[blockIdx.x] = a;
}

// kw_reduce_adam  (grid below): kw_grad_reduce fused with
// k_adam_tf for a single-process training step (hdg_train_step on the general path and on
// the model_4 fused path).  Slots in [seg_lo, seg_hi) are reduced from the partial rows as
// in kw_grad_reduce; the others (model_4 on the fused path) from the step kernel's
// per-block rows fp (frows rows of fstride floats, model_2 layout: slot p of the model_4
// vector is p2 = p, or p - f_shift from f_at on), as k_grad_reduce does.  Then TF1
// ApplyAdam for a parameter slot, with the loss terms and the Adam factor kw_derive put in
// D_AUX from the pre-update parameters, so no block depends on another; the CE slot's wave
// writes the loss stats, block 0 the new beta powers.  A fault in the step kernel's rows
// (a block-pair exchange timed out) skips every update, as in k_adam_tf.

// one slot's reduced value: the gradient out (the count slot as three 16-bit parts), the
// stats on the CE slot, and TF1 ApplyAdam on a parameter slot
__device__ __forceinline__ void reduce_adam_slot(int p, int np, float g, unsigned long long c,
                                                 float w, float m0, float v0, bool fault,
                                                 float* __restrict__ grad,
                                                 float* __restrict__ params,
                                                 float* __restrict__ mm, float* __restrict__ vv,
                                                 float* __restrict__ bpow,
                                                 const float* __restrict__ D, float lr,
                                                 float inv_pairs, float* __restrict__ stats) {
  if (p == np + HDG_TR_COUNT) {
    grad[p] = (float)(c & 0xFFFFull);
    grad[p + 1] = (float)((c >> 16) & 0xFFFFull);
    grad[p + 2] = (float)(c >> 32);
    if (stats) {                                   // stats[4..6]: the count's parts
      stats[4] = grad[p];
      stats[5] = grad[p + 1];
      stats[6] = grad[p + 2];
    }
    return;
  }
  grad[p] = g;
  if (p == np + HDG_TR_FAULT && stats) stats[7] = g;
  if (p == np + HDG_TR_CE && stats) {
    const float ce = g * inv_pairs;
    stats[0] = ce;
    stats[1] = D[D_AUX + 1];
    stats[2] = D[D_AUX + 0];
    stats[3] = 10.f * ce + 0.1f * D[D_AUX + 1] + D[D_AUX + 0];
  }
  if (p >= np || fault) return;
  const float b1 = 0.9f, b2 = 0.999f, ep = 1e-8f;
  const int TH1 = np - 4, TH2 = np - 2;
  float gg = g + 0.001f * w;
  if (p >= TH1 && p < TH1 + 2) gg += 0.001f * w / D[D_AUX + 2];
  if (p >= TH2 && p < TH2 + 2) gg += 0.001f * w / D[D_AUX + 3];
  float m = m0, v = v0;
  m += (gg - m) * (1.f - b1);
  v += (gg * gg - v) * (1.f - b2);
  mm[p] = m;
  vv[p] = v;
  params[p] = w - (lr * D[D_AUX + 4]) * m / (sqrtf(v) + ep);
  if (p == 0) {
    bpow[0] = D[D_AUX + 5];
    bpow[1] = D[D_AUX + 6];
  }
}

// grid (nfb + nsb), 256 threads.  Blocks [0, nfb): 16 consecutive slots of the step
// kernel's rows (fr, model_2 layout p2, mapped to the model_4 slot p) x 16 row phases, so
// each row's 16 slots are one 64-byte read; blocks [nfb, nfb + nsb): one wave per slot of
// [seg_lo, seg_hi) over its segment rows (contiguous per slot).
__global__ __launch_bounds__(NT) void kw_reduce_adam(
    const float* __restrict__ part, Segs sg, int np, int seg_lo, int seg_hi, int nfb,
    FusedRows fr, float* __restrict__ grad, float* __restrict__ params, float* __restrict__ mm,
    float* __restrict__ vv, float* __restrict__ bpow, const float* __restrict__ D, float lr,
    float inv_pairs, float* __restrict__ stats) {
  __shared__ float rs[16][17];
  __shared__ unsigned long long rc[16];
  const int t = threadIdx.x, lane = t & 63;
  const int pc = np + HDG_TR_COUNT;
  // Every load of the block (the fault slots, the Adam operands, the rows) is issued before
  // the first one is used, and the fault flag is OR-ed at the block's one barrier: the
  // kernel is one memory round trip deep.  Sums keep their fixed row order.
  bool bad = false;   // the step kernel's fault slot: any block-pair exchange timed out
  if (fr.ffault)
    for (int r = t; r < fr.frows; r += NT) bad |= fr.ffault[r] != 0.f;
  if ((int)blockIdx.x < nfb) {
    const int sl = t & 15, ph = t >> 4;
    const int p2 = blockIdx.x * 16 + sl;
    const int GL = fr.f_np + HDG_TRAILER;
    const int p = p2 < fr.f_at ? p2 : p2 + fr.f_shift;
    const bool ok = p2 < GL;
    const bool isc = p == pc;
    const bool isp = ok && ph == 0 && p < np;
    const float w = isp ? params[p] : 0.f, m0 = isp ? mm[p] : 0.f, v0 = isp ? vv[p] : 0.f;
    float a = 0.f;
    unsigned long long c = 0ull;
    constexpr int RU = 16;                       // rows of a phase in flight at once
    if (ok)
      for (int r0 = ph; r0 < fr.frows; r0 += 16 * RU) {
        float v[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int r = r0 + 16 * u;
          v[u] = r < fr.frows ? fr.fp[(size_t)r * fr.fstride + p2] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          if (r0 + 16 * u < fr.frows) {
            if (isc) c += (unsigned long long)v[u];
            else a += v[u];
          }
        }
      }
    rs[ph][sl] = a;
    if (isc) rc[ph] = c;
    const bool fault = __syncthreads_or(bad);
    if (ph == 0 && ok && !(p > pc && p <= pc + 2)) {   // count parts: the count slot's thread
      float g = 0.f;
      unsigned long long cc = 0ull;
#pragma unroll
      for (int q = 0; q < 16; ++q) g += rs[q][sl];     // fixed order
      if (isc)
        for (int q = 0; q < 16; ++q) cc += rc[q];
      reduce_adam_slot(p, np, g, cc, w, m0, v0, fault, grad, params, mm, vv, bpow, D, lr,
                       inv_pairs, stats);
    }
    return;
  }
  const int wv = t >> 6;
  const int p = seg_lo + ((int)blockIdx.x - nfb) * NW + wv;
  const bool live = p < seg_hi && !(p > pc && p <= pc + 2);   // count parts: the count slot's wave
  const bool isp = live && lane == 0 && p < np;
  const float w = isp ? params[p] : 0.f, m0 = isp ? mm[p] : 0.f, v0 = isp ? vv[p] : 0.f;
  float a = 0.f;
  unsigned long long c = 0ull;
  if (live)
    for (int q = 0; q < sg.count; ++q) {
      const Seg& sgq = sg.s[q];
      if (sgq.n > 0 && p >= sgq.p0 && p < sgq.p0 + sgq.n) {
        const float* src = part + sgq.off + (long long)(p - sgq.p0) * sgq.rows;
        constexpr int RU = 8;
        for (int r0 = lane; r0 < sgq.rows; r0 += 64 * RU) {
          float v[RU];
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            const int r = r0 + 64 * u;
            v[u] = r < sgq.rows ? src[r] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            if (r0 + 64 * u < sgq.rows) {
              if (p == pc) c += (unsigned long long)v[u];
              else a += v[u];
            }
          }
        }
        break;
      }
    }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  const float g = wsum(a);
  const bool fault = __syncthreads_or(bad);
  if (live && lane == 0)
    reduce_adam_slot(p, np, g, c, w, m0, v0, fault, grad, params, mm, vv, bpow, D, lr, inv_pairs,
                     stats);
}

// kw_prep_sort  grid (B), 1024 threads, dynamic LDS 2 Ne floats: stable rank sort of x,
// distinct values, counts below each distinct value and f64 prefix sums (any Ne)
__global__ __launch_bounds__(1024) void kw_prep_sort(const float* __restrict__ x,
                                                     uint32_t* __restrict__ prep, int Ne, int Nc) {
  extern __shared__ float xl[];
  float* xs = xl + Ne;
  const GenPrep GP = gen_prep(Ne, Nc);
  const int b = blockIdx.x, t = threadIdx.x;
  uint32_t* pb = prep + (size_t)b * GP.words;
  float* xsrt = reinterpret_cast<float*>(pb + GP.xsrt);
  int* perm = reinterpret_cast<int*>(pb + GP.perm);
  for (int i = t; i < Ne; i += 1024) xl[i] = x[(size_t)b * Ne + i];
  __syncthreads();
  for (int i = t; i < Ne; i += 1024) {
    const float xi = xl[i];
    int r = 0;
    for (int j = 0; j < Ne; ++j) {
      const float xj = xl[j];
      r += (xj < xi || (xj == xi && j < i)) ? 1 : 0;
    }
    xs[r] = xi;
    xsrt[r] = xi;
    perm[r] = i;
  }
  __syncthreads();
  if (t == 0) {   // serial over the sorted values, once per uploaded batch
    float* xu = reinterpret_cast<float*>(pb + GP.xu);
    int* cum = reinterpret_cast<int*>(pb + GP.cum);
    double* pxd = reinterpret_cast<double*>(pb + GP.pxd);
    int nd = 0;
    double acc = 0.0;
    for (int m = 0; m < Ne; ++m) {
      const float v = xs[m];
      if (m == 0 || v != xs[m - 1]) {
        xu[nd] = v;
        cum[nd] = m;
        pxd[nd] = acc;
        ++nd;
      }
      acc += (double)v;
    }
    cum[nd] = Ne;
    pxd[nd] = acc;
    pb[GP.meta] = (uint32_t)nd;
  }
}

// transposed class bits: out[b][j][w] bit l = in[b][32w + l][j]
__global__ __launch_bounds__(NT) void kw_prep_T(const uint32_t* __restrict__ in,
                                                uint32_t* __restrict__ out, int N) {
  const int b = blockIdx.y, W_ = (N + 31) >> 5;
  const uint32_t* ib = in + (size_t)b * N * W_;
  for (int e = blockIdx.x * NT + threadIdx.x; e < N * W_; e += gridDim.x * NT) {
    const int j = e / W_, w = e - j * W_;
    uint32_t bits = 0;
    for (int l = 0; l < 32; ++l) {
      const int i = 32 * w + l;
      if (i < N && i != j) bits |= ((ib[(size_t)i * W_ + (j >> 5)] >> (j & 31)) & 1u) << l;
    }
    out[(size_t)b * N * W_ + e] = bits;
  }
}

// kw_prep_lists  grid (ceil(Ne/4), B, 2), one wave per node and side: the set bits j != i of
// the node's a row (side 0) / aT row (side 1) as ascending u16 ids (list_layout); the wave
// scans the words' popcounts for each lane's write offset, then pads to 4 with Ne
// (the same kernel builds the hunk label lists: n = Nc, bits = ybits / yT, L = ylist_layout)
__global__ __launch_bounds__(NT) void kw_prep_lists(const uint32_t* __restrict__ abits,
                                                    const uint32_t* __restrict__ aT,
                                                    uint32_t* __restrict__ prep, int Ne,
                                                    ListLayout L) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * NW + (threadIdx.x >> 6);
  const int b = blockIdx.y, side = blockIdx.z, B = gridDim.y;
  if (i >= Ne) return;
  const int WE = (Ne + 31) >> 5, LS = list_stride(Ne);
  const size_t r = ((size_t)side * B + b) * Ne + i;
  const uint32_t* row = (side ? aT : abits) + ((size_t)b * Ne + i) * WE;
  uint16_t* out = reinterpret_cast<uint16_t*>(prep + L.ids) + r * LS;
  int base = 0;
  for (int w0 = 0; w0 < WE; w0 += 64) {
    const int w = w0 + lane;
    uint32_t m = w < WE ? row[w] : 0u;
    if (w == (i >> 5)) m &= ~(1u << (i & 31));
    const int pc = __builtin_popcount(m);
    int incl = pc;
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    int pos = base + incl - pc;
    while (m) {
      out[pos++] = (uint16_t)(32 * w + __builtin_ctz(m));
      m &= m - 1u;
    }
    base += __shfl(incl, 63);
  }
  for (int e = base + lane; e < ((base + 3) & ~3); e += 64) out[e] = (uint16_t)Ne;
  if (lane == 0) prep[L.cnt + r] = (uint32_t)base;
}

// ---------------------------------------------------------------------------------
// kw_prep_order  grid (1), 1024 threads, dynamic LDS te B ints: the entity-edge kernels'
// dispatch orders (ranks by decreasing work, ties by index; the layout note above):
// kw_ee_clsb's commits by relation rows, kw_ee_fwd's (commit, tile) pairs by their walk
// length (n for a tile holding index rows, T * TF < n; 0 for the others)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void rank_desc(const int* key, int N, uint32_t* __restrict__ out) {
  for (int e = threadIdx.x; e < N; e += blockDim.x) {
    const int re = key[e];
    int rank = 0;
    for (int f = 0; f < N; ++f) {
      const int rf = key[f];
      rank += (rf > re || (rf == re && f < e)) ? 1 : 0;
    }
    out[rank] = (uint32_t)e;
  }
}
__global__ __launch_bounds__(1024) void kw_prep_order(const int32_t* __restrict__ nleng, int B,
                                                      int Ne, uint32_t* __restrict__ order) {
  extern __shared__ int rk[];
  const int te = ee_fwd_tiles(Ne), N = te * B;
  for (int e = threadIdx.x; e < B; e += blockDim.x) rk[e] = ee_rows(nleng[e], Ne);
  __syncthreads();
  rank_desc(rk, B, order);
  __syncthreads();
  for (int e = threadIdx.x; e < N; e += blockDim.x) {
    const int b = e / te, T = e - b * te;
    int n = nleng[b];
    n = n < 0 ? 0 : (n > Ne ? Ne : n);
    rk[e] = (n >= 2 && T * TF < n) ? n : 0;
  }
  __syncthreads();
  rank_desc(rk, N, order + ((B + 3) & ~3));
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
bool has_ee(int v);
bool hunk_lists(const hdg_shape* s);
bool has_ent(int v);
// the prep words before the entity-edge order table (= the whole prep without model_4)
size_t ee_order_off(const hdg_shape* s) {
  const size_t B = s->batch, WE = (s->ne + 31) / 32, WC = (s->nc + 31) / 32;
  if (hunk_lists(s)) return ylist_layout(s->batch, s->ne, s->nc, has_ent(s->variant)).end;
  if (has_ent(s->variant)) return list_layout(s->batch, s->ne, s->nc).end;
  return B * gen_prep(s->ne, s->nc).words + B * s->ne * WE + B * s->nc * WC;
}
struct WideWork {
  size_t xp, ov, P, Eb, hE, rhoE;                 // entity stage   [B][Ne](*H)
  size_t R1, C1, Rn, Cn, rho, gmm, drho, dgam, phi, psi;   // EE     [B][Ne][H]
  size_t ncpart;                                  // u64 [B][tef][Nc][2] EE partial bins
  size_t nvec, alpha, beta, G, Hh, sig, tau, Dsig, Dtau, dG, dH, Dal, Dbe, dn;   // hunk
  size_t gam;                                     // [B][Nc][Nc]
  size_t D;                                       // derived weights
  size_t tab;                                     // f64 scan tables [2][B][H][2][Ne+1]
  size_t hsv, hsp, hsx, hsw;                      // sorted hunk tables (hunk_sorted)
  size_t htr, htc, hty;                           // one-sweep tile partials (hunk_tiled)
  size_t part;                                    // partial rows
  Segs segs;
  size_t total;
};

// the sorted-threshold form of the hunk relu / mask sums (kw_hunk_sort, _fwd_s, _wsum,
// _mlpb_s) instead of the dense sweeps (kw_hunk_fwd, kw_hunk_mlpb)
// automatic form by Nc (flags force one): tiled from HDG_HUNK_TILED_MIN_NC, sorted from
// HDG_HUNK_SORTED_MIN_NC below that, the dense two-pass sweep otherwise
bool hunk_tiled(const hdg_shape* s) {
  if (s->flags & (HDG_FLAG_HUNK_DENSE | HDG_FLAG_HUNK_SORTED)) return false;
  if (s->flags & HDG_FLAG_HUNK_TILED) return true;
  return s->nc >= HDG_HUNK_TILED_MIN_NC;
}
bool hunk_sorted(const hdg_shape* s) {
  if (s->flags & (HDG_FLAG_HUNK_DENSE | HDG_FLAG_HUNK_TILED)) return false;
  if (s->flags & HDG_FLAG_HUNK_SORTED) return true;
  return s->nc >= HDG_HUNK_SORTED_MIN_NC && !hunk_tiled(s);
}

// the hunk label id lists (the sorted passes' walks) are part of every general-path
// batch, whatever the flags: a batch's prep layout depends on its shape's path only
bool hunk_lists(const hdg_shape* s) { return hdg_resolve_path(s) == HDG_PATH_GENERAL; }

bool has_ent(int v) { return v == 2 || v == 4; }
bool has_ee(int v) { return v == 4; }

WideWork wide_layout(const hdg_shape* s) {
  WideWork w;
  memset(&w, 0, sizeof(w));
  const size_t B = s->batch, Ne = s->ne, Nc = s->nc;
  const int v = s->variant;
  const Off o = param_offsets(v);
  size_t off = 0;
  auto take = [&](size_t n) { const size_t r = off; off += (n + 63) & ~(size_t)63; return r; };
  const size_t NEH = B * Ne * H, NCH = B * Nc * H;
  if (has_ent(v)) {
    w.xp = take(B * Ne); w.ov = take(B * Ne);
    w.P = take(NEH); w.Eb = take(NEH); w.hE = take(NEH); w.rhoE = take(NEH);
  }
  if (has_ee(v)) {
    w.R1 = take(NEH); w.C1 = take(NEH); w.Rn = take(NEH); w.Cn = take(NEH);
    w.rho = take(NEH); w.gmm = take(NEH); w.dgam = take(NEH);
    w.drho = take(NEH * (size_t)ee_bwd_tiles((int)Ne));    // one partial per kw_ee_clsb tile
    w.phi = take(NEH); w.psi = take(NEH);
    w.ncpart = take(B * ee_fwd_tiles((int)Ne) * Nc * 4);
  }
  w.nvec = take(B * Nc * 4);
  w.alpha = take(NCH); w.beta = take(NCH); w.G = take(NCH); w.Hh = take(NCH);
  w.sig = take(NCH); w.tau = take(NCH); w.Dsig = take(NCH); w.Dtau = take(NCH);
  w.dG = take(NCH); w.dH = take(NCH); w.Dal = take(NCH); w.Dbe = take(NCH);
  w.dn = take(B * Nc * 4);
  w.gam = take(B * Nc * Nc);
  w.D = take(D_WORDS);
  if (has_ent(v) || has_ee(v)) w.tab = take(2 * 2 * B * H * 2 * (Ne + 1));   // doubles
  if (hunk_tiled(s)) {
    const size_t CC = (Nc + hunk_tile_cols() - 1) / hunk_tile_cols();
    const size_t RC = (Nc + hunk_tile_rows() - 1) / hunk_tile_rows();
    w.htr = take(B * CC * Nc * H);
    w.htc = take(B * RC * Nc * H);
    w.hty = take(B * RC * CC * H);
  }
  if (hunk_sorted(s)) {
    const size_t NcP = (Nc + 3) & ~(size_t)3;
    w.hsv = take(B * 2 * H * NcP);
    w.hsp = take(B * 2 * H * NcP);
    w.hsx = take(2 * B * 2 * H * (NcP + 1));                    // doubles
    w.hsw = take(2 * B * 2 * H * (NcP + 1));
  }
  const int te = (int)((Ne + TN - 1) / TN), tc = (int)((Nc + TN - 1) / TN);
  const int rc = (int)B * tc, re = (int)B * te;
  auto seg = [&](int id, int p0, int n, int rows) {
    w.segs.s[id].p0 = p0;
    w.segs.s[id].n = n;
    w.segs.s[id].rows = rows;
    w.segs.s[id].off = (long long)take((size_t)n * rows);
  };
  seg(SG_CLS, o.H2_W2, 42, CLS_SPLIT * rc);
  seg(SG_CE, o.NP, 2, CLS_SPLIT * rc);
  seg(SG_CLSB_H2, o.H2_W1, 460, 2 * rc);
  seg(SG_CLSB_H1, o.H1_W2, 420, 2 * rc);
  seg(SG_MLPB, o.H1_W1, 220, 2 * rc);
  if (has_ent(v)) {
    seg(SG_E3, o.E3_W1, 461, re);
    seg(SG_E1W5, o.E1_W5, 420, re);
    seg(SG_E1W1, o.E1_W1, 100, re);
  }
  if (has_ee(v)) {
    const int rb = (int)B * ee_bwd_tiles((int)Ne);      // kw_ee_clsb blocks
    seg(SG_ECW1A, o.EC_W1, 40, rb);
    seg(SG_ECB1, o.EC_B1, 62, rb);
    seg(SG_ECW1E, o.EC_W1 + 40, 400, re);
    seg(SG_EEW2, o.EE_W2, 420, re);
    seg(SG_EEW11, o.EE_W11, 80, re);
  }
  w.segs.count = SG_COUNT;
  w.part = 0;   // segment offsets are absolute (floats from the workspace base)
  w.total = off;
  return w;
}

#define WTRY(expr)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail((int)e_, "%s: %s", #expr, hipGetErrorString(e_));   \
  } while (0)

// kw_first_bwd's form by its grid: the 512-thread blocks (3 per CU at 76 VGPRs) while they
// fit one round, the 256-thread blocks (whole lists per wave) beyond
#ifndef HDG_FB_HALVES
#define HDG_FB_HALVES 0   // 0: by the grid; 1 / 2: forced
#endif
int first_bwd_halves(long long blocks) {
  if (HDG_FB_HALVES) return HDG_FB_HALVES;
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
              ? n : 256;
  }
  return blocks > 3LL * cus ? 1 : 2;
}

// kw_ent_fwd's form by its grid: 8 waves per block (2 blocks per CU at 126 VGPRs) while the
// tile blocks fit one round, 4 waves beyond
#ifndef HDG_EF_HALVES
#define HDG_EF_HALVES 0   // 0: by the grid; 1 / 2: forced
#endif
int ent_fwd_halves(long long blocks) {
  if (HDG_EF_HALVES) return HDG_EF_HALVES;
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
              ? n : 256;
  }
  return blocks <= 2LL * cus ? 2 : 1;
}

int set_wide_attrs() {
  static bool attr_set = false;   // > 64 KiB of dynamic LDS for Ne > 4000
  if (!attr_set) {
    WTRY(hipFuncSetAttribute((const void*)kw_ent_fwd<1>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_ent_fwd<2>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_first_bwd<2>,    // + 15 KiB static hand-over
                             hipFuncAttributeMaxDynamicSharedMemorySize, 112 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_first_bwd<1>,    // + 15 KiB static hand-over
                             hipFuncAttributeMaxDynamicSharedMemorySize, 112 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_ee_fwd<1, NWP>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_ee_fwd<2, HDG_EEF_WAVES>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_ee_fwd<0, HDG_EEF_WAVES>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_ee_clsb,      // 41 KiB static + 32 KiB at Ne 4096
                             hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    WTRY(hipFuncSetAttribute((const void*)kw_hunk_fwd_s,
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hs_lds_bytes(HS_ALL_MAX, 1)));
    WTRY(hipFuncSetAttribute((const void*)kw_hunk_mlpb_s,
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hs_lds_bytes(HS_ALL_MAX, 2)));
    WTRY(hipFuncSetAttribute((const void*)kw_hunk_fwd_g,
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hs_lds_bytes(HS_NC_MAX, 1)));
    WTRY(hipFuncSetAttribute((const void*)kw_hunk_mlpb_g,
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)hs_lds_bytes(HS_NC_MAX, 2)));
    attr_set = true;
  }
  return 0;
}

// the entity-edge kernels' dispatch order: snaking over rounds of one block per CU (the note
// above kw_ee_clsb), the ranks from the batch's prep (kw_prep_order); 0: blockIdx order
#ifndef HDG_EE_SNAKE
#define HDG_EE_SNAKE 1
#endif
int ee_snake(const hdg_shape* s) {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
              ? n : 0;
  }
  return (HDG_EE_SNAKE && (long long)ee_fwd_tiles(s->ne) * s->batch <= EE_ORDER_MAX) ? cus : 0;
}
size_t ee_clsb_lds(int Ne) { return (size_t)(Ne + TB * ((Ne + 31) / 32)) * 4; }   // Eq | a^T words

// kw_ee_fwd over the batch: both LDS tables up to EE_TAB_LDS_MAX nodes, the gam table alone
// while it fits the LDS, HBM reads beyond
int ee_snake(const hdg_shape* s);
size_t ee_order_off(const hdg_shape* s);
int launch_ee_fwd(const hdg_shape* s, const hdg_batch* bt, const float* params, const float* D,
                  const float* rho, const float* gmm, unsigned long long* ncpart, hipStream_t st) {
  const int B = s->batch, Ne = s->ne, Nc = s->nc;
  const Off o = param_offsets(s->variant);
  const dim3 grid(ee_fwd_tiles(Ne), B);
  const int tm = ee_fwd_mode(Ne, Nc);
  const int snake = ee_snake(s);
  const uint32_t* sorder = (const uint32_t*)bt->prep + ee_order_off(s) + ((B + 3) & ~3);
  if (tm == 1)
    hipLaunchKernelGGL((kw_ee_fwd<1, NWP>), grid, dim3(NTP), ee_fwd_lds(Ne, Nc), st, bt->abits,
                       bt->hid, bt->nlen, params, o, D, Ne, Nc, rho, gmm, ncpart, snake, sorder);
  else if (tm == 2)
    hipLaunchKernelGGL((kw_ee_fwd<2, HDG_EEF_WAVES>), grid, dim3(64 * HDG_EEF_WAVES),
                       ee_fwd_lds(Ne, Nc), st, bt->abits, bt->hid, bt->nlen, params, o, D, Ne,
                       Nc, rho, gmm, ncpart, snake, sorder);
  else
    hipLaunchKernelGGL((kw_ee_fwd<0, HDG_EEF_WAVES>), grid, dim3(64 * HDG_EEF_WAVES),
                       ee_fwd_lds(Ne, Nc), st, bt->abits, bt->hid, bt->nlen, params, o, D, Ne,
                       Nc, rho, gmm, ncpart, snake, sorder);
  WTRY(kmark("kw_ee_fwd", st));
  return 0;
}

}  // namespace

size_t wide_workspace_bytes(const hdg_shape* s) { return wide_layout(s).total * sizeof(float); }

// ---- model_4 on the fused path (hdgnn.hip): the entity-edge stage on this path's kernels
// around the fused step kernel, which runs the model_2-shaped rest of the step ----------
float* wide_dn(const hdg_shape* s, void* workspace) {
  return (float*)workspace + wide_layout(s).dn;
}

const unsigned long long* wide_ncpart(const hdg_shape* s, void* workspace) {
  return (const unsigned long long*)((float*)workspace + wide_layout(s).ncpart);
}
int wide_ncpart_tiles(const hdg_shape* s) { return ee_fwd_tiles(s->ne); }

int wide_ee_fwd(const hdg_shape* s, const hdg_batch* bt, const float* params, void* workspace,
                hipStream_t st, const float* bpow) {
  const int B = s->batch, Ne = s->ne, Nc = s->nc;
  const Off o = param_offsets(s->variant);
  const WideWork w = wide_layout(s);
  float* ws = (float*)workspace;
  auto F = [&](size_t off) { return ws + off; };
  const uint32_t* prep = (const uint32_t*)bt->prep;
  const uint32_t* aT = prep + (size_t)B * gen_prep(Ne, Nc).words;
  const int te = (Ne + TN - 1) / TN;
  if (int rc = set_wide_attrs()) return rc;
  const NodeFwdOut no{F(w.Eb), F(w.hE), F(w.ov), F(w.xp), F(w.Rn), F(w.Cn), F(w.rho), F(w.gmm)};
  if (ent_fwd_halves((long long)te * B) == 2)
    hipLaunchKernelGGL(kw_ent_fwd<2>, dim3(te + 1, B, 1), dim3(NTP), sort_lds_bytes(Ne), st,
                       bt->x, bt->abits, aT, prep, params, o, Ne, Nc, 0, F(w.P), F(w.R1),
                       F(w.C1), ws + w.D, bpow, no);
  else
    hipLaunchKernelGGL(kw_ent_fwd<1>, dim3(te + 1, B, 1), dim3(NT), sort_lds_bytes(Ne), st,
                       bt->x, bt->abits, aT, prep, params, o, Ne, Nc, 0, F(w.P), F(w.R1),
                       F(w.C1), ws + w.D, bpow, no);
  WTRY(kmark("kw_ent_fwd", st));
  unsigned long long* ncpart = (unsigned long long*)F(w.ncpart);
  return launch_ee_fwd(s, bt, params, ws + w.D, F(w.rho), F(w.gmm), ncpart, st);
}

int wide_ee_bwd(const hdg_shape* s, const hdg_batch* bt, const float* params, void* workspace,
                float* grad, hipStream_t st, const WideAdam* adam) {
  const int B = s->batch, Ne = s->ne, Nc = s->nc;
  const Off o = param_offsets(s->variant);
  const WideWork w = wide_layout(s);
  float* ws = (float*)workspace;
  auto F = [&](size_t off) { return ws + off; };
  const uint32_t* prep = (const uint32_t*)bt->prep;
  const uint32_t* aT = prep + (size_t)B * gen_prep(Ne, Nc).words;
  const int te = (Ne + TN - 1) / TN;
  float* part = ws;
  if (int rc = set_wide_attrs()) return rc;
  const int snake = ee_snake(s);
  hipLaunchKernelGGL(kw_ee_clsb, dim3(ee_bwd_tiles(Ne), B, 1), dim3(NT), ee_clsb_lds(Ne), st, aT,
                     bt->hid, bt->nlen, ws + w.D, Ne, Nc, snake, prep + ee_order_off(s), F(w.rho),
                     F(w.gmm), F(w.dn), F(w.drho), F(w.dgam), part, w.segs);
  WTRY(kmark("kw_ee_clsb", st));
  hipLaunchKernelGGL(kw_ee_nodeb, dim3(te, B), dim3(NT), 0, st, params, o, ws + w.D, Ne,
                     ee_bwd_tiles(Ne), bt->nlen, F(w.R1), F(w.C1), F(w.Rn), F(w.Cn), F(w.drho),
                     F(w.dgam), F(w.phi), F(w.psi), part, w.segs);
  WTRY(kmark("kw_ee_nodeb", st));
  hipLaunchKernelGGL(kw_scan, dim3(H, B, 1), dim3(NT), 0, st, prep, params, o, Ne, Nc, 1,
                     nullptr, F(w.psi), (double*)F(w.tab));
  WTRY(kmark("kw_scan", st));
  if (first_bwd_halves(te * B) == 2)
    hipLaunchKernelGGL(kw_first_bwd<2>, dim3(te, B), dim3(NTP), sort_lds_bytes(Ne), st, bt->x,
                       bt->abits, prep, params, o, Ne, Nc, 1, nullptr, F(w.phi), F(w.psi),
                       (const double*)F(w.tab), part, w.segs);
  else
    hipLaunchKernelGGL(kw_first_bwd<1>, dim3(te, B), dim3(NT), sort_lds_bytes(Ne), st, bt->x,
                       bt->abits, prep, params, o, Ne, Nc, 1, nullptr, F(w.phi), F(w.psi),
                       (const double*)F(w.tab), part, w.segs);
  WTRY(kmark("kw_first_bwd", st));
  // the entity-edge parameters [EE_W11, EC_B2 + 2): one contiguous block of the flat vector
  const int p0 = o.EE_W11, n = o.EC_B2 + 2 - o.EE_W11;
  if (adam) {
    hdg_state* S = adam->state;
    const FusedRows& fr = adam->fused;   // the step kernel's rows: every other slot
    const int nfb = (fr.f_np + HDG_TRAILER + 15) / 16, nsb = (n + NW - 1) / NW;
    hipLaunchKernelGGL(kw_reduce_adam, dim3(nfb + nsb), dim3(NT), 0, st, part, w.segs, o.NP,
                       p0, p0 + n, nfb, fr, grad, S->params, S->adam_m, S->adam_v, S->beta_pow,
                       ws + w.D, adam->lr, adam->inv_pairs, adam->stats);
  } else {
    hipLaunchKernelGGL(kw_grad_reduce, dim3(n), dim3(64), 0, st, part, w.segs, p0, o.NP,
                       grad + p0);
  }
  WTRY(kmark(adam ? "kw_reduce_adam" : "kw_grad_reduce", st));
  return 0;
}

void wide_prep_counts_layout(const hdg_shape* s, int64_t* stride, int64_t* ks, int64_t* kt,
                             int64_t* ncst) {
  const GenPrep GP = gen_prep(s->ne, s->nc);
  *stride = GP.words;
  *ks = GP.ks;
  *kt = GP.kt;
  *ncst = GP.ncst;
}

size_t wide_prep_bytes(const hdg_shape* s) {
  const size_t words = ee_order_off(s);
  const size_t ord = (((size_t)s->batch + 3) & ~(size_t)3) + (size_t)ee_fwd_tiles(s->ne) * s->batch;
  return (has_ee(s->variant) ? words + ord : words) * 4;
}

int wide_prepare(const hdg_shape* s, const hdg_batch* bt, hipStream_t st) {
  const GenPrep GP = gen_prep(s->ne, s->nc);
  WTRY(launch_prep_maps(s, bt, GP.words, GP.ks, GP.kt, GP.ncst, st));
  hipLaunchKernelGGL(kw_prep_sort, dim3(s->batch), dim3(1024), (size_t)2 * s->ne * 4, st, bt->x,
                     (uint32_t*)bt->prep, s->ne, s->nc);
  WTRY(kmark("kw_prep_sort", st));
  uint32_t* aT = (uint32_t*)bt->prep + (size_t)s->batch * GP.words;
  uint32_t* yT = aT + (size_t)s->batch * s->ne * ((s->ne + 31) / 32);
  hipLaunchKernelGGL(kw_prep_T, dim3(8, s->batch), dim3(NT), 0, st, bt->abits, aT, s->ne);
  WTRY(kmark("kw_prep_T", st));
  hipLaunchKernelGGL(kw_prep_T, dim3(4, s->batch), dim3(NT), 0, st, bt->ybits, yT, s->nc);
  WTRY(kmark("kw_prep_T", st));
  if (has_ent(s->variant)) {   // the entity walks' neighbour lists
    hipLaunchKernelGGL(kw_prep_lists, dim3((s->ne + NW - 1) / NW, s->batch, 2), dim3(NT), 0, st,
                       bt->abits, aT, (uint32_t*)bt->prep, s->ne,
                       list_layout(s->batch, s->ne, s->nc));
    WTRY(kmark("kw_prep_lists", st));
  }
  if (hunk_lists(s)) {         // the sorted hunk passes' label lists
    hipLaunchKernelGGL(kw_prep_lists, dim3((s->nc + NW - 1) / NW, s->batch, 2), dim3(NT), 0, st,
                       bt->ybits, yT, (uint32_t*)bt->prep, s->nc,
                       ylist_layout(s->batch, s->ne, s->nc, has_ent(s->variant)));
    WTRY(kmark("kw_prep_lists", st));
  }
  if (has_ee(s->variant) && ee_snake(s) > 0) {   // the entity-edge kernels' dispatch orders
    hipLaunchKernelGGL(kw_prep_order, dim3(1), dim3(1024),
                       (size_t)ee_fwd_tiles(s->ne) * s->batch * 4, st, bt->nlen, s->batch, s->ne,
                       (uint32_t*)bt->prep + ee_order_off(s));
    WTRY(kmark("kw_prep_order", st));
  }
  return 0;
}

// ---------------------------------------------------------------------------------
// kw_ehr  grid (1): loss_E_HR = 0.001 * l2_loss(C_edge_output) (model_2.py:122), the
// graph's unfetched regulariser of the hunk-pair effects (mlp_hunk_B2's output,
// model_2.py:245-277): C_edge_output[b][k][pq] = S_pk + T_qk with S = G V2 + (Nc-1) c2 and
// T = H V2 + (Nc-1) c2 (the second layer commutes with the row / column sums).
// Per commit and unit k, over the pairs p != q:
//   sum (S_p + T_q)^2 = (Nc-1)(sum S^2 + sum T^2) + 2 (sum S sum T - sum_p S_p T_p)
// so five additive per-unit sums suffice.  Thread (k = t % 20, slice t / 20) walks its
// nodes; f64 sums closed in a fixed order (deterministic).  G, H: [Nc][20] per commit at
// stride `cs` floats (the rows of kw_hunk_fwd, or those the fused step kernel parks).
// Forward-only diagnostic: one block, never on the training path.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void kw_ehr(const float* __restrict__ G,
                                               const float* __restrict__ Hh, size_t cs, int B,
                                               int Nc, const float* __restrict__ W, int oV2,
                                               int oc2, float* __restrict__ out) {
  constexpr int NSL = 1024 / H;                      // 51 node slices
  __shared__ double red[NSL][5][H];
  __shared__ double tot[H];
  const int t = threadIdx.x, k = t % H, sl = t / H;
  float v2[H];
#pragma unroll
  for (int l = 0; l < H; ++l) v2[l] = W[oV2 + l * H + k];
  const float off = (float)(Nc - 1) * W[oc2 + k];
  if (t < H) tot[t] = 0.0;
  for (int b = 0; b < B; ++b) {
    double sS = 0.0, sT = 0.0, sS2 = 0.0, sT2 = 0.0, sST = 0.0;
    if (sl < NSL) {
      for (int p = sl; p < Nc; p += NSL) {
        const float* g = G + (size_t)b * cs + (size_t)p * H;
        const float* h = Hh + (size_t)b * cs + (size_t)p * H;
        float S = 0.f, T = 0.f;
#pragma unroll
        for (int l = 0; l < H; ++l) {
          S = fmaf(g[l], v2[l], S);
          T = fmaf(h[l], v2[l], T);
        }
        const double Sd = (double)(S + off), Td = (double)(T + off);
        sS += Sd;
        sT += Td;
        sS2 += Sd * Sd;
        sT2 += Td * Td;
        sST += Sd * Td;
      }
      red[sl][0][k] = sS;
      red[sl][1][k] = sT;
      red[sl][2][k] = sS2;
      red[sl][3][k] = sT2;
      red[sl][4][k] = sST;
    }
    __syncthreads();
    if (t < H) {
      double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      for (int q = 0; q < NSL; ++q)
        for (int c = 0; c < 5; ++c) a[c] += red[q][c][t];
      tot[t] += (double)(Nc - 1) * (a[2] + a[3]) + 2.0 * (a[0] * a[1] - a[4]);
    }
    __syncthreads();
  }
  if (t == 0) {
    double s = 0.0;
    for (int q = 0; q < H; ++q) s += tot[q];
    out[0] = (float)(0.0005 * s);                    // 0.001 * l2_loss = 0.001 * sum / 2
  }
}

hipError_t launch_ehr(const float* G, const float* Hh, size_t cs, int B, int Nc,
                      const float* params, int variant, float* out, hipStream_t st) {
  const Off o = param_offsets(variant);
  hipLaunchKernelGGL(kw_ehr, dim3(1), dim3(1024), 0, st, G, Hh, cs, B, Nc, params, o.H1_W2,
                     o.H1_B2, out);
  return hipGetLastError();
}

int wide_run(const hdg_shape* s, const hdg_batch* bt, const float* params, float* grad,
             hdg_outputs* out, float* ce_sum, void* workspace, bool train, hipStream_t st,
             const WideAdam* adam) {
  const int B = s->batch, Ne = s->ne, Nc = s->nc, v = s->variant;
  const Off o = param_offsets(v);
  const WideWork w = wide_layout(s);
  float* ws = (float*)workspace;
  const uint32_t* prep = (const uint32_t*)bt->prep;
  const uint32_t* aT = prep + (size_t)B * gen_prep(Ne, Nc).words;
  const uint32_t* yT = aT + (size_t)B * Ne * ((Ne + 31) / 32);
  const int te = (Ne + TN - 1) / TN, tc = (Nc + TN - 1) / TN;
  const bool ent = has_ent(v), ee = has_ee(v);
  const int bg = s->batch_global > 0 ? s->batch_global : B;
  const float ce_scale = 10.f / ((float)bg * (float)(Nc * (Nc - 1)));
  float* D = ws + w.D;
  float* part = ws;   // segment offsets are absolute
  auto F = [&](size_t off) { return ws + off; };

  const size_t tlds = sort_lds_bytes(Ne);
  if (int rc = set_wide_attrs()) return rc;
  const float* bpow = train && adam ? adam->state->beta_pow : nullptr;
  if (!(ent || ee)) {
    hipLaunchKernelGGL(kw_derive, dim3(1), dim3(NT), 0, st, params, o, Nc, D, bpow);
    WTRY(kmark("kw_derive", st));
  }
  // ---- entity side ----
  if (ent || ee) {   // + kw_derive's work in one more block column, node_fwd_tile per tile
    const NodeFwdOut no{F(w.Eb), F(w.hE), F(w.ov), F(w.xp), F(w.Rn), F(w.Cn), F(w.rho),
                        F(w.gmm)};
    const int ez = (ent && ee) ? 2 : 1;
    if (ent_fwd_halves((long long)te * B * ez) == 2)
      hipLaunchKernelGGL(kw_ent_fwd<2>, dim3(te + 1, B, ez), dim3(NTP), tlds, st, bt->x,
                         bt->abits, aT, prep, params, o, Ne, Nc, ent ? 1 : 0, F(w.P), F(w.R1),
                         F(w.C1), D, bpow, no);
    else
      hipLaunchKernelGGL(kw_ent_fwd<1>, dim3(te + 1, B, ez), dim3(NT), tlds, st, bt->x,
                         bt->abits, aT, prep, params, o, Ne, Nc, ent ? 1 : 0, F(w.P), F(w.R1),
                         F(w.C1), D, bpow, no);
    WTRY(kmark("kw_ent_fwd", st));
  }
  unsigned long long* ncpart = ee ? (unsigned long long*)F(w.ncpart) : nullptr;
  if (ee) {
    if (int rc = launch_ee_fwd(s, bt, params, D, F(w.rho), F(w.gmm), ncpart, st)) return rc;
  }
  // ---- hunk side ----
  hipLaunchKernelGGL(kw_cross_fwd, dim3((Nc + NW - 1) / NW, B), dim3(NT), 0, st, prep,
                     ent ? F(w.xp) : bt->x, params, o, Ne, Nc, ncpart, ee_fwd_tiles(Ne), F(w.nvec), F(w.alpha),
                     F(w.beta));
  WTRY(kmark("kw_cross_fwd", st));
  const bool hs = hunk_sorted(s), ht = hunk_tiled(s);
  const ListLayout YL = ylist_layout(B, Ne, Nc, ent);
  const HTileSums hts{F(w.htr), F(w.htc), F(w.hty), (Nc + hunk_tile_cols() - 1) / hunk_tile_cols(),
                      (Nc + hunk_tile_rows() - 1) / hunk_tile_rows()};
  if (hs) {
    const dim3 gw(H, B, 2);
#define HDG_SORT(E_)                                                                            \
  hipLaunchKernelGGL(kw_hunk_sort<E_>, gw, dim3(NT), 0, st, F(w.alpha), F(w.beta), Nc, F(w.hsv), \
                     (int*)F(w.hsp), (double*)F(w.hsx))
    switch (hsort_e(Nc)) {
      case 1: HDG_SORT(1); break;
      case 2: HDG_SORT(2); break;
      case 4: HDG_SORT(4); break;
      default: HDG_SORT(8); break;
    }
#undef HDG_SORT
    WTRY(kmark("kw_hunk_sort", st));
    if (hs_all_shape(s)) {
      hipLaunchKernelGGL(kw_hunk_fwd_s, dim3((Nc + HSN - 1) / HSN, B, 2), dim3(HS_NT),
                         hs_shape_lds_bytes(s, 1), st, bt->ybits, yT, D, Nc, F(w.alpha), F(w.beta),
                         F(w.hsv), (const double*)F(w.hsx), prep, YL, F(w.G), F(w.Hh),
                         F(w.sig), F(w.tau));
      WTRY(kmark("kw_hunk_fwd_s", st));
    } else {
      hipLaunchKernelGGL(kw_hunk_fwd_g, dim3(4 * hs_tiles(Nc), B, 2), dim3(NT),
                         hs_shape_lds_bytes(s, 1), st, bt->ybits, yT, D, Nc, F(w.alpha), F(w.beta),
                         F(w.hsv), (const double*)F(w.hsx), prep, YL, F(w.G), F(w.Hh));
      WTRY(kmark("kw_hunk_fwd_g", st));
      hipLaunchKernelGGL(kw_hunk_sig, dim3(tc, B, 2), dim3(NT), 0, st, D, Nc, F(w.G), F(w.Hh),
                         F(w.sig), F(w.tau));
      WTRY(kmark("kw_hunk_sig", st));
    }
  } else if (ht) {
    HTileArgs ha{Nc, F(w.alpha), F(w.beta), nullptr, nullptr, nullptr, D + D_DLT, bt->ybits,
                 F(w.htr), F(w.htc), F(w.hty)};
    WTRY(launch_hunk_tile(0, ha, B, st));
    hipLaunchKernelGGL(kw_hunk_fin0, dim3(tc, B, 2), dim3(NTP), 0, st, hts, D, Nc, F(w.alpha),
                       F(w.beta), F(w.G), F(w.Hh), F(w.sig), F(w.tau));
    WTRY(kmark("kw_hunk_fin0", st));
  } else {
    hipLaunchKernelGGL(kw_hunk_fwd, dim3(tc, B, 2), dim3(NTP), 0, st, bt->ybits, yT, D, Nc,
                       F(w.alpha), F(w.beta), F(w.G), F(w.Hh), F(w.sig), F(w.tau));
    WTRY(kmark("kw_hunk_fwd", st));
  }
  float* probs = out ? out->probs : nullptr;
  float* logits = out ? out->logits : nullptr;
  if (!train) {
    hipLaunchKernelGGL(kw_hunk_cls<false>, dim3(tc, B, CLS_SPLIT), dim3(NTP), 0, st, yT, params,
                       o, D,
                       Nc, F(w.sig), F(w.tau), probs, logits, F(w.gam), ce_scale, part, w.segs, 0);
    WTRY(kmark("kw_hunk_cls", st));
    if (ce_sum) {
      hipLaunchKernelGGL(kw_grad_reduce, dim3(1), dim3(64), 0, st, part, w.segs, o.NP, o.NP,
                         ce_sum);
      WTRY(kmark("kw_grad_reduce", st));
    }
    if (out && out->ehr) {
      WTRY(launch_ehr(F(w.G), F(w.Hh), (size_t)Nc * H, B, Nc, params, v, out->ehr, st));
    }
    return 0;
  }
  // the two-pass classifier backward rebuilds gamma from the probabilities when the step
  // writes them (a training sess.run fetches C_edge_output2): 4 B per pair not stored
  const float* gprobs = (!ht && HDG_GAM_FROM_PROBS) ? probs : nullptr;
  hipLaunchKernelGGL(kw_hunk_cls<true>, dim3(tc, B, CLS_SPLIT), dim3(NTP), 0, st, yT, params,
                     o, D, Nc,
                     F(w.sig), F(w.tau), probs, logits, F(w.gam), ce_scale, part, w.segs,
                     gprobs ? 0 : 1);
  WTRY(kmark("kw_hunk_cls", st));
  if (ht) {
    HTileArgs ha{Nc, F(w.sig), F(w.tau), nullptr, nullptr, F(w.gam), D + D_EPS, bt->ybits,
                 F(w.htr), F(w.htc), F(w.hty)};
    WTRY(launch_hunk_tile(2, ha, B, st));
    hipLaunchKernelGGL(kw_hunk_fin2, dim3(tc, B, 2), dim3(NTP), 0, st, hts, params, o, D, Nc,
                       F(w.G), F(w.Hh), F(w.Dsig), F(w.Dtau), F(w.dG), F(w.dH), part, w.segs);
    WTRY(kmark("kw_hunk_fin2", st));
  } else {
    hipLaunchKernelGGL(kw_hunk_clsb, dim3(tc, B, 2), dim3(NTP), 0, st, bt->ybits, yT, params, o,
                       D, Nc, F(w.sig), F(w.tau), F(w.gam), F(w.G), F(w.Hh), F(w.Dsig),
                       F(w.Dtau), F(w.dG), F(w.dH), part, w.segs, gprobs, ce_scale);
    WTRY(kmark("kw_hunk_clsb", st));
  }
  if (hs) {
    const dim3 gw(H, B, 2);
#define HDG_WSUM(E_)                                                                        \
  hipLaunchKernelGGL(kw_hunk_wsum<E_>, gw, dim3(NT), 0, st, (const int*)F(w.hsp), F(w.dG), \
                     F(w.dH), Nc, (double*)F(w.hsw))
    switch (hsort_e(Nc)) {
      case 1: HDG_WSUM(1); break;
      case 2: HDG_WSUM(2); break;
      case 4: HDG_WSUM(4); break;
      default: HDG_WSUM(8); break;
    }
#undef HDG_WSUM
    WTRY(kmark("kw_hunk_wsum", st));
    if (hs_all_shape(s)) {
      hipLaunchKernelGGL(kw_hunk_mlpb_s, dim3((Nc + HSN - 1) / HSN, B, 2), dim3(HS_NT),
                         hs_shape_lds_bytes(s, 2), st, bt->ybits, yT, D, Nc, F(w.alpha), F(w.beta),
                         F(w.dG), F(w.dH), F(w.nvec), F(w.hsv), (const double*)F(w.hsw), prep,
                         YL, F(w.Dal), F(w.Dbe), part, w.segs);
      WTRY(kmark("kw_hunk_mlpb_s", st));
    } else {
      hipLaunchKernelGGL(kw_hunk_mlpb_g, dim3(4 * hs_tiles(Nc), B, 2), dim3(NT),
                         hs_shape_lds_bytes(s, 2), st, bt->ybits, yT, D, Nc, F(w.alpha), F(w.beta),
                         F(w.dG), F(w.dH), F(w.nvec), F(w.hsv), (const double*)F(w.hsw), prep,
                         YL, F(w.Dal), F(w.Dbe), part, w.segs);
      WTRY(kmark("kw_hunk_mlpb_g", st));
    }
  } else if (ht) {
    HTileArgs ha{Nc, F(w.alpha), F(w.beta), F(w.dG), F(w.dH), nullptr, D + D_DLT, bt->ybits,
                 F(w.htr), F(w.htc), F(w.hty)};
    WTRY(launch_hunk_tile(1, ha, B, st));
    hipLaunchKernelGGL(kw_hunk_fin1, dim3(tc, B, 2), dim3(NTP), 0, st, hts, D, Nc, F(w.alpha),
                       F(w.beta), F(w.dG), F(w.dH), F(w.nvec), F(w.Dal), F(w.Dbe), part, w.segs);
    WTRY(kmark("kw_hunk_fin1", st));
  } else {
    hipLaunchKernelGGL(kw_hunk_mlpb, dim3(tc, B, 2), dim3(NTP), 0, st, bt->ybits, yT, D, Nc,
                       F(w.alpha), F(w.beta), F(w.dG), F(w.dH), F(w.nvec), F(w.Dal), F(w.Dbe),
                       part, w.segs);
    WTRY(kmark("kw_hunk_mlpb", st));
  }
  if (ee) {   // kw_ee_clsb reads dn; with the entity stage alone kw_node_bwd forms it itself
    hipLaunchKernelGGL(kw_dn, dim3(tc, B), dim3(NT), 0, st, params, o, Nc, F(w.Dal), F(w.Dbe),
                       F(w.dn));
    WTRY(kmark("kw_dn", st));
  }
  if (ent) {
    hipLaunchKernelGGL(kw_node_bwd, dim3(te, B), dim3(NT), 0, st, prep, bt->x, params, o, Ne, Nc,
                       ee ? F(w.dn) : nullptr, F(w.ov), F(w.P), F(w.Eb), F(w.hE), F(w.rhoE), part,
                       w.segs, F(w.Dal), F(w.Dbe));
    WTRY(kmark("kw_node_bwd", st));
  }
  if (ee) {
    const int snake = ee_snake(s);
    hipLaunchKernelGGL(kw_ee_clsb, dim3(ee_bwd_tiles(Ne), B, 1), dim3(NT), ee_clsb_lds(Ne), st,
                       aT, bt->hid, bt->nlen, D, Ne, Nc, snake, prep + ee_order_off(s), F(w.rho),
                       F(w.gmm), F(w.dn), F(w.drho), F(w.dgam), part, w.segs);
    WTRY(kmark("kw_ee_clsb", st));
    hipLaunchKernelGGL(kw_ee_nodeb, dim3(te, B), dim3(NT), 0, st, params, o, D, Ne,
                       ee_bwd_tiles(Ne), bt->nlen, F(w.R1), F(w.C1), F(w.Rn), F(w.Cn), F(w.drho),
                       F(w.dgam), F(w.phi), F(w.psi), part, w.segs);
    WTRY(kmark("kw_ee_nodeb", st));
  }
  if (ent || ee) {   // the first-layer backward of both stages: one scan, one launch
    const int mode0 = ent ? 0 : 1, stages = (ent && ee) ? 2 : 1;
    hipLaunchKernelGGL(kw_scan, dim3(H, B, stages), dim3(NT), 0, st, prep, params, o, Ne, Nc,
                       mode0, F(w.rhoE), F(w.psi), (double*)F(w.tab));
    WTRY(kmark("kw_scan", st));
    if (first_bwd_halves(te * B * stages) == 2)
      hipLaunchKernelGGL(kw_first_bwd<2>, dim3(te, B, stages), dim3(NTP), tlds, st, bt->x,
                         bt->abits, prep, params, o, Ne, Nc, mode0, F(w.rhoE), F(w.phi),
                         F(w.psi), (const double*)F(w.tab), part, w.segs);
    else
      hipLaunchKernelGGL(kw_first_bwd<1>, dim3(te, B, stages), dim3(NT), tlds, st, bt->x,
                         bt->abits, prep, params, o, Ne, Nc, mode0, F(w.rhoE), F(w.phi),
                         F(w.psi), (const double*)F(w.tab), part, w.segs);
    WTRY(kmark("kw_first_bwd", st));
  }
  if (adam) {
    hdg_state* S = adam->state;
    const int nsb = (o.NP + HDG_TRAILER + NW - 1) / NW;
    hipLaunchKernelGGL(kw_reduce_adam, dim3(nsb), dim3(NT), 0, st, part, w.segs, o.NP, 0,
                       o.NP + HDG_TRAILER, 0, FusedRows{}, grad, S->params, S->adam_m,
                       S->adam_v, S->beta_pow, D, adam->lr, adam->inv_pairs, adam->stats);
  } else {
    hipLaunchKernelGGL(kw_grad_reduce, dim3(o.NP + HDG_TRAILER), dim3(64), 0, st, part, w.segs,
                       0, o.NP, grad);
  }
  WTRY(kmark(adam ? "kw_reduce_adam" : "kw_grad_reduce", st));
  return 0;
}

}  // namespace hdg

#ifdef HDG_WSTAMP
extern "C" int hdg_wstamp_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(hdg::g_wst), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif
