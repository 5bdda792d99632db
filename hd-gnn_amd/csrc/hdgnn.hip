// hdgnn.hip -- MI355X (gfx950, CDNA4) engine for the HD-GNN/S training step.
//
// One training step of model_2.graph2graph (model_2.py:86-130 forward, 336-338
// loss + Adam) runs as five launches on the caller's stream:
//
//   k_entity_fwd  [5 x B]   entity pair grid, relu(u_i + v_j + a_ij d) row+col sums
//                           (mlp_entity_B1 + agg_entity_B1 with W5 hoisted out of the
//                           pair sum: model_2.py:161-188)
//   k_commit_mid  [B]       per-commit: E3 node MLP, entity->hunk cross-graph sum,
//                           hunk pair MLP sums, edge classifier + softmax-CE (fwd+bwd),
//                           all node-level backward, rho = dL/dP  (model_2.py:94-130)
//   k_entity_bwd  [5 x B]   entity pair grid backward -> dW1 / db1 partials
//   k_grad_reduce [P/256]   deterministic per-commit partial sum (fixed commit order)
//   k_adam_tf     [1]       loss_para / loss_map gradients + TF1 ApplyAdam
//
// Algebra used (exact up to fp32 re-association; derivation in DESIGN.md section 3):
//   first-layer pre-activation of a pair MLP on [x_i, x_j, 1-a, a] = u_i + v_j + a*d,
//   so a pair costs ~5 VALU ops per hidden unit; second layers are linear and commute
//   with the row/column sums, so they run once per NODE.  The diagonal (i == j) is
//   summed with the tile and subtracted once per node.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "hdgnn.h"

namespace {

constexpr int HS = 20;              // h_size = De_e = De_er (model_2.py:163, 192, 247, 306)
constexpr int NT_MID = 1024;        // k_commit_mid block
constexpr int KK_MID = 5;           // hidden units per pair-tile chunk in k_commit_mid
constexpr int KK_E = 4;             // hidden units per block in the entity kernels
constexpr int NCHUNK_E = HS / KK_E;

// model_2 flat parameter offsets (tf.global_variables order)
namespace m2 {
constexpr int E1_W1 = 0, E1_B1 = 80, E1_W5 = 100, E1_B5 = 500;
constexpr int E3_W1 = 520, E3_B1 = 940, E3_W2 = 960, E3_B2 = 980;
constexpr int H1_W1 = 981, H1_B1 = 1181, H1_W2 = 1201, H1_B2 = 1601;
constexpr int H2_W1 = 1621, H2_B1 = 2061, H2_W2 = 2081, H2_B2 = 2121;
constexpr int TH1 = 2123, TH2 = 2125, NP = 2127;
}  // namespace m2
constexpr int NPART = 2132;        // per-commit partial row: NP grads + CE sum, padded
constexpr int GRAD_LEN = m2::NP + 4;

// ------------------------------------------------------------------------------
// cross-lane helpers (wave64)
// ------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}

// Sum over a 16-lane DPP row; every lane of the row receives the total.
__device__ __forceinline__ float row16_sum(float v) {
  v += dppf<0x140>(v);  // row_mirror        lane i <- 15-i
  v += dppf<0x141>(v);  // row_half_mirror   lane i <- 7-i (per 8)
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}

// Sum over the 4 DPP rows of a wave for every lane column: lane l gets
// v[l] + v[l^16] + v[l^32] + v[l^48].  v_permlane{32,16}_swap in the VALU (no LDS);
// inline asm because the ROCm 7.2 builtins mis-assign the two results, with the two
// wait states the swap needs after a VALU write of its operands inside the string.
__device__ __forceinline__ float xrow_sum4(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  const float s = x + y;
  float p = s, q = s;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(p), "+v"(q));
  return p + q;
}

__device__ __forceinline__ float wave_sum(float v) { return xrow_sum4(row16_sum(v)); }

__device__ __forceinline__ float reluf(float v) { return fmaxf(v, 0.f); }

__device__ __forceinline__ uint32_t getbit(const uint32_t* rowbits, int j) {
  return (rowbits[j >> 5] >> (j & 31)) & 1u;
}

// q = r / d, rem = r % d for 0 <= r < 2^22, 1 <= d < 2^12: float estimate + one select
// correction, 24-bit multiplies, no branches (keeps unrolled loads in flight)
__device__ __forceinline__ void divmod_bf(int r, int d, float inv, int& q, int& rem) {
  int q0 = (int)((float)r * inv);
  int r0 = r - __mul24(q0, d);
  const bool lo = r0 < 0, hi = r0 >= d;
  q = lo ? q0 - 1 : (hi ? q0 + 1 : q0);
  rem = lo ? r0 + d : (hi ? r0 - d : r0);
}

// ------------------------------------------------------------------------------
// Pair-tile engine: one 256-thread group sweeps an N x N pair grid for KK hidden
// units [k0, k0+KK).  Thread (ti, tj) = (t>>4, t&15) owns rows i = ti+16s and
// columns j = tj+16c.  Row sums close with a 16-lane DPP reduction per row; column
// partials stay in registers for the whole sweep and close once through LDS.
//   z_ij  = A[i] + B[j] + y_ij * dl          (y_ij = bit j of row i)
//   MODE 0  e = relu(z)                                       (forward sums)
//   MODE 1  e = [z > 0] * (wr[i] + wc[j])  , ysum += y*e      (backward, node weights)
//   MODE 2  e = [z > 0] * gam[i][j]        , ysum += y*e,  zsum += z*e   (pair weights)
//   Rout[i] = sum_j e_ij   Cout[j] = sum_i e_ij   (diagonal INCLUDED for MODE 0/1:
//   callers subtract it; MODE 2 masks it)
// A, B, wr, wc, Rout, Cout: LDS [node][LD] (rows/cols >= N padded with -inf in A/B).
// Rout may alias A and Cout may alias B (rows are consumed before they are written,
// columns are written after the closing barrier).  cred: 4*16*SMAX*KK + 8*KK words.
// Every thread of the BLOCK must call this the same number of times (barriers).
// ------------------------------------------------------------------------------
template <int SMAX, int KK>
constexpr int tile_cred_words() { return 4 * 16 * SMAX * KK + 8 * KK; }

template <int KK, int SMAX, int MODE, int LD>
__device__ __forceinline__ void pair_tile(
    const int N, const int t, const float* A, const float* Bv, const int k0,
    const float* __restrict__ dl, const uint32_t* __restrict__ bits, const int W,
    const float* __restrict__ wr, const float* __restrict__ wc,
    const float* __restrict__ gam, const int gld, float* Rout, float* Cout,
    float* __restrict__ ysum, float* __restrict__ zsum, float* __restrict__ cred) {
  constexpr int NP16 = 16 * SMAX;
  constexpr int NW = (SMAX + 1) / 2;
  const int tj = t & 15, ti = t >> 4, lane = t & 63, wv = t >> 6;
  const int S = (N + 15) >> 4;

  float cacc[SMAX][KK];
#pragma unroll
  for (int c = 0; c < SMAX; ++c)
#pragma unroll
    for (int k = 0; k < KK; ++k) cacc[c][k] = 0.f;
  float yacc[KK], zacc[KK], dk[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) { yacc[k] = 0.f; zacc[k] = 0.f; dk[k] = dl[k0 + k]; }

  for (int s = 0; s < S; ++s) {
    const int i = ti + 16 * s;
    const bool iv = i < N;
    float a[KK], rw[KK], racc[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      a[k] = A[i * LD + k0 + k];
      rw[k] = (MODE == 1) ? wr[i * LD + k0 + k] : 0.f;
      racc[k] = 0.f;
    }
    uint32_t wrow[NW];
    const int ib = iv ? i : 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {      // branch-free: clamped load, masked value
      const uint32_t w = bits[ib * W + (q < W ? q : 0)];
      wrow[q] = (iv && q < W) ? w : 0u;
    }
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
      const int j = tj + 16 * c;
      const float af = (float)((wrow[c >> 1] >> (tj + 16 * (c & 1))) & 1u);
      float g = 0.f;
      if constexpr (MODE == 2) {   // branch-free: clamped load, masked value
        const int ic = iv ? i : N - 1, jc = j < N ? j : N - 1;
        g = gam[ic * gld + jc] * ((iv && j < N && j != i) ? 1.f : 0.f);
      }
#pragma unroll
      for (int k = 0; k < KK; ++k) {
        const float z = a[k] + fmaf(af, dk[k], Bv[j * LD + k0 + k]);
        float e;
        if constexpr (MODE == 0) {
          e = reluf(z);
        } else {
          const float w = (MODE == 1) ? (rw[k] + wc[j * LD + k0 + k]) : g;
          e = (z > 0.f) ? w : 0.f;
          yacc[k] = fmaf(af, e, yacc[k]);
          if constexpr (MODE == 2) zacc[k] = fmaf(reluf(z), e, zacc[k]);   // z may be -inf
        }
        racc[k] += e;
        cacc[c][k] += e;
      }
    }
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const float r = row16_sum(racc[k]);
      if (tj == 0 && iv) Rout[i * LD + k0 + k] = r;
    }
  }
  // close the column partials: 4 ti per wave by shuffles, then 4 waves via LDS
  float* credy = cred + 4 * NP16 * KK;
  float* credz = credy + 4 * KK;
#pragma unroll
  for (int c = 0; c < SMAX; ++c)
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const float v = xrow_sum4(cacc[c][k]);
      if (lane < 16) cred[(wv * NP16 + tj + 16 * c) * KK + k] = v;
    }
  if constexpr (MODE != 0) {
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const float v = wave_sum(yacc[k]);
      if (lane == 0) credy[wv * KK + k] = v;
      if constexpr (MODE == 2) {
        const float vz = wave_sum(zacc[k]);
        if (lane == 0) credz[wv * KK + k] = vz;
      }
    }
  }
  __syncthreads();
  for (int e = t; e < NP16 * KK; e += 256) {
    const int j = e / KK, k = e - j * KK;
    const float v = cred[e] + cred[e + NP16 * KK] + cred[e + 2 * NP16 * KK] + cred[e + 3 * NP16 * KK];
    if (j < N) Cout[j * LD + k0 + k] = v;
  }
  if constexpr (MODE != 0) {
    if (t < KK) ysum[k0 + t] = credy[t] + credy[KK + t] + credy[2 * KK + t] + credy[3 * KK + t];
    if constexpr (MODE == 2) {
      if (t < KK) zsum[k0 + t] = credz[t] + credz[KK + t] + credz[2 * KK + t] + credz[3 * KK + t];
    }
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------
// Row/column sweep over an N x N relation grid by NG 256-thread groups, columns
// split across groups (group g owns column blocks c = g, g+NG, ...):
//   Rout[i][w] = sum_j f(i,j)[w],  Cout[j][w] = sum_i f(i,j)[w]
// f(i,j,v) must be branch-free and safe on any i,j in [0,N) (it is called on clamped
// indices and masked: i == j and out-of-range slots contribute 0).
// scratch: sweep_scratch_words(SMAX, VW, NG) words.
// ------------------------------------------------------------------------------
__host__ __device__ constexpr int sweep_scratch_words(int smax, int vw, int ng) {
  return (ng + 4) * 16 * smax * vw;
}

template <int VW, int SMAX, int NG, class F>
__device__ __forceinline__ void grid_sweep(const int N, const int t, F f, float* __restrict__ Rout,
                                           float* __restrict__ Cout, float* __restrict__ scratch) {
  constexpr int NP16 = 16 * SMAX;
  constexpr int CPG = SMAX / NG;       // column blocks per group
  static_assert(SMAX % NG == 0, "SMAX must be a multiple of NG");
  const int g = t >> 8, tg = t & 255;
  const int tj = tg & 15, ti = tg >> 4, lane = t & 63, wg = tg >> 6;
  const int S = (N + 15) >> 4;
  float* Rpart = scratch;                          // [NG][NP16][VW]
  float* Cpart = scratch + NG * NP16 * VW;         // [NG][4][16*CPG][VW]
  float cacc[CPG][VW];
#pragma unroll
  for (int c = 0; c < CPG; ++c)
#pragma unroll
    for (int w = 0; w < VW; ++w) cacc[c][w] = 0.f;
  for (int s = 0; s < S; ++s) {
    const int i = ti + 16 * s;
    const int ic = i < N ? i : N - 1;
    float racc[VW];
#pragma unroll
    for (int w = 0; w < VW; ++w) racc[w] = 0.f;
#pragma unroll
    for (int cc = 0; cc < CPG; ++cc) {
      const int j = tj + 16 * (g + NG * cc);
      const int jc = j < N ? j : N - 1;
      const float m = (i < N && j < N && i != j) ? 1.f : 0.f;
      float v[VW];
      f(ic, jc, v);
#pragma unroll
      for (int w = 0; w < VW; ++w) {
        racc[w] = fmaf(m, v[w], racc[w]);
        cacc[cc][w] = fmaf(m, v[w], cacc[cc][w]);
      }
    }
#pragma unroll
    for (int w = 0; w < VW; ++w) {
      const float r = row16_sum(racc[w]);
      if (tj == 0) Rpart[(g * NP16 + i) * VW + w] = r;
    }
  }
#pragma unroll
  for (int cc = 0; cc < CPG; ++cc)
#pragma unroll
    for (int w = 0; w < VW; ++w) {
      const float v = xrow_sum4(cacc[cc][w]);
      if (lane < 16) Cpart[((g * 4 + wg) * 16 * CPG + tj + 16 * cc) * VW + w] = v;
    }
  __syncthreads();
  for (int e = t; e < N * VW; e += 256 * NG) {
    const int i = e / VW, w = e - i * VW;
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < NG; ++q) r += Rpart[(q * NP16 + i) * VW + w];
    Rout[e] = r;
    const int jb = i >> 4, gq = jb % NG, cc = jb / NG, tq = i & 15;
    float c = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) c += Cpart[((gq * 4 + q) * 16 * CPG + tq + 16 * cc) * VW + w];
    Cout[e] = c;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------
// Entity stage (shared set-up of the forward and backward entity kernels)
//   u_i = x_i W1[0] + W1[2] + b1      v_j = x_j W1[1]      d = W1[3] - W1[2]
// so W1^T [x_i, x_j, [a=0], [a=1]] + b1 = u_i + v_j + a_ij d   (model_2.py:165-170)
// ------------------------------------------------------------------------------
template <int SMAX>
struct EntSmem {
  static constexpr int NP16 = 16 * SMAX;
  alignas(16) float u[NP16 * KK_E];
  alignas(16) float v[NP16 * KK_E];
  alignas(16) float R[NP16 * KK_E];
  alignas(16) float C[NP16 * KK_E];
  alignas(16) float rho[NP16 * KK_E];
  alignas(16) float cred[tile_cred_words<SMAX, KK_E>()];
  alignas(16) float xs[NP16];
  float dl[KK_E];
  float ysum[KK_E];
  uint32_t bits[NP16 * ((NP16 + 31) / 32)];
};

template <int SMAX>
__device__ __forceinline__ void entity_setup(EntSmem<SMAX>& sm, const float* __restrict__ x,
                                             const uint32_t* __restrict__ abits,
                                             const float* __restrict__ Wp, int Ne, int b,
                                             int k0, int t) {
  constexpr int NP16 = 16 * SMAX;
  using namespace m2;
  const int WE = (Ne + 31) >> 5;
  const float* xb = x + (size_t)b * Ne;
  for (int i = t; i < NP16; i += 256) {
    const float xi = (i < Ne) ? xb[i] : 0.f;
    sm.xs[i] = xi;
#pragma unroll
    for (int k = 0; k < KK_E; ++k) {
      const int kk = k0 + k;
      sm.u[i * KK_E + k] = (i < Ne) ? fmaf(xi, Wp[E1_W1 + kk], Wp[E1_W1 + 40 + kk] + Wp[E1_B1 + kk])
                                    : -INFINITY;
      sm.v[i * KK_E + k] = (i < Ne) ? xi * Wp[E1_W1 + 20 + kk] : -INFINITY;
    }
  }
  if (t < KK_E) sm.dl[t] = Wp[E1_W1 + 60 + k0 + t] - Wp[E1_W1 + 40 + k0 + t];
  const uint32_t* ab = abits + (size_t)b * Ne * WE;
  for (int w = t; w < Ne * WE; w += 256) sm.bits[w] = ab[w];
}

// P[b][i][k] = sum_{j!=i} relu(z_ij) + sum_{j!=i} relu(z_ji)   (so that
// E_bar_i = P_i W5 + 2(Ne-1) b5, model_2.py:175 + 186)
template <int SMAX>
__global__ __launch_bounds__(256) void k_entity_fwd(const float* __restrict__ x,
                                                    const uint32_t* __restrict__ abits,
                                                    const float* __restrict__ Wp,
                                                    float* __restrict__ Pout, int Ne) {
  __shared__ EntSmem<SMAX> sm;
  const int kc = blockIdx.x, b = blockIdx.y, t = threadIdx.x, k0 = kc * KK_E;
  entity_setup<SMAX>(sm, x, abits, Wp, Ne, b, k0, t);
  __syncthreads();
  pair_tile<KK_E, SMAX, 0, KK_E>(Ne, t, sm.u, sm.v, 0, sm.dl, sm.bits, (Ne + 31) >> 5, nullptr,
                                 nullptr, nullptr, 0, sm.R, sm.C, nullptr, nullptr, sm.cred);
  float* Pb = Pout + (size_t)b * Ne * HS;
  for (int e = t; e < Ne * KK_E; e += 256) {
    const int i = e / KK_E, k = e - i * KK_E;
    const float diag = reluf(sm.u[i * KK_E + k] + sm.v[i * KK_E + k]);
    Pb[i * HS + k0 + k] = (sm.R[e] + sm.C[e]) - 2.f * diag;
  }
}

// dz_ij = [z_ij > 0] (rho_i + rho_j)  (rho = dL/dP from k_commit_mid)
// dW1[0] = sum x_i dz, dW1[1] = sum x_j dz, dW1[3] = sum a dz, dW1[2] = sum (1-a) dz, db1 = sum dz
template <int SMAX>
__global__ __launch_bounds__(256) void k_entity_bwd(const float* __restrict__ x,
                                                    const uint32_t* __restrict__ abits,
                                                    const float* __restrict__ Wp,
                                                    const float* __restrict__ rho,
                                                    float* __restrict__ part, int Ne) {
  constexpr int NP16 = 16 * SMAX;
  __shared__ EntSmem<SMAX> sm;
  const int kc = blockIdx.x, b = blockIdx.y, t = threadIdx.x, k0 = kc * KK_E;
  entity_setup<SMAX>(sm, x, abits, Wp, Ne, b, k0, t);
  const float* rb = rho + (size_t)b * Ne * HS;
  for (int e = t; e < NP16 * KK_E; e += 256) {
    const int i = e / KK_E, k = e - i * KK_E;
    sm.rho[e] = (i < Ne) ? rb[i * HS + k0 + k] : 0.f;
  }
  __syncthreads();
  pair_tile<KK_E, SMAX, 1, KK_E>(Ne, t, sm.u, sm.v, 0, sm.dl, sm.bits, (Ne + 31) >> 5, sm.rho,
                                 sm.rho, nullptr, 0, sm.R, sm.C, sm.ysum, nullptr, sm.cred);
  // remove the diagonal term the tile included (a_ii = 0)
  for (int e = t; e < Ne * KK_E; e += 256) {
    const float z = sm.u[e] + sm.v[e];
    const float dz = (z > 0.f) ? (sm.rho[e] + sm.rho[e]) : 0.f;
    sm.R[e] -= dz;
    sm.C[e] -= dz;
  }
  __syncthreads();
  // 12 sums over nodes: (k, which) -> one 16-lane row each
  const int row = t >> 4, tj = t & 15;
  if (row < 3 * KK_E) {
    const int k = row % KK_E, which = row / KK_E;
    float acc = 0.f;
    for (int i = tj; i < Ne; i += 16) {
      const float du = sm.R[i * KK_E + k], dv = sm.C[i * KK_E + k], xi = sm.xs[i];
      acc += (which == 0) ? xi * du : (which == 1) ? xi * dv : du;
    }
    acc = row16_sum(acc);
    if (tj == 0) {
      using namespace m2;
      float* pb = part + (size_t)b * NPART;
      const int kk = k0 + k;
      if (which == 0) pb[E1_W1 + kk] = acc;
      if (which == 1) pb[E1_W1 + 20 + kk] = acc;
      if (which == 2) {
        const float ya = sm.ysum[k];
        pb[E1_W1 + 60 + kk] = ya;
        pb[E1_W1 + 40 + kk] = acc - ya;
        pb[E1_B1 + kk] = acc;
      }
    }
  }
}

// ------------------------------------------------------------------------------
// k_commit_mid: everything between the two entity pair sweeps, one 1024-thread
// block per commit.  Node arrays live in LDS; one union region U is re-carved per
// phase (entity staging -> X1 sweep -> hunk buffers -> X1 backward -> E3 backward).
// E_bar and the E3 hidden layer are parked in the workspace across the hunk phases.
// Node matvecs use a (k, slice) thread map with the weight column held in registers.
// ------------------------------------------------------------------------------
constexpr int NG_MID = NT_MID / 256;            // 4 pair-tile groups, one k-chunk each
constexpr int NBUF_H = 6;                       // hunk node buffers [NC16][HS]
constexpr int NSL = NT_MID / HS;                // 51 node slices for (k, slice) matvecs

struct MidLayout {   // offsets in 4-byte words into the dynamic LDS arena
  int W, xs, xps, os, dxr, dxc, hid, ab, yb, nb, dnb, misc, Mm, Xm, red, U, Uwords, total;
};

__host__ __device__ inline MidLayout mid_layout(int Ne, int Nc, int smaxc) {
  MidLayout L;
  const int NC16 = 16 * smaxc;
  const int NE4 = (Ne + 3) & ~3;
  const int WE = (Ne + 31) >> 5, WC = (Nc + 31) >> 5;
  const int cred = 4 * 16 * smaxc * KK_MID + 8 * KK_MID;
  int o = 0;
  L.W = o;    o += (m2::NP + 3) & ~3;
  L.xs = o;   o += NE4;
  L.xps = o;  o += NE4;
  L.os = o;   o += NE4;
  L.dxr = o;  o += NE4;
  L.dxc = o;  o += NE4;
  L.hid = o;  o += NE4;
  L.ab = o;   o += (Ne * WE + 3) & ~3;
  L.yb = o;   o += (Nc * WC + 3) & ~3;
  L.nb = o;   o += 4 * NC16;
  L.dnb = o;  o += 4 * NC16;
  L.misc = o; o += 8 * HS;            // dlt eps cvec ysumv s0 t0 sumD zsumv
  L.Mm = o;   o += HS * HS;           // V2 . U1e
  L.Xm = o;   o += HS * HS;           // sum_p G_p (x) Dsig_p + H_p (x) Dtau_p
  L.red = o;  o += (NT_MID / 64) * 32;
  int u = 3 * NE4 * HS;                                            // P | E_bar | h
  const int ux1 = 8 * NE4 + sweep_scratch_words(16, 4, NG_MID);    // X1 forward
  const int uh = NBUF_H * NC16 * HS + NG_MID * cred;               // hunk phases
  const int ux2 = 6 * NE4 + sweep_scratch_words(16, 2, NG_MID);    // X1 backward
  const int ueb = 5 * NE4 * HS;                                    // E3 backward
  if (ux1 > u) u = ux1;
  if (uh > u) u = uh;
  if (ux2 > u) u = ux2;
  if (ueb > u) u = ueb;
  L.U = o; L.Uwords = u; o += u;
  L.total = o;
  return L;
}

// dot of a 20-float LDS row (16-B aligned) with 20 register weights
__device__ __forceinline__ float dot20(const float* row, const float (&w)[HS], float acc) {
  const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll
  for (int v = 0; v < HS / 4; ++v) {
    const float4 q = r4[v];
    acc = fmaf(q.x, w[4 * v], acc);
    acc = fmaf(q.y, w[4 * v + 1], acc);
    acc = fmaf(q.z, w[4 * v + 2], acc);
    acc = fmaf(q.w, w[4 * v + 3], acc);
  }
  return acc;
}

template <int SMAXC, bool TRAIN, bool STAMPS = false>
__global__ __launch_bounds__(NT_MID) void k_commit_mid(
    const float* __restrict__ x, const uint32_t* __restrict__ abits,
    const uint32_t* __restrict__ ybits, const int32_t* __restrict__ hidg,
    const int32_t* __restrict__ nleng, const float* __restrict__ Wg,
    const float* __restrict__ Pg, float* __restrict__ Esave, float* __restrict__ rhog,
    float* __restrict__ gamg, float* __restrict__ part, float* __restrict__ probs,
    float* __restrict__ logits, int Ne, int Nc, float ce_scale,
    unsigned long long* __restrict__ stamps) {
  using namespace m2;
  constexpr int NC16 = 16 * SMAXC;
  constexpr int CRED = tile_cred_words<SMAXC, KK_MID>();
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const MidLayout L = mid_layout(Ne, Nc, SMAXC);
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6, g = t >> 8, tg = t & 255;
  const int mk = t % HS, msl = t / HS;            // (k, slice) map; msl == NSL idles
  const int WE = (Ne + 31) >> 5, WC = (Nc + 31) >> 5;
  const int NE4 = (Ne + 3) & ~3;
  const int Pc = Nc * (Nc - 1);
  int nstamp = 0;
#define MID_STAMP()                                                                     \
  do {                                                                                  \
    if constexpr (STAMPS) {                                                             \
      if (threadIdx.x == 0) stamps[blockIdx.x * 32 + nstamp] = __builtin_amdgcn_s_memrealtime(); \
      ++nstamp;                                                                         \
    }                                                                                   \
  } while (0)
  MID_STAMP();
  float* Ws = lds + L.W;
  float* xs = lds + L.xs;
  float* xps = lds + L.xps;
  float* os = lds + L.os;
  float* dxr = lds + L.dxr;
  float* dxc = lds + L.dxc;
  int* hid = (int*)(lds + L.hid);
  uint32_t* ab = (uint32_t*)(lds + L.ab);
  uint32_t* yb = (uint32_t*)(lds + L.yb);
  float* nb = lds + L.nb;
  float* dnb = lds + L.dnb;
  float* dlt = lds + L.misc;        // V1[9]-V1[8]
  float* eps = dlt + HS;            // U1[1]-U1[0]
  float* cvec = eps + HS;           // U2[:,1]-U2[:,0]
  float* ysumv = cvec + HS;
  float* s0v = ysumv + HS;          // sigma offset
  float* t0v = s0v + HS;            // tau offset
  float* sumD = t0v + HS;
  float* zsumv = sumD + HS;
  float* Mm = lds + L.Mm;
  float* Xm = lds + L.Xm;
  float* red = lds + L.red;
  float* U = lds + L.U;

  const float* Pb = Pg + (size_t)b * Ne * HS;
  float* EbG = Esave + (size_t)b * 2 * Ne * HS;
  float* hEG = EbG + Ne * HS;
  float* pb = part + (size_t)b * NPART;
  float* gam = gamg + (size_t)b * NC16 * NC16;
  int n = nleng[b];
  n = n < 0 ? 0 : (n > Ne ? Ne : n);
  const int nrel = n * (n - 1);
  const float Nc1 = (float)(Nc - 1);
  const float twoNe1 = 2.f * (float)(Ne - 1);

  // ---- M0: stage weights, commit inputs and P (k_entity_fwd output) -----------------
  float* Ps = U;
  float* Eb = U + NE4 * HS;
  float* hE = U + 2 * NE4 * HS;
  for (int i = t; i < NP; i += NT_MID) Ws[i] = Wg[i];
  for (int i = t; i < Ne; i += NT_MID) {
    xs[i] = x[(size_t)b * Ne + i];
    hid[i] = hidg[(size_t)b * Ne + i];
  }
  for (int w = t; w < Ne * WE; w += NT_MID) ab[w] = abits[(size_t)b * Ne * WE + w];
  for (int w = t; w < Nc * WC; w += NT_MID) yb[w] = ybits[(size_t)b * Nc * WC + w];
  {
    const float4* src = reinterpret_cast<const float4*>(Pb);
    float4* dst = reinterpret_cast<float4*>(Ps);
    for (int e = t; e < Ne * HS / 4; e += NT_MID) dst[e] = src[e];
  }
  __syncthreads();
  MID_STAMP();

  // ---- M1: E_bar = P W5 + 2(Ne-1) b5   (agg_entity_B1, model_2.py:181-188) ----------
  if (msl < NSL) {
    float w[HS];
#pragma unroll
    for (int m = 0; m < HS; ++m) w[m] = Ws[E1_W5 + m * HS + mk];
    const float bias = twoNe1 * Ws[E1_B5 + mk];
    for (int i = msl; i < Ne; i += NSL) {
      const float v = dot20(Ps + i * HS, w, 0.f) + bias;
      Eb[i * HS + mk] = v;
      EbG[i * HS + mk] = v;
    }
  }
  __syncthreads();
  MID_STAMP();
  // ---- M2: mlp2_entity_B1 (model_2.py:190-205) --------------------------------------
  if (msl < NSL) {
    float w[HS];
#pragma unroll
    for (int m = 0; m < HS; ++m) w[m] = Ws[E3_W1 + (1 + m) * HS + mk];
    const float w0 = Ws[E3_W1 + mk], bb = Ws[E3_B1 + mk];
    for (int i = msl; i < Ne; i += NSL) {
      const float v = reluf(dot20(Eb + i * HS, w, fmaf(xs[i], w0, bb)));
      hE[i * HS + mk] = v;
      hEG[i * HS + mk] = v;
    }
  }
  __syncthreads();
  MID_STAMP();
  {
    float w[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) w[k] = Ws[E3_W2 + k];
    for (int i = t; i < Ne; i += NT_MID) {
      const float o = dot20(hE + i * HS, w, Ws[E3_B2]);
      os[i] = o;
      xps[i] = reluf(o);
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M3: marshalling_B2 cross-graph sum (model_2.py:146-150, utils2.py:111-137) -----
  // n_c = sum_r ([s_r=c]+[t_r=c]) B2_r,  B2_r = [x'_I, x'_J, [a=0], [a=1]] on the Ne-grid,
  // s_r = hid[i'(r)], t_r = hid[j'(r)] on the n-grid (stride n-1): row sums (segS) and
  // column sums (segT) of the n x n grid of B2 values, then binned by hid.
  float* segS = U;
  float* segT = U + 4 * NE4;
  if (n >= 2) {
    const int Ne1 = Ne - 1, n1 = n - 1;
    const float invNe1 = 1.f / (float)Ne1;
    grid_sweep<4, 16, NG_MID>(n, t, [&](int ip, int jp, float* v) {
      const int r = __mul24(ip, n1) + jp - (jp > ip ? 1 : 0);
      int I, jj;
      divmod_bf(r < 0 ? 0 : r, Ne1, invNe1, I, jj);
      const int J = jj + (jj >= I ? 1 : 0);
      const float a = (float)((ab[__mul24(I, WE) + (J >> 5)] >> (J & 31)) & 1u);
      v[0] = xps[I];
      v[1] = xps[J];
      v[2] = 1.f - a;
      v[3] = a;
    }, segS, segT, U + 8 * NE4);
  }
  for (int e = t; e < NC16 * 4; e += NT_MID) {
    const int c = e >> 2, m = e & 3;
    float acc = 0.f;
    if (c < Nc && n >= 2) {
      const int4* h4 = reinterpret_cast<const int4*>(hid);
      for (int q = 0; q < (n + 3) >> 2; ++q) {
        const int4 h = h4[q];
        const int ip = 4 * q;
        if (h.x == c) acc += segS[4 * ip + m] + segT[4 * ip + m];
        if (h.y == c && ip + 1 < n) acc += segS[4 * ip + 4 + m] + segT[4 * ip + 4 + m];
        if (h.z == c && ip + 2 < n) acc += segS[4 * ip + 8 + m] + segT[4 * ip + 8 + m];
        if (h.w == c && ip + 3 < n) acc += segS[4 * ip + 12 + m] + segT[4 * ip + 12 + m];
      }
    }
    nb[e] = acc;
  }
  // per-block constants: delta, eps, c, M = V2 U1e, sigma/tau offsets
  if (t < HS) {
    dlt[t] = Ws[H1_W1 + 9 * HS + t] - Ws[H1_W1 + 8 * HS + t];
    eps[t] = Ws[H2_W1 + HS + t] - Ws[H2_W1 + t];
    cvec[t] = Ws[H2_W2 + 2 * t + 1] - Ws[H2_W2 + 2 * t];
    float cu = 0.f;                       // (Nc-1) c2 U1e
#pragma unroll
    for (int m = 0; m < HS; ++m) cu = fmaf(Ws[H1_B2 + m], Ws[H2_W1 + (2 + m) * HS + t], cu);
    cu *= Nc1;
    t0v[t] = cu;
    s0v[t] = cu + (Ws[H2_W1 + t] + Ws[H2_B1 + t]);
  }
  for (int e = t; e < HS * HS; e += NT_MID) {
    const int l = e / HS, k = e - l * HS;
    float acc = 0.f;
#pragma unroll
    for (int m = 0; m < HS; ++m) acc = fmaf(Ws[H1_W2 + l * HS + m], Ws[H2_W1 + (2 + m) * HS + k], acc);
    Mm[e] = acc;
  }
  __syncthreads();
  MID_STAMP();

  // ---- M4: first layer of mlp_hunk_B2 split per node (model_2.py:257-260) ----------
  //   alpha_p = n_p V1[0:4] + V1[8] + c1,   beta_q = n_q V1[4:8],   delta = V1[9]-V1[8]
  float* Bf[NBUF_H];
#pragma unroll
  for (int q = 0; q < NBUF_H; ++q) Bf[q] = U + q * NC16 * HS;
  float* credg = U + NBUF_H * NC16 * HS + g * CRED;
  float* alpha = Bf[0];
  float* beta = Bf[1];
  if (msl < NSL) {
    float wa[4], wb[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      wa[m] = Ws[H1_W1 + m * HS + mk];
      wb[m] = Ws[H1_W1 + (4 + m) * HS + mk];
    }
    const float a0 = Ws[H1_W1 + 8 * HS + mk] + Ws[H1_B1 + mk];
    for (int p = msl; p < NC16; p += NSL) {
      float al = -INFINITY, be = -INFINITY;
      if (p < Nc) {
        const float4 nv = reinterpret_cast<const float4*>(nb)[p];
        al = fmaf(nv.w, wa[3], fmaf(nv.z, wa[2], fmaf(nv.y, wa[1], fmaf(nv.x, wa[0], a0))));
        be = fmaf(nv.w, wb[3], fmaf(nv.z, wb[2], fmaf(nv.y, wb[1], nv.x * wb[0])));
      }
      alpha[p * HS + mk] = al;
      beta[p * HS + mk] = be;
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M5: hunk pair sums G_p = sum_q g1_pq, H_q = sum_p g1_pq (model_2.py:260-275) ---
  float* G = Bf[2];
  float* Hh = Bf[3];
  pair_tile<KK_MID, SMAXC, 0, HS>(Nc, tg, alpha, beta, g * KK_MID, dlt, yb, WC, nullptr, nullptr,
                                  nullptr, 0, G, Hh, nullptr, nullptr, credg);
  for (int e = t; e < Nc * HS; e += NT_MID) {
    const float dg = reluf(alpha[e] + beta[e]);
    G[e] -= dg;
    Hh[e] -= dg;
  }
  __syncthreads();
  MID_STAMP();

  // ---- M6: classifier first layer on eff = S_p + T_q, S = G V2 + (Nc-1) c2:
  //   sigma_p = G_p M + (Nc-1) c2 U1e + U1[0] + d1,  tau_q = H_q M + (Nc-1) c2 U1e
  float* sig = Bf[4];
  float* tau = Bf[5];
  if (msl < NSL) {
    float w[HS];
#pragma unroll
    for (int l = 0; l < HS; ++l) w[l] = Mm[l * HS + mk];
    const float s0 = s0v[mk], t0 = t0v[mk];
    for (int p = msl; p < NC16; p += NSL) {
      float as = -INFINITY, at = -INFINITY;
      if (p < Nc) {
        as = dot20(G + p * HS, w, s0);
        at = dot20(Hh + p * HS, w, t0);
      }
      sig[p * HS + mk] = as;
      tau[p * HS + mk] = at;
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M7: edge classifier + softmax CE per hunk pair (model_2.py:304-324, 115-118) ----
  float* prb = probs ? probs + (size_t)b * 2 * Pc : nullptr;
  float* lgb = logits ? logits + (size_t)b * 2 * Pc : nullptr;
  float ce_acc = 0.f, gsum = 0.f;
  {
    const int Nc1i = Nc - 1;
    const float invNc1 = 1.f / (float)Nc1i;
    float w0[HS], w1[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) {
      w0[k] = Ws[H2_W2 + 2 * k];
      w1[k] = Ws[H2_W2 + 2 * k + 1];
    }
    const float b0 = Ws[H2_B2], b1 = Ws[H2_B2 + 1];
    const float4* ep4 = reinterpret_cast<const float4*>(eps);
    for (int e = t; e < Pc; e += NT_MID) {
      int p, qq;
      divmod_bf(e, Nc1i, invNc1, p, qq);
      const int q = qq + (qq >= p ? 1 : 0);
      const float yf = (float)((yb[__mul24(p, WC) + (q >> 5)] >> (q & 31)) & 1u);
      const float4* sp = reinterpret_cast<const float4*>(sig + p * HS);
      const float4* tq = reinterpret_cast<const float4*>(tau + q * HS);
      float z0 = b0, z1 = b1;
#pragma unroll
      for (int v = 0; v < HS / 4; ++v) {
        const float4 a = sp[v], c = tq[v], ee = ep4[v];
        const float k0 = reluf(a.x + fmaf(yf, ee.x, c.x));
        const float k1 = reluf(a.y + fmaf(yf, ee.y, c.y));
        const float k2 = reluf(a.z + fmaf(yf, ee.z, c.z));
        const float k3 = reluf(a.w + fmaf(yf, ee.w, c.w));
        z0 = fmaf(k3, w0[4 * v + 3], fmaf(k2, w0[4 * v + 2], fmaf(k1, w0[4 * v + 1], fmaf(k0, w0[4 * v], z0))));
        z1 = fmaf(k3, w1[4 * v + 3], fmaf(k2, w1[4 * v + 2], fmaf(k1, w1[4 * v + 1], fmaf(k0, w1[4 * v], z1))));
      }
      const float mx = fmaxf(z0, z1);
      const float e0 = __expf(z0 - mx), e1 = __expf(z1 - mx);
      const float ssum = e0 + e1;
      const float inv = 1.f / ssum;
      const float p0 = e0 * inv, p1 = e1 * inv;
      ce_acc += (__logf(ssum) + mx) - (yf > 0.f ? z1 : z0);
      if (prb) { prb[e] = p0; prb[Pc + e] = p1; }
      if (lgb) { lgb[e] = z0; lgb[Pc + e] = z1; }
      if constexpr (TRAIN) {
        if (qq == p) gam[p * NC16 + p] = 0.f;     // defined diagonal (read masked in M8)
        const float gmm = ce_scale * (p1 - yf);   // dL/dz1 = -dL/dz0
        gam[p * NC16 + q] = gmm;
        gsum += gmm;
      }
    }
  }
  {
    const float s0 = wave_sum(ce_acc), s1 = wave_sum(gsum);
    if (lane == 0) { red[wv * 32] = s0; red[wv * 32 + 1] = s1; }
  }
  __syncthreads();
  MID_STAMP();
  if (t < 2) {
    float s = 0.f;
    for (int w = 0; w < NT_MID / 64; ++w) s += red[w * 32 + t];
    if (t == 0) pb[NP] = s;
    if constexpr (TRAIN) {
      if (t == 1) { pb[H2_B2] = -s; pb[H2_B2 + 1] = s; }
    }
  }
  if constexpr (!TRAIN) return;   // uniform exit: forward-only launch

  // ---- M8: classifier backward: dkappa_pq = c (.) [kappa_pq > 0] gamma_pq,
  //          row sums Dsig (in place over sigma), column sums Dtau (over tau);
  //          zsum_k = sum relu(kappa_k) gamma -> dU2 ---------------------------------
  float* Dsig = sig;
  float* Dtau = tau;
  pair_tile<KK_MID, SMAXC, 2, HS>(Nc, tg, sig, tau, g * KK_MID, eps, yb, WC, nullptr, nullptr,
                                  gam, NC16, Dsig, Dtau, ysumv, zsumv, credg);
  for (int e = t; e < Nc * HS; e += NT_MID) {
    const int k = e % HS;
    Dsig[e] *= cvec[k];
    Dtau[e] *= cvec[k];
  }
  if (t < HS) { pb[H2_W2 + 2 * t] = -zsumv[t]; pb[H2_W2 + 2 * t + 1] = zsumv[t]; }
  __syncthreads();
  MID_STAMP();
  // ---- M9: X = sum_p G_p (x) Dsig_p + H_p (x) Dtau_p; classifier / hunk-MLP grads ----
  for (int e = t; e < HS * HS + HS; e += NT_MID) {
    const int l = e / HS, k = e - l * HS;
    if (l < HS) {
      float a0 = 0.f, a1 = 0.f;
      int p = 0;
      for (; p + 1 < Nc; p += 2) {
        a0 = fmaf(G[p * HS + l], Dsig[p * HS + k], fmaf(Hh[p * HS + l], Dtau[p * HS + k], a0));
        a1 = fmaf(G[(p + 1) * HS + l], Dsig[(p + 1) * HS + k],
                  fmaf(Hh[(p + 1) * HS + l], Dtau[(p + 1) * HS + k], a1));
      }
      if (p < Nc) a0 = fmaf(G[p * HS + l], Dsig[p * HS + k], fmaf(Hh[p * HS + l], Dtau[p * HS + k], a0));
      Xm[e] = a0 + a1;
    } else {
      float dd1 = 0.f, dt = 0.f;
      for (int p = 0; p < Nc; ++p) { dd1 += Dsig[p * HS + k]; dt += Dtau[p * HS + k]; }
      sumD[k] = dd1 + dt;
      const float dy1 = cvec[k] * ysumv[k];
      pb[H2_B1 + k] = dd1;
      pb[H2_W1 + HS + k] = dy1;
      pb[H2_W1 + k] = dd1 - dy1;
    }
  }
  __syncthreads();
  MID_STAMP();
  for (int e = t; e < 2 * HS * HS + HS; e += NT_MID) {
    if (e < HS * HS) {                    // dU1e[m][k] = sum_l V2[l][m] X[l][k] + (Nc-1)c2[m] sumD[k]
      const int m = e / HS, k = e - m * HS;
      float acc = Nc1 * Ws[H1_B2 + m] * sumD[k];
#pragma unroll
      for (int l = 0; l < HS; ++l) acc = fmaf(Ws[H1_W2 + l * HS + m], Xm[l * HS + k], acc);
      pb[H2_W1 + (2 + m) * HS + k] = acc;
    } else if (e < 2 * HS * HS) {         // dV2[l][m] = sum_k X[l][k] U1e[m][k]
      const int f = e - HS * HS, l = f / HS, m = f - l * HS;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < HS; ++k) acc = fmaf(Xm[l * HS + k], Ws[H2_W1 + (2 + m) * HS + k], acc);
      pb[H1_W2 + f] = acc;
    } else {                              // dc2[m] = (Nc-1) sum_k U1e[m][k] sumD[k]
      const int m = e - 2 * HS * HS;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < HS; ++k) acc = fmaf(Ws[H2_W1 + (2 + m) * HS + k], sumD[k], acc);
      pb[H1_B2 + m] = Nc1 * acc;
    }
  }
  float* dG = G;       // G, H dead once X is formed
  float* dH = Hh;
  if (msl < NSL) {     // dG_p[l] = sum_k M[l][k] Dsig_p[k]
    float w[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) w[k] = Mm[mk * HS + k];
    for (int p = msl; p < NC16; p += NSL) {
      float ag = 0.f, ah = 0.f;
      if (p < Nc) {
        ag = dot20(Dsig + p * HS, w, 0.f);
        ah = dot20(Dtau + p * HS, w, 0.f);
      }
      dG[p * HS + mk] = ag;
      dH[p * HS + mk] = ah;
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M10: hunk pair backward: dgamma = [g1 > 0](dG_p + dH_q) -----------------------
  float* Dal = Bf[4];   // Dsig/Dtau dead after dG/dH
  float* Dbe = Bf[5];
  pair_tile<KK_MID, SMAXC, 1, HS>(Nc, tg, alpha, beta, g * KK_MID, dlt, yb, WC, dG, dH, nullptr, 0,
                                  Dal, Dbe, ysumv, nullptr, credg);
  for (int e = t; e < Nc * HS; e += NT_MID) {
    const float dz = (alpha[e] + beta[e] > 0.f) ? (dG[e] + dH[e]) : 0.f;
    Dal[e] -= dz;
    Dbe[e] -= dz;
  }
  __syncthreads();
  MID_STAMP();
  for (int e = t; e < 10 * HS; e += NT_MID) {       // dV1 rows 0..9, dc1
    const int r = e / HS, k = e - r * HS;
    float acc = 0.f;
    if (r < 4) {
      for (int p = 0; p < Nc; ++p) acc = fmaf(nb[4 * p + r], Dal[p * HS + k], acc);
    } else if (r < 8) {
      for (int p = 0; p < Nc; ++p) acc = fmaf(nb[4 * p + r - 4], Dbe[p * HS + k], acc);
    } else {
      float dc1 = 0.f;
      for (int p = 0; p < Nc; ++p) dc1 += Dal[p * HS + k];
      acc = (r == 9) ? ysumv[k] : dc1 - ysumv[k];
      if (r == 8) pb[H1_B1 + k] = dc1;
    }
    pb[H1_W1 + e] = acc;
  }
  for (int e = t; e < NC16 * 2; e += NT_MID) {      // dn_c[m], m in {0,1} (x' components)
    const int c = e >> 1, m = e & 1;
    float acc = 0.f;
    if (c < Nc) {
#pragma unroll
      for (int k = 0; k < HS; ++k)
        acc = fmaf(Ws[H1_W1 + m * HS + k], Dal[c * HS + k],
                   fmaf(Ws[H1_W1 + (4 + m) * HS + k], Dbe[c * HS + k], acc));
    }
    dnb[e] = acc;
  }
  __syncthreads();
  MID_STAMP();

  // ---- M11: cross-graph backward: dx'_I += D_r[0], dx'_J += D_r[1], D_r = dn_s + dn_t --
  //   one sweep over the Ne-grid: row sums of D[0] -> dxr, column sums of D[1] -> dxc
  {
    float* gv = U;                      // [Ne][2] dn of the index line's hunk (0 if none)
    float* R2 = U + 2 * NE4;            // [Ne][2]
    float* C2 = U + 4 * NE4;            // [Ne][2]
    for (int e = t; e < 2 * Ne; e += NT_MID) {
      const int ip = e >> 1, m = e & 1;
      const int h = (ip < n) ? hid[ip] : -1;
      gv[e] = (h >= 0) ? dnb[2 * h + m] : 0.f;
    }
    __syncthreads();
    if (nrel > 0) {
      const int Ne1 = Ne - 1, n1 = n - 1;
      const float invn1 = 1.f / (float)n1;
      grid_sweep<2, 16, NG_MID>(Ne, t, [&](int i, int j, float* v) {
        const int r = __mul24(i, Ne1) + j - (j > i ? 1 : 0);
        const float live = r < nrel ? 1.f : 0.f;
        const int rc = r < nrel ? (r < 0 ? 0 : r) : nrel - 1;
        int Ip, jj;
        divmod_bf(rc, n1, invn1, Ip, jj);
        const int Jp = jj + (jj >= Ip ? 1 : 0);
        const float2 gs = reinterpret_cast<const float2*>(gv)[Ip];
        const float2 gt = reinterpret_cast<const float2*>(gv)[Jp];
        v[0] = live * (gs.x + gt.x);
        v[1] = live * (gs.y + gt.y);
      }, R2, C2, U + 6 * NE4);
      for (int i = t; i < Ne; i += NT_MID) {
        dxr[i] = R2[2 * i];
        dxc[i] = C2[2 * i + 1];
      }
    } else {
      for (int i = t; i < Ne; i += NT_MID) { dxr[i] = 0.f; dxc[i] = 0.f; }
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M12: mlp2_entity_B1 backward (U re-carved: P | E_bar | h | dq | dE) ------------
  float* dq = U + 3 * NE4 * HS;
  float* dE = U + 4 * NE4 * HS;
  for (int i = t; i < Ne; i += NT_MID) {
    const float dxp = dxr[i] + dxc[i];
    dxr[i] = (os[i] > 0.f) ? dxp : 0.f;             // d o_i
  }
  {
    const float4* s0 = reinterpret_cast<const float4*>(Pb);
    const float4* s1 = reinterpret_cast<const float4*>(EbG);
    const float4* s2 = reinterpret_cast<const float4*>(hEG);
    float4* d0 = reinterpret_cast<float4*>(Ps);
    float4* d1 = reinterpret_cast<float4*>(Eb);
    float4* d2 = reinterpret_cast<float4*>(hE);
    for (int e = t; e < Ne * HS / 4; e += NT_MID) { d0[e] = s0[e]; d1[e] = s1[e]; d2[e] = s2[e]; }
  }
  __syncthreads();
  MID_STAMP();
  for (int e = t; e < Ne * HS; e += NT_MID) {
    const int i = e / HS, k = e - i * HS;
    dq[e] = (hE[e] > 0.f) ? Ws[E3_W2 + k] * dxr[i] : 0.f;
  }
  if (t >= NT_MID - 64) {                           // one wave: dw2' (20), db2' (1)
    const int k = t - (NT_MID - 64);
    if (k <= HS) {
      float acc = 0.f;
      if (k < HS) {
        for (int i = 0; i < Ne; ++i) acc = fmaf(hE[i * HS + k], dxr[i], acc);
        pb[E3_W2 + k] = acc;
      } else {
        for (int i = 0; i < Ne; ++i) acc += dxr[i];
        pb[E3_B2] = acc;
      }
    }
  }
  __syncthreads();
  MID_STAMP();
  for (int e = t; e < 22 * HS; e += NT_MID) {       // dW1' (21 rows) + db1'
    const int r = e / HS, k = e - r * HS;
    float a0 = 0.f, a1 = 0.f;
    const float* src = (r == 0) ? xs : Eb + (r - 1);
    const int sst = (r == 0) ? 1 : HS;
    if (r <= HS) {
      int i = 0;
      for (; i + 1 < Ne; i += 2) {
        a0 = fmaf(src[i * sst], dq[i * HS + k], a0);
        a1 = fmaf(src[(i + 1) * sst], dq[(i + 1) * HS + k], a1);
      }
      if (i < Ne) a0 = fmaf(src[i * sst], dq[i * HS + k], a0);
      pb[E3_W1 + r * HS + k] = a0 + a1;
    } else {
      for (int i = 0; i < Ne; ++i) a0 += dq[i * HS + k];
      pb[E3_B1 + k] = a0;
    }
  }
  if (msl < NSL) {      // dE_i[m] = sum_k W1'[1+m][k] dq_i[k]
    float w[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) w[k] = Ws[E3_W1 + (1 + mk) * HS + k];
    for (int i = msl; i < Ne; i += NSL) dE[i * HS + mk] = dot20(dq + i * HS, w, 0.f);
  }
  __syncthreads();
  MID_STAMP();
  // ---- M13: agg_entity_B1 / mlp_entity_B1 second layer backward ----------------------
  for (int e = t; e < HS * HS + HS; e += NT_MID) {
    const int m = e / HS, k = e - m * HS;
    float a0 = 0.f, a1 = 0.f;
    if (m < HS) {
      int i = 0;
      for (; i + 1 < Ne; i += 2) {
        a0 = fmaf(Ps[i * HS + m], dE[i * HS + k], a0);
        a1 = fmaf(Ps[(i + 1) * HS + m], dE[(i + 1) * HS + k], a1);
      }
      if (i < Ne) a0 = fmaf(Ps[i * HS + m], dE[i * HS + k], a0);
      pb[E1_W5 + e] = a0 + a1;
    } else {
      for (int i = 0; i < Ne; ++i) a0 += dE[i * HS + k];
      pb[E1_B5 + k] = twoNe1 * a0;
    }
  }
  float* rb = rhog + (size_t)b * Ne * HS;
  if (msl < NSL) {      // rho_i[m] = sum_k W5[m][k] dE_i[k]
    float w[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) w[k] = Ws[E1_W5 + mk * HS + k];
    for (int i = msl; i < Ne; i += NSL) rb[i * HS + mk] = dot20(dE + i * HS, w, 0.f);
  }
  if (t < 4) pb[TH1 + t] = 0.f;                     // map_theta*: data-independent
  if (t < 4) pb[NP + 1 + t] = 0.f;                  // trailer / pad
  __syncthreads();
  MID_STAMP();
#undef MID_STAMP
}

// ------------------------------------------------------------------------------
// deterministic reduction of per-commit partial rows (fixed commit order per lane,
// fixed 4-way combine): block = 64 parameters x 4 commit phases
// ------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_grad_reduce(const float* __restrict__ part, int B,
                                                     int p_begin, int p_end,
                                                     float* __restrict__ out) {
  __shared__ float sh[4][64];
  const int pl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int p = p_begin + blockIdx.x * 64 + pl;
  float acc = 0.f;
  if (p < p_end) {
    int b = ph;
    for (; b + 12 < B; b += 16) {
      const float v0 = part[(size_t)b * NPART + p];
      const float v1 = part[(size_t)(b + 4) * NPART + p];
      const float v2 = part[(size_t)(b + 8) * NPART + p];
      const float v3 = part[(size_t)(b + 12) * NPART + p];
      acc += v0; acc += v1; acc += v2; acc += v3;
    }
    for (; b < B; b += 4) acc += part[(size_t)b * NPART + p];
  }
  sh[ph][pl] = acc;
  __syncthreads();
  if (ph == 0 && p < p_end) out[p - p_begin] = (sh[0][pl] + sh[1][pl]) + (sh[2][pl] + sh[3][pl]);
}

// ------------------------------------------------------------------------------
// TF1 Adam (model_2.py:336-338): train_loss = 10 CE + 0.1 loss_map + loss_para.
//   g = dCE-part (from the reduction, already x10/(B Pc)) + 0.001 v
//       + [theta] 0.1*0.01*theta/|theta|
//   lr_t = lr sqrt(1-b2^t)/(1-b1^t);  m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   var -= lr_t m / (sqrt(v) + eps)     (tensorflow/core/kernels/training_ops.cc ApplyAdam)
// ------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_adam_tf(float* __restrict__ params,
                                                  float* __restrict__ mm,
                                                  float* __restrict__ vv,
                                                  float* __restrict__ bpow,
                                                  const float* __restrict__ grad, int np,
                                                  float lr, float inv_pairs,
                                                  float* __restrict__ stats) {
  using namespace m2;
  __shared__ float red[16 * 4];
  __shared__ float sh[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float l2 = 0.f, t1 = 0.f, t2 = 0.f;
  for (int p = t; p < np; p += 1024) {
    const float w = params[p];
    l2 = fmaf(w, w, l2);
    if (p >= TH1 && p < TH1 + 2) t1 = fmaf(w, w, t1);
    if (p >= TH2 && p < TH2 + 2) t2 = fmaf(w, w, t2);
  }
  l2 = wave_sum(l2);
  t1 = wave_sum(t1);
  t2 = wave_sum(t2);
  if (lane == 0) { red[wv * 4] = l2; red[wv * 4 + 1] = t1; red[wv * 4 + 2] = t2; }
  __syncthreads();
  if (t < 3) {
    float s = 0.f;
    for (int w = 0; w < 16; ++w) s += red[w * 4 + t];
    sh[t] = s;
  }
  __syncthreads();
  const float n1 = sqrtf(sh[1]), n2 = sqrtf(sh[2]);
  const float b1p = bpow[0], b2p = bpow[1];
  const float lr_t = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  if (t == 0 && stats) {
    const float ce = grad[NP] * inv_pairs;
    const float lmap = 0.01f * (n2 + n1);
    const float lpara = 0.0005f * sh[0];
    stats[0] = ce;
    stats[1] = lmap;
    stats[2] = lpara;
    stats[3] = 10.f * ce + 0.1f * lmap + lpara;
  }
  const float b1 = 0.9f, b2 = 0.999f, ep = 1e-8f;
  for (int p = t; p < np; p += 1024) {
    const float w = params[p];
    float g = grad[p] + 0.001f * w;
    if (p >= TH1 && p < TH1 + 2) g += 0.001f * w / n1;
    if (p >= TH2 && p < TH2 + 2) g += 0.001f * w / n2;
    float m = mm[p], v = vv[p];
    m += (g - m) * (1.f - b1);
    v += (g * g - v) * (1.f - b2);
    mm[p] = m;
    vv[p] = v;
    params[p] = w - lr_t * m / (sqrtf(v) + ep);
  }
  __syncthreads();
  if (t == 0) { bpow[0] = b1p * b1; bpow[1] = b2p * b2; }
}

// ------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int smax_e(int ne) { return ne <= 128 ? 8 : 16; }
int smax_c(int nc) { return nc <= 80 ? 5 : (nc <= 128 ? 8 : 10); }

struct Work {   // workspace carve (floats)
  size_t P, rho, Esave, gam, part, total;
};

Work work_layout(const hdg_shape* s) {
  Work w;
  const size_t B = s->batch, Ne = s->ne;
  const size_t NC16 = 16 * (size_t)smax_c(s->nc);
  size_t o = 0;
  auto take = [&](size_t n) { size_t r = o; o += (n + 63) & ~(size_t)63; return r; };
  w.P = take(B * Ne * HS);
  w.rho = take(B * Ne * HS);
  w.Esave = take(2 * B * Ne * HS);
  w.gam = take(B * NC16 * NC16);
  w.part = take(B * (size_t)NPART);
  w.total = o;
  return w;
}

int check_shape(const hdg_shape* s) {
  if (!s) return fail(HDG_EINVAL, "shape is NULL");
  if (s->variant != 2)
    return fail(HDG_EINVAL, "variant %d not built (this engine implements model_2)", s->variant);
  if (s->batch < 1) return fail(HDG_EINVAL, "batch must be >= 1 (got %d)", s->batch);
  if (s->ne < 2 || s->ne > 256) return fail(HDG_EINVAL, "ne must be in [2,256] (got %d)", s->ne);
  if (s->nc < 2 || s->nc > 160) return fail(HDG_EINVAL, "nc must be in [2,160] (got %d)", s->nc);
  const MidLayout L = mid_layout(s->ne, s->nc, smax_c(s->nc));
  if ((size_t)L.total * 4 > 160 * 1024)
    return fail(HDG_EINVAL, "ne=%d nc=%d needs %zu B of LDS in k_commit_mid (> 160 KiB)", s->ne,
                s->nc, (size_t)L.total * 4);
  return 0;
}

int check_batch(const hdg_batch* bt) {
  if (!bt || !bt->x || !bt->abits || !bt->ybits || !bt->hid || !bt->nlen)
    return fail(HDG_EINVAL, "batch has a NULL device pointer");
  return 0;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail((int)e_, "%s: %s", #expr, hipGetErrorString(e_));   \
  } while (0)

template <int SMAXC, bool TRAIN>
hipError_t launch_mid(const hdg_shape* s, const hdg_batch* bt, const float* params, float* ws,
                      const Work& w, float* probs, float* logits, float ce_scale,
                      hipStream_t st) {
  const MidLayout L = mid_layout(s->ne, s->nc, SMAXC);
  const size_t lds = (size_t)L.total * 4;
  static bool attr_set = false;   // the attribute is per function; 160 KiB covers every shape
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_commit_mid<SMAXC, TRAIN>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_commit_mid<SMAXC, TRAIN>), dim3(s->batch), dim3(NT_MID), lds, st, bt->x,
                     bt->abits, bt->ybits, bt->hid, bt->nlen, params, ws + w.P, ws + w.Esave,
                     ws + w.rho, ws + w.gam, ws + w.part, probs, logits, s->ne, s->nc, ce_scale,
                     nullptr);
  return hipGetLastError();
}

template <bool TRAIN>
hipError_t dispatch_mid(const hdg_shape* s, const hdg_batch* bt, const float* params, float* ws,
                        const Work& w, float* probs, float* logits, float ce_scale,
                        hipStream_t st) {
  switch (smax_c(s->nc)) {
    case 5: return launch_mid<5, TRAIN>(s, bt, params, ws, w, probs, logits, ce_scale, st);
    case 8: return launch_mid<8, TRAIN>(s, bt, params, ws, w, probs, logits, ce_scale, st);
    default: return launch_mid<10, TRAIN>(s, bt, params, ws, w, probs, logits, ce_scale, st);
  }
}

hipError_t launch_entity(bool fwd, const hdg_shape* s, const hdg_batch* bt, const float* params,
                         float* ws, const Work& w, hipStream_t st) {
  dim3 grid(NCHUNK_E, s->batch);
  if (smax_e(s->ne) == 8) {
    if (fwd) hipLaunchKernelGGL(k_entity_fwd<8>, grid, dim3(256), 0, st, bt->x, bt->abits, params, ws + w.P, s->ne);
    else hipLaunchKernelGGL(k_entity_bwd<8>, grid, dim3(256), 0, st, bt->x, bt->abits, params, ws + w.rho, ws + w.part, s->ne);
  } else {
    if (fwd) hipLaunchKernelGGL(k_entity_fwd<16>, grid, dim3(256), 0, st, bt->x, bt->abits, params, ws + w.P, s->ne);
    else hipLaunchKernelGGL(k_entity_bwd<16>, grid, dim3(256), 0, st, bt->x, bt->abits, params, ws + w.rho, ws + w.part, s->ne);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" {

int hdg_version(void) { return HDG_ABI_VERSION; }
const char* hdg_last_error(void) { return g_err; }
int hdg_param_count(int32_t variant) { return variant == 2 ? m2::NP : -1; }
int hdg_grad_len(int32_t variant) { return variant == 2 ? GRAD_LEN : -1; }

size_t hdg_workspace_bytes(const hdg_shape* shape) {
  if (check_shape(shape)) return 0;
  return work_layout(shape).total * sizeof(float);
}

int hdg_fwd_bwd_events(const hdg_shape* s, const hdg_batch* bt, const float* params,
                       float* grad, hdg_outputs* out, void* workspace, void* stream,
                       void* const* events) {
  if (int rc = check_shape(s)) return rc;
  if (int rc = check_batch(bt)) return rc;
  if (!params || !grad || !workspace) return fail(HDG_EINVAL, "NULL params/grad/workspace");
  hipStream_t st = (hipStream_t)stream;
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const int bg = s->batch_global > 0 ? s->batch_global : s->batch;
  const float ce_scale = 10.f / ((float)bg * (float)(s->nc * (s->nc - 1)));
  auto mark = [&](int k) -> hipError_t {
    return events ? hipEventRecord((hipEvent_t)events[k], st) : hipSuccess;
  };
  HIP_TRY(mark(0));
  HIP_TRY(launch_entity(true, s, bt, params, ws, w, st));
  HIP_TRY(mark(1));
  HIP_TRY(dispatch_mid<true>(s, bt, params, ws, w, out ? out->probs : nullptr,
                             out ? out->logits : nullptr, ce_scale, st));
  HIP_TRY(mark(2));
  HIP_TRY(launch_entity(false, s, bt, params, ws, w, st));
  HIP_TRY(mark(3));
  hipLaunchKernelGGL(k_grad_reduce, dim3((GRAD_LEN + 63) / 64), dim3(256), 0, st,
                     ws + w.part, s->batch, 0, GRAD_LEN, grad);
  HIP_TRY(hipGetLastError());
  HIP_TRY(mark(4));
  return 0;
}

int hdg_fwd_bwd(const hdg_shape* s, const hdg_batch* bt, const float* params, float* grad,
                hdg_outputs* out, void* workspace, void* stream) {
  return hdg_fwd_bwd_events(s, bt, params, grad, out, workspace, stream, nullptr);
}

int hdg_debug_mid_stamps(const hdg_shape* s, const hdg_batch* bt, const float* params,
                         void* workspace, unsigned long long* stamps, void* stream) {
  if (int rc = check_shape(s)) return rc;
  if (int rc = check_batch(bt)) return rc;
  if (smax_c(s->nc) != 5) return fail(HDG_EINVAL, "phase stamps are built for nc <= 80");
  hipStream_t st = (hipStream_t)stream;
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const MidLayout L = mid_layout(s->ne, s->nc, 5);
  HIP_TRY(hipFuncSetAttribute((const void*)k_commit_mid<5, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipLaunchKernelGGL((k_commit_mid<5, true, true>), dim3(s->batch), dim3(NT_MID),
                     (size_t)L.total * 4, st, bt->x, bt->abits, bt->ybits, bt->hid, bt->nlen,
                     params, ws + w.P, ws + w.Esave, ws + w.rho, ws + w.gam, ws + w.part, nullptr,
                     nullptr, s->ne, s->nc, 1.f, stamps);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_adam_tf(const hdg_shape* s, hdg_state* state, const float* grad, float lr, float* stats,
                void* stream) {
  if (int rc = check_shape(s)) return rc;
  if (!state || !state->params || !state->adam_m || !state->adam_v || !state->beta_pow || !grad)
    return fail(HDG_EINVAL, "NULL state/grad pointer");
  const int bg = s->batch_global > 0 ? s->batch_global : s->batch;
  const float inv_pairs = 1.f / ((float)bg * (float)(s->nc * (s->nc - 1)));
  hipLaunchKernelGGL(k_adam_tf, dim3(1), dim3(1024), 0, (hipStream_t)stream, state->params,
                     state->adam_m, state->adam_v, state->beta_pow, grad, m2::NP, lr, inv_pairs,
                     stats);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_train_step(const hdg_shape* s, const hdg_batch* bt, hdg_state* state, float lr,
                   hdg_outputs* out, float* grad, void* workspace, void* stream) {
  if (!state) return fail(HDG_EINVAL, "NULL state");
  if (int rc = hdg_fwd_bwd(s, bt, state->params, grad, out, workspace, stream)) return rc;
  return hdg_adam_tf(s, state, grad, lr, out ? out->stats : nullptr, stream);
}

int hdg_forward(const hdg_shape* s, const hdg_batch* bt, const float* params, hdg_outputs* out,
                float* ce_sum, void* workspace, void* stream) {
  if (int rc = check_shape(s)) return rc;
  if (int rc = check_batch(bt)) return rc;
  if (!params || !workspace) return fail(HDG_EINVAL, "NULL params/workspace");
  hipStream_t st = (hipStream_t)stream;
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  HIP_TRY(launch_entity(true, s, bt, params, ws, w, st));
  HIP_TRY(dispatch_mid<false>(s, bt, params, ws, w, out ? out->probs : nullptr,
                              out ? out->logits : nullptr, 0.f, st));
  if (ce_sum) {
    hipLaunchKernelGGL(k_grad_reduce, dim3(1), dim3(256), 0, st, ws + w.part, s->batch, m2::NP,
                       m2::NP + 1, ce_sum);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

}  // extern "C"
