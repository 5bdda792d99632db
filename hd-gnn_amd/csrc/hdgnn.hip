// hdgnn.hip -- MI355X (gfx950, CDNA4) engine for the HD-GNN/S training step.
//
// One training step of model_2.graph2graph (model_2.py:86-130 forward, 336-338
// loss + Adam) runs as three launches on the caller's stream:
//
//   k_commit_step [B]       one 1024-thread block per commit: entity pair stage,
//                           E3 node MLP, entity->hunk cross-graph sum, hunk pair MLP
//                           sums, edge classifier + softmax-CE (fwd+bwd), the whole
//                           backward down to dW1 of the entity pair MLP
//                           (model_2.py:94-130, 161-324)
//   k_grad_reduce [P/64]    deterministic per-commit partial sum (fixed commit order)
//   k_adam_tf     [1]       loss_para / loss_map gradients + TF1 ApplyAdam
//
// plus, once per uploaded batch, k_prep_sort / k_prep_counts (hdg_prepare): the
// parameter-independent tables of a commit (x sort order, transposed class bits,
// cross-graph count matrices).
//
// Algebra used (exact up to fp32 re-association; derivation in DESIGN.md section 3):
//   first-layer pre-activation of a pair MLP on [x_i, x_j, 1-a, a] = u_i + v_j + a*d;
//   second layers are linear and commute with the row/column sums, so they run once
//   per NODE.  Entity pairs: u, v are affine in the scalar x, so the a = 0 relu sums
//   are prefix/suffix sums over the x-sorted order (O(Ne log nd) per hidden unit)
//   plus sparse corrections for a = 1.  Hunk pairs run as dense register tiles.
#include <hip/hip_runtime.h>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "hdgnn.h"
#include "hdgnn_internal.h"

namespace {

constexpr int HS = 20;              // h_size = De_e = De_er (model_2.py:163, 192, 247, 306)
constexpr int NT_MID = 1024;        // k_commit_step block
constexpr int KK_MID = 5;           // hidden units per pair-tile chunk in k_commit_step

// model_2 flat parameter offsets (tf.global_variables order)
namespace m2 {
constexpr int E1_W1 = 0, E1_B1 = 80, E1_W5 = 100, E1_B5 = 500;
constexpr int E3_W1 = 520, E3_B1 = 940, E3_W2 = 960, E3_B2 = 980;
constexpr int H1_W1 = 981, H1_B1 = 1181, H1_W2 = 1201, H1_B2 = 1601;
constexpr int H2_W1 = 1621, H2_B1 = 2061, H2_W2 = 2081, H2_B2 = 2121;
constexpr int TH1 = 2123, TH2 = 2125, NP = 2127;
}  // namespace m2
constexpr int GRAD_LEN = m2::NP + HDG_TRAILER;
constexpr int NPART = (GRAD_LEN + 3) & ~3;   // per-block partial row: NP grads + trailer

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

// row16_sum of N values as fused v_add_f32_dpp (one VALU op per value and step; the
// compiler otherwise splits some into v_mov_dpp + v_add).  A DPP read needs 2 wait states
// after the VALU write of its operand, and the compiler's hazard recognizer does not look
// inside inline asm: it may schedule a producer (or a register copy) right before any asm
// statement.  So each group of 3-4 values is reduced by ONE asm block that opens with the
// s_nop covering its producers; inside, the steps run over the group's values in turn
// (each DPP read >= 2 instructions after the write it depends on).
#define HDG_DPP_STEP(ctl, n) "v_add_f32_dpp %" #n ", %" #n ", %" #n " " ctl \
  " row_mask:0xf bank_mask:0xf\n\t"
#define HDG_DPP_STEP3(ctl) HDG_DPP_STEP(ctl, 0) HDG_DPP_STEP(ctl, 1) HDG_DPP_STEP(ctl, 2)
#define HDG_DPP_STEP4(ctl) HDG_DPP_STEP3(ctl) HDG_DPP_STEP(ctl, 3)
#define HDG_DPP_STEP5(ctl) HDG_DPP_STEP4(ctl) HDG_DPP_STEP(ctl, 4)
#define HDG_DPP_BLOCK(S) "s_nop 1\n\t" S("row_mirror") S("row_half_mirror") \
  S("quad_perm:[2,3,0,1]") S("quad_perm:[1,0,3,2]")
__device__ __forceinline__ void row16_sum3(float* v) {
  asm volatile(HDG_DPP_BLOCK(HDG_DPP_STEP3) : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]));
}
__device__ __forceinline__ void row16_sum4(float* v) {
  asm volatile(HDG_DPP_BLOCK(HDG_DPP_STEP4) : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
__device__ __forceinline__ void row16_sum5(float* v) {
  asm volatile(HDG_DPP_BLOCK(HDG_DPP_STEP5)
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]));
}
#undef HDG_DPP_BLOCK
#undef HDG_DPP_STEP5
#undef HDG_DPP_STEP4
#undef HDG_DPP_STEP3
#undef HDG_DPP_STEP
#ifndef HDG_SETPRIO  // wave priority by progress in the pair passes, E1, E2 and M7 (0 = off)
#define HDG_SETPRIO 1
#endif
// Wave priority by progress.  The SIMD's issue arbiter favours the oldest wave, so in a
// phase of equal per-wave work wave 0 of each SIMD finishes first and the youngest runs its
// last trips alone, with nothing to hide its latencies (the per-wave stamps show the
// stagger: E1 done at 1.8 / 2.1 / 2.6 / 3.1 us for waves 0-3 / 4-7 / 8-11 / 12-15).  A wave
// lowers its priority as it passes trips / milestones, so waves that are behind get the
// issue slots first and the SIMD's waves finish together: pair passes M5 / M8 / M10
// 4.60 / 5.56 / 7.04 -> 4.20 / 5.08 / 6.52 us, E1 3.12 -> 2.80, median block 54.8 -> 53.2 us
// (tools/gpu_ph_ab.sh, two runs each).  Priority 3, 2, 1, 0 for trips 0, 1, 2, later
// (s_setprio takes an immediate).
__device__ __forceinline__ void trip_prio(int s) {
  if (s == 0) __builtin_amdgcn_s_setprio(3);
  else if (s == 1) __builtin_amdgcn_s_setprio(2);
  else if (s == 2) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
#ifndef HDG_HOIST   // pair tiles: the columns' B (and MODE 1 wc) operands held in registers
#define HDG_HOIST 1  // for the whole sweep instead of re-read from LDS every 16-row trip
#endif
#ifndef HDG_XROW
#define HDG_XROW 1
#endif
#ifndef HDG_QMAP   // pair tiles: quad unit map (16-byte unit quads, ds_read_b128; below)
#define HDG_QMAP 1
#endif
#ifndef HDG_QTAIL  // quad map: tail units of the column operands by 8-byte reads (1 B, 2 wc)
#define HDG_QTAIL 0
#endif
// Row sums of 5 values over a 16-lane DPP row as a transposed butterfly: 12 DPP adds
// instead of 20, no selects -- at the two bank-crossing levels (row_mirror: lanes 0-7 vs
// 8-15; row_half_mirror: banks 0, 2 vs 1, 3) one register takes the a-values' sums in
// one half of the lanes and the b-values' in the other through the DPP bank mask; the
// last two levels reduce the remaining two values in full.  Afterwards (tj = lane & 15):
//   tj 0-3: y0 = v0, y1 = v1;  4-7: y0 = v2, y1 = v1;  8-11: y0 = v3, y1 = v4;
//   12-15: y0 = v2, y1 = v4   (every lane of a group holds the same bits).
// Hazards: one s_nop 1 for the producers of v, then every DPP read >= 2 wait states after
// the write of its operand (the instruction order and the two inner s_nops ensure it).
__device__ __forceinline__ void row16_xsum5(const float* v, float& y0, float& y1) {
  float x0, x1, x2;
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %2, %7, %7 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %0, %5, %5 row_mirror row_mask:0xf bank_mask:0x3\n\t"
      "v_add_f32_dpp %0, %8, %8 row_mirror row_mask:0xf bank_mask:0xc\n\t"
      "v_add_f32_dpp %1, %6, %6 row_mirror row_mask:0xf bank_mask:0x3\n\t"
      "v_add_f32_dpp %1, %9, %9 row_mirror row_mask:0xf bank_mask:0xc\n\t"
      "v_add_f32_dpp %3, %0, %0 row_half_mirror row_mask:0xf bank_mask:0x5\n\t"
      "v_add_f32_dpp %3, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xa\n\t"
      "v_add_f32_dpp %4, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %3, %3, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %4, %4, %4 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_add_f32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %4, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(y0), "=&v"(y1)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]));
}

// N = 3 G + R (R < 3): G - 1 groups of 3 and one of 3 + R
template <int N>
__device__ __forceinline__ void row16_sums(float (&v)[N]) {
  static_assert(N >= 3, "row16_sums needs >= 3 values (groups of 3-5 per asm block)");
  constexpr int G = N / 3, R = N % 3;
#pragma unroll
  for (int g = 0; g + 1 < G; ++g) row16_sum3(v + 3 * g);
  if constexpr (R == 0) row16_sum3(v + 3 * (G - 1));
  else if constexpr (R == 1) row16_sum4(v + 3 * (G - 1));
  else row16_sum5(v + 3 * (G - 1));
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

// x <-> y exchange of DPP rows: swap32 trades x's lanes 32-63 for y's lanes 0-31, swap16
// x's rows 1, 3 for y's rows 0, 2 (v_permlane{32,16}_swap, same hazard handling as above)
__device__ __forceinline__ void swap32(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void swap16(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}

// Transposed cross-row reduction of N per-lane values: value n summed over the 4 DPP rows
// (lane columns kept apart) with one swap + one add per PAIR of values at each of the two
// levels, instead of two swaps + two adds per value.  Afterwards vector i (i < H2) holds
// value i in row 0, i + H2 in row 1, i + H in row 2 and i + H + H2 in row 3, H = ceil(N/2),
// H2 = ceil(H/2); store(n, row_value) is called by every lane for the valid n of its row.
template <int N, class F>
__device__ __forceinline__ void xrow_sums(const float (&v)[N], const int lane, F store) {
  constexpr int H = (N + 1) / 2, H2 = (H + 1) / 2;
  float a[H], b[H2];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    float x = v[i], y = (i + H < N) ? v[i + H] : 0.f;
    swap32(x, y);
    a[i] = x + y;              // rows 0,1: value i; rows 2,3: value i + H
  }
#pragma unroll
  for (int i = 0; i < H2; ++i) {
    float x = a[i], y = (i + H2 < H) ? a[i + H2] : 0.f;
    swap16(x, y);
    b[i] = x + y;
  }
  const int r = lane >> 4;
  const int off = ((r & 1) ? H2 : 0) + ((r & 2) ? H : 0);
#pragma unroll
  for (int i = 0; i < H2; ++i) {
    const bool ok = ((r & 1) ? (i + H2 < H) : true) && (i + off < N);
    if (ok) store(i + off, b[i]);
  }
}

// Full 64-lane sums of N values: xrow_sums, then one 16-lane DPP reduction per vector;
// store(n, total) runs on lane 0 of the row that holds n.
template <int N, class F>
__device__ __forceinline__ void wave_sums(const float (&v)[N], const int lane, F store) {
  constexpr int H = (N + 1) / 2, H2 = (H + 1) / 2;
  float a[H], b[H2];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    float x = v[i], y = (i + H < N) ? v[i + H] : 0.f;
    swap32(x, y);
    a[i] = x + y;
  }
#pragma unroll
  for (int i = 0; i < H2; ++i) {
    float x = a[i], y = (i + H2 < H) ? a[i + H2] : 0.f;
    swap16(x, y);
    b[i] = row16_sum(x + y);
  }
  if ((lane & 15) == 0) {
    const int r = lane >> 4;
    const int off = ((r & 1) ? H2 : 0) + ((r & 2) ? H : 0);
#pragma unroll
    for (int i = 0; i < H2; ++i) {
      const bool ok = ((r & 1) ? (i + H2 < H) : true) && (i + off < N);
      if (ok) store(i + off, b[i]);
    }
  }
}

__device__ __forceinline__ float reluf(float v) { return fmaxf(v, 0.f); }
// ln x for x in [1, 2] (the two-class CE's log(1 + e^-|d|)): v_log_f32 (log2, ~1 ulp, no
// denormal range to guard) times ln 2 -- 2 VALU ops where logf expands to a denormal-scaled,
// split-constant sequence of ~11
__device__ __forceinline__ float ln_1to2(float x) { return __builtin_amdgcn_logf(x) * 0.693147182f; }

// padding / masked-row value of the pair-tile operands: far below any real pre-activation
// but finite, so that z [z > 0] (MODE 0) and [z > 0] w (MODE 1, 2) are 0, never inf * 0
constexpr float PADNEG = -1e30f;

typedef float f2 __attribute__((ext_vector_type(2)));   // packed fp32 (v_pk_* ops)

// [z > 0] for two lanes of a packed pair in ONE VALU op: clamp(z * 2^126, 0, 1) on
// v_pk_mul_f32 (exact for every normal z; -0, NaN -> 0).  Used as step2(z) * w, which
// needs w finite wherever z <= 0 (padding rows / columns are kept finite).
__device__ __forceinline__ f2 step2(f2 z) {
  f2 r;
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(z), "v"((f2){0x1p126f, 0x1p126f}));
  return r;
}

// [x + c > 0] for a packed pair in ONE op where only the step of the sum is used (the
// backward passes' masks): clamp(fma(x, 2^64, c 2^64)).  The fma rounds the exact
// (x + c) 2^64 once: 0 for x + c <= 0 (-0, NaN: 0), 1 for every x + c >= 2^-64, so it
// differs from step2(fl(x + c)) only for 0 < x + c < 2^-64.  cs = c 2^64 (exact and finite
// for |c| < 2^63; PADNEG 2^64 = -inf masks the pair).
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
//   MODE 2  e = [z > 0] * gam[i][j]        , ysum += y*e                 (pair weights;
//           GFULL: gam (in LDS) finite on every swept row for j < 16 SMAX, 0 on the diagonal
//           and for j >= N, read unmasked; else clamped reads, diagonal / padding masked)
//   Rout[i] = sum_j e_ij   Cout[j] = sum_i e_ij   (diagonal INCLUDED for MODE 0/1:
//   callers subtract it; MODE 2 masks it)
// Rows swept: i = rmul * r + radd, r = 0, 1, ... while i < N (a block pair splits the rows
// by parity: rmul = 2, radd = half); Cout then holds the partial column sums of those rows.
// A, B, wr, wc, Rout, Cout: LDS [node][LD] (rows/cols >= N padded with PADNEG or -inf in
// A/B; MODE 0 needs the finite PADNEG).
// Rout may alias A and Cout may alias B (rows are consumed before they are written,
// columns are written after the closing barrier).  cred: 4*16*SMAX*KK + 8*KK words.
// Every thread of the BLOCK must call this the same number of times (barriers).
// ------------------------------------------------------------------------------
template <int SMAX, int KK>
constexpr int tile_cred_words() { return 4 * 16 * SMAX * KK + 8 * KK; }

// quad unit map of the pair tiles: 4 groups of KK = 5 of the 20 units, group g's pairs are
// the 16-byte-aligned units 4g..4g+3 of a row (row pitch LD a multiple of 4 words)
template <int KK, int LD>
constexpr bool pair_qmap() { return HDG_QMAP && KK == 5 && LD % 4 == 0; }

// the KP packed pairs of units p0, p0 + 1, ... at q (LDS): one 16-byte read when QM
template <bool QM, int KP>
__device__ __forceinline__ void ld_pairs(const float* q, f2* out) {
  if constexpr (QM && KP == 2) {
    const float4 v = *reinterpret_cast<const float4*>(q);
    out[0] = (f2){v.x, v.y};
    out[1] = (f2){v.z, v.w};
  } else {
#pragma unroll
    for (int p = 0; p < KP; ++p) out[p] = *reinterpret_cast<const f2*>(q + 2 * p);
  }
}

// a row's tail unit (row base r): QM reads the 8-byte pair {16 + (g & ~1), +1} -- a
// ds_read_b64 (mod-64 banks: 16 columns at pitch 20 on distinct banks) instead of a
// 4-byte read whose mod-32 banks repeat every 8 columns -- and takes its half
template <bool QM>
__device__ __forceinline__ float ld_tail(const float* r, const int ktl, const int grp) {
  if constexpr (QM) {
    const f2 v = *reinterpret_cast<const f2*>(r + 16 + (grp & ~1));
    return (grp & 1) ? v.y : v.x;
  } else {
    return r[ktl];
  }
}

// Column closing of a pair pass: element e = (node j, local unit k) of the group's
// column sums is the fixed-order sum of the 4 waves' partials in cred.  Every partial
// of the thread is loaded before the first add (one LDS round trip).  fix(j, unit, v)
// stores it (NoFix: Cout[j][unit] = v); a caller's fix also finishes node j's row value
// (diagonal pair removed, classifier c applied) -- rows are complete at this point.
struct NoFix {};
template <int NEL, int KK, class KOF, class FIX, class DFL>
__device__ __forceinline__ void close_columns(const float* cred, const int N, const int t,
                                              KOF kof, FIX fix, DFL dfl) {
  constexpr int NU = (NEL + 255) / 256;
  float c[NU][4];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int e = t + 256 * u;
#pragma unroll
    for (int q = 0; q < 4; ++q) c[u][q] = e < NEL ? cred[e + q * NEL] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int e = t + 256 * u;
    const int j = e / KK, k = e - j * KK;
    const float v = ((c[u][0] + c[u][1]) + c[u][2]) + c[u][3];
    if (e < NEL && j < N) {
      if constexpr (__is_same(FIX, NoFix)) dfl(j, kof(k), v);
      else fix(j, kof(k), v);
    }
  }
}

template <int KK, int SMAX, int MODE, int LD, int ABL = 0, bool GFULL = false, class FIX = NoFix>
__device__ __forceinline__ void pair_tile(
    const int N, const int t, const float* A, const float* Bv, const int k0,
    const float* __restrict__ dl, const uint32_t* __restrict__ bits, const int W,
    const float* __restrict__ wr, const float* __restrict__ wc,
    const float* __restrict__ gam, const int gld, float* Rout, float* Cout,
    float* __restrict__ ysum, float* __restrict__ cred, const int rmul = 1, const int radd = 0,
    FIX fix = FIX{}, const int ncol = -1, const int wstride = -1, const int doff = 0) {
  typedef float p2 __attribute__((ext_vector_type(2)));
  constexpr int NP16 = 16 * SMAX;
  // a rectangular block of the pair grid (the general path's tiled passes): N rows, NCOL
  // columns, the rows' bit words at stride WS (W of them from the block's first column on),
  // global column = global row + doff on the diagonal; the fused kernel's square grid by
  // default
  const int NCOL = ncol < 0 ? N : ncol, WS = wstride < 0 ? W : wstride;
  constexpr int NW = (SMAX + 1) / 2;
  constexpr int KP = KK / 2, KT = KK & 1;      // packed fp32 pairs (v_pk_*) + odd tail
  // SIMD balance: waves 4g + w of a block share one SIMD for every group g (workgroup waves
  // are dealt to the 4 SIMDs cyclically), so group g's wave w takes the tile rows of
  // ti-block (w + g) & 3, and a wave whose rows of a trip all lie past the sweep skips the
  // trip: the partial last trip's work lands on different SIMDs in the 4 groups
  const int grp = k0 / KK;
  const int tj = t & 15, ti = ((t >> 4) + 4 * grp) & 15, lane = t & 63, wv = t >> 6;
  const int wrow = __builtin_amdgcn_readfirstlane(4 * ((wv + grp) & 3));   // wave's first ti
  // hidden units of the group: the packed pairs start at the even unit kpb, so every pair
  // is one 8-byte-aligned LDS read at an immediate offset from a per-thread base; the unit
  // left over is the tail ktl.  Quad map (QM): group g takes units 4g..4g+3 (one 16-byte
  // read per row: ds_read_b128, whose 16-lane groups see 16 distinct columns on 64 banks)
  // and the tail 16 + g; otherwise units [k0, k0 + KK), pairs from k0 or k0 + 1 (the
  // compiler merges the two 8-byte reads into a ds_read2_b64, whose mod-32 banks put
  // columns j and j + 8 of a row pitch of 20 words on one bank: 2-way on every read)
  constexpr bool QM = pair_qmap<KK, LD>();
  const int kpb = QM ? 4 * grp : k0 + (k0 & 1);
  const int ktl = QM ? 16 + grp : ((k0 & 1) ? k0 : k0 + KK - 1);
  auto kof = [&](const int k) { return k < 2 * KP ? kpb + k : ktl; };   // local -> unit
  const int nown = (N - radd + rmul - 1) / rmul;   // rows i = rmul r + radd < N
  const int S = (nown + 15) >> 4;
  const p2 z2 = {0.f, 0.f};
  // row16_xsum5's storing lanes and their units (KK = 5)
  const bool xst = tj == 0 || tj == 4 || tj == 8;
  const int xk0 = kof(tj == 0 ? 0 : (tj == 4 ? 2 : 3)), xk1 = kof(tj < 8 ? 1 : 4);

  p2 cacc2[SMAX][KP > 0 ? KP : 1];
  float cacct[SMAX];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) {
#pragma unroll
    for (int p = 0; p < KP; ++p) cacc2[c][p] = z2;
    cacct[c] = 0.f;
  }
  p2 yacc2[KP > 0 ? KP : 1], dk2[KP > 0 ? KP : 1];
  float yacct = 0.f, dkt = KT ? dl[ktl] : 0.f;
#pragma unroll
  for (int p = 0; p < KP; ++p) yacc2[p] = z2;
  ld_pairs<QM, KP>(dl + kpb, dk2);

  // loop-invariant column operands (the trip loop's stores to Rout may alias A in general,
  // so the compiler does not hoist these LDS reads itself; B / wc are not written in the loop)
  // HDG_HOIST bits: 1 MODE 0's B (M5), 2 MODE 1's wc, 4 MODE 2's B (M8), 8 MODE 1's B (M10)
  constexpr bool HB = (MODE == 0 && (HDG_HOIST & 1)) || (MODE == 2 && (HDG_HOIST & 4)) ||
                      (MODE == 1 && (HDG_HOIST & 8));
  constexpr bool HW = (HDG_HOIST & 2) && MODE == 1;
  p2 bcol[HB ? SMAX : 1][KP > 0 ? KP : 1], wcol[HW ? SMAX : 1][KP > 0 ? KP : 1];
  float bcolt[HB ? SMAX : 1], wcolt[HW ? SMAX : 1];
  if constexpr (HB || HW) {
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
      const int j = tj + 16 * c;
      if constexpr (HB) ld_pairs<QM, KP>(Bv + j * LD + kpb, bcol[c]);
      if constexpr (HW) ld_pairs<QM, KP>(wc + j * LD + kpb, wcol[c]);
      if constexpr (HB) bcolt[c] = KT ? ld_tail<QM && (HDG_QTAIL & 1)>(Bv + j * LD, ktl, grp) : 0.f;
      if constexpr (HW) wcolt[c] = KT ? ld_tail<QM && (HDG_QTAIL & 2)>(wc + j * LD, ktl, grp) : 0.f;
    }
  }
  for (int s = 0; s < S; ++s) {
    // waves still on an earlier trip get the issue arbiter first (it otherwise favours
    // the oldest wave, which finishes its trips first and leaves the SIMD to one wave at
    // the end of the pass)
    if constexpr (HDG_SETPRIO) trip_prio(s);
    if (wrow + 16 * s >= nown) continue;    // wave-uniform: no row of this wave in the trip
    const int r = ti + 16 * s;
    const int i = rmul * r + radd;
    const bool iv = r < nown;
    p2 a2[KP > 0 ? KP : 1], rw2[KP > 0 ? KP : 1], racc2[KP > 0 ? KP : 1];
    // rows past the sweep read the first swept row and are masked to A = PADNEG, w = 0
    // (e = 0): the sweep may run past the padded buffer when the rows are split by parity
    const int ib = iv ? i : radd;       // past the sweep: the first swept row (own, finite)
    const float* Ai = A + ib * LD;
    // masks applied arithmetically (that row's values are finite): every load of the sweep's
    // row operands is unconditional, so none of them is sunk into an exec-masked branch
    // with its own LDS round trip
    const float addm = iv ? 0.f : PADNEG, mulm = iv ? 1.f : 0.f;
    const p2 addm2 = {addm, addm}, mulm2 = {mulm, mulm};
    ld_pairs<QM, KP>(Ai + kpb, a2);
    if constexpr (MODE == 1) ld_pairs<QM, KP>(wr + ib * LD + kpb, rw2);
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      a2[p] += addm2;
      if constexpr (MODE != 0 && HDG_STEPF) a2[p] *= (p2){STEP_S, STEP_S};   // stepf2's c
      if constexpr (MODE == 1)
        rw2[p] *= mulm2;
      else
        rw2[p] = z2;
      racc2[p] = z2;
    }
    const float at = KT ? Ai[ktl] + addm : 0.f;
    const float rwt = (MODE == 1 && KT) ? wr[ib * LD + ktl] * mulm : 0.f;
    float racct = 0.f;
    uint32_t wrow[NW];
    const uint32_t bmask = iv ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int q = 0; q < NW; ++q)        // clamped load, masked value
      wrow[q] = bits[ib * WS + (q < W ? q : 0)] & (q < W ? bmask : 0u);
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
      const int j = tj + 16 * c;
      const float af = (ABL & 1) ? 0.f : (float)((wrow[c >> 1] >> (tj + 16 * (c & 1))) & 1u);
      const p2 af2 = {af, af};
      float g = 0.f;
      if constexpr (MODE == 2 && GFULL) {   // rows past the sweep read the first swept row
        g = gam[(iv ? i : radd) * gld + j];  // (A = -inf zeroes their terms)
      } else if constexpr (MODE == 2) {      // clamped load, selected (not multiplied:
        const int ic = iv ? i : N - 1, jc = j < NCOL ? j : NCOL - 1;   // garbage * 0 can be NaN)
        const float gl = gam[ic * gld + jc];
        g = (iv && j < NCOL && j + doff != i) ? gl : 0.f;
      }
      const float gy = af * g;             // MODE 2: exact (af is 0 or 1)
      const float* Bj = Bv + j * LD;
      p2 bbv[KP > 0 ? KP : 1], wcv[KP > 0 ? KP : 1];
      if constexpr (!HB) ld_pairs<QM, KP>(Bj + kpb, bbv);
      if constexpr (MODE == 1 && !HW) ld_pairs<QM, KP>(wc + j * LD + kpb, wcv);
#pragma unroll
      for (int p = 0; p < KP; ++p) {
        p2 bb;
        if constexpr (HB) bb = bcol[c][p];
        else bb = bbv[p];
        const p2 zb = __builtin_elementwise_fma(af2, dk2[p], bb);
        const p2 z = a2[p] + zb;          // used by MODE 0 (MODE 1, 2: stepf2(zb, a 2^64))
        if constexpr (MODE == 0) {
          // relu(z) accumulated as z [z > 0]: one packed step and two packed fma (no packed
          // max on gfx950: relu was two scalar v_max plus two packed adds)
          const p2 sz = step2(z);
          racc2[p] = __builtin_elementwise_fma(z, sz, racc2[p]);
          cacc2[c][p] = __builtin_elementwise_fma(z, sz, cacc2[c][p]);
        } else if constexpr (MODE == 2) {
          // w = g is one value per pair: [z > 0] g and [z > 0] a g as one fma each (the
          // products are exact: the same bits as multiply, then add)
          const p2 sz = HDG_STEPF ? stepf2(zb, a2[p]) : step2(z), g2 = {g, g}, gy2 = {gy, gy};
          yacc2[p] = __builtin_elementwise_fma(sz, gy2, yacc2[p]);
          racc2[p] = __builtin_elementwise_fma(sz, g2, racc2[p]);
          cacc2[c][p] = __builtin_elementwise_fma(sz, g2, cacc2[c][p]);
        } else {
          p2 w;
          if constexpr (HW) w = rw2[p] + wcol[c][p];
          else w = rw2[p] + wcv[p];
          const p2 e = (HDG_STEPF ? stepf2(zb, a2[p]) : step2(z)) * w;
          yacc2[p] = __builtin_elementwise_fma(af2, e, yacc2[p]);
          racc2[p] += e;
          cacc2[c][p] += e;
        }
      }
      if constexpr (KT) {
        const float z = at + fmaf(af, dkt, HB ? bcolt[c] : ld_tail<QM && (HDG_QTAIL & 1)>(Bj, ktl, grp));
        float e;
        if constexpr (MODE == 0) {
          e = reluf(z);
        } else {
          const float w =
              (MODE == 1) ? (rwt + (HW ? wcolt[c] : ld_tail<QM && (HDG_QTAIL & 2)>(wc + j * LD, ktl, grp))) : g;
          e = (z > 0.f) ? w : 0.f;
          yacct = fmaf(af, e, yacct);
        }
        racct += e;
        cacct[c] += e;
      }
    }
    float rs[KK];
#pragma unroll
    for (int p = 0; p < KP; ++p) {     // unpack first: DPP adds do not fuse on 64-bit halves
      rs[2 * p] = racc2[p].x;
      rs[2 * p + 1] = racc2[p].y;
    }
    if constexpr (KT) rs[KK - 1] = racct;
    if constexpr (KK == 5 && HDG_XROW && !(ABL & 2)) {
      // transposed: lanes tj = 0, 4, 8 store two row values each (tj = 4's y1 is v1, the
      // same bits tj = 0 stores at the same address)
      float y0, y1;
      row16_xsum5(rs, y0, y1);
      if (xst && iv) {
        Rout[i * LD + xk0] = y0;
        Rout[i * LD + xk1] = y1;
      }
    } else {
      if constexpr (!(ABL & 2)) row16_sums(rs);
      if (tj == 0 && iv) {     // one predicated block: no per-value branch / address spill
#pragma unroll
        for (int k = 0; k < KK; ++k) Rout[i * LD + kof(k)] = rs[k];
      }
    }
  }
  float cacc[SMAX][KK], yacc[KK];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      cacc[c][2 * p] = cacc2[c][p].x;
      cacc[c][2 * p + 1] = cacc2[c][p].y;
    }
    if constexpr (KT) cacc[c][KK - 1] = cacct[c];
  }
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    yacc[2 * p] = yacc2[p].x;
    yacc[2 * p + 1] = yacc2[p].y;
  }
  if constexpr (KT) yacc[KK - 1] = yacct;
  if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(0);
  // close the column partials: 4 ti per wave by shuffles, then 4 waves via LDS
  float* credy = cred + 4 * NP16 * KK;
  {                          // column partials summed over the wave's 4 rows (transposed)
    float cf[SMAX * KK];
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
#pragma unroll
      for (int k = 0; k < KK; ++k) cf[c * KK + k] = cacc[c][k];
    float* cw = cred + (wv * NP16 + tj) * KK;
    xrow_sums(cf, lane, [&](int n, float x) {
      const int c = n / KK, k = n - c * KK;
      cw[16 * c * KK + k] = x;
    });
  }
  if constexpr (MODE != 0) {
    wave_sums(yacc, lane, [&](int k, float x) { credy[wv * KK + k] = x; });
  }
  __syncthreads();
  close_columns<NP16 * KK, KK>(cred, NCOL, t, kof, fix,
                               [&](int j, int kk, float v) { Cout[j * LD + kk] = v; });
  if constexpr (MODE != 0) {
    if (t < KK) ysum[kof(t)] = credy[t] + credy[KK + t] + credy[2 * KK + t] + credy[3 * KK + t];
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------
// pair_tile32: the same passes (same arguments, buffers and results as pair_tile) on
// 8 x 32 thread tiles, for the wide hunk grids (NC16 = 128, 160: Nc in (80, 160]).
// Thread (ti, tj) = (t>>5, t&31) owns rows i = ti + 8s and columns j = tj + 32c, so a
// thread holds SMAX16/2 column accumulators per unit instead of SMAX16: the 16-wide
// tiles' 40-50 accumulators spilled to scratch inside the sweeps (448 B per lane at
// SMAX16 = 10).  A wave is two tile rows: row sums close with a 16-lane DPP reduction
// plus one permlane16 swap (the two DPP rows of a half-wave), column partials with one
// permlane32 swap per pair of values, then the 4 waves through LDS as in pair_tile.
// ------------------------------------------------------------------------------
template <int KK, int SMAX16, int MODE, int LD, bool GFULL = false, class FIX = NoFix>
__device__ __forceinline__ void pair_tile32(
    const int N, const int t, const float* A, const float* Bv, const int k0,
    const float* __restrict__ dl, const uint32_t* __restrict__ bits, const int W,
    const float* __restrict__ wr, const float* __restrict__ wc,
    const float* __restrict__ gam, const int gld, float* Rout, float* Cout,
    float* __restrict__ ysum, float* __restrict__ cred, const int rmul = 1, const int radd = 0,
    FIX fix = FIX{}) {
  typedef float p2 __attribute__((ext_vector_type(2)));
  static_assert(SMAX16 % 2 == 0, "32-wide tiles cover an even count of 16-column tiles");
  constexpr int NP16 = 16 * SMAX16;
  constexpr int SMAX = SMAX16 / 2;
  constexpr int KP = KK / 2, KT = KK & 1;
  const int grp = k0 / KK;                     // SIMD-balanced rows, as in pair_tile
  const int tj = t & 31, ti = ((t >> 5) + 2 * grp) & 7, lane = t & 63, wv = t >> 6;
  const int wrow = __builtin_amdgcn_readfirstlane(2 * ((wv + grp) & 3));
  constexpr bool QM = pair_qmap<KK, LD>();     // the quad unit map of pair_tile
  const int kpb = QM ? 4 * grp : k0 + (k0 & 1);
  const int ktl = QM ? 16 + grp : ((k0 & 1) ? k0 : k0 + KK - 1);
  auto kof = [&](const int k) { return k < 2 * KP ? kpb + k : ktl; };
  const int nown = (N - radd + rmul - 1) / rmul;
  const int S = (nown + 7) >> 3;
  const p2 z2 = {0.f, 0.f};

  p2 cacc2[SMAX][KP > 0 ? KP : 1];
  float cacct[SMAX];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) {
#pragma unroll
    for (int p = 0; p < KP; ++p) cacc2[c][p] = z2;
    cacct[c] = 0.f;
  }
  p2 yacc2[KP > 0 ? KP : 1], dk2[KP > 0 ? KP : 1];
  float yacct = 0.f, dkt = KT ? dl[ktl] : 0.f;
#pragma unroll
  for (int p = 0; p < KP; ++p) yacc2[p] = z2;
  ld_pairs<QM, KP>(dl + kpb, dk2);

  for (int s = 0; s < S; ++s) {
    // waves still on an earlier trip get the issue arbiter first (it otherwise favours
    // the oldest wave, which finishes its trips first and leaves the SIMD to one wave at
    // the end of the pass)
    if constexpr (HDG_SETPRIO) trip_prio(s);
    if (wrow + 8 * s >= nown) continue;     // wave-uniform skip
    const int r = ti + 8 * s;
    const int i = rmul * r + radd;
    const bool iv = r < nown;
    p2 a2[KP > 0 ? KP : 1], rw2[KP > 0 ? KP : 1], racc2[KP > 0 ? KP : 1];
    const int ib = iv ? i : radd;       // past the sweep: the first swept row (own, finite)
    const float* Ai = A + ib * LD;
    const float addm = iv ? 0.f : PADNEG, mulm = iv ? 1.f : 0.f;
    const p2 addm2 = {addm, addm}, mulm2 = {mulm, mulm};
    ld_pairs<QM, KP>(Ai + kpb, a2);
    if constexpr (MODE == 1) ld_pairs<QM, KP>(wr + ib * LD + kpb, rw2);
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      a2[p] += addm2;
      if constexpr (MODE != 0 && HDG_STEPF) a2[p] *= (p2){STEP_S, STEP_S};   // stepf2's c
      if constexpr (MODE == 1)
        rw2[p] *= mulm2;
      else
        rw2[p] = z2;
      racc2[p] = z2;
    }
    const float at = KT ? Ai[ktl] + addm : 0.f;
    const float rwt = (MODE == 1 && KT) ? wr[ib * LD + ktl] * mulm : 0.f;
    float racct = 0.f;
    uint32_t wrow[SMAX];
    const uint32_t bmask = iv ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int q = 0; q < SMAX; ++q)      // clamped load, masked value
      wrow[q] = bits[ib * W + (q < W ? q : 0)] & (q < W ? bmask : 0u);
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
      const int j = tj + 32 * c;
      const float af = (float)((wrow[c] >> tj) & 1u);
      const p2 af2 = {af, af};
      float g = 0.f;
      if constexpr (MODE == 2 && GFULL) {
        g = gam[(iv ? i : radd) * gld + j];
      } else if constexpr (MODE == 2) {
        const int ic = iv ? i : N - 1, jc = j < N ? j : N - 1;
        const float gl = gam[ic * gld + jc];
        g = (iv && j < N && j != i) ? gl : 0.f;
      }
      const float gy = af * g;             // MODE 2: exact (af is 0 or 1)
      const float* Bj = Bv + j * LD;
      p2 bbv[KP > 0 ? KP : 1], wcv[KP > 0 ? KP : 1];
      ld_pairs<QM, KP>(Bj + kpb, bbv);
      if constexpr (MODE == 1) ld_pairs<QM, KP>(wc + j * LD + kpb, wcv);
#pragma unroll
      for (int p = 0; p < KP; ++p) {
        const p2 bb = bbv[p];
        const p2 zb = __builtin_elementwise_fma(af2, dk2[p], bb);
        const p2 z = a2[p] + zb;          // used by MODE 0 (MODE 1, 2: stepf2(zb, a 2^64))
        if constexpr (MODE == 0) {
          // relu(z) accumulated as z [z > 0]: one packed step and two packed fma (no packed
          // max on gfx950: relu was two scalar v_max plus two packed adds)
          const p2 sz = step2(z);
          racc2[p] = __builtin_elementwise_fma(z, sz, racc2[p]);
          cacc2[c][p] = __builtin_elementwise_fma(z, sz, cacc2[c][p]);
        } else if constexpr (MODE == 2) {   // as pair_tile: one exact fma per sum
          const p2 sz = HDG_STEPF ? stepf2(zb, a2[p]) : step2(z), g2 = {g, g}, gy2 = {gy, gy};
          yacc2[p] = __builtin_elementwise_fma(sz, gy2, yacc2[p]);
          racc2[p] = __builtin_elementwise_fma(sz, g2, racc2[p]);
          cacc2[c][p] = __builtin_elementwise_fma(sz, g2, cacc2[c][p]);
        } else {
          const p2 w = rw2[p] + wcv[p];
          const p2 e = (HDG_STEPF ? stepf2(zb, a2[p]) : step2(z)) * w;
          yacc2[p] = __builtin_elementwise_fma(af2, e, yacc2[p]);
          racc2[p] += e;
          cacc2[c][p] += e;
        }
      }
      if constexpr (KT) {
        const float z = at + fmaf(af, dkt, ld_tail<QM && (HDG_QTAIL & 1)>(Bj, ktl, grp));
        float e;
        if constexpr (MODE == 0) {
          e = reluf(z);
        } else {
          const float w = (MODE == 1) ? (rwt + ld_tail<QM && (HDG_QTAIL & 2)>(wc + j * LD, ktl, grp)) : g;
          e = (z > 0.f) ? w : 0.f;
          yacct = fmaf(af, e, yacct);
        }
        racct += e;
        cacct[c] += e;
      }
    }
    float rs[KK];
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      rs[2 * p] = racc2[p].x;
      rs[2 * p + 1] = racc2[p].y;
    }
    if constexpr (KT) rs[KK - 1] = racct;
    row16_sums(rs);
#pragma unroll
    for (int k = 0; k < KK; ++k) {    // + the other DPP row of the half-wave
      float x = rs[k], y = rs[k];
      swap16(x, y);
      rs[k] = x + y;
    }
    if (tj == 0 && iv) {
#pragma unroll
      for (int k = 0; k < KK; ++k) Rout[i * LD + kof(k)] = rs[k];
    }
  }
  if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(0);
  float cf[SMAX * KK], yacc[KK];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) {
#pragma unroll
    for (int p = 0; p < KP; ++p) {
      cf[c * KK + 2 * p] = cacc2[c][p].x;
      cf[c * KK + 2 * p + 1] = cacc2[c][p].y;
    }
    if constexpr (KT) cf[c * KK + KK - 1] = cacct[c];
  }
#pragma unroll
  for (int p = 0; p < KP; ++p) {
    yacc[2 * p] = yacc2[p].x;
    yacc[2 * p + 1] = yacc2[p].y;
  }
  if constexpr (KT) yacc[KK - 1] = yacct;
  float* credy = cred + 4 * NP16 * KK;
  {   // the wave's two tile rows: value n in lanes 0-31, value n + HV in lanes 32-63
    constexpr int NV = SMAX * KK, HV = (NV + 1) / 2;
    float* cw = cred + wv * NP16 * KK;
#pragma unroll
    for (int q = 0; q < HV; ++q) {
      float x = cf[q], y = (q + HV < NV) ? cf[q + HV] : 0.f;
      swap32(x, y);
      const float v = x + y;
      const int n = lane < 32 ? q : q + HV;
      if (n < NV) {
        const int c = n / KK, k = n - c * KK;
        cw[(tj + 32 * c) * KK + k] = v;
      }
    }
  }
  if constexpr (MODE != 0) {
    wave_sums(yacc, lane, [&](int k, float x) { credy[wv * KK + k] = x; });
  }
  __syncthreads();
  close_columns<NP16 * KK, KK>(cred, N, t, kof, fix,
                               [&](int j, int kk, float v) { Cout[j * LD + kk] = v; });
  if constexpr (MODE != 0) {
    if (t < KK) ysum[kof(t)] = credy[t] + credy[KK + t] + credy[2 * KK + t] + credy[3 * KK + t];
  }
  __syncthreads();
}

// the hunk pair passes: 16 x 16 thread tiles up to NC16 = 80 (glide), 8 x 32 beyond
template <int KK, int SMAX16, int MODE, int LD, bool GFULL = false, class FIX = NoFix,
          class... Args>
__device__ __forceinline__ void pair_pass(Args... args) {
  if constexpr (SMAX16 > 5)
    pair_tile32<KK, SMAX16, MODE, LD, GFULL, FIX>(args...);
  else
    pair_tile<KK, SMAX16, MODE, LD, 0, GFULL, FIX>(args...);
}

// ------------------------------------------------------------------------------
// scans / searches
// ------------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ T wave_incl_scan(T v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T n = __shfl_up(v, o);
    if (lane >= o) v += n;
  }
  return v;
}

// For every neighbour j in list[0..d) of the node owned by this lane's group (GL lanes
// starting at lane gbase) call f(j, x_j).  Lane r of the group loads neighbour c0+r and
// its x once; the group reads (j, x_j) back with ds_bpermute (LDS pipe, not VALU), four
// neighbours per trip so their bpermutes are in flight together.  All lanes of a group
// share the trip count, so bpermute sources are active.  list may point to LDS or HBM.
// (ds_bpermute byte addresses are formed once per trip; the 4 reads use the immediate
// offset field, so a neighbour costs no address arithmetic.)
template <int GL, bool NEED_J, class F>
__device__ __forceinline__ void for_each_nbr(const uint8_t* list, const int d, const int gbase,
                                             const int r, const float* xs, F f) {
  for (int c0 = 0; c0 < d; c0 += GL) {
    const int jl = (c0 + r < d) ? (int)list[c0 + r] : 0;
    const int xl = __builtin_bit_cast(int, xs[jl]);
    const int nn = (d - c0 < GL) ? d - c0 : GL;
    int n = 0;
    for (; n + 4 <= nn; n += 4) {
      const int a0 = (gbase + n) << 2;
      float x[4];
      int j[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        x[q] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(a0 + 4 * q, xl));
        j[q] = NEED_J ? __builtin_amdgcn_ds_bpermute(a0 + 4 * q, jl) : 0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) f(j[q], x[q]);
    }
    for (; n < nn; ++n) {
      const int a0 = (gbase + n) << 2;
      f(NEED_J ? __builtin_amdgcn_ds_bpermute(a0, jl) : 0,
        __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(a0, xl)));
    }
  }
}

// the same with x taken from the low / high half of a packed pair (op_sel: no copy of the
// half into a register of its own)
__device__ __forceinline__ f2 clamp_fma2_lo(const f2 x, const f2 a, const f2 b) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(r) : "v"(x), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 clamp_fma2_hi(const f2 x, const f2 a, const f2 b) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1] clamp"
      : "=v"(r) : "v"(x), "v"(a), "v"(b));
  return r;
}




// inclusive scan over the 64 lanes of a wave with DPP only (GFX9 row_shr + row_bcast):
// no LDS round trips.  Lanes shifted in from outside a row read 0 (bound_ctrl).
template <int CTRL, int RMASK>
__device__ __forceinline__ float dpp_in(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                               RMASK, 0xF, true));
}
__device__ __forceinline__ float wave_incl_scan_dpp(float v) {
  v += dpp_in<0x111, 0xF>(v);   // row_shr:1
  v += dpp_in<0x112, 0xF>(v);   // row_shr:2
  v += dpp_in<0x114, 0xF>(v);   // row_shr:4
  v += dpp_in<0x118, 0xF>(v);   // row_shr:8
  v += dpp_in<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  v += dpp_in<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ __forceinline__ int top_pow2(int n) {   // largest power of two <= n (n >= 1)
  return 1 << (31 - __builtin_clz((unsigned)n));
}

// ------------------------------------------------------------------------------
// Prepared batch (hdg_prepare: once per uploaded batch, independent of the parameters).
// Per commit, in 4-byte words:
//   xsrt[NE4]    x sorted ascending            perm[NE4]  node at sorted slot m
//   xu[NE4]      the nd distinct x values      cum[NE4+4] cum[q] = #nodes with x < xu[q]
//   pxd[NE4+4]   f64 pxd[q] = sum of x over nodes with x < xu[q]      meta[4] = {nd}
//   offr, offc   CSR offsets of the a = 1 neighbours of each node (rows of a, of a^T)
//   lists        u8 ids of the row neighbours, padded like the row x-lists (xoffr)
//   ks, kt       [Nc][Ne] u16 cross-graph counts (k_prep_counts)
//   ncst[Nc][2]  f32 count of relations binned to hunk c with a = 0 / a = 1
// ------------------------------------------------------------------------------
using hdg::PrepLayout;
using hdg::prep_layout;

// sort x (stable rank count), distinct values + f64 prefix sums, transposed class bits
__global__ __launch_bounds__(256) void k_prep_sort(const float* __restrict__ x,
                                                   const uint32_t* __restrict__ abits,
                                                   uint32_t* __restrict__ prep, int Ne, int Nc) {
  const PrepLayout L = prep_layout(Ne, Nc);
  const int b = blockIdx.x, t = threadIdx.x;
  const int WE = (Ne + 31) >> 5;
  __shared__ float xl[256], xsl[256];
  __shared__ uint32_t al[256 * 8];
  uint32_t* pb = prep + (size_t)b * L.words;
  float* xsrt = (float*)(pb + L.xsrt);
  int* perm = (int*)(pb + L.perm);
  float* xu = (float*)(pb + L.xu);
  int* cum = (int*)(pb + L.cum);
  double* pxd = (double*)(pb + L.pxd);
  if (t < Ne) xl[t] = x[(size_t)b * Ne + t];
  for (int w = t; w < Ne * WE; w += 256) al[w] = abits[(size_t)b * Ne * WE + w];
  __syncthreads();
  if (t < Ne) al[t * WE + (t >> 5)] &= ~(1u << (t & 31));      // a_ii is not a relation
  __syncthreads();
  if (t < Ne) {
    const float xi = xl[t];
    int r = 0;
    for (int j = 0; j < Ne; ++j) {
      const float xj = xl[j];
      r += (xj < xi || (xj == xi && j < t)) ? 1 : 0;
    }
    xsl[r] = xi;
    xsrt[r] = xi;
    perm[r] = t;
  }
  __shared__ uint32_t atl[256 * 8];
  __shared__ int offl[2][260];
  for (int e = t; e < Ne * WE; e += 256) {          // a^T bits
    const int j = e / WE, w = e - j * WE;
    uint32_t bits = 0;
    for (int l = 0; l < 32; ++l) {
      const int i = 32 * w + l;
      if (i < Ne) bits |= ((al[i * WE + (j >> 5)] >> (j & 31)) & 1u) << l;
    }
    atl[e] = bits;
  }
  __syncthreads();
  __shared__ int xof[2][260];
  if (t < Ne) {
    int dr = 0, dc = 0;
    for (int w = 0; w < WE; ++w) {
      dr += __builtin_popcount(al[t * WE + w]);
      dc += __builtin_popcount(atl[t * WE + w]);
    }
    offl[0][t] = dr;
    offl[1][t] = dc;
    xof[0][t] = (dr + 3) & ~3;
    xof[1][t] = (dc + 3) & ~3;
  }
  __syncthreads();
  if (t == 0) {            // serial scans of the padded x-list lengths, rows then columns
    int acc = 0;
    for (int s2 = 0; s2 < 2; ++s2) {
      int* dst = (int*)(pb + (s2 ? L.xoffc : L.xoffr));
      for (int i = 0; i < Ne; ++i) {
        const int d = xof[s2][i];
        xof[s2][i] = acc;
        dst[i] = acc;
        acc += d;
      }
      xof[s2][Ne] = acc;
      dst[Ne] = acc;
    }
  }
  if (t < 2) {                                       // serial exclusive scans, once per batch
    int acc = 0;
    for (int i = 0; i < Ne; ++i) {
      const int d = offl[t][i];
      offl[t][i] = acc;
      ((int*)(pb + (t ? L.offc : L.offr)))[i] = acc;
      acc += d;
    }
    offl[t][Ne] = acc;
    ((int*)(pb + (t ? L.offc : L.offr)))[Ne] = acc;
  }
  __syncthreads();
  const int cbase = (offl[0][Ne] + 3) & ~3;
  if (t == 0) {
    pb[L.meta + 1] = (uint32_t)offl[0][Ne];
    pb[L.meta + 2] = (uint32_t)offl[1][Ne];
    pb[L.meta + 3] = (uint32_t)cbase;
  }
  if (t < Ne) {
    uint8_t* lb = reinterpret_cast<uint8_t*>(pb + L.lists);
    float* xlp = reinterpret_cast<float*>(pb + L.xl);
    int xr = xof[0][t], xc = xof[1][t];
    for (int w = 0; w < WE; ++w) {
      uint32_t m = al[t * WE + w];
      while (m) {
        const int j = 32 * w + __builtin_ctz(m);
        lb[xr] = (uint8_t)j;
        xlp[xr++] = xl[j];
        m &= m - 1u;
      }
      m = atl[t * WE + w];
      while (m) {
        xlp[xc++] = xl[32 * w + __builtin_ctz(m)];
        m &= m - 1u;
      }
    }
    const float qnan = __builtin_nanf("");      // clamp_fma2(NaN) = 0: pads add nothing
    for (; xr < xof[0][t + 1]; ++xr) { xlp[xr] = qnan; lb[xr] = 0; }
    for (; xc < xof[1][t + 1]; ++xc) xlp[xc] = qnan;
  }
  __syncthreads();
  if (t == 0) {   // serial over <= 256 sorted values, once per batch
    int nd = 0;
    double s = 0.0;
    for (int m = 0; m < Ne; ++m) {
      const float v = xsl[m];
      if (m == 0 || v != xsl[m - 1]) {
        xu[nd] = v;
        cum[nd] = m;
        pxd[nd] = s;
        ++nd;
      }
      s += (double)v;
    }
    cum[nd] = Ne;
    pxd[nd] = s;
    pb[L.meta] = (uint32_t)nd;
  }
}

// Cross-graph aggregation counts.  marshalling_B2 (model_2.py:146-150, dense maps of
// utils2.py:111-137) is n_c = sum_r ([s_r = c] + [t_r = c]) B2_r with
// B2_r = [x'_I, x'_J, [a_IJ = 0], [a_IJ = 1]], (I, J) = relation r on the Ne-grid and
// s_r = hid[i'], t_r = hid[j'] with (i', j') = relation r on the n-grid (r < n(n-1)).
// Only x' changes between steps, so
//   n_c[0] = sum_I ks[c][I] x'_I,  n_c[1] = sum_J kt[c][J] x'_J,  n_c[2:4] = ncst[c]
// ks[c][I] = #{r in Ne-row I : s_r = c} + #{r in Ne-row I : t_r = c}, kt over Ne-columns.
//
// k_prep_counts grid (ceil(Ne / TI), B, 2): block (tile, b, z) owns TI Ne-rows (z = 0: ks,
// plus the class counts) or TI Ne-columns (z = 1: kt) of commit b and visits each of their
// relations once, counting into an LDS histogram [Nc][TI] (integer, order-independent).
// Lanes hold consecutive relations of a row (or column), whose hunk ids repeat in runs
// (s_r is constant over n-1 consecutive relations): each run of equal counter addresses in
// consecutive lanes is one LDS atomic by its first lane (ballot masks), not a same-address
// conflict per lane.  The tile's counters are written as coalesced u16 rows; the class
// counts are summed over tiles with global u32 atomics into ncst (zeroed, then converted to
// f32 in place by k_prep_ncst).  The count arrays live at word offsets (o_ks, o_kt, o_ncst)
// of each commit's prep block of `stride` words (fused layout: prep_layout; general path:
// its own layout).
// ------------------------------------------------------------------------------
__device__ __forceinline__ void divmod_exact(int r, int d, float inv, int& q, int& rem) {
  q = (int)((float)r * inv);
  rem = r - q * d;
  while (rem < 0) { --q; rem += d; }
  while (rem >= d) { ++q; rem -= d; }
}

// counter[key] += (number of consecutive valid lanes from this lane with the same key),
// issued by the first lane of each run; invalid lanes end runs.  All 64 lanes take part.
__device__ __forceinline__ void run_add(uint32_t* counter, int key, bool valid, int lane) {
  const int kp = __shfl_up(key, 1, 64);
  const unsigned long long V = __ballot(valid);
  const bool pv = lane > 0 && ((V >> (lane - 1)) & 1ull);   // previous lane in a run
  const bool lead = valid && (!pv || kp != key);
  const unsigned long long L = __ballot(lead);
  if (lead) {
    const unsigned long long stop =
        (L | ~V) & (lane == 63 ? 0ull : (~0ull << (lane + 1)));
    const int nxt = stop ? __builtin_ctzll(stop) : 64;
    atomicAdd(&counter[key], (uint32_t)(nxt - lane));
  }
}

__global__ __launch_bounds__(512) void k_prep_counts(const uint32_t* __restrict__ abits,
                                                     const int32_t* __restrict__ hidg,
                                                     const int32_t* __restrict__ nleng,
                                                     uint32_t* __restrict__ prep, int Ne, int Nc,
                                                     int TI, int stride, int o_ks, int o_kt,
                                                     int o_ncst) {
  extern __shared__ uint32_t hist[];   // [Nc][TI + 1] | class counts [Nc][2] | hid [Ne] |
                                       // the tile's a-rows [TI][WE] (z = 0)
  const int z = blockIdx.z, b = blockIdx.y, L0 = blockIdx.x * TI, t = threadIdx.x;
  const int lane = t & 63;
  const int WE = (Ne + 31) >> 5;
  uint32_t* pb = prep + (size_t)b * stride;
  const int TP = TI + 1;               // odd row stride: the hunks of one row / column of the
                                       // tile fall in different LDS banks
  uint32_t* ncl = hist + Nc * TP;
  int32_t* hid = reinterpret_cast<int32_t*>(ncl + 2 * Nc);   // LDS copies: the per-relation
  uint32_t* ab = ncl + 2 * Nc + Ne;                          // lookups stay on-chip
  int n = nleng[b];
  n = n < 0 ? 0 : (n > Ne ? Ne : n);
  const int nrel = n >= 2 ? n * (n - 1) : 0;
  const int n1 = n >= 2 ? n - 1 : 1, Ne1 = Ne - 1;
  const float invn = 1.f / (float)n1, invE = 1.f / (float)(Ne1 > 0 ? Ne1 : 1);
  const int nl = Ne - L0 < TI ? Ne - L0 : TI;
  for (int e = t; e < Ne; e += 512) hid[e] = hidg[(size_t)b * Ne + e];
  if (z == 0)
    for (int e = t; e < nl * WE; e += 512) ab[e] = abits[((size_t)b * Ne + L0) * WE + e];
  for (int e = t; e < Nc * TP + 2 * Nc; e += 512) hist[e] = 0;
  __syncthreads();
  const int items = nl * Ne1;
  for (int e0 = 0; e0 < items; e0 += 512) {   // block-uniform trips: every lane takes part
    const int e = e0 + t;
    int li = 0, k = 0, I = 0, jj = 0, J = 0;
    if (e < items) divmod_exact(e, Ne1, invE, li, k);
    if (z == 0) { I = L0 + li; jj = k; J = jj + (jj >= I ? 1 : 0); }
    else { J = L0 + li; I = k + (k >= J ? 1 : 0); jj = J - (J > I ? 1 : 0); }
    const int r = I * Ne1 + jj;
    const bool in = e < items && r < nrel;
    int hs = -1, ht = -1, a = 0;
    if (in) {
      int ip, jjp;
      divmod_exact(r, n1, invn, ip, jjp);
      const int jp = jjp + (jjp >= ip ? 1 : 0);
      hs = hid[ip];
      ht = hid[jp];
      if (z == 0) a = (int)((ab[li * WE + (J >> 5)] >> (J & 31)) & 1u);
    }
    const bool vs = hs >= 0 && hs < Nc, vt = ht >= 0 && ht < Nc;
    run_add(hist, vs ? hs * TP + li : 0, vs, lane);
    run_add(hist, vt ? ht * TP + li : 0, vt, lane);
    if (z == 0) {
      run_add(ncl, vs ? 2 * hs + a : 0, vs, lane);
      run_add(ncl, vt ? 2 * ht + a : 0, vt, lane);
    }
  }
  __syncthreads();
  uint16_t* out = (uint16_t*)(pb + (z ? o_kt : o_ks));
  for (int e = t; e < Nc * TI; e += 512) {
    const int c = e / TI, i = e - c * TI;
    if (i < nl) out[(size_t)c * Ne + L0 + i] = (uint16_t)hist[c * TP + i];
  }
  if (z == 0) {
    uint32_t* nc = pb + o_ncst;
    for (int e = t; e < 2 * Nc; e += 512)
      if (ncl[e]) atomicAdd(&nc[e], ncl[e]);
  }
}

// Upload-time marshalling (hdg_pack_classes): (B, N, N) u8 class grid -> (B, N, ceil(N/32))
// u32 rows, bit j of row i = (class(i, j) == 1), diagonal cleared -- the E_edge / C_edge
// one-hots of utils2.py:82, 105 as hdg_batch's abits / ybits.  One thread per word.
__global__ __launch_bounds__(256) void k_pack_classes(const uint8_t* __restrict__ cls, const int N,
                                                      const int W, const long long words,
                                                      uint32_t* __restrict__ bits) {
  const long long w = (long long)blockIdx.x * 256 + threadIdx.x;
  if (w >= words) return;
  const long long row = w / W;
  const int wi = (int)(w - row * W), i = (int)(row % N), j0 = 32 * wi;
  const uint8_t* src = cls + row * N + j0;
  const int n = N - j0 < 32 ? N - j0 : 32;
  uint32_t b = 0u;
  for (int l = 0; l < n; ++l) b |= (src[l] == 1 ? 1u : 0u) << l;
  if (i >= j0 && i < j0 + 32) b &= ~(1u << (i - j0));   // a_ii is not a relation
  bits[w] = b;
}

// grid (B): mode 0 zeroes the class-count words of each commit, mode 1 turns the summed
// u32 counts into the f32 values the step kernels read (exact: counts < 2^24)
__global__ __launch_bounds__(256) void k_prep_ncst(uint32_t* __restrict__ prep, int Nc,
                                                   int stride, int o_ncst, int mode) {
  uint32_t* nc = prep + (size_t)blockIdx.x * stride + o_ncst;
  for (int e = threadIdx.x; e < 2 * Nc; e += 256) {
    if (mode == 0) nc[e] = 0u;
    else nc[e] = __float_as_uint((float)nc[e]);
  }
}

// ------------------------------------------------------------------------------
// k_commit_step: the whole per-commit forward + backward, one 1024-thread block per
// commit.  Node arrays live in LDS; one union region U is re-carved per phase
// (entity stage -> hunk buffers -> E3 backward -> entity backward).  P, E_bar and the
// E3 hidden layer are parked in the workspace across the hunk phases.  Node matvecs
// use a (k, slice) thread map with the weight column held in registers.
// ------------------------------------------------------------------------------
constexpr int NG_MID = NT_MID / 256;            // 4 pair-tile groups, one k-chunk each
// hunk node buffers [NC16][HS]: alpha beta G H sigma tau (+ tau+eps when it fits)
__host__ __device__ constexpr int nbuf_h(int smaxc) { return smaxc <= 8 ? 7 : 6; }
// the classifier's dL/dz1 matrix gamma [NC16][NC16] lives in LDS (after the pair-tile
// scratch) when Nc <= 80; larger hunk graphs keep it in the workspace
__host__ __device__ constexpr bool gam_lds(int smaxc) { return smaxc <= 5; }
constexpr int NSL = NT_MID / HS;                // 51 node slices for (k, slice) matvecs

struct StepLayout {   // offsets in 4-byte words into the dynamic LDS arena
  int W, xs, xps, os, dxp, xsrt, perm, xu, cum, pxd, offr, offc, yb, nb, dnb, misc, u2, Mm, Xm,
      red, U, Uwords, total;
};

__host__ __device__ inline StepLayout step_layout(int Ne, int Nc, int smaxc) {
  StepLayout L;
  const int NC16 = 16 * smaxc;
  const int NE4 = (Ne + 3) & ~3;
  const int WC = (Nc + 31) >> 5;
  const int cred = 4 * 16 * smaxc * KK_MID + 8 * KK_MID;
  int o = 0;
  L.W = o;    o += (m2::NP + 3) & ~3;
  L.xs = o;   o += NE4;
  L.xps = o;  o += NE4;
  L.os = o;   o += NE4;
  L.dxp = o;  o += NE4;
  L.xsrt = o; o += NE4;
  L.perm = o; o += NE4;
  L.xu = o;   o += 2 * NE4;           // nd values, then +inf padding (E1's clamp-free search)
  L.cum = o;  o += NE4 + 4;
  L.pxd = o;  o += 2 * (NE4 + 4);     // f64 (offset is a multiple of 4 words)
  L.offr = o; o += NE4 + 4;           // CSR offsets of the entity neighbour lists
  L.offc = o; o += NE4 + 4;
  L.yb = o;   o += (Nc * WC + 3) & ~3;
  L.nb = o;   o += 4 * NC16;
  L.dnb = o;  o += 2 * NC16;
  L.misc = o; o += 8 * HS;            // dlt eps cvec ysumv s0 t0 sumD (spare)
  L.u2 = o;   o += 2 * HS;            // U2 (classifier output layer), 16-B aligned copy
  L.Mm = o;   o += HS * HS;           // V2 . U1e
  L.Xm = o;   o += HS * HS;           // sum_p G_p (x) Dsig_p + H_p (x) Dtau_p
  L.red = o;  o += (NT_MID / 64) * 32;
  int u = 3 * NE4 * HS;                                            // P | E_bar | h
  const int uh = nbuf_h(smaxc) * NC16 * HS + NG_MID * cred +      // hunk phases
                 (gam_lds(smaxc) ? NC16 * (NC16 + 8) : 0);
  int ueb = 5 * NE4 * HS;                         // E3 bwd: P | E_bar | dq | dE | h/rho
  const int ue2 = 2 * NE4 * HS + 2 * HS * (NE4 + 4) + (NT_MID / 64) * 4 * HS;   // E2 + rho
  if (ue2 > ueb) ueb = ue2;
  if (uh > u) u = uh;
  if (ueb > u) u = ueb;
  L.U = o; L.Uwords = u; o += u;
  L.total = o;
  return L;
}

using hdg::f4v;
using hdg::mfma_tile16_p;

// One 16x16 tile of C = A.B on v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate; exact
// f32 fmaf-chain numerics).  fa(r, k) = A[row0 + r][k], fb(k, c) = B[k][col0 + c], both
// 0 outside the matrix, so K is zero-padded to a multiple of 4.  Lane l's fragment holds
// C[row0 + 4*(l>>4) + i][col0 + (l&15)] in c[i].  Wave-uniform call (MFMA needs all lanes).
template <class FA, class FB>
__device__ __forceinline__ f4v mfma_tile16(FA fa, FB fb, const int K, const int lane) {
  const int r = lane & 15, q = lane >> 4;
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  int k = 0;
  for (; k + 16 <= K; k += 16) {      // operands of 4 steps issued before their MFMAs
    float a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = fa(r, k + 4 * u + q);
      b[u] = fb(k + 4 * u + q, r);
    }
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c1, 0, 0, 0);
  }
  for (; k < K; k += 4)
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(fa(r, k + q), fb(k + q, r), c0, 0, 0, 0);
  return c0 + c1;
}

// mfma_tile16_p (strided operands): hdgnn_internal.h, shared with the general path

// Two 16x16 tiles sharing the A rows (the two 16-column halves of a 20-wide output):
// one A read per k step feeds both MFMAs, the two accumulation chains interleave.
__device__ __forceinline__ void mfma_tile16x2_p(const float* pa, const int sa, const float* pb0,
                                                const int sb0, const float* pb1, const int sb1,
                                                const int K, const int lane, f4v& o0, f4v& o1) {
  const int q = lane >> 4;
  const float* a = pa + q * sa;
  const float* b0 = pb0 + q * sb0;
  const float* b1 = pb1 + q * sb1;
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  int k = 0;
  for (; k + 16 <= K; k += 16) {
    float av[4], bv0[4], bv1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      av[u] = a[4 * u * sa];
      bv0[u] = b0[4 * u * sb0];
      bv1[u] = b1[4 * u * sb1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv0[u], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv1[u], c1, 0, 0, 0);
    }
    a += 16 * sa;
    b0 += 16 * sb0;
    b1 += 16 * sb1;
  }
  for (; k + 4 <= K; k += 4) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b0[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b1[0], c1, 0, 0, 0);
    a += 4 * sa;
    b0 += 4 * sb0;
    b1 += 4 * sb1;
  }
  if (k < K) {                       // K % 4 tail, as in mfma_tile16_p
    const bool ok = k + q < K;
    const float av = ok ? a[0] : 0.f;
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, ok ? b0[0] : 0.f, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, ok ? b1[0] : 0.f, c1, 0, 0, 0);
  }
  o0 = c0;
  o1 = c1;
}

// first layer of mlp_entity_B1 for hidden unit kk (model_2.py:165-170):
//   W1^T [x_i, x_j, [a=0], [a=1]] + b1 = u_i + v_j + a_ij d,
//   u = fma(x, W1[0], W1[2] + b1), v = x * W1[1], d = W1[3] - W1[2]
// z_ij = u_i + v_j (a = 0) or u_i + (v_j + d) (a = 1), each op rounded (no contraction),
// so the forward sets, the sparse corrections and the backward masks agree exactly.
struct EntUnit {
  float w0, w1, c0, d;
};
__device__ __forceinline__ EntUnit ent_unit(const float* Ws, int kk) {
  using namespace m2;
  EntUnit e;
  e.w0 = Ws[E1_W1 + kk];
  e.w1 = Ws[E1_W1 + HS + kk];
  const float w2 = Ws[E1_W1 + 2 * HS + kk];
  e.c0 = w2 + Ws[E1_B1 + kk];
  e.d = Ws[E1_W1 + 3 * HS + kk] - w2;
  return e;
}

// Entity-stage lane map: a wave takes EG_N = 6 nodes, a node group is EG_L = 10 lanes,
// lane kp of a group owns hidden units (2kp, 2kp+1) as one packed fp32 pair.
constexpr int EG_L = HS / 2, EG_N = 6;

// E1 body (phase comment in k_commit_step).  Rounding contract (no fma contraction):
//   z0_ij = fl(u_i + fl(x_j w1)),  u = fma(x, w0, c0);   z1_ij = fl(z0_ij + d)
// shared by the dense sets, the sparse corrections and the backward masks.
// ABL: ablation bits for the microbenchmark (1 = skip search, 2 = skip dense sums,
// 4 = skip row bits, 8 = skip column bits); 0 in the engine.
template <int ABL = 0>
__device__ __forceinline__ void entity_fwd(const int t, const float* Ws,
                                           const float* xs, const float* xu, const int* cum,
                                           const double* pxd, const int nd,
                                           const int* offr, const int* offc,
                                           const float* xlr, const float* xlc,
                                           const int n0, const int n1, float* Ps,
                                           float* __restrict__ EG, uint16_t* __restrict__ rq) {
#pragma clang fp contract(off)
  // block-wide lane map (no cross-lane traffic left in E1): thread t takes node group
  // sub = t / 10 (102 nodes per pass), hidden units (2 kp, 2 kp + 1), kp = t % 10
  const int sub = t / EG_L, kp = t - sub * EG_L, k0 = 2 * kp;
  const EntUnit ea = ent_unit(Ws, k0 < HS ? k0 : 0), eb = ent_unit(Ws, k0 < HS ? k0 + 1 : 1);
  const f2 w0 = {ea.w0, eb.w0}, w1 = {ea.w1, eb.w1}, c0 = {ea.c0, eb.c0}, dd = {ea.d, eb.d};
  const bool ra[2] = {ea.w1 >= 0.f, eb.w1 >= 0.f}, ca[2] = {ea.w0 >= 0.f, eb.w0 >= 0.f};
  constexpr int NG = NT_MID / EG_L;                // 102 node groups per pass
  for (int base = n0; base < n1; base += NG) {       // block-uniform
    if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(3);   // milestones: see trip_prio
    const int i = base + sub;
    const bool live = sub < NG && i < n1;
    const int ic = live ? i : 0;
    const float xi = xs[ic];
    const f2 u = __builtin_elementwise_fma((f2){xi, xi}, w0, c0);
    const f2 v = xi * w1;
    // binary searches over the nd distinct values, padded with +inf up to 2 top_pow2(nd)
    // (k_commit_step's stage): a probe past nd has z = +-inf (w = 0: NaN), which never
    // moves a search whose answer is < nd; an answer of nd runs into the padding and is
    // clamped once at the end -- no per-probe index clamp
    int br[2] = {0, 0}, bc[2] = {0, 0};
    for (int s = (ABL & 1) ? 0 : top_pow2(nd); s > 0; s >>= 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float xr = xu[br[h] + s - 1], xc = xu[bc[h] + s - 1];
        const bool fr = (u[h] + xr * w1[h]) > 0.f;
        const bool fc = (fmaf(xc, w0[h], c0[h]) + v[h]) > 0.f;
        br[h] = (fr != ra[h]) ? br[h] + s : br[h];
        bc[h] = (fc != ca[h]) ? bc[h] + s : bc[h];
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      br[h] = br[h] < nd ? br[h] : nd;
      bc[h] = bc[h] < nd ? bc[h] : nd;
    }
    if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(2);
    // the a = 0 set sums: cnt u + w1 sum x (row side), cnt (v + c0) + w0 sum x (column
    // side).  The x sums are differences of the f64 prefix table (exact to 2^-53 of the
    // set, rounded once to f32); the rest in f32 with fma: the same rounding order as the
    // reference graph's own f32 pair sums (f64 arithmetic costs ~5x f32 on gfx950)
    float tot[2] = {0.f, 0.f};
    if constexpr (!(ABL & 2)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rlo = ra[h] ? br[h] : 0, rhi = ra[h] ? nd : br[h];
        const int clo = ca[h] ? bc[h] : 0, chi = ca[h] ? nd : bc[h];
        const float sxr = (float)(pxd[rhi] - pxd[rlo]), sxc = (float)(pxd[chi] - pxd[clo]);
        const float nr = (float)(cum[rhi] - cum[rlo]), nc = (float)(cum[chi] - cum[clo]);
        float acc = fmaf(nr, u[h], w1[h] * sxr);
        acc += fmaf(nc, v[h] + c0[h], w0[h] * sxc);
        tot[h] = fmaf(-2.f, reluf(u[h] + v[h]), acc);
      }
    }
    // a = 1 corrections relu(z0 + d) - relu(z0) = d clamp((s z0 + t) / d, 0, 1) with
    // (s, t) = (1, d) for d >= 0 and (-1, 0) for d < 0: z0 is affine in x_j, so the
    // clamp argument is x_j A + B and a neighbour costs ONE clamped packed fma (+ the
    // accumulate); d multiplies the sum once.  |d| < 2^-100 counts as d = 0 (the
    // correction is then below the sum's rounding).
    f2 sp = {0.f, 0.f};
    const f2 sg = {dd.x >= 0.f ? 1.f : -1.f, dd.y >= 0.f ? 1.f : -1.f};
    const f2 tg = {dd.x >= 0.f ? dd.x : 0.f, dd.y >= 0.f ? dd.y : 0.f};
    const f2 rd = {fabsf(dd.x) >= 0x1p-100f ? 1.f / dd.x : 0.f,
                   fabsf(dd.y) >= 0x1p-100f ? 1.f / dd.y : 0.f};
    // neighbour x values come from the prepared NaN-padded x-lists (offr / offc here are
    // their 4-aligned float offsets), four per 16-byte read, identical across the 10
    // lanes of a node group (LDS broadcast): no id lookup, no cross-lane traffic
    // (eight per trip: two 16-byte reads in flight; xlr / xlc point into LDS when staged,
    // so the reads are ds_read_b128, not flat)
    // (two accumulation chains; the x values used in place as packed halves)
    auto xsum = [&](const float* xl, int o, const int o1, const f2 ca, const f2 cb) {
      f2 s0 = {0.f, 0.f}, s1 = s0;
      for (; o + 8 <= o1; o += 8) {
        const float4 xa = *reinterpret_cast<const float4*>(xl + o);
        const float4 xb = *reinterpret_cast<const float4*>(xl + o + 4);
        const f2 a0 = {xa.x, xa.y}, a1 = {xa.z, xa.w}, b0 = {xb.x, xb.y}, b1 = {xb.z, xb.w};
        s0 += clamp_fma2_lo(a0, ca, cb);
        s1 += clamp_fma2_hi(a0, ca, cb);
        s0 += clamp_fma2_lo(a1, ca, cb);
        s1 += clamp_fma2_hi(a1, ca, cb);
        s0 += clamp_fma2_lo(b0, ca, cb);
        s1 += clamp_fma2_hi(b0, ca, cb);
        s0 += clamp_fma2_lo(b1, ca, cb);
        s1 += clamp_fma2_hi(b1, ca, cb);
      }
      if (o < o1) {
        const float4 xa = *reinterpret_cast<const float4*>(xl + o);
        const f2 a0 = {xa.x, xa.y}, a1 = {xa.z, xa.w};
        s0 += clamp_fma2_lo(a0, ca, cb);
        s1 += clamp_fma2_hi(a0, ca, cb);
        s0 += clamp_fma2_lo(a1, ca, cb);
        s1 += clamp_fma2_hi(a1, ca, cb);
      }
      sp += s0 + s1;
    };
    xsum(xlr, ((ABL & 4) || !live) ? 0 : offr[ic], ((ABL & 4) || !live) ? 0 : offr[ic + 1],
         sg * w1 * rd, __builtin_elementwise_fma(sg, u, tg) * rd);
    if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(1);
    xsum(xlc, ((ABL & 8) || !live) ? 0 : offc[ic], ((ABL & 8) || !live) ? 0 : offc[ic + 1],
         sg * w0 * rd, __builtin_elementwise_fma(sg, c0 + v, tg) * rd);
    sp *= dd;
    if (live && kp < EG_L) {
      const float2 P = make_float2(tot[0] + sp.x, tot[1] + sp.y);
      *reinterpret_cast<float2*>(Ps + i * HS + k0) = P;
      *reinterpret_cast<float2*>(EG + i * HS + k0) = P;
      rq[i * HS + k0] = (uint16_t)br[0];
      rq[i * HS + k0 + 1] = (uint16_t)br[1];
    }
  }
  if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(0);
}

// E2 body: per-wave partial sums S0..S3 (dW1 rows, model_2.py:165-170 backward) for
// the wave's nodes -> red2[wv][4][HS].  Same lane map and rounding contract as E1.
__device__ __forceinline__ void entity_bwd(const int lane, const int wv, const float* Ws,
                                           const float* xs, const int* cum, const double* pxd,
                                           const int nd, const uint16_t* __restrict__ rq,
                                           const float* rho, const float* Tr, const float* Tx,
                                           const int TL, const int* xoff, const int* coff,
                                           const uint8_t* idl, const float* xlr,
                                           const int n0, const int n1, float* red2,
                                           const int ne) {
#pragma clang fp contract(off)
  const int sub = lane / EG_L, kp = lane - sub * EG_L, k0 = 2 * kp;
  const EntUnit ea = ent_unit(Ws, k0 < HS ? k0 : 0), eb = ent_unit(Ws, k0 < HS ? k0 + 1 : 1);
  const f2 w0 = {ea.w0, eb.w0}, w1 = {ea.w1, eb.w1}, c0 = {ea.c0, eb.c0}, dd = {ea.d, eb.d};
  const f2 ddS = dd * (f2){STEP_S, STEP_S};       // stepf2's c for [z0 + d > 0]
  const bool ra[2] = {ea.w1 >= 0.f, eb.w1 >= 0.f};
  f2 S0 = {0.f, 0.f}, S1 = S0, S2 = S0, S3 = S0;
  // rounds of 96 nodes; wave w takes nodes w + 16 s (s < 6) of a round, so the last,
  // partial round's nodes land on as many waves -- and SIMDs -- as there are nodes
  constexpr int NWV = NT_MID / 64;
  int ms = 0;                                      // progress milestones (trip_prio)
  for (int base = n0; base + wv < n1; base += EG_N * NWV) {   // wave-uniform
    if constexpr (HDG_SETPRIO) trip_prio(ms++);
    const int i = base + wv + NWV * sub;
    const bool live = sub < EG_N && i < n1;
    const int ic = live ? i : 0;
    const float xi = xs[ic];
    const f2 u = __builtin_elementwise_fma((f2){xi, xi}, w0, c0);
    const f2 vi = xi * w1;
    const f2 ri = *reinterpret_cast<const f2*>(rho + ic * HS + (k0 < HS ? k0 : 0));
    f2 s0, s1, s2, s3 = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = (k0 < HS ? k0 : 0) + h;
      const int q = rq[ic * HS + k];
      const int lo = ra[h] ? q : 0, hi = ra[h] ? nd : q;
      const float cnt = (float)(cum[hi] - cum[lo]);
      const float sx = (float)(pxd[hi] - pxd[lo]);
      const int bm = cum[q];
      const int ts = k * TL + 3 + (ra[h] ? ne - bm : bm);       // the set's scan-order count
      float rs = fmaf(cnt, ri[h], Tr[ts]);                      // sum_{j in set} rho_i + rho_j
      float a0 = xi * rs, a1 = fmaf(ri[h], sx, Tx[ts]);
      if ((u[h] + vi[h]) > 0.f) {                                // remove j == i
        const float r2 = 2.f * ri[h];
        rs -= r2;
        a0 -= xi * r2;
        a1 -= xi * r2;
      }
      s0[h] = a0;
      s1[h] = a1;
      s2[h] = rs;
    }
    if constexpr (HDG_SETPRIO) trip_prio(ms++);
    f2 sd = {0.f, 0.f}, sx = sd;                     // sum dm, sum x_j dm
    // row neighbours from the padded (id, x) lists: 4 ids in one u32 and 4 x values in one
    // 16-byte read per step, identical across the node group's lanes (LDS broadcast)
    // [z1 > 0] as stepf2(z0, d 2^64) (no z1 add); dm = ([z1 > 0] - [z0 > 0]) gs and s3 += [z1 > 0] gs
    // as one fma: the same values as m1 gs - m0 gs and s3 + m1 gs (the steps are 0 or 1)
    auto nbr = [&](const int j, const float xj) {
      const f2 rj = *reinterpret_cast<const f2*>(rho + j * HS + k0);
      const f2 z0 = u + xj * w1;
      const f2 gs = ri + rj;                 // finite: step2(z) * gs == [z > 0] gs
      const f2 st0 = step2(z0);
      const f2 st1 = HDG_STEPF ? stepf2(z0, ddS) : step2(z0 + dd);
      const f2 dm = (st1 - st0) * gs;
      sd += dm;
      sx = __builtin_elementwise_fma((f2){xj, xj}, dm, sx);
      s3 = __builtin_elementwise_fma(st1, gs, s3);
    };
    const int o0 = live ? xoff[ic] : 0;
    const int d = live ? coff[ic + 1] - coff[ic] : 0;
    int q = 0;
    for (; q + 4 <= d; q += 4) {
      const float4 xv = *reinterpret_cast<const float4*>(xlr + o0 + q);
      const uint32_t jw = *reinterpret_cast<const uint32_t*>(idl + o0 + q);
      nbr(jw & 0xffu, xv.x);
      nbr((jw >> 8) & 0xffu, xv.y);
      nbr((jw >> 16) & 0xffu, xv.z);
      nbr(jw >> 24, xv.w);
    }
    if (q < d) {                             // 1-3 left (group-uniform); pads are skipped
      const float4 xv = *reinterpret_cast<const float4*>(xlr + o0 + q);
      const uint32_t jw = *reinterpret_cast<const uint32_t*>(idl + o0 + q);
      nbr(jw & 0xffu, xv.x);
      if (q + 1 < d) nbr((jw >> 8) & 0xffu, xv.y);
      if (q + 2 < d) nbr((jw >> 16) & 0xffu, xv.z);
    }
    s0 = __builtin_elementwise_fma((f2){xi, xi}, sd, s0);
    s1 += sx;
    s2 += sd;
    if (live) { S0 += s0; S1 += s1; S2 += s2; S3 += s3; }
  }
  if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(0);
  // fold the 6 node groups (lanes kp + 10 s), then lanes 0..9 write the wave's sums
  f2 sv[4] = {S0, S1, S2, S3};
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float a = sv[w][h];
      a += __shfl_down(a, 3 * EG_L);
      a += __shfl_down(a, EG_L) + __shfl_down(a, 2 * EG_L);
      sv[w][h] = a;
    }
  if (lane < EG_L) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      red2[(wv * 4 + w) * HS + k0] = sv[w].x;
      red2[(wv * 4 + w) * HS + k0 + 1] = sv[w].y;
    }
  }
}

// ------------------------------------------------------------------------------
// Block-pair exchange (split mode: the two blocks of a commit split the hunk rows).
// pair_send + pair_recv_add: v[0..n) (LDS) += the partner block's v[0..n); both blocks
// end with the same bits (fp32 addition commutes).  Values travel as (value, tag) 8-byte
// pairs, two per 16-byte write-through store (global_store_dwordx4 sc0 sc1: system scope,
// to memory) into the partner's inbox: no L2 writeback fence (the 8 XCD L2s are not
// coherent; an agent-scope release writes back the whole dirty L2, 5-11 us,
// tools/probe/xchg2.hip).  The receiver polls its own inbox with L2-bypassing loads
// (sc0 sc1) until both tags match (1.6 us per 1480-value exchange measured, hidden behind
// independent work between send and receive); tags change every launch (xtag).  The pair
// is co-resident on an otherwise idle GPU (host: 2 B blocks <= CUs, one block per CU),
// which a plain launch does not guarantee (another process, CU masking): a partner that
// never arrives ends the wait after ~20 ms and the launch is failed loudly (xch_fault:
// status word, NaN CE / probs / logits, fault slot that makes the Adam kernels skip the
// update), never a hang.  v must not change between send and receive; n is even.
// ------------------------------------------------------------------------------
// tag of exchange slot s (1..5) in the pair's launch epoch e (a per-commit counter the
// pair reads at its start and block 0 advances after the last exchange): stale words
// of earlier launches carry other tags, so the inboxes are never cleared; the xor keeps
// a tag different from the word's own fill pattern in a garbage workspace
__device__ __forceinline__ uint32_t xtag(const uint32_t epoch, const int slot) {
  return (epoch * 8u + (uint32_t)slot) ^ 0xC0DE5A5Au;
}
constexpr int XSLOTS = 4;                       // H, D_tau, dn partials; n partial + o rows
constexpr int XRHO = 256 * HS / 2;              // + the rho rows of a node half (Ne <= 256)
constexpr unsigned long long XWAIT = 2000000ull;   // s_memrealtime ticks (100 MHz) = 20 ms
typedef uint32_t xu4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void xstore(xu4* p, const xu4 w) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ void xstore1(uint32_t* p, const uint32_t w) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ xu4 xload(const xu4* p) {
  xu4 w;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(w) : "v"(p) : "memory");
  return w;
}
// The send does not wait for this thread's earlier memory operations: the partner reads
// nothing of this block's but the mailbox words themselves (value and tag in one 16-byte
// store), and the receive's polls wait for every outstanding operation (vmcnt(0)), which
// orders a thread's earlier stores before a fault path's poison of the same slots.  (A
// vmcnt(0) here cost 0.3 us per launch, the waves stalling on stores before the send's
// overlapped work.)
__device__ __forceinline__ void pair_send(const float* v, const int n, xu4* __restrict__ out,
                                          const uint32_t tag, const int t) {
  for (int e = t; 2 * e < n; e += NT_MID)
    xstore(out + e, (xu4){__float_as_uint(v[2 * e]), tag, __float_as_uint(v[2 * e + 1]), tag});
}

template <bool ADD = true>
__device__ __forceinline__ bool pair_recv_add(float* v, const int n, xu4* __restrict__ in,
                                              const uint32_t tag, const int t) {
  bool late = false;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int e = t; 2 * e < n; e += NT_MID) {
    xu4 w = xload(in + e);
    while (w.y != tag || w.w != tag) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > XWAIT) { late = true; break; }
      w = xload(in + e);
    }
    if (ADD) {
      v[2 * e] += __uint_as_float(w.x);
      v[2 * e + 1] += __uint_as_float(w.z);
    } else {                                 // the partner's own rows: taken as they are
      v[2 * e] = __uint_as_float(w.x);
      v[2 * e + 1] = __uint_as_float(w.z);
    }
  }
  __syncthreads();
  return late;
}

// A pair exchange of a forward-only launch timed out (split mode; block-uniform call):
// fail the launch loudly.  The CE slot and this block's own probs / logits rows
// (p = rmul r + radd) become NaN and the caller's status word gets HDG_STATUS_XCH_TIMEOUT.
// Thread 0 wrote pb[NP] before, so program order keeps the poison last.  (Training
// launches handle a timeout in their tail: CE NaN, fault slot, status.)
__device__ __forceinline__ void xch_fault(float* __restrict__ pb, uint32_t* __restrict__ status,
                                       float* __restrict__ probs, float* __restrict__ logits,
                                       const int b, const int Nc, const int rmul,
                                       const int radd, const int t) {
  const float qnan = __builtin_nanf("");
  if (t == 0) pb[m2::NP + HDG_TR_CE] = qnan;
  if (t == 0 && status) xstore1(status, HDG_STATUS_XCH_TIMEOUT);
  const int Nc1 = Nc - 1, Pc = Nc * Nc1;
  const int rows = (Nc - radd + rmul - 1) / rmul;
  const size_t base = (size_t)b * 2 * Pc;
  for (int e = t; e < rows * Nc1; e += NT_MID) {
    const int r = (rmul * (e / Nc1) + radd) * Nc1 + e % Nc1;
    if (probs) { probs[base + r] = qnan; probs[base + Pc + r] = qnan; }
    if (logits) { logits[base + r] = qnan; logits[base + Pc + r] = qnan; }
  }
}

template <int SMAXC, bool TRAIN, bool STAMPS = false, bool SPLIT = false>
__global__ __launch_bounds__(NT_MID) void k_commit_step(
    const float* __restrict__ x, const uint32_t* __restrict__ abits,
    const uint32_t* __restrict__ ybits, const uint32_t* __restrict__ prep,
    const float* __restrict__ Wg, float* __restrict__ Esave, uint16_t* __restrict__ rowq,
    float* __restrict__ gamg, float* __restrict__ part, float* __restrict__ probs,
    float* __restrict__ logits, int Ne, int Nc, float ce_scale,
    unsigned long long* __restrict__ stamps, float* __restrict__ aux,
    const float* __restrict__ bpow, const int B, unsigned long long* __restrict__ xch,
    uint32_t* __restrict__ status, const uint32_t xfault, const int ee_ins,
    const unsigned long long* __restrict__ ncpart, const int ncpt, float* __restrict__ dnout,
    const int ehr_park) {
  // model_4 on this kernel (hdg hybrid path): ee_ins = the entity-edge parameter block's
  // length in the flat vector (the model_2-shaped parameters after it are staged at their
  // model_2 offsets); ncpart [B][ncpt][Nc][2] = kw_ee_fwd's per-tile partial bins of the
  // entity-edge aggregate n_c[2:4] (2^-32 fixed point), summed here in tile order, replacing
  // the static class counts (model_4.py:95-97); dnout [B][Nc][4] receives dn for the
  // entity-edge backward.  model_2: 0, nullptr, 0, nullptr.
  using namespace m2;
  constexpr int NC16 = 16 * SMAXC;
  constexpr int CRED = tile_cred_words<SMAXC, KK_MID>();
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const StepLayout L = step_layout(Ne, Nc, SMAXC);
  const PrepLayout PL = prep_layout(Ne, Nc);
  // split mode: commit b runs on two blocks h = 0, 1; block h owns the hunk rows p = 2r + h
  // and the entity nodes of its half for E2.  The pair's block ids are 8 apart (blocks are
  // dealt round-robin over the 8 XCDs, so b and b + 8 share one: the pair's exchanges and
  // its shared input reads stay in one XCD's L2 -- speed only, the protocol does not
  // assume it): ids 16q + 8h + r (r < 8) run commit 8q + r; the grid is padded to whole
  // groups of 16 and the padding commits (b >= B) exit at once.
  int b, h;
  if constexpr (SPLIT) {
    b = ((blockIdx.x >> 1) & ~7) | (blockIdx.x & 7);
    h = (blockIdx.x >> 3) & 1;
  } else {
    b = blockIdx.x;
    h = 0;
  }
  if (b >= B) return;                                // (uniform: split-mode padding)
  const int rmul = SPLIT ? 2 : 1, radd = h;          // own hunk rows p = rmul r + radd
  const int prow = SPLIT ? 2 * b + h : b;            // this block's partial-gradient row
  bool xlate = false;
  constexpr int XS = 16 * SMAXC * HS / 2;            // 16-byte words per inbox slot
  constexpr int XB = XSLOTS * XS + XRHO;             // per block inbox
  xu4* xin = SPLIT ? reinterpret_cast<xu4*>(xch) + (size_t)(2 * b + h) * XB : nullptr;
  xu4* xout = SPLIT ? reinterpret_cast<xu4*>(xch) + (size_t)(2 * b + 1 - h) * XB : nullptr;
  // per-commit launch epoch of the pair's exchange tags (after the 2B inboxes)
  uint32_t* xctr = SPLIT ? reinterpret_cast<uint32_t*>(reinterpret_cast<xu4*>(xch) +
                                                      (size_t)2 * B * XB) + b
                         : nullptr;
  const uint32_t epoch = SPLIT ? *xctr : 0u;
  // send tags: xtag(epoch, slot) ^ xsend; xsend != 0 only under the HDG_DEBUG_XCH_FAULT
  // knob (block 1 of every pair sends words its partner never accepts: forced timeouts)
  const uint32_t xsend = h ? xfault : 0u;
  // Thread ids are re-derived from an opaque copy of threadIdx.x at every phase
  // boundary (PHASE()), so the compiler cannot keep addresses derived from them live
  // across phases: this kernel runs at the 128-VGPR ceiling of 1024-thread blocks.
  int t = threadIdx.x;
  int lane = t & 63, wv = t >> 6, g = t >> 8, tg = t & 255;
  int mk = t % HS, msl = t / HS;                  // (k, slice) map; msl == NSL idles
  const int WC = (Nc + 31) >> 5;
  const int NE4 = (Ne + 3) & ~3;
  const int Pc = Nc * (Nc - 1);
  int nstamp = 0;
  // HDG_STOP_AFTER=n (counter-attribution builds only, tools/lds_phases.sh): every block
  // returns at the n-th top-level phase boundary, so PMC totals of builds n and n+1 differ
  // by phase n's work (outputs are void in such a build)
#ifndef HDG_STOP_AFTER
#define HDG_STOP_AFTER -1
#endif
  int nphase = 0;
#define MID_STAMP()                                                                     \
  do {                                                                                  \
    if constexpr (STAMPS) {                                                             \
      if (threadIdx.x == 0) stamps[prow * 32 + nstamp] = __builtin_amdgcn_s_memrealtime(); \
      ++nstamp;                                                                         \
    }                                                                                   \
    if constexpr (HDG_STOP_AFTER >= 0) {                                                \
      if (nphase++ == HDG_STOP_AFTER) return;                                           \
    }                                                                                   \
    asm volatile("" : "+v"(t));                                                         \
    lane = t & 63;                                                                      \
    wv = __builtin_amdgcn_readfirstlane(t >> 6);                                        \
    g = __builtin_amdgcn_readfirstlane(t >> 8);                                         \
    tg = t & 255;                                                                       \
    mk = t % HS;                                                                        \
    msl = t / HS;                                                                       \
  } while (0)
  MID_STAMP();
  // diagnostic (STAMPS builds only): lane 0 of every wave stamps slot s of its own row
  // [2B][16 waves][8] after the 32-slot phase rows
#define WAVE_STAMP(s)                                                                   \
  do {                                                                                  \
    if constexpr (STAMPS) {                                                             \
      if ((threadIdx.x & 63) == 0)                                                      \
        stamps[(size_t)(SPLIT ? 2 * B : B) * 32 + (prow * 16 + (threadIdx.x >> 6)) * 8 + (s)] = \
            __builtin_amdgcn_s_memrealtime();                                           \
    }                                                                                   \
  } while (0)
  float* Ws = lds + L.W;
  float* xs = lds + L.xs;
  float* xps = lds + L.xps;
  float* os = lds + L.os;
  float* dxp = lds + L.dxp;
  float* xsrt = lds + L.xsrt;
  int* perm = (int*)(lds + L.perm);
  float* xu = lds + L.xu;
  int* cum = (int*)(lds + L.cum);
  double* pxd = (double*)(lds + L.pxd);
  int* offr = (int*)(lds + L.offr);
  int* offc = (int*)(lds + L.offc);
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
  float* kzero = sumD + HS;         // 0.f, 1.f: stride-0 operand rows of mfma_tile16_p
  const float* kone = kzero + 1;
  float* Mm = lds + L.Mm;
  float* Xm = lds + L.Xm;
  float* red = lds + L.red;
  float* U = lds + L.U;

  const uint32_t* pp = prep + (size_t)b * PL.words;
  const int nd = (int)pp[PL.meta];
  float* EG = Esave + (size_t)b * 3 * Ne * HS;     // P | E_bar | h
  float* EbG = EG + Ne * HS;
  float* hEG = EbG + Ne * HS;
  float* pb = part + (size_t)prow * NPART;
  // the rows' fault slots again, contiguous past the 2B rows (work_layout): the reduction
  // reads 2B consecutive floats instead of one cache line per row
  float* fsl = part + (size_t)2 * B * NPART;
  constexpr bool GAML = gam_lds(SMAXC);
  // LDS gamma row stride: 8 words past NC16 puts rows 2 apart (the two rows a 32-lane
  // group of pass B reads in split mode) 16 banks apart: no 2-way conflict on its reads
  constexpr int GLD = GAML ? NC16 + 8 : NC16;
  float* gamG = gamg + (size_t)b * NC16 * NC16;
  uint16_t* rq = rowq + (size_t)b * Ne * HS;
  const float Nc1 = (float)(Nc - 1);
  const float twoNe1 = 2.f * (float)(Ne - 1);

  // ---- M0: stage weights, commit inputs, sorted-x tables and entity class bits --------
  float* Ps = U;
  float* Eb = U + NE4 * HS;
  // neighbour lists (u8 ids, rows | columns): staged behind P when they fit, else read
  // from the prepared buffer in HBM through the same (generic) pointer
  // neighbour x-lists (rows | columns, NaN-padded, k_prep_sort): staged behind P when they
  // fit, else read from the prepared buffer in HBM through the same (generic) pointer
  const int xwords = (int)pp[PL.xoffc + Ne];
  const bool lfit = xwords <= L.Uwords - NE4 * HS;
  const float* xlistg = reinterpret_cast<const float*>(pp + PL.xl);
  // every global load of the stage is issued before the first LDS write (one HBM round
  // trip instead of one per array); Ne, nd < NT_MID and Nc * WC < NT_MID on this path
  constexpr int WQ = (NP + NT_MID - 1) / NT_MID;
  constexpr int LQ = 2;                            // x-list float4 per thread in the batch
  float wr_[WQ];
#pragma unroll
  for (int u = 0; u < WQ; ++u) {
    const int q = t + u * NT_MID;
    wr_[u] = q < NP ? Wg[q + (q >= H1_W1 ? ee_ins : 0)] : 0.f;
  }
  float xv = 0.f, xsv = 0.f, xuv = 0.f;
  int pmv = 0, cmv = 0, orv = 0, ocv = 0;
  double pxv = 0.0;
  uint32_t ybv = 0u;
  if (t < Ne) {
    xv = x[(size_t)b * Ne + t];
    xsv = reinterpret_cast<const float*>(pp + PL.xsrt)[t];
    pmv = reinterpret_cast<const int*>(pp + PL.perm)[t];
  }
  if (t <= Ne) {   // nd <= Ne: loaded without waiting for nd (stored below for t <= nd)
    if (t < Ne) xuv = reinterpret_cast<const float*>(pp + PL.xu)[t];
    cmv = reinterpret_cast<const int*>(pp + PL.cum)[t];
    pxv = reinterpret_cast<const double*>(pp + PL.pxd)[t];
  }
  if (t <= Ne) {   // x-list offsets (E1); the id offsets for E2 are restaged before E2
    orv = reinterpret_cast<const int*>(pp + PL.xoffr)[t];
    ocv = reinterpret_cast<const int*>(pp + PL.xoffc)[t];
  }
  if (t < Nc * WC) ybv = ybits[(size_t)b * Nc * WC + t];
  // the first LQ x-list float4 per thread are loaded without waiting for xwords (reads
  // bounded by the list region's static size, stored below only when they belong)
  const int xlcap = 2 * Ne * (Ne - 1) + 6 * Ne + 8;      // prep_layout's x-list words
  float4 lv[LQ];
#pragma unroll
  for (int u = 0; u < LQ; ++u) {
    const int w = 4 * (t + u * NT_MID);
    lv[u] = w + 4 <= xlcap ? *reinterpret_cast<const float4*>(pp + PL.xl + w)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float l2 = 0.f;
#pragma unroll
  for (int u = 0; u < WQ; ++u) {
    if (t + u * NT_MID < NP) Ws[t + u * NT_MID] = wr_[u];
    l2 = fmaf(wr_[u], wr_[u], l2);
  }
  if (aux && b == 0 && h == 0) {           // pre-update loss_para / loss_map / Adam factor
    l2 = wave_sum(l2);
    if (lane == 0) red[wv * 32] = l2;
  }
  if (t < Ne) {
    xs[t] = xv;
    xsrt[t] = xsv;
    perm[t] = pmv;
  }
  if (t <= nd) {
    cum[t] = cmv;
    pxd[t] = pxv;
  }
  // the nd distinct values, +inf past them up to 2 NE4 >= 2 top_pow2(nd): E1's binary
  // search probes indices < 2 top_pow2(nd) without clamping (entity_fwd)
  if (t < 2 * NE4) xu[t] = t < nd ? xuv : INFINITY;     // 2 NE4 <= 512 < NT_MID
  if (t <= Ne) {
    offr[t] = orv;
    offc[t] = ocv;
  }
  if (t < Nc * WC) yb[t] = ybv;
#pragma unroll
  for (int u = 0; u < LQ; ++u) {
    const int w = 4 * (t + u * NT_MID);
    if (lfit && w < xwords) *reinterpret_cast<float4*>(U + NE4 * HS + w) = lv[u];
  }
  if (lfit)                                // the rest of long lists
    for (int w = 4 * (t + LQ * NT_MID); w < xwords; w += 4 * NT_MID)
      *reinterpret_cast<float4*>(U + NE4 * HS + w) =
          *reinterpret_cast<const float4*>(pp + PL.xl + w);
  if (t == 0) { kzero[0] = 0.f; kzero[1] = 1.f; }
  __syncthreads();
  if (aux && b == 0 && h == 0 && t == 0) {   // model_2.py:123-130, 326-333; TF ApplyAdam lr_t
    float s2 = 0.f;
    for (int w = 0; w < NT_MID / 64; ++w) s2 += red[w * 32];
    const float n1 = sqrtf(Ws[TH1] * Ws[TH1] + Ws[TH1 + 1] * Ws[TH1 + 1]);
    const float n2 = sqrtf(Ws[TH2] * Ws[TH2] + Ws[TH2 + 1] * Ws[TH2 + 1]);
    const float b1p = bpow[0], b2p = bpow[1];
    aux[0] = 0.0005f * s2;
    aux[1] = 0.01f * (n2 + n1);
    aux[2] = n1;
    aux[3] = n2;
    aux[4] = sqrtf(1.f - b2p) / (1.f - b1p);
    aux[5] = b1p * 0.9f;
    aux[6] = b2p * 0.999f;
  }
  MID_STAMP();

  // ---- E1: mlp_entity_B1 pair sums (model_2.py:161-175, agg model_2.py:181-188) -----
  //   P_i[k] = sum_{j!=i} relu(z_ij) + sum_{j!=i} relu(z_ji)  (E_bar = P W5 + 2(Ne-1) b5)
  //   a = 0 part over ALL j: {j : u_i + v_j > 0} is a prefix or suffix of the x-sorted
  //   order (v_j monotone in x_j), found by binary search over the nd distinct x values;
  //   its sum is cnt*u_i + w1*sum(x_j) from f64 prefix sums.  Likewise the column side
  //   {j : u_j + v_i > 0}.  a_ij = 1 entries add relu(z + d) - relu(z) (set bits of row
  //   i of a and of a^T); the diagonal is removed once.  Lane map: a wave takes 3 nodes,
  //   lane = (node sub, hidden unit k), so the 20 lanes of a node walk its bits together.
  //   The row-set boundaries are kept for the backward.
  // split mode: each block of the pair takes its half of the nodes through E1 -> M3 and
  // M11 -> E2; the P, E_bar and h rows it parks in the workspace are read back by itself
  const int nlo = SPLIT && h ? (Ne + 1) / 2 : 0, nhi = SPLIT && !h ? (Ne + 1) / 2 : Ne;
  if (lfit)        // two inlined copies: the staged lists are read as LDS, not flat
    entity_fwd(t, Ws, xs, xu, cum, pxd, nd, offr, offc, U + NE4 * HS, U + NE4 * HS, nlo, nhi, Ps,
               EG, rq);
  else
    entity_fwd(t, Ws, xs, xu, cum, pxd, nd, offr, offc, xlistg, xlistg, nlo, nhi, Ps, EG, rq);
  WAVE_STAMP(0);
  __syncthreads();
  MID_STAMP();

  // ---- M1/M2: per 16-row block, one wave runs the row-local chain (MFMA tiles):
  //   E_bar = P W5 + 2(Ne-1) b5          (agg_entity_B1, model_2.py:181-188)
  //   h = relu([x, E_bar] W1' + b1')     (mlp2_entity_B1, model_2.py:190-205)
  //   o = h w2' + b2',  x' = relu(o)
  for (int rb = (nlo >> 4) + wv; rb <= ((nhi - 1) >> 4); rb += NT_MID / 64) {   // wave-uniform
    const int row0 = rb * 16;
    const int ir = row0 + (lane & 15);                         // this lane's A row
    const bool rv = ir >= nlo && ir < nhi;
    {                                  // both 16-column halves, shared A reads
      f4v cc[2];
      const int m0 = lane & 15, m1 = 16 + (lane & 15);
      mfma_tile16x2_p(rv ? Ps + ir * HS : kzero, rv ? 1 : 0, Ws + E1_W5 + m0, HS,
                      m1 < HS ? Ws + E1_W5 + m1 : kzero, m1 < HS ? HS : 0, HS, lane, cc[0], cc[1]);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col0 = cb * 16;
        const f4v c = cc[cb];
        const int m = col0 + (lane & 15);
        if (m < HS) {
          const float bias = twoNe1 * Ws[E1_B5 + m];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = row0 + 4 * (lane >> 4) + q;
            if (i >= nlo && i < nhi) {
              Eb[i * HS + m] = c[q] + bias;
              EbG[i * HS + m] = c[q] + bias;
            }
          }
        }
      }
    }
    {                                  // both 16-column halves, shared A reads
      f4v cc[2];
      const int m0 = lane & 15, m1 = 16 + (lane & 15);
      mfma_tile16x2_p(rv ? Eb + ir * HS : kzero, rv ? 1 : 0, Ws + E3_W1 + HS + m0, HS,
                      m1 < HS ? Ws + E3_W1 + HS + m1 : kzero, m1 < HS ? HS : 0, HS, lane, cc[0], cc[1]);
      // h = relu(...) in the tile registers; o = h w2' + b2' as a 16-lane row sum of the
      // lanes' h w2' products (no LDS round trip for h)
      float ow[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {   // same wave: its E_bar rows are complete (LDS in order)
        const int col0 = cb * 16;        // [x, E_bar] W1' = E_bar W1'[1:] (MFMA) + x W1'[0]
        const f4v c = cc[cb];
        const int m = col0 + (lane & 15);
        if (m < HS) {
          const float bias = Ws[E3_B1 + m], w0 = Ws[E3_W1 + m], w2 = Ws[E3_W2 + m];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = row0 + 4 * (lane >> 4) + q;
            const bool own = i >= nlo && i < nhi;
            const float v = reluf(fmaf(xs[own ? i : nlo], w0, c[q]) + bias);
            if (own) hEG[i * HS + m] = v;
            ow[q] = fmaf(v, w2, ow[q]);
          }
        }
      }
      row16_sums(ow);
      const int q = lane & 15, i = row0 + 4 * (lane >> 4) + q;
      if (q < 4 && i >= nlo && i < nhi) {
        const float o = (q == 0 ? ow[0] : q == 1 ? ow[1] : q == 2 ? ow[2] : ow[3]) + Ws[E3_B2];
        os[i] = o;
        xps[i] = reluf(o);
      }
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M3: marshalling_B2 (model_2.py:146-150) as two count-matrix matvecs -----------
  //   n_c = [sum_I ks[c][I] x'_I, sum_J kt[c][J] x'_J, ncst[c][0], ncst[c][1]]  (k_prep_counts)
  {
    const uint16_t* ks = reinterpret_cast<const uint16_t*>(pp + PL.ks);
    const uint16_t* kt = reinterpret_cast<const uint16_t*>(pp + PL.kt);
    const float* ncst = reinterpret_cast<const float*>(pp + PL.ncst);
    // 4 tasks (c, m) per trip, each lane's <= QN elements per task unrolled: all global
    // loads of a trip are in flight before the first reduction.  Split mode: the block's
    // own nodes only; the partial n and the own o rows go through one pair exchange.
    constexpr int QN = SPLIT ? 2 : 4;                 // Ne <= 256: a half is <= 128 nodes
    float* xsc = Ps;                                  // [2 Nc n partials | NE4 o rows]
    // a wave takes MT consecutive tasks (c, m) per trip: all MT * QN count loads are in
    // flight before the products, and the MT wave sums close together (wave_sums)
    constexpr int MT = 10;
    float xv[QN];
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int I = nlo + lane + 64 * q;
      xv[q] = I < nhi ? xps[I] : 0.f;
    }
    for (int t0 = MT * wv; t0 < 2 * Nc; t0 += MT * (NT_MID / 64)) {   // wave-uniform
      float kv[MT][QN];
#pragma unroll
      for (int u = 0; u < MT; ++u) {
        const int task = t0 + u < 2 * Nc ? t0 + u : 2 * Nc - 1;
        const uint16_t* kr = ((task & 1) ? kt : ks) + (size_t)(task >> 1) * Ne;
#pragma unroll
        for (int q = 0; q < QN; ++q) {
          const int I = nlo + lane + 64 * q;
          kv[u][q] = (float)kr[I < nhi ? I : nlo];
        }
      }
      float a[MT];
#pragma unroll
      for (int u = 0; u < MT; ++u) {
        a[u] = 0.f;
#pragma unroll
        for (int q = 0; q < QN; ++q) a[u] = fmaf(kv[u][q], xv[q], a[u]);
      }
      wave_sums(a, lane, [&](int u, float v) {
        const int task = t0 + u;
        if (task < 2 * Nc) {
          if (SPLIT) xsc[task] = v;
          else nb[4 * (task >> 1) + (task & 1)] = v;
        }
      });
    }
    if (ncpart) {   // model_4: the EE aggregate, tile partials in tile order (as kw_cross_fwd)
      const unsigned long long* pr = ncpart + (size_t)b * ncpt * 2 * Nc;
      for (int e = t; e < 2 * Nc; e += NT_MID) {
        unsigned long long a = 0ull;
        for (int tl = 0; tl < ncpt; tl += 8) {   // 8 tiles' loads in flight (integer sum:
          unsigned long long v[8];               // any order gives the same bits)
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = tl + u < ncpt ? pr[(size_t)(tl + u) * 2 * Nc + e] : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u) a += v[u];
        }
        nb[4 * (e >> 1) + 2 + (e & 1)] = (float)((double)a * (1.0 / 4294967296.0));
      }
    } else {
      for (int c = t; c < Nc; c += NT_MID) {
        nb[4 * c + 2] = ncst[2 * c];
        nb[4 * c + 3] = ncst[2 * c + 1];
      }
    }
    if constexpr (SPLIT) {
      for (int i = t; i < NE4; i += NT_MID) xsc[2 * Nc + i] = (i >= nlo && i < nhi) ? os[i] : 0.f;
      __syncthreads();
      pair_send(xsc, 2 * Nc + NE4, xout + 3 * XS, xtag(epoch, 4) ^ xsend, t);   // constants overlap
    }
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
  if (t < 2 * HS) lds[L.u2 + t] = Ws[H2_W2 + t];
  for (int e = t; e < HS * HS; e += NT_MID) {
    const int l = e / HS, k = e - l * HS;
    float acc = 0.f;
#pragma unroll
    for (int m = 0; m < HS; ++m) acc = fmaf(Ws[H1_W2 + l * HS + m], Ws[H2_W1 + (2 + m) * HS + k], acc);
    Mm[e] = acc;
  }
  if constexpr (SPLIT) {
    float* xsc = Ps;
    xlate |= pair_recv_add(xsc, 2 * Nc + NE4, xin + 3 * XS, xtag(epoch, 4), t);
    for (int e = t; e < 2 * Nc; e += NT_MID) nb[4 * (e >> 1) + (e & 1)] = xsc[e];
    for (int i = t; i < Ne; i += NT_MID) os[i] = xsc[2 * Nc + i];
  }
  __syncthreads();
  MID_STAMP();

  // ---- M4: first layer of mlp_hunk_B2 split per node (model_2.py:257-260) ----------
  //   alpha_p = n_p V1[0:4] + V1[8] + c1,   beta_q = n_q V1[4:8],   delta = V1[9]-V1[8]
  constexpr int NBUF_H = nbuf_h(SMAXC);
  constexpr bool TAUE = NBUF_H == 7;
  float* Bf[7];
#pragma unroll
  for (int q = 0; q < NBUF_H; ++q) Bf[q] = U + q * NC16 * HS;
  float* credg = U + NBUF_H * NC16 * HS + g * CRED;
  float* gam = GAML ? U + NBUF_H * NC16 * HS + NG_MID * CRED : gamG;   // compile-time choice
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
      float al = PADNEG, be = PADNEG;   // finite: MODE 0 accumulates z [z > 0]
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
  {
    // the pass includes the diagonal pair (p, p) of every swept row (y_pp = 0): removed from
    // both sums of the own rows when the columns close
    auto m5fix = [&](int j, int kk, float v) {
      const int e = j * HS + kk;
      if (!SPLIT || (j & 1) == h) {
        const float dg = reluf(alpha[e] + beta[e]);
        G[e] -= dg;
        v -= dg;
      }
      Hh[e] = v;
    };
    pair_pass<KK_MID, SMAXC, 0, HS, false, decltype(m5fix)>(
        Nc, tg, alpha, beta, g * KK_MID, dlt, yb, WC, nullptr, nullptr, nullptr, 0, G, Hh,
        nullptr, credg, rmul, radd, m5fix);
  }
  if constexpr (SPLIT) pair_send(Hh, Nc * HS, xout, xtag(epoch, 1) ^ xsend, t);   // received in M6
  MID_STAMP();

  // ---- M6: classifier first layer on eff = S_p + T_q, S = G V2 + (Nc-1) c2:
  //   sigma_p = G_p M + (Nc-1) c2 U1e + U1[0] + d1,  tau_q = H_q M + (Nc-1) c2 U1e
  float* sig = Bf[4];
  float* tau = Bf[5];
  float* tauE = TAUE ? Bf[6] : nullptr;     // tau + eps: the y = 1 column operand of pass A
  // sigma tiles first, tau tiles after the H exchange (split mode: the sigma tiles
  // overlap the exchange latency)
  auto m6_tiles = [&](const int which) {
    for (int tile = wv; tile < 2 * SMAXC; tile += NT_MID / 64) {     // wave-uniform
      const int row0 = (tile >> 1) * 16, col0 = (tile & 1) * 16;
      const float* src = which ? Hh : G;
      const int pr = row0 + (lane & 15), mc = col0 + (lane & 15);
      const f4v c = mfma_tile16_p(pr < Nc ? src + pr * HS : kzero, pr < Nc ? 1 : 0,
                                  mc < HS ? Mm + mc : kzero, mc < HS ? HS : 0, HS, lane);
      const int m = col0 + (lane & 15);
      if (m < HS) {
        const float off = which ? t0v[m] : s0v[m], ek = eps[m];
        float* dst = which ? tau : sig;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = row0 + 4 * (lane >> 4) + q;
          const float v = p < Nc ? c[q] + off : -INFINITY;
          dst[p * HS + m] = v;
          if constexpr (TAUE) {
            if (which) tauE[p * HS + m] = v + ek;
          }
        }
      }
    }
  };
  m6_tiles(0);
  if constexpr (SPLIT) {
    if constexpr (STAMPS) MID_STAMP();
    xlate |= pair_recv_add(Hh, Nc * HS, xin, xtag(epoch, 1), t);
  }
  m6_tiles(1);
  __syncthreads();
  if constexpr (!TRAIN) {
    if (ehr_park) {   // loss_E_HR (hdg_forward only): G's own rows and H (block 0) to gamma's
                      // workspace slot, unused by a forward launch, for kw_ehr
      for (int e = t; e < Nc * HS; e += NT_MID) {
        if (!SPLIT || ((e / HS) & 1) == h) gamG[e] = G[e];
        if (h == 0) gamG[Nc * HS + e] = Hh[e];
      }
    }
  }
  MID_STAMP();

  // ---- M7: edge classifier + softmax CE per hunk pair (model_2.py:304-324, 115-118) ----
  float* prb = probs ? probs + (size_t)b * 2 * Pc : nullptr;
  float* lgb = logits ? logits + (size_t)b * 2 * Pc : nullptr;
  float ce_acc = 0.f, gsum = 0.f, corr = 0.f;
  // dU2 = sum relu(kappa) gamma (model_2.py:318-321) is not accumulated per pair: it is
  // rebuilt after the classifier backward from its row / column sums (M9)
  {
    const int Nc1i = Nc - 1;
    const float invNc1 = 1.f / (float)Nc1i;
    // U2 rows (w0_k, w1_k) read as broadcast LDS float4 pairs: keeps 40 VGPRs free
    const float4* u2 = reinterpret_cast<const float4*>(lds + L.u2);
    const float b0 = Ws[H2_B2], b1 = Ws[H2_B2 + 1];
    const int Pown = ((Nc - radd + rmul - 1) / rmul) * Nc1i;    // pairs of the own rows
    // (row r, column slot qq) of pair el advance by a fixed step with one carry per trip
    int r, qq;
    divmod_bf(t, Nc1i, invNc1, r, qq);
    const int dr = NT_MID / Nc1i, dqq = NT_MID - dr * Nc1i;
    const int npad = NC16 - Nc;
    if (TRAIN && npad > 0) {   // gamma's padding columns [Nc, NC16) of the own rows:
                               // pass B reads the gamma rows unmasked (GFULL)
      for (int e = t; e < ((Nc - radd + rmul - 1) / rmul) * npad; e += NT_MID) {
        const int r2 = e / npad;
        gam[(rmul * r2 + radd) * GLD + Nc + (e - r2 * npad)] = 0.f;
      }
    }
    int trip = 0;
    for (int el = t; el < Pown; el += NT_MID) {
      if constexpr (HDG_SETPRIO) trip_prio(trip++);
      const int p = rmul * r + radd;
      const int e = SPLIT ? p * Nc1i + qq : el;
      const int q = qq + (qq >= p ? 1 : 0);
      const float yf = (float)((yb[__mul24(p, WC) + (q >> 5)] >> (q & 31)) & 1u);
      const float4* sp = reinterpret_cast<const float4*>(sig + p * HS);
      const float4* tq =
          reinterpret_cast<const float4*>((TAUE && yf > 0.f ? tauE : tau) + q * HS);
      const float4* ep4 = reinterpret_cast<const float4*>(eps);
      const float ey = TAUE ? 0.f : yf;       // without tau+eps: add y*eps here
      // two classes: softmax / CE / gradient need only d = z1 - z0 = sum_k relu(kappa_k) c_k
      // + (b1 - b0) (c = U2[:,1] - U2[:,0]): one fma per unit instead of two (the logits
      // themselves only when requested); two accumulation chains
      const float4* cv4 = reinterpret_cast<const float4*>(cvec);
      float da = b1 - b0, dbb = 0.f;
      float kap[HS];
#pragma unroll
      for (int v = 0; v < HS / 4; ++v) {
        const float4 a = sp[v];
        float4 c = tq[v];
        if constexpr (!TAUE) {
          const float4 ee = ep4[v];
          c.x = fmaf(ey, ee.x, c.x);
          c.y = fmaf(ey, ee.y, c.y);
          c.z = fmaf(ey, ee.z, c.z);
          c.w = fmaf(ey, ee.w, c.w);
        }
        kap[4 * v] = reluf(a.x + c.x);
        kap[4 * v + 1] = reluf(a.y + c.y);
        kap[4 * v + 2] = reluf(a.z + c.z);
        kap[4 * v + 3] = reluf(a.w + c.w);
        const float4 cw = cv4[v];
        da = fmaf(kap[4 * v], cw.x, da);
        dbb = fmaf(kap[4 * v + 1], cw.y, dbb);
        da = fmaf(kap[4 * v + 2], cw.z, da);
        dbb = fmaf(kap[4 * v + 3], cw.w, dbb);
      }
      float d = da + dbb;
      if (lgb) {                              // C_edge_output2_logits (model_2.py:321-323)
        typedef float p2 __attribute__((ext_vector_type(2)));
        p2 zz = {b0, b1}, zy = {0.f, 0.f};
#pragma unroll
        for (int v = 0; v < HS / 4; ++v) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const float4 w = u2[2 * v + hh];      // w0_k, w1_k, w0_k+1, w1_k+1
            zz = __builtin_elementwise_fma((p2){kap[4 * v + 2 * hh], kap[4 * v + 2 * hh]},
                                           (p2){w.x, w.y}, zz);
            zy = __builtin_elementwise_fma((p2){kap[4 * v + 2 * hh + 1], kap[4 * v + 2 * hh + 1]},
                                           (p2){w.z, w.w}, zy);
          }
        }
        zz += zy;
        lgb[e] = zz.x;
        lgb[Pc + e] = zz.y;
        d = zz.y - zz.x;   // probs = softmax of the returned logits, as the graph defines them
      }
      // p1 = 1 / (1 + e^-d), p0 = e^-d p1, evaluated with e = e^-|d| in (0, 1] (no overflow);
      // CE = softplus(d) (y = 0) or softplus(-d) (y = 1) = max(+-d, 0) + log(1 + e)
      const float ex = __expf(-fabsf(d));
      const float inv = __builtin_amdgcn_rcpf(1.f + ex);   // 1 + e in (1, 2]: 1-ulp rcp
      const float pbig = inv, psmall = ex * inv;
      const float p1 = d >= 0.f ? pbig : psmall, p0 = d >= 0.f ? psmall : pbig;
      ce_acc += ln_1to2(1.f + ex) + reluf(yf > 0.f ? -d : d);
      corr += ((p1 > p0) == (yf > 0.f)) ? 1.f : 0.f;   // top_ACC: np.argmax, ties -> 0
      if (prb) { prb[e] = p0; prb[Pc + e] = p1; }
      if constexpr (TRAIN) {
        if (qq == p || (p == Nc1i && qq == Nc1i - 1))   // defined diagonal, every row
          gam[p * GLD + p] = 0.f;
        const float gmm = ce_scale * (p1 - yf);   // dL/dz1 = -dL/dz0
        gam[p * GLD + q] = gmm;
        gsum += gmm;
      }
      qq += dqq;                              // next pair of this thread
      r += dr;
      if (qq >= Nc1i) {
        qq -= Nc1i;
        ++r;
      }
    }
  }
  if constexpr (HDG_SETPRIO) __builtin_amdgcn_s_setprio(0);
  WAVE_STAMP(1);
  if constexpr (TRAIN) {   // red[wv][0] CE, [1] sum gamma, [2 + HS] count
    float v[3] = {ce_acc, gsum, corr};
    float* rw = red + wv * 32;
    wave_sums(v, lane, [&](int n, float x) { rw[n < 2 ? n : 2 + HS] = x; });
  } else {
    const float s0 = wave_sum(ce_acc);
    const float sc = wave_sum(corr);
    if (lane == 0) { red[wv * 32] = s0; red[wv * 32 + 2 + HS] = sc; }
  }
  __syncthreads();
  MID_STAMP();
  if (t < 3 + HS && (t < 2 || t == 2 + HS)) {
    float s = 0.f;
    for (int w = 0; w < NT_MID / 64; ++w) s += red[w * 32 + t];
    if (t == 0) pb[NP] = s;
    if (t == 2 + HS) pb[NP + 1] = s;        // correct-prediction count (integer, exact)
    if constexpr (TRAIN) {
      if (t == 1) { pb[H2_B2] = -s; pb[H2_B2 + 1] = s; }
    }
  }
  if constexpr (!TRAIN) {         // uniform exit: forward-only launch (the H exchange was
    if (SPLIT && h == 0 && t == 0) *xctr = epoch + 1u;   // the pair's last: next epoch)
    if constexpr (SPLIT) {        // block-wide vote through word 31 of each wave's red row
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own probs stores land first
      const bool wl = __ballot(xlate) != 0ull;            // (no __syncthreads_or: its
      if (lane == 0) red[wv * 32 + 31] = wl ? 1.f : 0.f;  // static LDS word would push the
      __syncthreads();                                     // block past 160 KiB)
      bool any = false;
      for (int w = 0; w < NT_MID / 64; ++w) any |= red[w * 32 + 31] != 0.f;
      if (any) xch_fault(pb, status, probs, logits, b, Nc, rmul, radd, t);
    }
    return;
  }

  // ---- M8: classifier backward: dkappa_pq = c (.) [kappa_pq > 0] gamma_pq,
  //          row sums Dsig (in place over sigma), column sums Dtau (over tau) -------
  float* Dsig = sig;
  float* Dtau = tau;
  // Dsig / Dtau here are the sums of [kappa > 0] gamma WITHOUT the factor c of
  // dkappa = c (.) [kappa > 0] gamma: M9 applies c to the sums it forms, and the dG / dH
  // tiles take it in M c (c scales a column of the sums, so nothing is lost)
  pair_pass<KK_MID, SMAXC, 2, HS, true>(Nc, tg, sig, tau, g * KK_MID, eps, yb, WC, nullptr,
                                           nullptr, gam, GLD, Dsig, Dtau, ysumv, credg, rmul,
                                           radd);
  if constexpr (SPLIT) pair_send(Dtau, Nc * HS, xout + XS, xtag(epoch, 2) ^ xsend, t);   // received in M9
  MID_STAMP();
  // ---- M9: X = sum_p G_p (x) Dsig_p + H_p (x) Dtau_p; classifier / hunk-MLP grads ----
  //   one MFMA GEMM [G^T; 1; 0 | H^T; 0; 1] (22 x 2Nc) . [Dsig; Dtau] (2Nc x 20): rows
  //   20, 21 are sum_p Dsig, sum_p Dtau.  4 tiles x 4 K-quarters (two per half: waves 0-7
  //   take the G / Dsig half, waves 8-15 the H / Dtau half, after the D_tau exchange in
  //   split mode), partials in the pair-tile scratch (dead after pass B), then one
  //   fixed-order sum.  Split mode sums over the block's own rows p only.
  {
    float* xpart = U + NBUF_H * NC16 * HS;            // [4 kq][4 tiles][256]
    const int Nc4 = (Nc + 3) & ~3;
    const int kq = wv >> 2, tl = wv & 3, half = kq >> 1;
    const int row0 = (tl >> 1) * 16, col0 = (tl & 1) * 16;
    const int mq = ((Nc4 / 2) + 3) & ~3;
    const int kl = (kq & 1) * mq;
    const int kh = (kl + mq < Nc4) ? kl + mq : Nc4;
    auto xtile = [&]() {
      const f4v c = mfma_tile16(
          [&](int r, int k) {
            const int p = kl + k, l = row0 + r;
            if (p >= Nc || (SPLIT && (p & 1) != h)) return 0.f;     // own rows
            if (l < HS) return (half ? Hh : G)[p * HS + l];
            return (l == HS + half) ? 1.f : 0.f;
          },
          [&](int k, int j) {
            const int p = kl + k, m = col0 + j;
            return (p < Nc && m < HS && (!SPLIT || (p & 1) == h)) ? (half ? Dtau : Dsig)[p * HS + m]
                                                                  : 0.f;
          }, kh > kl ? kh - kl : 0, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        xpart[(kq * 4 + tl) * 256 + (4 * (lane >> 4) + q) * 16 + (lane & 15)] = c[q];
    };
    if (half == 0) xtile();
    if constexpr (SPLIT) {
      if constexpr (STAMPS) MID_STAMP();
      xlate |= pair_recv_add(Dtau, Nc * HS, xin + XS, xtag(epoch, 2), t);
    }
    if (half == 1) xtile();
    __syncthreads();
    float* Xp = xpart + 16 * 256;                      // X' (no c) [22][HS], then M c [HS][HS]
    float* Mc = Xp + 22 * HS;
    {
      const int tl2 = t >> 8, e = t & 255;
      const float v = (xpart[(0 * 4 + tl2) * 256 + e] + xpart[(1 * 4 + tl2) * 256 + e]) +
                      (xpart[(2 * 4 + tl2) * 256 + e] + xpart[(3 * 4 + tl2) * 256 + e]);
      const int l = (tl2 >> 1) * 16 + (e >> 4), m = (tl2 & 1) * 16 + (e & 15);
      if (m < HS && l < HS + 2) {
        Xp[l * HS + m] = v;
        const float vc = v * cvec[m];                   // dkappa's factor c (see M8)
        if (l < HS) Xm[l * HS + m] = vc;
        else if (l == HS) sumD[m] = vc;                 // sum_p Dsig (completed below)
        else red[m] = vc;                               // sum_p Dtau
      }
      if (t < HS * HS) Mc[t] = Mm[t] * cvec[t % HS];   // dG = Dsig' (M c)^T
    }
    __syncthreads();
    if (t < HS) {
      const float dd1 = sumD[t], dt = red[t];
      const float dy1 = cvec[t] * ysumv[t];
      pb[H2_B1 + t] = dd1;
      pb[H2_W1 + HS + t] = dy1;
      pb[H2_W1 + t] = dd1 - dy1;
      sumD[t] = dd1 + dt;
      // dU2 (model_2.py:318-321): Z_k = sum_pq relu(kappa_pq,k) gamma_pq
      //   = sum_pq [kappa > 0] gamma (sigma_pk + tau_qk + y eps_k)
      //   = sum_l M_lk X'_lk + s0_k sum_p Dsig'_pk + t0_k sum_q Dtau'_qk + eps_k ysum_k
      // (sigma = G M + s0, tau = H M + t0; X' = sum_p G_p (x) Dsig'_p + H_p (x) Dtau'_p):
      // the per-pair accumulation of the classifier pass, from sums this block has anyway
      float z = fmaf(s0v[t], Xp[HS * HS + t], fmaf(t0v[t], Xp[(HS + 1) * HS + t], eps[t] * ysumv[t]));
#pragma unroll
      for (int l = 0; l < HS; ++l) z = fmaf(Mm[l * HS + t], Xp[l * HS + t], z);
      pb[H2_W2 + 2 * t] = -z;
      pb[H2_W2 + 2 * t + 1] = z;
    }
  }
  __syncthreads();
  MID_STAMP();
  // dU1e = V2^T X + (Nc-1) c2 (x) sumD and dV2 = X U1e^T as 16x16 MFMA tiles (4 each,
  // tiles 0-7), then dG = Dsig M^T, dH = Dtau M^T (tiles 8..); dc2 on the last wave
  float* dG = G;       // G, H dead once X is formed
  float* dH = Hh;
  for (int tile = wv; tile < 8 + 4 * SMAXC; tile += NT_MID / 64) {   // wave-uniform
    if (tile < 8) {
      const int which = tile >> 2, row0 = ((tile >> 1) & 1) * 16, col0 = (tile & 1) * 16;
      const int ra = row0 + (lane & 15), cb = col0 + (lane & 15);
      const f4v c = which == 0
          ? mfma_tile16_p(ra < HS ? Ws + H1_W2 + ra : kzero, ra < HS ? HS : 0,     // V2^T
                          cb < HS ? Xm + cb : kzero, cb < HS ? HS : 0, HS, lane)    // X
          : mfma_tile16_p(ra < HS ? Xm + ra * HS : kzero, ra < HS ? 1 : 0,          // X
                          cb < HS ? Ws + H2_W1 + (2 + cb) * HS : kzero, cb < HS ? 1 : 0,
                          HS, lane);                                                  // U1e^T
      const int cc = col0 + (lane & 15);
      if (cc < HS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = row0 + 4 * (lane >> 4) + q;
          if (rr < HS) {
            if (which == 0) pb[H2_W1 + (2 + rr) * HS + cc] = fmaf(Nc1 * Ws[H1_B2 + rr], sumD[cc], c[q]);
            else pb[H1_W2 + rr * HS + cc] = c[q];
          }
        }
      }
      continue;
    }
    const int tt = tile - 8;
    const int which = tt & 1, row0 = (tt >> 2) * 16, col0 = ((tt >> 1) & 1) * 16;
    const float* src = which ? Dtau : Dsig;
    const int pr = row0 + (lane & 15), lc = col0 + (lane & 15);
    const float* Mcm = U + NBUF_H * NC16 * HS + 16 * 256 + 22 * HS;   // M c (M9)
    const f4v c = mfma_tile16_p(pr < Nc ? src + pr * HS : kzero, pr < Nc ? 1 : 0,
                                lc < HS ? Mcm + lc * HS : kzero, lc < HS ? 1 : 0, HS, lane);
    const int l = col0 + (lane & 15);
    if (l < HS) {
      float* dst = which ? dH : dG;
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // padding rows (from -inf sigma / tau) kept finite
        const int pr = row0 + 4 * (lane >> 4) + q;
        dst[pr * HS + l] = pr < Nc ? c[q] : 0.f;
      }
    }
  }
  if (wv == NT_MID / 64 - 1 && lane < HS) {   // dc2[m] = (Nc-1) sum_k U1e[m][k] sumD[k]
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < HS; ++k) acc = fmaf(Ws[H2_W1 + (2 + lane) * HS + k], sumD[k], acc);
    pb[H1_B2 + lane] = Nc1 * acc;
  }
  __syncthreads();
  MID_STAMP();

  // ---- M10: hunk pair backward: dgamma = [g1 > 0](dG_p + dH_q) -----------------------
  float* Dal = Bf[4];   // Dsig/Dtau dead after dG/dH
  float* Dbe = Bf[5];
  {
    auto m10fix = [&](int j, int kk, float v) {
      const int e = j * HS + kk;
      if (SPLIT && (j & 1) != h) {                  // partner's rows: no D_alpha here
        Dal[e] = 0.f;
      } else {                                      // minus the diagonal pair of an own row
        const float dz = (alpha[e] + beta[e] > 0.f) ? (dG[e] + dH[e]) : 0.f;
        Dal[e] -= dz;
        v -= dz;
      }
      Dbe[e] = v;
    };
    pair_pass<KK_MID, SMAXC, 1, HS, false, decltype(m10fix)>(
        Nc, tg, alpha, beta, g * KK_MID, dlt, yb, WC, dG, dH, nullptr, 0, Dal, Dbe, ysumv, credg,
        rmul, radd, m10fix);
  }
  MID_STAMP();
  // dn_c[m] = Dalpha_c V1[m] + Dbeta_c V1[4+m]: m in {0,1} (x' parts) for M11, m in {2,3}
  // (class parts, [NC16][2] in the pair-tile scratch: dead after M10, below M11's dx'
  // partials) only when model_4's entity-edge backward needs them
  const int ndm = dnout ? 4 : 2;
  float* dnc = U + NBUF_H * NC16 * HS;
  if (wv < SMAXC) {   // MFMA row tiles
    const int row0 = wv * 16, rr = row0 + (lane & 15), m = lane & 15;
    const bool rv = rr < Nc, mv = m < ndm;
    const f4v c = mfma_tile16_p(rv ? Dal + rr * HS : kzero, rv ? 1 : 0,
                                mv ? Ws + H1_W1 + m * HS : kzero, mv ? 1 : 0, HS, lane) +
                  mfma_tile16_p(rv ? Dbe + rr * HS : kzero, rv ? 1 : 0,
                                mv ? Ws + H1_W1 + (4 + m) * HS : kzero, mv ? 1 : 0, HS, lane);
    if (mv) {
      float* dst = m < 2 ? dnb + m : dnc + (m - 2);
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[2 * (row0 + 4 * (lane >> 4) + q)] = c[q];   // 0 past Nc
    }
  }
  __syncthreads();
  if constexpr (SPLIT) {
    pair_send(dnb, 2 * Nc, xout + 2 * XS, xtag(epoch, 3) ^ xsend, t);   // dV1 overlaps
    if (dnout) pair_send(dnc, 2 * Nc, xout + 2 * XS + Nc, xtag(epoch, 3) ^ xsend, t);
    // waves 4-15 warm this XCD's L2 with the count matrices (M11 reads every column; M3
    // fetched only the own half) while waves 0-3 run dV1
    if (wv >= 4) {
      const int nw = PL.ncst - PL.ks;                     // ks | kt words
      uint32_t acc = 0;
      for (int w = (t - 256) * 16; w < nw; w += (NT_MID - 256) * 16) acc ^= pp[PL.ks + w];
      asm volatile("" ::"v"(acc));
    }
  }
  if (wv < 4) {         // dV1 rows 0..7 and dc1: [n^T; 1] . Dalpha, n^T . Dbeta  (MFMA)
    const int side = wv >> 1, col0 = (wv & 1) * 16;
    const float* D = side ? Dbe : Dal;
    const int r = lane & 15, mc = col0 + (lane & 15);
    const float* pa = r < 4 ? nb + r : ((r == 4 && side == 0) ? kone : kzero);
    const f4v c = mfma_tile16_p(pa, r < 4 ? 4 : 0, mc < HS ? D + mc : kzero, mc < HS ? HS : 0, Nc,
                                lane);
    const int m = col0 + (lane & 15);
    if (m < HS) {
      if (lane < 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pb[H1_W1 + (4 * side + q) * HS + m] = c[q];
      } else if (lane < 32 && side == 0) {            // row 4: dc1 = sum_p Dalpha
        const float dc1 = c[0];
        pb[H1_B1 + m] = dc1;
        pb[H1_W1 + 8 * HS + m] = dc1 - ysumv[m];
        pb[H1_W1 + 9 * HS + m] = ysumv[m];
      }
    }
  }
  if constexpr (SPLIT) {
    if constexpr (STAMPS) MID_STAMP();
    xlate |= pair_recv_add(dnb, 2 * Nc, xin + 2 * XS, xtag(epoch, 3), t);
    if (dnout) xlate |= pair_recv_add(dnc, 2 * Nc, xin + 2 * XS + Nc, xtag(epoch, 3), t);
  } else {
    __syncthreads();
  }
  if (dnout) {                                 // the whole dn for the entity-edge backward
    if (h == 0)
      for (int e = t; e < 4 * Nc; e += NT_MID) {
        const int c = e >> 2, m = e & 3;
        dnout[(size_t)b * 4 * Nc + e] = m < 2 ? dnb[2 * c + m] : dnc[2 * c + m - 2];
      }
    __syncthreads();
  }
  MID_STAMP();

  // ---- M11: cross-graph backward: dx'_I = sum_c dn_c[0] ks[c][I] + dn_c[1] kt[c][I] ----
  //   4 hunk ranges (one per group) -> partial rows in the dq slot of U
  float* dxpart = U + 3 * NE4 * HS;
  {
    const uint16_t* ks = reinterpret_cast<const uint16_t*>(pp + PL.ks);
    const uint16_t* kt = reinterpret_cast<const uint16_t*>(pp + PL.kt);
    // split mode: the own node half only, 8 hunk ranges x 128 nodes
    constexpr int NGX = SPLIT ? 8 : NG_MID, TX = NT_MID / NGX;
    const int gx = t / TX, tx = t - gx * TX;
    const int cq = (Nc + NGX - 1) / NGX;
    const int cb0 = gx * cq, cb1 = (cb0 + cq < Nc) ? cb0 + cq : Nc;
    for (int I = nlo + tx; I < nhi; I += TX) {
      float a0 = 0.f, a1 = 0.f;
      for (int c = cb0; c < cb1; ++c) {
        a0 = fmaf(dnb[2 * c], (float)ks[(size_t)c * Ne + I], a0);
        a1 = fmaf(dnb[2 * c + 1], (float)kt[(size_t)c * Ne + I], a1);
      }
      dxpart[gx * NE4 + I] = a0 + a1;
    }
  }
  __syncthreads();
  MID_STAMP();

  // ---- M12: mlp2_entity_B1 backward.  U re-carved: P | E_bar | dq | dE | ... | h (-> rho)
  float* dq = U + 2 * NE4 * HS;
  float* dE = U + 3 * NE4 * HS;
  const int rho_off = (4 * NE4 * HS > NE4 * HS + 2 * HS * (NE4 + 4) + (NT_MID / 64) * 4 * HS)
                          ? 4 * NE4 * HS
                          : NE4 * HS + 2 * HS * (NE4 + 4) + (NT_MID / 64) * 4 * HS;
  float* hB = U + rho_off;                          // h, overwritten by rho row block by row block
  float* rho = hB;
  float* dw2p = Xm;                                 // [row block][21] partial dw2', db2'
  for (int i = nlo + t; i < nhi; i += NT_MID) {
    float d = (dxpart[i] + dxpart[NE4 + i]) + (dxpart[2 * NE4 + i] + dxpart[3 * NE4 + i]);
    if constexpr (SPLIT)
      d += (dxpart[4 * NE4 + i] + dxpart[5 * NE4 + i]) + (dxpart[6 * NE4 + i] + dxpart[7 * NE4 + i]);
    dxp[i] = (os[i] > 0.f) ? d : 0.f;               // d o_i (x' = relu(o))
  }
  {
    const float4* s0 = reinterpret_cast<const float4*>(EG);
    const float4* s1 = reinterpret_cast<const float4*>(EbG);
    const float4* s2 = reinterpret_cast<const float4*>(hEG);
    float4* d0 = reinterpret_cast<float4*>(Ps);
    float4* d1 = reinterpret_cast<float4*>(Eb);
    float4* d2 = reinterpret_cast<float4*>(hB);
    // the own node half's rows (this block parked them: same L2, plain loads)
    for (int e = nlo * HS / 4 + t; e < nhi * HS / 4; e += NT_MID) {
      d0[e] = s0[e];
      d1[e] = s1[e];
      d2[e] = s2[e];
    }
  }
  __syncthreads();
  MID_STAMP();
  // E2's row neighbour lists and row CSR offsets: fetched here into registers (one HBM
  // round trip hidden behind M12 / M13 and the rho exchange), written to LDS after the
  // exchange (the P slot they go to is read by dW5)
  const int rl = (int)pp[PL.xoffc];                 // padded row-list length (multiple of 4)
  const bool rfit = rl / 4 + rl <= NE4 * HS;
  const int xl2o = (rl / 4 + 3) & ~3;              // staged x values after the ids
  uint32_t e2id = 0u;
  float4 e2x = make_float4(0.f, 0.f, 0.f, 0.f);
  int e2off = 0;
  if (rfit) {
    if (t < rl / 4) e2id = pp[PL.lists + t];
    if (4 * t < rl) e2x = *reinterpret_cast<const float4*>(pp + PL.xl + 4 * t);
  }
  if (t <= Ne) e2off = reinterpret_cast<const int*>(pp + PL.offr)[t];
  // row-local chain per 16-row block: dq = [h > 0] w2' do;  dE = dq W1'[1:]^T;
  // rho = dE W5^T (into h's rows, consumed first); partial dw2' / db2' of the block
  for (int rb = (nlo >> 4) + wv; rb <= ((nhi - 1) >> 4); rb += NT_MID / 64) {   // wave-uniform
    const int row0 = rb * 16;
    for (int e = lane; e < 16 * HS; e += 64) {
      const int i = row0 + e / HS, k = e - (e / HS) * HS;
      if (i >= nlo && i < nhi) dq[i * HS + k] = (hB[i * HS + k] > 0.f) ? Ws[E3_W2 + k] * dxp[i] : 0.f;
    }
    {   // dw2' / db2' partials of the block: lane = (row r = lane / 4, units k = kq + 4 j)
      const int r = lane >> 2, kq = lane & 3, i = row0 + r;
      const bool ok = i >= nlo && i < nhi;
      const float d = ok ? dxp[i] : 0.f;
      float v[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int k = kq + 4 * j;
        v[j] = (ok && k < HS) ? hB[i * HS + k] * d : (k == HS ? d : 0.f);
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {                 // sum over the 16 rows (lane bits 2..5):
        v[j] += dppf<0x124>(v[j]);                  // DPP row_ror:4, row_ror:8 keep lane & 3;
        v[j] += dppf<0x128>(v[j]);                  // lanes 0-3 (r = 0) hold the stored sums
        v[j] = xrow_sum4(v[j]);
      }
      if (r == 0) {
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (kq + 4 * j <= HS) dw2p[rb * 21 + kq + 4 * j] = v[j];
      }
    }
    const int ir = row0 + (lane & 15);
    const bool rv = ir >= nlo && ir < nhi;
    {                                  // both 16-column halves, shared A reads
      f4v cc[2];
      const int m0 = lane & 15, m1 = 16 + (lane & 15);
      mfma_tile16x2_p(rv ? dq + ir * HS : kzero, rv ? 1 : 0, Ws + E3_W1 + (1 + m0) * HS, 1,
                      m1 < HS ? Ws + E3_W1 + (1 + m1) * HS : kzero, m1 < HS ? 1 : 0, HS, lane, cc[0], cc[1]);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col0 = cb * 16;
        const f4v c = cc[cb];
        const int m = col0 + (lane & 15);
        if (m < HS) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = row0 + 4 * (lane >> 4) + q;
            if (i >= nlo && i < nhi) dE[i * HS + m] = c[q];
          }
        }
      }
    }
    {                                  // both 16-column halves, shared A reads
      f4v cc[2];
      const int m0 = lane & 15, m1 = 16 + (lane & 15);
      mfma_tile16x2_p(rv ? dE + ir * HS : kzero, rv ? 1 : 0, Ws + E1_W5 + m0 * HS, 1,
                      m1 < HS ? Ws + E1_W5 + m1 * HS : kzero, m1 < HS ? 1 : 0, HS, lane, cc[0], cc[1]);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col0 = cb * 16;
        const f4v c = cc[cb];
        const int m = col0 + (lane & 15);
        if (m < HS) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = row0 + 4 * (lane >> 4) + q;
            if (i >= nlo && i < nhi) rho[i * HS + m] = c[q];
          }
        }
      }
    }
  }
  __syncthreads();
  // trailer zeros (fault slot: t = 2) before the rho send, whose vmcnt(0) completes them:
  // a late thread's fault store at the end then lands after them
  if (t < HDG_TRAILER - 2) pb[NP + 2 + t] = 0.f;
  if (t == 2) fsl[prow] = 0.f;                      // same thread as the fault slot
  if constexpr (SPLIT) pair_send(rho + nlo * HS, (nhi - nlo) * HS, xout + XSLOTS * XS, xtag(epoch, 5) ^ xsend, t);
  MID_STAMP();
  // ---- M13: reductions over rows: dW1' = [x, E_bar, 1]^T dq (waves 0-3),
  //      dW5 = [P, 1]^T dE (waves 4-7; row 20 -> db5 / 2(Ne-1)), dw2' / db2' (wave 8);
  //      split mode: over the own node half (partial gradients), the rho exchange overlaps
  if (wv < 4) {
    const int row0 = (wv >> 1) * 16, col0 = (wv & 1) * 16;
    const int lr = row0 + (lane & 15), kc = col0 + (lane & 15);
    const float* pa = lr == 0 ? xs : (lr <= HS ? Eb + lr - 1 : (lr == HS + 1 ? kone : kzero));
    const int sa = lr == 0 ? 1 : (lr <= HS ? HS : 0);
    const f4v c = mfma_tile16_p(pa + nlo * sa, sa, kc < HS ? dq + kc + nlo * HS : kzero,
                                kc < HS ? HS : 0, nhi - nlo, lane);
    const int k = col0 + (lane & 15);
    if (k < HS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int l = row0 + 4 * (lane >> 4) + q;
        if (l <= HS) pb[E3_W1 + l * HS + k] = c[q];
        else if (l == HS + 1) pb[E3_B1 + k] = c[q];
      }
    }
  } else if (wv < 8) {
    const int row0 = ((wv - 4) >> 1) * 16, col0 = ((wv - 4) & 1) * 16;
    const int lr = row0 + (lane & 15), kc = col0 + (lane & 15);
    const f4v c = mfma_tile16_p(lr < HS ? Ps + lr + nlo * HS : (lr == HS ? kone : kzero),
                                lr < HS ? HS : 0, kc < HS ? dE + kc + nlo * HS : kzero,
                                kc < HS ? HS : 0, nhi - nlo, lane);
    const int k = col0 + (lane & 15);
    if (k < HS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int l = row0 + 4 * (lane >> 4) + q;
        if (l < HS) pb[E1_W5 + l * HS + k] = c[q];
        else if (l == HS) pb[E1_B5 + k] = twoNe1 * c[q];
      }
    }
  } else if (wv == 8 && lane <= HS) {
    float acc = 0.f;
    for (int rb = nlo >> 4; rb <= ((nhi - 1) >> 4); ++rb) acc += dw2p[rb * 21 + lane];
    pb[lane < HS ? E3_W2 + lane : E3_B2] = acc;
  }
  if (t < 4) pb[TH1 + t] = 0.f;                     // map_theta*: data-independent
  if constexpr (SPLIT) {                             // the partner half's rho rows
    const int plo = h ? 0 : (Ne + 1) / 2, phi = h ? (Ne + 1) / 2 : Ne;
    xlate |= pair_recv_add<false>(rho + plo * HS, (phi - plo) * HS, xin + XSLOTS * XS,
                                  xtag(epoch, 5), t);
    if (h == 0 && t == 0) *xctr = epoch + 1u;     // last exchange of the pair: next epoch
  } else {
    __syncthreads();
  }
  MID_STAMP();

  // ---- E2: mlp_entity_B1 first-layer backward -----------------------------------------
  //   dz_ij = [z_ij > 0] (rho_i + rho_j)  (P_i holds row i AND column i of the grid)
  //   S0 = sum x_i dz, S1 = sum x_j dz, S2 = sum dz, S3 = sum a dz  ->
  //   dW1[0] = S0, dW1[1] = S1, dW1[2] = S2 - S3, dW1[3] = S3, db1 = S2.
  //   The a = 0 part reuses the forward's row sets: per k, sums of rho and of x*rho over
  //   every suffix (w1 >= 0) or prefix (w1 < 0) of the x-sorted order, one wave per scan,
  //   so each set sum is one table read.  a = 1 corrections over the set bits of row i,
  //   same (node, k) lane map as E1.
  const int TL = NE4 + 4;
  float* Tr = U + NE4 * HS;                // [HS][TL]   (E_bar, dq, dE slots are dead)
  float* Tx = Tr + HS * TL;                // [HS][TL]
  float* red2 = Tx + HS * TL;              // [16 waves][4][HS]  (ends below rho_off)
  // row neighbour (id, x) lists (padded, offsets xoffr still in offr), staged into the P
  // slot (dead after dW5) when they fit (rl <= 4096 < 4 NT_MID: one id word and one x
  // float4 per thread, fetched before M12); offc <- the compact row CSR (degrees)
  if (rfit) {
    if (t < rl / 4) Ps[t] = __builtin_bit_cast(float, e2id);
    if (4 * t < rl) *reinterpret_cast<float4*>(Ps + xl2o + 4 * t) = e2x;
  }
  if (t <= Ne) offc[t] = e2off;
  WAVE_STAMP(3);
  // The scan inputs in scan order, unit-major: Tr[k][4 + s] = rho of the node at scan slot
  // s (sorted slot m = s for the prefix units, w1 < 0; Ne - 1 - s for the suffix units), Tx
  // likewise x rho -- one block-wide pass over rho's rows (a node's 20 units on 20 lanes),
  // instead of each unit's wave gathering its column through perm: a column of the 20-word
  // row pitch lies on 8 of the 32 banks, a 4-way conflict on every gathered read.
  for (int e = t; e < Ne * HS; e += NT_MID) {
    const int m = e / HS, k = e - m * HS;
    const float v = rho[perm[m] * HS + k];
    const int sl = Ws[E1_W1 + HS + k] >= 0.f ? Ne - 1 - m : m;
    Tr[k * TL + 4 + sl] = v;
    Tx[k * TL + 4 + sl] = v * xsrt[m];
  }
  __syncthreads();
  // Per-unit inclusive scans in place: T[k][3 + c] = the sum over the first c scan slots
  // (T[k][3] = 0), so a suffix unit's set [m, Ne) is c = Ne - m and a prefix unit's [0, m)
  // is c = m (entity_bwd).  A lane owns 4 consecutive slots: one 16-byte read and write.
  // TB: 1 = the rho table, 2 = the x rho table, 3 = both
  auto unit_scan = [&](const int k, auto tbc) {
    constexpr int TB = decltype(tbc)::value;
    float* T0 = Tr + k * TL;
    float* T1 = Tx + k * TL;
    const int s0 = 4 * lane;                      // NE4 <= 256: one float4 per lane
    float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
    if (s0 < Ne) {
      if constexpr (TB & 1) a0 = *reinterpret_cast<const float4*>(T0 + 4 + s0);
      if constexpr (TB & 2) a1 = *reinterpret_cast<const float4*>(T1 + 4 + s0);
    }
    const float v0[4] = {a0.x, a0.y, a0.z, a0.w}, v1[4] = {a1.x, a1.y, a1.z, a1.w};
    float run0[4], run1[4];
    float r0 = 0.f, r1 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool in = s0 + q < Ne;                  // slots past Ne hold no node
      r0 += in ? v0[q] : 0.f;
      r1 += in ? v1[q] : 0.f;
      run0[q] = r0;
      run1[q] = r1;
    }
    const float off0 = (TB & 1) ? wave_incl_scan_dpp(r0) - r0 : 0.f;
    const float off1 = (TB & 2) ? wave_incl_scan_dpp(r1) - r1 : 0.f;
    if (s0 < Ne) {
      if constexpr (TB & 1)
        *reinterpret_cast<float4*>(T0 + 4 + s0) =
            make_float4(off0 + run0[0], off0 + run0[1], off0 + run0[2], off0 + run0[3]);
      if constexpr (TB & 2)
        *reinterpret_cast<float4*>(T1 + 4 + s0) =
            make_float4(off1 + run1[0], off1 + run1[1], off1 + run1[2], off1 + run1[3]);
    }
    if (lane == 0) {
      if constexpr (TB & 1) T0[3] = 0.f;
      if constexpr (TB & 2) T1[3] = 0.f;
    }
  };
  // units 0..15: both tables on wave k; units 16.. (HS > 16): one table each on waves
  // 4, 5, ...: the second unit no longer runs alone on waves 0-3 at the phase's tail
  constexpr int NWV = NT_MID / 64;
  static_assert(HS <= NWV + (NWV - 4) / 2, "scan map: extra units beyond waves 4..15");
  if (wv < HS) unit_scan(wv, std::integral_constant<int, 3>{});
  if (wv >= 4 && wv < 4 + 2 * (HS - NWV)) {
    const int k = NWV + ((wv - 4) >> 1);
    if ((wv - 4) & 1) unit_scan(k, std::integral_constant<int, 2>{});
    else unit_scan(k, std::integral_constant<int, 1>{});
  }
  WAVE_STAMP(4);
  __syncthreads();
  MID_STAMP();
  if (rfit)
    entity_bwd(lane, wv, Ws, xs, cum, pxd, nd, rq, rho, Tr, Tx, TL, offr, offc,
               reinterpret_cast<const uint8_t*>(Ps), Ps + xl2o, nlo, nhi, red2, Ne);
  else
    entity_bwd(lane, wv, Ws, xs, cum, pxd, nd, rq, rho, Tr, Tx, TL, offr, offc,
               reinterpret_cast<const uint8_t*>(pp + PL.lists),
               reinterpret_cast<const float*>(pp + PL.xl), nlo, nhi, red2, Ne);
  WAVE_STAMP(2);
  __syncthreads();
  if (t < 4 * HS) {
    const int w = t / HS, k = t - w * HS;
    float s = 0.f;
    for (int q = 0; q < NT_MID / 64; ++q) s += red2[(q * 4 + w) * HS + k];
    red[w * 32 + k] = s;
  }
  __syncthreads();
  if (t < HS) {
    const float s0 = red[t], s1 = red[32 + t], s2 = red[64 + t], s3 = red[96 + t];
    pb[E1_W1 + t] = s0;
    pb[E1_W1 + HS + t] = s1;
    pb[E1_W1 + 2 * HS + t] = s2 - s3;
    pb[E1_W1 + 3 * HS + t] = s3;
    pb[E1_B1 + t] = s2;
  }
  // a pair exchange timed out: every late thread poisons the CE slot, sets the fault slot
  // and the status word (identical values; thread 0's earlier CE store completed at its
  // polls' vmcnt(0) in the M9 receive, before the barriers that precede this).  No
  // block-wide vote here: the tail sits at the VGPR ceiling.
  // The step's probs stay as computed; the status word and the NaN CE void them.
  if (SPLIT && xlate) {
    pb[NP + HDG_TR_CE] = __builtin_nanf("");
    pb[NP + HDG_TR_FAULT] = 1.f;
    fsl[prow] = 1.f;
    if (status) xstore1(status, HDG_STATUS_XCH_TIMEOUT);
  }
  MID_STAMP();
#undef MID_STAMP
#undef WAVE_STAMP
}

// ------------------------------------------------------------------------------
// deterministic reduction of the partial rows (one per block of k_commit_step): a
// 1024-thread block takes RED_P = 16 parameters x 64 row phases (row r -> phase r % 64,
// fixed order); a thread's <= 4 rows per trip are loaded before they are added (one
// memory round trip up to 256 rows), the 4 phases of a wave close with two permlane
// swaps, the 16 waves in a fixed-order LDS sum.  Bitwise reproducible.  The correct-
// prediction count (slot NP + HDG_TR_COUNT, an exact integer per row) is summed as an
// integer alongside and returned in `count` (thread pl of that slot's block).
// ------------------------------------------------------------------------------
constexpr int RED_P = 16, RED_PH = NT_MID / RED_P;   // 16 parameters x 64 phases
constexpr int CNT_SLOT = m2::NP + HDG_TR_COUNT;

struct RedShared {
  float s[NT_MID / 64][RED_P];
  uint32_t c[NT_MID / 16];             // per (wave, phase lane group) count partials
};

__device__ __forceinline__ float reduce_commits(const float* __restrict__ part, int R, int p,
                                                bool valid, RedShared& sh, uint32_t& count) {
  const int pl = threadIdx.x & (RED_P - 1), ph = threadIdx.x / RED_P;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool isc = p == CNT_SLOT;
  float acc = 0.f;
  uint32_t accu = 0u;
  if (valid) {
    for (int b0 = ph; b0 < R; b0 += 4 * RED_PH) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int b = b0 + u * RED_PH;
        v[u] = b < R ? part[(size_t)b * NPART + p] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += v[u];
      if (isc) {
#pragma unroll
        for (int u = 0; u < 4; ++u) accu += (uint32_t)v[u];
      }
    }
  }
  acc = xrow_sum4(acc);                 // the wave's 4 phases (lanes pl, pl+16, +32, +48)
  if (lane < RED_P) sh.s[wv][pl] = acc;
  if (isc) sh.c[wv * 4 + (lane >> 4)] = accu;
  __syncthreads();
  float g = 0.f;
  count = 0u;
  if (threadIdx.x < RED_P) {
#pragma unroll
    for (int q = 0; q < NT_MID / 64; ++q) g += sh.s[q][pl];
    if (isc)
      for (int q = 0; q < NT_MID / 16; ++q) count += sh.c[q];
  }
  return g;
}

// the trailer's count slots from the integer total (each part < 2^16: exact under any
// float all-reduce of up to 256 ranks)
__device__ __forceinline__ void put_count(float* __restrict__ out, const uint32_t c) {
  out[0] = (float)(c & 0xFFFFu);
  out[1] = (float)(c >> 16);
  out[2] = 0.f;
}

// slots [p_begin, p_end) -> out[p - p_begin], those >= shift_at moved by shift (model_4 on
// the fused path: the model_2-layout slots past the entity-edge block)
__global__ __launch_bounds__(1024) void k_grad_reduce(const float* __restrict__ part, int B,
                                                      int p_begin, int p_end, int shift_at,
                                                      int shift, float* __restrict__ out) {
  __shared__ RedShared sh;
  const int p = p_begin + blockIdx.x * RED_P + (threadIdx.x & (RED_P - 1));
  uint32_t cnt;
  const float g = reduce_commits(part, B, p, p < p_end, sh, cnt);
  if (threadIdx.x >= RED_P || p >= p_end) return;
  float* o = out + (p - p_begin) + (p >= shift_at ? shift : 0);
  if (p == CNT_SLOT && p + 2 < p_end) put_count(o, cnt);
  else if (p < CNT_SLOT || p > CNT_SLOT + 2) o[0] = g;
}

// Single-process training step tail: the reduction above fused with TF1 Adam for the
// block's 64 parameters.  aux (written by block 0 of k_commit_step from the pre-update
// parameters): [lpara, lmap, |theta1|, |theta2|, sqrt(1-b2^t)/(1-b1^t), b1^(t+1),
// b2^(t+1)], so no block here depends on another.
__global__ __launch_bounds__(1024) void k_reduce_adam(const float* __restrict__ part, int B,
                                                      float* __restrict__ params,
                                                      float* __restrict__ mm,
                                                      float* __restrict__ vv,
                                                      float* __restrict__ bpow,
                                                      const float* __restrict__ aux, float lr,
                                                      float inv_pairs, float* __restrict__ stats,
                                                      float* __restrict__ grad, int fault_rows) {
  using namespace m2;
  __shared__ RedShared sh;
  const int p = blockIdx.x * RED_P + (threadIdx.x & (RED_P - 1));
  bool upd = threadIdx.x < RED_P && p < NP;
  // the update's operands are fetched before the reduction so both latencies overlap
  const float w = upd ? params[p] : 0.f, m0 = upd ? mm[p] : 0.f, v0 = upd ? vv[p] : 0.f;
  const float lr_t = lr * aux[4], n1 = aux[2], n2 = aux[3];
  // split mode: any block whose pair exchange timed out voids the whole update (the rows'
  // fault slots, contiguous past the rows: k_commit_step's fsl)
  bool bad = false;
  for (int r = threadIdx.x; r < fault_rows; r += NT_MID)
    bad |= part[(size_t)fault_rows * NPART + r] != 0.f;
  uint32_t cnt;
  const float g = reduce_commits(part, B, p, p < GRAD_LEN, sh, cnt);
  if (fault_rows > 0 && __syncthreads_or(bad)) upd = false;
  if (threadIdx.x >= RED_P) return;
  if (p == CNT_SLOT) put_count(grad + p, cnt);
  else if (p < CNT_SLOT || (p > CNT_SLOT + 2 && p < GRAD_LEN)) grad[p] = g;
  if (stats && p == CNT_SLOT) put_count(stats + 4, cnt);
  if (stats && p == NP + HDG_TR_FAULT) stats[7] = g;
  if (p == NP) {
    const float ce = g * inv_pairs;
    if (stats) {
      stats[0] = ce;
      stats[1] = aux[1];
      stats[2] = aux[0];
      stats[3] = 10.f * ce + 0.1f * aux[1] + aux[0];
    }
  }
  if (upd) {
    const float b1 = 0.9f, b2 = 0.999f, ep = 1e-8f;
    float gg = g + 0.001f * w;
    if (p >= TH1 && p < TH1 + 2) gg += 0.001f * w / n1;
    if (p >= TH2 && p < TH2 + 2) gg += 0.001f * w / n2;
    float m = m0, v = v0;
    m += (gg - m) * (1.f - b1);
    v += (gg * gg - v) * (1.f - b2);
    mm[p] = m;
    vv[p] = v;
    params[p] = w - lr_t * m / (sqrtf(v) + ep);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && upd) {
    bpow[0] = aux[5];
    bpow[1] = aux[6];
  }
}

// ------------------------------------------------------------------------------
// TF1 Adam (model_2.py:336-338): train_loss = 10 CE + 0.1 loss_map + loss_para.
//   g = dCE-part (from the reduction, already x10/(B Pc)) + 0.001 v
//       + [theta] 0.1*0.01*theta/|theta|
//   lr_t = lr sqrt(1-b2^t)/(1-b1^t);  m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   var -= lr_t m / (sqrt(v) + eps)     (tensorflow/core/kernels/training_ops.cc ApplyAdam)
// ------------------------------------------------------------------------------
constexpr int ADAM_PT = 4;   // parameters per thread: 4 x 1024 >= every variant's count

__global__ __launch_bounds__(1024) void k_adam_tf(float* __restrict__ params,
                                                  float* __restrict__ mm,
                                                  float* __restrict__ vv,
                                                  float* __restrict__ bpow,
                                                  const float* __restrict__ grad, int np,
                                                  float lr, float inv_pairs,
                                                  float* __restrict__ stats) {
  const int TH1 = np - 4, TH2 = np - 2;   // map_conv thetas close every variant
  __shared__ float red[16 * 4];
  __shared__ float sh[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // every operand of the thread's parameters is loaded up front: one memory round trip
  float w[ADAM_PT], g[ADAM_PT], m[ADAM_PT], v[ADAM_PT];
#pragma unroll
  for (int u = 0; u < ADAM_PT; ++u) {
    const int p = t + u * 1024;
    const bool ok = p < np;
    w[u] = ok ? params[p] : 0.f;
    g[u] = ok ? grad[p] : 0.f;
    m[u] = ok ? mm[p] : 0.f;
    v[u] = ok ? vv[p] : 0.f;
  }
  __shared__ float bp[2];          // beta powers through LDS: only thread 0 touches bpow
  if (t == 0) { bp[0] = bpow[0]; bp[1] = bpow[1]; }
  const float ce_sum = grad[np + HDG_TR_CE], fault = grad[np + HDG_TR_FAULT];
  float l2 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
  for (int u = 0; u < ADAM_PT; ++u) {
    const int p = t + u * 1024;
    l2 = fmaf(w[u], w[u], l2);
    if (p >= TH1 && p < TH1 + 2) t1 = fmaf(w[u], w[u], t1);
    if (p >= TH2 && p < TH2 + 2) t2 = fmaf(w[u], w[u], t2);
  }
  l2 = wave_sum(l2);
  t1 = wave_sum(t1);
  t2 = wave_sum(t2);
  if (lane == 0) { red[wv * 4] = l2; red[wv * 4 + 1] = t1; red[wv * 4 + 2] = t2; }
  __syncthreads();
  if (t < 3) {
    float s = 0.f;
    for (int q = 0; q < 16; ++q) s += red[q * 4 + t];
    sh[t] = s;
  }
  __syncthreads();
  const float n1 = sqrtf(sh[1]), n2 = sqrtf(sh[2]);
  const float b1p = bp[0], b2p = bp[1];
  const float lr_t = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  if (t == 0 && stats) {
    const float ce = ce_sum * inv_pairs;
    const float lmap = 0.01f * (n2 + n1);
    const float lpara = 0.0005f * sh[0];
    stats[0] = ce;
    stats[1] = lmap;
    stats[2] = lpara;
    stats[3] = 10.f * ce + 0.1f * lmap + lpara;
    for (int q = 0; q < 4; ++q) stats[4 + q] = grad[np + HDG_TR_COUNT + q];   // count, fault
  }
  if (fault != 0.f) return;   // a pair exchange timed out on some rank: no update
  const float b1 = 0.9f, b2 = 0.999f, ep = 1e-8f;
#pragma unroll
  for (int u = 0; u < ADAM_PT; ++u) {
    const int p = t + u * 1024;
    if (p >= np) break;
    float gg = g[u] + 0.001f * w[u];
    if (p >= TH1 && p < TH1 + 2) gg += 0.001f * w[u] / n1;
    if (p >= TH2 && p < TH2 + 2) gg += 0.001f * w[u] / n2;
    float mv = m[u], vq = v[u];
    mv += (gg - mv) * (1.f - b1);
    vq += (gg * gg - vq) * (1.f - b2);
    mm[p] = mv;
    vv[p] = vq;
    params[p] = w[u] - lr_t * mv / (sqrtf(vq) + ep);
  }
  if (t == 0) { bpow[0] = b1p * b1; bpow[1] = b2p * b2; }
}

// ------------------------------------------------------------------------------
// Data-parallel tail over xGMI (include/hdgnn.h hdg_*_dp).
// Every rank owns a mailbox of uncached device memory that each peer maps through HIP
// IPC.  Block k of the tail kernel owns gradient slots [16k, 16k + 16): it forms its
// local values (the fixed-order sum of the partial rows, or the rank's reduced gradient),
// writes each as an 8-byte (value, tag) word with a system-scope write-through store into
// slot (parity, rank, p) of EVERY peer's mailbox (xGMI, one hop, all peers at once; the
// 8-byte word is single-copy atomic, as in RCCL's LL protocol), polls its own mailbox for
// the peers' words with L2-bypassing loads, and sums the world's values in rank order
// 0..W-1: every rank holds the same bits, so the replicas stay bitwise equal.
//   tag = epoch << 1 | fault: epoch is a per-block launch counter kept in the own mailbox
//   (all ranks issue the same launches); parity = epoch & 1 double-buffers the words, so
//   a rank one launch ahead writes over words every peer has already read (it needed the
//   peers' words of its previous launch, which they sent after reading theirs).  A peer
//   that never arrives ends the wait after wait_ticks: HDG_STATUS_DP_TIMEOUT, NaN loss,
//   no update on that block -- never a hang.
// ------------------------------------------------------------------------------
namespace dpk {
constexpr int MAXW = HDG_DP_MAX_WORLD;
constexpr int GLENP = HDG_DP_MAX_LEN;               // >= every variant's grad length, x16
constexpr int NBLK = GLENP / RED_P;
constexpr size_t DATA_WORDS = 2ull * MAXW * GLENP;  // u64 (value, tag) words
constexpr size_t OFF_EPOCH = DATA_WORDS * 8;        // u32 [256] per-block launch counters
constexpr size_t OFF_AUX = OFF_EPOCH + 256 * 4;     // f32 [8] loss terms + Adam factor
constexpr size_t OFF_GLOC = OFF_AUX + 8 * 4;        // f32 [GLENP] the rank's own gradient
constexpr size_t BYTES = OFF_GLOC + GLENP * 4;      //   (general path, hdg_train_step_dp)
constexpr unsigned long long WAIT_DEFAULT = 1000000000ull;   // 10 s of s_memrealtime
static_assert(GLENP % RED_P == 0 && NBLK <= 256, "mailbox layout");
static_assert(GLENP >= 3129 + HDG_TRAILER, "every variant's gradient fits a mailbox row");
enum { SUM = 0, PART = 1, GRAD = 2 };
}  // namespace dpk
// SUM / GRAD blocks only move 16 words per rank: 256 threads (16 ranks x 16 slots), so
// the grid stays small and resident even when several ranks share one device (tests);
// PART runs k_reduce_adam's 1024-thread reduction first
constexpr int DP_NT_LIGHT = dpk::MAXW * RED_P;

struct DpArgs {
  uint32_t* box[dpk::MAXW];
  int rank, world;
  unsigned long long wait;
};

typedef uint32_t xu2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void dstore2(uint32_t* p, const xu2 w) {
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ xu2 dload2(const uint32_t* p) {
  xu2 w;
  asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(w) : "v"(p) : "memory");
  return w;
}
__device__ __forceinline__ uint32_t* dp_slot(uint32_t* box, uint32_t par, int src, int p) {
  return box + 2 * (((size_t)par * dpk::MAXW + src) * dpk::GLENP + p);
}

// MODE SUM:  gout = world sum of src[0..glen)                       (hdg_dp_allreduce)
// MODE PART: local = fixed-order sum of R partial rows (k_reduce_adam's reduction), then
//            world sum -> gout, TF Adam with aux from k_commit_step   (hdg_train_step_dp)
// MODE GRAD: local = src[0..glen) (a rank's reduced gradient), aux from k_dp_aux (hdg_adam_dp)
template <int MODE>
__global__ __launch_bounds__(1024) void k_dp_tail(const float* __restrict__ src, const int R,
                                                  const int np, const int glen,
                                                  float* __restrict__ gout,
                                                  float* __restrict__ params,
                                                  float* __restrict__ mm, float* __restrict__ vv,
                                                  float* __restrict__ bpow,
                                                  const float* __restrict__ aux, const float lr,
                                                  const float inv_pairs,
                                                  float* __restrict__ stats,
                                                  uint32_t* __restrict__ status,
                                                  const int fault_rows, const DpArgs d) {
  __shared__ RedShared sh;
  __shared__ float gl[RED_P];
  __shared__ float vals[dpk::MAXW][RED_P];
  __shared__ uint32_t s_ep, s_cnt;
  const int t = threadIdx.x, blk = blockIdx.x;
  const int l = t & (RED_P - 1), r = t / RED_P;
  const int p = blk * RED_P + l;
  uint32_t* own = d.box[d.rank];
  uint32_t* ep = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(own) + dpk::OFF_EPOCH);
  if (t == 0) s_ep = ep[blk] + 1u;
  // the update's operands are fetched first so their latency overlaps the reduction
  bool upd = MODE != dpk::SUM && t < RED_P && p < np;
  const float w = upd ? params[p] : 0.f, m0 = upd ? mm[p] : 0.f, v0 = upd ? vv[p] : 0.f;
  float g = 0.f;
  bool bad = false;
  if constexpr (MODE == dpk::PART) {
    for (int q = t; q < fault_rows; q += 1024)             // k_commit_step's fsl
      bad |= src[(size_t)fault_rows * NPART + q] != 0.f;
    uint32_t cnt;
    g = reduce_commits(src, R, p, p < glen, sh, cnt);
    if (t < RED_P && p == CNT_SLOT) s_cnt = cnt;
  } else {
    if (t < RED_P && p < glen) g = src[p];
    if constexpr (MODE == dpk::GRAD) bad = t == 0 && src[np + HDG_TR_FAULT] != 0.f;
  }
  bad = __syncthreads_or(bad);               // also publishes s_ep and s_cnt
  if (t < RED_P) {
    if (MODE == dpk::PART && p >= CNT_SLOT && p <= CNT_SLOT + 2)   // three 16-bit parts
      g = p == CNT_SLOT ? (float)(s_cnt & 0xFFFFu) : (p == CNT_SLOT + 1 ? (float)(s_cnt >> 16) : 0.f);
    gl[l] = g;
  }
  __syncthreads();
  const uint32_t e = s_ep, par = e & 1u;
  const bool mine = r < d.world && p < glen;
  if (mine && r != d.rank)                    // to every peer at once
    dstore2(dp_slot(d.box[r], par, d.rank, p),
            (xu2){__float_as_uint(gl[l]), (e << 1) | (bad ? 1u : 0u)});
  bool late = false, rbad = false;
  if (mine) {
    float v = gl[l];
    if (r != d.rank) {
      const uint32_t* in = dp_slot(own, par, r, p);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      xu2 wd = dload2(in);
      while ((wd.y >> 1) != (e & 0x7FFFFFFFu)) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > d.wait) { late = true; break; }
        __builtin_amdgcn_s_sleep(1);
        wd = dload2(in);
      }
      v = __uint_as_float(wd.x);
      rbad = (wd.y & 1u) != 0u;
    }
    vals[r][l] = v;
  }
  const bool anylate = __syncthreads_or(late);
  const bool anybad = __syncthreads_or(rbad) || bad;
  if (t == 0) ep[blk] = e;                    // this block's launch is consumed
  if (t >= RED_P || p >= glen) return;
  float tot = 0.f;
  for (int q = 0; q < d.world; ++q) tot += vals[q][l];
  if (MODE != dpk::SUM && p == np + HDG_TR_CE && anylate) tot = __builtin_nanf("");
  gout[p] = tot;
  if (anylate && t == 0 && status) xstore1(status, HDG_STATUS_DP_TIMEOUT);
  if constexpr (MODE == dpk::SUM) return;
  const int TH1 = np - 4, TH2 = np - 2;
  if (stats && p >= np + HDG_TR_COUNT && p <= np + HDG_TR_FAULT)   // count parts, fault
    stats[4 + (p - np - HDG_TR_COUNT)] = tot;
  if (p == np + HDG_TR_CE && stats) {
    const float ce = tot * inv_pairs;
    stats[0] = ce;
    stats[1] = aux[1];
    stats[2] = aux[0];
    stats[3] = 10.f * ce + 0.1f * aux[1] + aux[0];
  }
  if (anylate || anybad) upd = false;
  if (upd) {
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
    const float lr_t = lr * aux[4], n1 = aux[2], n2 = aux[3];
    float gg = tot + 0.001f * w;
    if (p >= TH1 && p < TH1 + 2) gg += 0.001f * w / n1;
    if (p >= TH2 && p < TH2 + 2) gg += 0.001f * w / n2;
    float m = m0, v = v0;
    m += (gg - m) * (1.f - b1);
    v += (gg * gg - v) * (1.f - b2);
    mm[p] = m;
    vv[p] = v;
    params[p] = w - lr_t * m / (sqrtf(v) + eps);
  }
  if (blk == 0 && t == 0 && upd) {
    bpow[0] = aux[5];
    bpow[1] = aux[6];
  }
}

// k_dp_tail's SUM / GRAD modes for ranks that share a device (hdg_dp.flags HDG_DP_SHARED):
// G blocks per rank (dp_shared_grid: (W - 1) G <= CUs / 2, G >= HDG_DP_SHARED_BLOCKS),
// block b owning the slot groups b, b + G, ... .  A
// block first sends the words of all its groups (the values are src[p], the epoch of group
// k is ep[k] + 1 as in k_dp_tail), then receives, sums and updates its groups in order:
// the same words, tags, rank-order sums and Adam arithmetic as one k_dp_tail block per
// group, so the two kernels give the same bits and keep the same per-group launch counters.
// Only G blocks per rank spin, so the W-1 ranks waiting for the last one cover at most
// half the CUs and the last rank's step kernel always finds CUs to run on.
template <int MODE>
__global__ __launch_bounds__(DP_NT_LIGHT) void k_dp_tail_shared(
    const float* __restrict__ src, const int np, const int glen, float* __restrict__ gout,
    float* __restrict__ params, float* __restrict__ mm, float* __restrict__ vv,
    float* __restrict__ bpow, const float* __restrict__ aux, const float lr,
    const float inv_pairs, float* __restrict__ stats, uint32_t* __restrict__ status,
    const DpArgs d) {
  static_assert(MODE != dpk::PART, "the shared-device tail exchanges a reduced gradient");
  __shared__ float vals[dpk::MAXW][RED_P];
  const int t = threadIdx.x, l = t & (RED_P - 1), r = t / RED_P;
  const int ngrp = (glen + RED_P - 1) / RED_P;
  uint32_t* own = d.box[d.rank];
  uint32_t* ep = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(own) + dpk::OFF_EPOCH);
  const bool bad = MODE == dpk::GRAD && src[np + HDG_TR_FAULT] != 0.f;
  // 1. every word of this block's groups to every peer
  if (r < d.world && r != d.rank) {
    for (int k = blockIdx.x; k < ngrp; k += gridDim.x) {
      const int p = k * RED_P + l;
      const uint32_t e = ep[k] + 1u;
      if (p < glen)
        dstore2(dp_slot(d.box[r], e & 1u, d.rank, p),
                (xu2){__float_as_uint(src[p]), (e << 1) | (bad ? 1u : 0u)});
    }
  }
  // 2. per group: the peers' words, the rank-order sum, TF Adam
  for (int k = blockIdx.x; k < ngrp; k += gridDim.x) {
    const int p = k * RED_P + l;
    const uint32_t e = ep[k] + 1u, par = e & 1u;
    bool upd = MODE != dpk::SUM && t < RED_P && p < np;
    const float w = upd ? params[p] : 0.f, m0 = upd ? mm[p] : 0.f, v0 = upd ? vv[p] : 0.f;
    bool late = false, rbad = false;
    if (r < d.world && p < glen) {
      float v;
      if (r != d.rank) {
        const uint32_t* in = dp_slot(own, par, r, p);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        xu2 wd = dload2(in);
        while ((wd.y >> 1) != (e & 0x7FFFFFFFu)) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > d.wait) { late = true; break; }
          __builtin_amdgcn_s_sleep(1);
          wd = dload2(in);
        }
        v = __uint_as_float(wd.x);
        rbad = (wd.y & 1u) != 0u;
      } else {
        v = src[p];
      }
      vals[r][l] = v;
    }
    const bool anylate = __syncthreads_or(late);
    const bool anybad = __syncthreads_or(rbad) || bad;
    if (t == 0) ep[k] = e;                      // this group's launch is consumed
    if (t < RED_P && p < glen) {
      float tot = 0.f;
      for (int q = 0; q < d.world; ++q) tot += vals[q][l];
      if (MODE != dpk::SUM && p == np + HDG_TR_CE && anylate) tot = __builtin_nanf("");
      gout[p] = tot;
      if (anylate && t == 0 && status) xstore1(status, HDG_STATUS_DP_TIMEOUT);
      if constexpr (MODE == dpk::GRAD) {
        const int TH1 = np - 4, TH2 = np - 2;
        if (stats && p >= np + HDG_TR_COUNT && p <= np + HDG_TR_FAULT)
          stats[4 + (p - np - HDG_TR_COUNT)] = tot;
        if (p == np + HDG_TR_CE && stats) {
          const float ce = tot * inv_pairs;
          stats[0] = ce;
          stats[1] = aux[1];
          stats[2] = aux[0];
          stats[3] = 10.f * ce + 0.1f * aux[1] + aux[0];
        }
        if (anylate || anybad) upd = false;
        if (upd) {
          const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
          const float lr_t = lr * aux[4], n1 = aux[2], n2 = aux[3];
          float gg = tot + 0.001f * w;
          if (p >= TH1 && p < TH1 + 2) gg += 0.001f * w / n1;
          if (p >= TH2 && p < TH2 + 2) gg += 0.001f * w / n2;
          float m = m0, v = v0;
          m += (gg - m) * (1.f - b1);
          v += (gg * gg - v) * (1.f - b2);
          mm[p] = m;
          vv[p] = v;
          params[p] = w - lr_t * m / (sqrtf(v) + eps);
        }
        if (k == 0 && t == 0 && upd) {
          bpow[0] = aux[5];
          bpow[1] = aux[6];
        }
      }
    }
    __syncthreads();                            // vals is rewritten by the next group
  }
}

// aux for MODE GRAD (k_commit_step's block 0 writes it on the fused path): loss terms of
// the pre-update parameters (model_2.py:123-130, 326-333) and TF ApplyAdam's lr factor,
// in k_adam_tf's summation order
__global__ __launch_bounds__(1024) void k_dp_aux(const float* __restrict__ params, const int np,
                                                 const float* __restrict__ bpow,
                                                 float* __restrict__ aux) {
  const int TH1 = np - 4, TH2 = np - 2;
  __shared__ float red[16 * 4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float l2 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
  for (int u = 0; u < ADAM_PT; ++u) {
    const int p = t + u * 1024;
    const float w = p < np ? params[p] : 0.f;
    l2 = fmaf(w, w, l2);
    if (p >= TH1 && p < TH1 + 2) t1 = fmaf(w, w, t1);
    if (p >= TH2 && p < TH2 + 2) t2 = fmaf(w, w, t2);
  }
  l2 = wave_sum(l2);
  t1 = wave_sum(t1);
  t2 = wave_sum(t2);
  if (lane == 0) { red[wv * 4] = l2; red[wv * 4 + 1] = t1; red[wv * 4 + 2] = t2; }
  __syncthreads();
  if (t == 0) {
    float s[3] = {0.f, 0.f, 0.f};
    for (int q = 0; q < 16; ++q)
      for (int c = 0; c < 3; ++c) s[c] += red[q * 4 + c];
    const float n1 = sqrtf(s[1]), n2 = sqrtf(s[2]);
    const float b1p = bpow[0], b2p = bpow[1];
    aux[0] = 0.0005f * s[0];
    aux[1] = 0.01f * (n2 + n1);
    aux[2] = n1;
    aux[3] = n2;
    aux[4] = sqrtf(1.f - b2p) / (1.f - b1p);
    aux[5] = b1p * 0.9f;
    aux[6] = b2p * 0.999f;
  }
}

// ------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------
int smax_c(int nc) { return nc <= 80 ? 5 : (nc <= 128 ? 8 : 10); }

struct Work {   // workspace carve (floats)
  size_t Esave, rowq, gam, part, aux, xch, total;
};

Work work_layout(const hdg_shape* s) {
  Work w;
  const size_t B = s->batch, Ne = s->ne;
  const size_t NC16 = 16 * (size_t)smax_c(s->nc);
  size_t o = 0;
  auto take = [&](size_t n) { size_t r = o; o += (n + 63) & ~(size_t)63; return r; };
  w.Esave = take(3 * B * Ne * HS);
  w.rowq = take((B * Ne * HS + 1) / 2);     // u16
  w.gam = take(B * NC16 * NC16);
  // one partial row per block (2 per commit split), then the rows' fault slots (2B floats)
  w.part = take(2 * B * (size_t)NPART + 2 * B);
  w.aux = take(8);
  // block-pair inboxes (split mode): [B][2 halves][XSLOTS][NC16*HS] u64 (value, tag) words;
  // zero at allocation, left zero by every completed launch
  w.xch = take(2 * B * 4 * ((size_t)XSLOTS * NC16 * HS / 2 + XRHO) + B);   // + epochs
  w.total = o;
  return w;
}

// k_prep_counts tile width: TI Ne-rows / -columns per block (<= 64 KiB of counters where
// possible, two blocks per CU), and the LDS words it needs
int prep_lds_words(int ne, int nc, int ti) {
  return (ti + 1) * nc + 2 * nc + ne + ti * ((ne + 31) / 32);
}
int prep_tile(int ne, int nc) {
  int ti = 64;
  while (ti > 16 && ti * nc > 16384) ti >>= 1;
  while (ti > 1 && prep_lds_words(ne, nc, ti) > 38 * 1024) ti >>= 1;
  return ti;
}

// ------------------------------------------------------------------------------
// kh_tile<MODE>  grid (ceil(Nc / HTC), ceil(Nc / HTR), B), 1024 threads = 4 groups of 256
// (one per five hidden units): the general path's hunk pair sums on one HTR-row x
// HTC-column block of the commit's pair grid with the fused kernel's pair tiles -- row sums
// and column sums from ONE sweep (the two-pass kernels sweep every pair twice, once per
// side), block partials reduced in a fixed order by kw_hunk_fin*:
//   MODE 0  relu(z), z = alpha_p + beta_q + y delta           (kw_hunk_fwd's G / H)
//   MODE 1  [z > 0] (dG_p + dH_q)                            (kw_hunk_mlpb's D alpha / D beta)
//   MODE 2  [kappa > 0] gamma_pq, kappa = sigma_p + tau_q + y eps   (kw_hunk_clsb's sums)
// Rpart [B][CC][Nc][20] row sums over the block's columns, Cpart [B][RC][Nc][20] column sums
// over its rows, ysp [B][RC][CC][20] sum y e (MODE 1, 2).  The diagonal pair is inside the
// sweep for MODE 0 / 1 (removed by kw_hunk_fin0 / fin1); gamma's diagonal is 0.
// ------------------------------------------------------------------------------
constexpr int HTR = 256, HTC = 64, HT_SMAX = HTC / 16;

template <int MODE>
__global__ __launch_bounds__(NT_MID) void kh_tile(hdg::HTileArgs a) {
  constexpr int CRW = tile_cred_words<HT_SMAX, KK_MID>();
  __shared__ __attribute__((aligned(16))) float Al[HTR * HS];
  __shared__ __attribute__((aligned(16))) float Bl[HTC * HS];
  __shared__ __attribute__((aligned(16))) float Wr[MODE == 1 ? HTR * HS : 4];
  __shared__ __attribute__((aligned(16))) float Wc[MODE == 1 ? HTC * HS : 4];
  __shared__ float cred[NG_MID * CRW];
  const int cc = blockIdx.x, rc = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int Nc = a.Nc, CC = gridDim.x, RC = gridDim.y, WC = (Nc + 31) >> 5;
  const int j0 = cc * HTC, r0 = rc * HTR;
  const int nr = Nc - r0 < HTR ? Nc - r0 : HTR, ncol = Nc - j0 < HTC ? Nc - j0 : HTC;
  const size_t cb = (size_t)b * Nc * HS;
  {   // 16-byte copies, every load of a thread issued before its stores
    const float4* ra = reinterpret_cast<const float4*>(a.rows + cb + (size_t)r0 * HS);
    const float4* ca = reinterpret_cast<const float4*>(a.cols + cb + (size_t)j0 * HS);
    const int nra = nr * HS / 4, nca = HTC * HS / 4, ncv = ncol * HS / 4;
    const float4 pad = make_float4(PADNEG, PADNEG, PADNEG, PADNEG), zero4 = {0.f, 0.f, 0.f, 0.f};
    float4 v0 = t < nra ? ra[t] : pad, v1 = t + NT_MID < nra ? ra[t + NT_MID] : pad;
    float4 w0 = zero4, w1 = zero4, u = pad, uw = zero4;
    if constexpr (MODE == 1) {
      const float4* rw = reinterpret_cast<const float4*>(a.wrow + cb + (size_t)r0 * HS);
      w0 = t < nra ? rw[t] : zero4;
      w1 = t + NT_MID < nra ? rw[t + NT_MID] : zero4;
    }
    if (t < nca) {
      u = t < ncv ? ca[t] : pad;
      if constexpr (MODE == 1)
        uw = t < ncv ? reinterpret_cast<const float4*>(a.wcol + cb + (size_t)j0 * HS)[t] : zero4;
    }
    float4* A4 = reinterpret_cast<float4*>(Al);
    if (t < HTR * HS / 4) A4[t] = v0;
    if (t + NT_MID < HTR * HS / 4) A4[t + NT_MID] = v1;
    if constexpr (MODE == 1) {
      float4* W4 = reinterpret_cast<float4*>(Wr);
      if (t < HTR * HS / 4) W4[t] = w0;
      if (t + NT_MID < HTR * HS / 4) W4[t + NT_MID] = w1;
    }
    if (t < nca) {
      reinterpret_cast<float4*>(Bl)[t] = u;
      if constexpr (MODE == 1) reinterpret_cast<float4*>(Wc)[t] = uw;
    }
  }
  __syncthreads();
  const int g = t >> 8, tg = t & 255;
  const uint32_t* bits = a.ybits + ((size_t)b * Nc + r0) * WC + (j0 >> 5);
  float* Rout = a.rpart + (((size_t)b * CC + cc) * Nc + r0) * HS;
  float* Cout = a.cpart + (((size_t)b * RC + rc) * Nc + j0) * HS;
  float* ysum = a.ysp + (((size_t)b * RC + rc) * CC + cc) * HS;
  const float* gam = MODE == 2 ? a.gam + ((size_t)b * Nc + r0) * Nc + j0 : nullptr;
  pair_tile<KK_MID, HT_SMAX, MODE, HS, 0, false>(
      nr, tg, Al, Bl, g * KK_MID, a.dl, bits, WC - (j0 >> 5), Wr, Wc, gam, Nc, Rout, Cout, ysum,
      cred + g * CRW, 1, 0, NoFix{}, ncol, WC, j0 - r0);
}

}  // namespace

namespace hdg {

hipError_t launch_hunk_tile(int mode, const HTileArgs& a, int B, hipStream_t st) {
  const dim3 grid((a.Nc + HTC - 1) / HTC, (a.Nc + HTR - 1) / HTR, B);
  switch (mode) {
    case 0: hipLaunchKernelGGL(kh_tile<0>, grid, dim3(NT_MID), 0, st, a); break;
    case 1: hipLaunchKernelGGL(kh_tile<1>, grid, dim3(NT_MID), 0, st, a); break;
    default: hipLaunchKernelGGL(kh_tile<2>, grid, dim3(NT_MID), 0, st, a); break;
  }
  return kmark(mode == 0 ? "kh_tile<0>" : (mode == 1 ? "kh_tile<1>" : "kh_tile<2>"), st);
}
int hunk_tile_cols() { return HTC; }
int hunk_tile_rows() { return HTR; }

}  // namespace hdg

namespace {

}  // namespace

namespace hdg {

thread_local char g_err[512] = "";
thread_local KTrace* g_ktrace = nullptr;

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

hipError_t launch_prep_maps(const hdg_shape* s, const hdg_batch* bt, int stride, int o_ks,
                            int o_kt, int o_ncst, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_prep_counts,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ti = prep_tile(s->ne, s->nc);
  const size_t lds = (size_t)prep_lds_words(s->ne, s->nc, ti) * 4;
  uint32_t* prep = (uint32_t*)bt->prep;
  hipLaunchKernelGGL(k_prep_ncst, dim3(s->batch), dim3(256), 0, st, prep, s->nc, stride, o_ncst,
                     0);
  hipLaunchKernelGGL(k_prep_counts, dim3((s->ne + ti - 1) / ti, s->batch, 2), dim3(512), lds, st,
                     bt->abits, bt->hid, bt->nlen, prep, s->ne, s->nc, ti, stride, o_ks, o_kt,
                     o_ncst);
  hipLaunchKernelGGL(k_prep_ncst, dim3(s->batch), dim3(256), 0, st, prep, s->nc, stride, o_ncst,
                     1);
  return hipGetLastError();
}

// tf.global_variables() order per variant: E1 E3 | EE EC | H1 H2 TH
Off param_offsets(int v) {
  Off o;
  memset(&o, 0xff, sizeof(o));   // -1 everywhere
  if (v < 1 || v > 4) return o;
  int p = 0;
  if (v == 2 || v == 4) {
    o.E1_W1 = p; p += 80;  o.E1_B1 = p; p += 20;  o.E1_W5 = p; p += 400; o.E1_B5 = p; p += 20;
    o.E3_W1 = p; p += 420; o.E3_B1 = p; p += 20;  o.E3_W2 = p; p += 20;  o.E3_B2 = p; p += 1;
  }
  if (v == 3 || v == 4) {
    o.EE_W11 = p; p += 20; o.EE_W12 = p; p += 40; o.EE_B1 = p; p += 20;
    o.EE_W2 = p; p += 400; o.EE_B2 = p; p += 20;
    o.EC_W1 = p; p += 440; o.EC_B1 = p; p += 20; o.EC_W2 = p; p += 40; o.EC_B2 = p; p += 2;
  }
  o.H1_W1 = p; p += 200; o.H1_B1 = p; p += 20; o.H1_W2 = p; p += 400; o.H1_B2 = p; p += 20;
  o.H2_W1 = p; p += 440; o.H2_B1 = p; p += 20; o.H2_W2 = p; p += 40;  o.H2_B2 = p; p += 2;
  o.TH1 = p; p += 2; o.TH2 = p; p += 2;
  o.NP = p;
  return o;
}

}  // namespace hdg

namespace {

using hdg::fail;

bool fused_fits(const hdg_shape* s) {
  if ((s->variant != 2 && s->variant != 4) || s->ne > 256 || s->nc > 160) return false;
  const StepLayout L = step_layout(s->ne, s->nc, smax_c(s->nc));
  return (size_t)L.total * 4 <= 160 * 1024;
}

// validates the shape; returns the resolved path (HDG_PATH_FUSED / _GENERAL) or -1
int resolve(const hdg_shape* s) {
  if (!s) return fail(HDG_EINVAL, "shape is NULL"), -1;
  if (s->variant < 1 || s->variant > 4)
    return fail(HDG_EINVAL, "variant must be 1..4 (model_<variant>.py), got %d", s->variant), -1;
  if (s->batch < 1) return fail(HDG_EINVAL, "batch must be >= 1 (got %d)", s->batch), -1;
  if (s->ne < 2 || s->ne > 4096) return fail(HDG_EINVAL, "ne must be in [2,4096] (got %d)", s->ne), -1;
  if (s->nc < 2 || s->nc > 2048) return fail(HDG_EINVAL, "nc must be in [2,2048] (got %d)", s->nc), -1;
  if (s->path == HDG_PATH_GENERAL) return HDG_PATH_GENERAL;
  const bool fits = fused_fits(s);
  if (s->path == HDG_PATH_FUSED) {
    if (!fits)
      return fail(HDG_EINVAL, "the fused path runs model_2 / model_4 with ne <= 256, "
                              "nc <= 160 (got variant %d, ne=%d, nc=%d)", s->variant, s->ne,
                  s->nc), -1;
    return HDG_PATH_FUSED;
  }
  if (s->path != HDG_PATH_AUTO) return fail(HDG_EINVAL, "unknown path %d", s->path), -1;
  return fits ? HDG_PATH_FUSED : HDG_PATH_GENERAL;
}

int check_batch(const hdg_batch* bt) {
  if (!bt || !bt->x || !bt->abits || !bt->ybits || !bt->hid || !bt->nlen || !bt->prep)
    return fail(HDG_EINVAL, "batch has a NULL device pointer");
  return 0;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail((int)e_, "%s: %s", #expr, hipGetErrorString(e_));   \
  } while (0)

#define RESOLVE(s, var)                          \
  const int var = resolve(s);                    \
  if (var < 0) return HDG_EINVAL

// Split mode (two blocks per commit, hunk rows split by parity, block-pair exchanges)
// needs both blocks of a pair resident at once.  The host asks for it only when the
// whole grid fits the device at the kernel's occupancy (2 B <= CUs x blocks per CU, one
// 1024-thread block per CU in practice); that holds on an otherwise idle GPU, and a pair
// that still cannot meet (another process holding CUs, CU masking) fails its launch
// loudly (xch_fault) rather than hanging.  A cooperative launch would check residency at
// launch time but costs +17-20 us per replay (MI355X_MICROARCH price list), a quarter of
// the step.  HDG_FUSED_SPLIT=0 forces one block per commit.
int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return n;
}

template <int SMAXC, bool TRAIN, bool STAMPS, bool SPLIT>
hipError_t set_step_attr() {
  static bool attr_set = false;   // the attribute is per function; 160 KiB covers every shape
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_commit_step<SMAXC, TRAIN, STAMPS, SPLIT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  return hipSuccess;
}

// resident split-mode blocks per CU for this shape: the kernel's register / wave limit
// (occupancy query, memoized per device and tile count: it does not depend on the
// shape) combined per call with the shape's LDS bytes
template <int SMAXC>
int split_blocks_per_cu(const hdg_shape* s) {
  static int regs_cache[16] = {0};   // idempotent memo of a device query
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  int nb = __atomic_load_n(&regs_cache[dev], __ATOMIC_RELAXED);
  if (nb == 0) {
    if (set_step_attr<SMAXC, true, false, true>() != hipSuccess) return 0;
    // registers / waves from the occupancy query (without dynamic LDS: the query rejects
    // sizes above the default 64 KiB limit)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, (const void*)k_commit_step<SMAXC, true, false, true>, NT_MID, 0) != hipSuccess) {
      (void)hipGetLastError();      // leave no sticky error for the launch's check
      return 0;
    }
    nb = nb > 0 ? nb : -1;
    __atomic_store_n(&regs_cache[dev], nb, __ATOMIC_RELAXED);
  }
  if (nb < 0) return 0;
  const size_t lds = (size_t)step_layout(s->ne, s->nc, SMAXC).total * 4;   // this shape
  const int by_lds = lds > 0 ? (int)((160 * 1024) / lds) : nb;
  return nb < by_lds ? nb : by_lds;
}

// split-mode grid: two blocks per commit, padded to whole groups of 16 (k_commit_step's
// XCD-paired block map)
int split_grid(int batch) { return (2 * batch + 15) & ~15; }

bool use_split(const hdg_shape* s) {
  if (s->flags & HDG_FLAG_NO_SPLIT) return false;
  const char* e = getenv("HDG_FUSED_SPLIT");
  if (e && e[0] == '0') return false;
  int per_cu = 0;
  switch (smax_c(s->nc)) {
    case 5: per_cu = split_blocks_per_cu<5>(s); break;
    case 8: per_cu = split_blocks_per_cu<8>(s); break;
    default: per_cu = split_blocks_per_cu<10>(s); break;
  }
  return split_grid(s->batch) <= cu_count() * per_cu;
}

int part_rows(const hdg_shape* s, bool split) { return split ? 2 * s->batch : s->batch; }

// HDG_DEBUG_XCH_FAULT=1 (tests only): block 1 of every pair sends exchange words with a
// tag its partner never accepts, forcing the timeout path of every exchange
uint32_t debug_xfault() {
  const char* e = getenv("HDG_DEBUG_XCH_FAULT");
  return (e && e[0] && e[0] != '0') ? 0x40000000u : 0u;
}

struct StepOut {
  float* probs;
  float* logits;
  uint32_t* status;
  float* ehr;
};
StepOut step_out(const hdg_outputs* out) {
  return out ? StepOut{out->probs, out->logits, out->status, out->ehr}
             : StepOut{nullptr, nullptr, nullptr, nullptr};
}

// model_4 hooks of the step kernel (k_commit_step's ee_ins / ncpart / dnout); all zero for
// model_2
struct Hyb {
  int ins;
  const unsigned long long* ncpart;
  int ncpt;
  float* dnout;
};

template <int SMAXC, bool TRAIN, bool STAMPS, bool SPLIT>
hipError_t launch_step(const hdg_shape* s, const hdg_batch* bt, const float* params, float* ws,
                       const Work& w, const StepOut& o, float ce_scale,
                       unsigned long long* stamps, const float* bpow, hipStream_t st,
                       const Hyb& hy) {
  const StepLayout L = step_layout(s->ne, s->nc, SMAXC);
  const size_t lds = (size_t)L.total * 4;
  if (hipError_t e = set_step_attr<SMAXC, TRAIN, STAMPS, SPLIT>(); e != hipSuccess) return e;
  const int grid = SPLIT ? split_grid(s->batch) : s->batch;
  hipLaunchKernelGGL((k_commit_step<SMAXC, TRAIN, STAMPS, SPLIT>), dim3(grid), dim3(NT_MID), lds,
                     st, bt->x, bt->abits, bt->ybits, (const uint32_t*)bt->prep, params,
                     ws + w.Esave, (uint16_t*)(ws + w.rowq), ws + w.gam, ws + w.part, o.probs,
                     o.logits, s->ne, s->nc, ce_scale, stamps, bpow ? ws + w.aux : nullptr, bpow,
                     s->batch, (unsigned long long*)(ws + w.xch), o.status,
                     SPLIT ? debug_xfault() : 0u, hy.ins, hy.ncpart, hy.ncpt, hy.dnout,
                     (!TRAIN && o.ehr) ? 1 : 0);
  return hdg::kmark("k_commit_step", st);
}

template <bool TRAIN, bool STAMPS = false>
hipError_t dispatch_step(const hdg_shape* s, const hdg_batch* bt, const float* params, float* ws,
                         const Work& w, const StepOut& o, float ce_scale,
                         unsigned long long* stamps, hipStream_t st, bool split,
                         const float* bpow = nullptr, const Hyb& hy = Hyb{0, nullptr, 0, nullptr}) {
#define HDG_STEP(SM)                                                                              \
  return split ? launch_step<SM, TRAIN, STAMPS, true>(s, bt, params, ws, w, o, ce_scale, stamps, \
                                                      bpow, st, hy)                               \
               : launch_step<SM, TRAIN, STAMPS, false>(s, bt, params, ws, w, o, ce_scale, stamps,\
                                                       bpow, st, hy)
  switch (smax_c(s->nc)) {
    case 5: HDG_STEP(5);
    case 8: HDG_STEP(8);
    default: HDG_STEP(10);
  }
#undef HDG_STEP
}

// loss_E_HR of a fused forward launch: the step kernel parked G / H in gamma's slot
hipError_t fused_ehr(const hdg_shape* s, float* ws, const Work& w, const float* params,
                     const hdg_outputs* out, hipStream_t st) {
  if (!out || !out->ehr) return hipSuccess;
  const size_t cs = (size_t)16 * smax_c(s->nc) * 16 * smax_c(s->nc);   // NC16^2 per commit
  return hdg::launch_ehr(ws + w.gam, ws + w.gam + (size_t)s->nc * HS, cs, s->batch, s->nc,
                         params, s->variant, out->ehr, st);
}

float pair_count(const hdg_shape* s) {
  const int bg = s->batch_global > 0 ? s->batch_global : s->batch;
  return (float)bg * (float)(s->nc * (s->nc - 1));
}

// ---- model_4 on the fused path ("hybrid"): the entity-edge stage runs on the general
// path's kernels (hdg::wide_ee_fwd / wide_ee_bwd) around k_commit_step, which runs the
// model_2-shaped rest of the step (entity pair MLP, E3, cross-graph, hunk stage,
// classifier, their backward) with model_4's parameters, the entity-edge aggregate as
// the class part of n_c and dn exported for the entity-edge backward.  model_4 is model_2
// plus that stage (model_4.py:92-97): the two meet only at n_c[2:4] and dn_c[2:4].
// prep = [fused prep | general prep]; workspace = [fused | general].
bool is_hybrid(const hdg_shape* s, int path) { return path == HDG_PATH_FUSED && s->variant == 4; }

size_t fused_prep_bytes(const hdg_shape* s) {
  return (size_t)s->batch * prep_layout(s->ne, s->nc).words * 4;
}

struct HybWork {
  size_t wide, total;   // float offsets
};
HybWork hyb_layout(const hdg_shape* s) {
  HybWork h;
  auto up = [](size_t n) { return (n + 63) & ~(size_t)63; };
  h.wide = up(work_layout(s).total);
  h.total = h.wide + up(hdg::wide_workspace_bytes(s) / 4);
  return h;
}

hdg_batch wide_half(const hdg_batch* bt, const hdg_shape* s) {
  hdg_batch bw = *bt;
  bw.prep = (char*)bt->prep + fused_prep_bytes(s);
  return bw;
}

// train: grad = the full model_4 gradient + trailer (the fused rows' model_2-layout slots
// mapped past the entity-edge block, the EE block from the general path's rows);
// !train: forward only, CE sum -> *ce_sum.  events[0..2] as hdg_fwd_bwd_events.
int hybrid_run(const hdg_shape* s, const hdg_batch* bt, const float* params, float* grad,
               hdg_outputs* out, float* ce_sum, void* workspace, bool train, hipStream_t st,
               void* const* events, const hdg::WideAdam* adam = nullptr) {
  const HybWork hw = hyb_layout(s);
  float* ws = (float*)workspace;
  float* wws = ws + hw.wide;
  const hdg_batch bw = wide_half(bt, s);
  const int ins = hdg::param_offsets(4).H1_W1 - m2::H1_W1;   // the entity-edge block (1002)
  auto mark = [&](int k) -> hipError_t {
    return events ? hipEventRecord((hipEvent_t)events[k], st) : hipSuccess;
  };
  HIP_TRY(mark(0));
  if (int rc = hdg::wide_ee_fwd(s, &bw, params, wws, st,
                                adam && train ? adam->state->beta_pow : nullptr))
    return rc;
  const Work w = work_layout(s);
  const bool split = use_split(s);
  const float pairs = pair_count(s);
  const Hyb hy{ins, hdg::wide_ncpart(s, wws), hdg::wide_ncpart_tiles(s),
               train ? hdg::wide_dn(s, wws) : nullptr};
  if (!train) {
    HIP_TRY(dispatch_step<false>(s, bt, params, ws, w, step_out(out), 0.f, nullptr, st, split,
                                 nullptr, hy));
    if (ce_sum) {
      hipLaunchKernelGGL(k_grad_reduce, dim3(1), dim3(1024), 0, st, ws + w.part,
                         part_rows(s, split), m2::NP, m2::NP + 1, GRAD_LEN, 0, ce_sum);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(fused_ehr(s, ws, w, params, out, st));
    HIP_TRY(mark(1));
    HIP_TRY(mark(2));
    return 0;
  }
  HIP_TRY(dispatch_step<true>(s, bt, params, ws, w, step_out(out), 10.f / pairs, nullptr, st,
                              split, nullptr, hy));
  const int R = part_rows(s, split);
  if (adam) {   // the fused rows are reduced inside the final reduce + Adam kernel
    hdg::WideAdam ad = *adam;
    ad.fused = hdg::FusedRows{ws + w.part, R, NPART, m2::H1_W1, ins, m2::NP,
                              split ? ws + w.part + (size_t)R * NPART : nullptr};
    if (int rc = hdg::wide_ee_bwd(s, &bw, params, wws, grad, st, &ad)) return rc;
  } else {
    // the fused rows: [0, H1_W1) in place, [H1_W1, GRAD_LEN) past the entity-edge block
    hipLaunchKernelGGL(k_grad_reduce, dim3((GRAD_LEN + RED_P - 1) / RED_P), dim3(1024), 0, st,
                       ws + w.part, R, 0, GRAD_LEN, m2::H1_W1, ins, grad);
    HIP_TRY(hdg::kmark("k_grad_reduce", st));
    if (int rc = hdg::wide_ee_bwd(s, &bw, params, wws, grad, st)) return rc;
  }
  HIP_TRY(mark(1));
  HIP_TRY(mark(2));
  return 0;
}

}  // namespace

extern "C" {

int hdg_version(void) { return HDG_ABI_VERSION; }
const char* hdg_last_error(void) { return hdg::g_err; }
int hdg_resolve_path(const hdg_shape* shape) { return resolve(shape); }
int hdg_param_count(int32_t variant) {
  const int np = hdg::param_offsets(variant).NP;
  if (np < 0) fail(HDG_EINVAL, "variant must be 1..4 (model_1 .. model_4), got %d", (int)variant);
  return np < 0 ? -1 : np;
}
int hdg_grad_len(int32_t variant) {
  const int np = hdg_param_count(variant);
  return np < 0 ? -1 : np + HDG_TRAILER;
}

size_t hdg_workspace_bytes(const hdg_shape* shape) {
  const int path = resolve(shape);
  if (path < 0) return 0;
  if (path == HDG_PATH_GENERAL) return hdg::wide_workspace_bytes(shape);
  if (is_hybrid(shape, path)) return hyb_layout(shape).total * sizeof(float);
  return work_layout(shape).total * sizeof(float);
}

size_t hdg_prep_bytes(const hdg_shape* shape) {
  const int path = resolve(shape);
  if (path < 0) return 0;
  if (path == HDG_PATH_GENERAL) return hdg::wide_prep_bytes(shape);
  if (is_hybrid(shape, path)) return fused_prep_bytes(shape) + hdg::wide_prep_bytes(shape);
  return fused_prep_bytes(shape);
}

int hdg_prep_counts_layout(const hdg_shape* s, int64_t* stride, int64_t* ks, int64_t* kt,
                           int64_t* ncst) {
  RESOLVE(s, path);
  if (!stride || !ks || !kt || !ncst) return fail(HDG_EINVAL, "NULL output pointer");
  if (path == HDG_PATH_GENERAL) {
    hdg::wide_prep_counts_layout(s, stride, ks, kt, ncst);
    return 0;
  }
  const PrepLayout L = prep_layout(s->ne, s->nc);
  *stride = L.words;
  *ks = L.ks;
  *kt = L.kt;
  *ncst = L.ncst;
  return 0;
}

int hdg_pack_classes(const uint8_t* cls, int32_t batch, int32_t n, uint32_t* bits,
                     void* stream) {
  if (!cls || !bits || batch < 1 || n < 1)
    return fail(HDG_EINVAL, "hdg_pack_classes: NULL pointer or batch=%d n=%d", batch, n);
  const int W = (n + 31) / 32;
  const long long words = (long long)batch * n * W;
  hipLaunchKernelGGL(k_pack_classes, dim3((unsigned)((words + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cls, n, W, words, bits);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_prepare(const hdg_shape* s, const hdg_batch* bt, void* stream) {
  RESOLVE(s, path);
  if (int rc = check_batch(bt)) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (path == HDG_PATH_GENERAL) return hdg::wide_prepare(s, bt, st);
  hipLaunchKernelGGL(k_prep_sort, dim3(s->batch), dim3(256), 0, st, bt->x, bt->abits,
                     (uint32_t*)bt->prep, s->ne, s->nc);
  HIP_TRY(hipGetLastError());
  const PrepLayout L = prep_layout(s->ne, s->nc);
  HIP_TRY(hdg::launch_prep_maps(s, bt, L.words, L.ks, L.kt, L.ncst, st));
  if (is_hybrid(s, path)) {        // + the general path's tables for the entity-edge stage
    const hdg_batch bw = wide_half(bt, s);
    return hdg::wide_prepare(s, &bw, st);
  }
  return 0;
}

int hdg_fwd_bwd_events(const hdg_shape* s, const hdg_batch* bt, const float* params,
                       float* grad, hdg_outputs* out, void* workspace, void* stream,
                       void* const* events) {
  RESOLVE(s, path);
  if (int rc = check_batch(bt)) return rc;
  if (!params || !grad || !workspace) return fail(HDG_EINVAL, "NULL params/grad/workspace");
  hipStream_t st = (hipStream_t)stream;
  auto mark = [&](int k) -> hipError_t {
    return events ? hipEventRecord((hipEvent_t)events[k], st) : hipSuccess;
  };
  if (path == HDG_PATH_GENERAL) {
    HIP_TRY(mark(0));
    if (int rc = hdg::wide_run(s, bt, params, grad, out, nullptr, workspace, true, st)) return rc;
    HIP_TRY(mark(1));
    HIP_TRY(mark(2));
    return 0;
  }
  if (is_hybrid(s, path)) return hybrid_run(s, bt, params, grad, out, nullptr, workspace, true, st, events);
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const bool split = use_split(s);
  HIP_TRY(mark(0));
  HIP_TRY(dispatch_step<true>(s, bt, params, ws, w, step_out(out), 10.f / pair_count(s), nullptr,
                              st, split));
  HIP_TRY(mark(1));
  hipLaunchKernelGGL(k_grad_reduce, dim3((GRAD_LEN + RED_P - 1) / RED_P), dim3(1024), 0, st,
                     ws + w.part, part_rows(s, split), 0, GRAD_LEN, GRAD_LEN, 0, grad);
  HIP_TRY(hdg::kmark("k_grad_reduce", st));
  HIP_TRY(mark(2));
  return 0;
}

int hdg_fwd_bwd_kernel_events(const hdg_shape* s, const hdg_batch* bt, const float* params,
                              float* grad, hdg_outputs* out, void* workspace, void* stream,
                              void* const* events, int32_t n_events, const char** names,
                              int32_t* n_kernels) {
  if (!events || n_events < 2 || !names || !n_kernels)
    return fail(HDG_EINVAL, "hdg_fwd_bwd_kernel_events: need >= 2 events, names, n_kernels");
  hdg::KTrace t{events, (int)n_events, 0, names};
  HIP_TRY(hipEventRecord((hipEvent_t)events[0], (hipStream_t)stream));
  hdg::g_ktrace = &t;
  const int rc = hdg_fwd_bwd_events(s, bt, params, grad, out, workspace, stream, nullptr);
  hdg::g_ktrace = nullptr;
  *n_kernels = t.n;
  return rc;
}

int hdg_fwd_bwd(const hdg_shape* s, const hdg_batch* bt, const float* params, float* grad,
                hdg_outputs* out, void* workspace, void* stream) {
  return hdg_fwd_bwd_events(s, bt, params, grad, out, workspace, stream, nullptr);
}

int hdg_debug_step_stamps(const hdg_shape* s, const hdg_batch* bt, const float* params,
                          void* workspace, unsigned long long* stamps, void* stream) {
  RESOLVE(s, path);
  if (path != HDG_PATH_FUSED || s->variant != 2)
    return fail(HDG_EINVAL, "phase stamps exist on the fused path for model_2 only");
  if (int rc = check_batch(bt)) return rc;
  if (!stamps || !workspace || !params) return fail(HDG_EINVAL, "NULL stamps/workspace/params");
  const Work w = work_layout(s);
  const hipError_t e = dispatch_step<true, true>(s, bt, params, (float*)workspace, w,
                                                 step_out(nullptr), 1.f, stamps,
                                                 (hipStream_t)stream, use_split(s));
  HIP_TRY(e);
  return 0;
}

int hdg_adam_tf(const hdg_shape* s, hdg_state* state, const float* grad, float lr, float* stats,
                void* stream) {
  RESOLVE(s, path);
  (void)path;
  if (hdg::param_offsets(s->variant).NP > ADAM_PT * 1024)
    return fail(HDG_EINVAL, "k_adam_tf holds at most %d parameters", ADAM_PT * 1024);
  if (!state || !state->params || !state->adam_m || !state->adam_v || !state->beta_pow || !grad)
    return fail(HDG_EINVAL, "NULL state/grad pointer");
  hipLaunchKernelGGL(k_adam_tf, dim3(1), dim3(1024), 0, (hipStream_t)stream, state->params,
                     state->adam_m, state->adam_v, state->beta_pow, grad,
                     hdg::param_offsets(s->variant).NP, lr, 1.f / pair_count(s), stats);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_train_step(const hdg_shape* s, const hdg_batch* bt, hdg_state* state, float lr,
                   hdg_outputs* out, float* grad, void* workspace, void* stream) {
  if (!state || !state->params || !state->adam_m || !state->adam_v || !state->beta_pow)
    return fail(HDG_EINVAL, "NULL state pointer");
  RESOLVE(s, path);
  if (int rc = check_batch(bt)) return rc;
  if (!grad || !workspace) return fail(HDG_EINVAL, "NULL grad/workspace");
  hipStream_t st = (hipStream_t)stream;
  if (path == HDG_PATH_GENERAL || is_hybrid(s, path)) {
    // TF Adam inside the final reduction (kw_reduce_adam): no separate k_adam_tf launch
    const hdg::WideAdam adam{state, lr, 1.f / pair_count(s), out ? out->stats : nullptr, {}};
    return path == HDG_PATH_GENERAL
        ? hdg::wide_run(s, bt, state->params, grad, out, nullptr, workspace, true, st, &adam)
        : hybrid_run(s, bt, state->params, grad, out, nullptr, workspace, true, st, nullptr,
                     &adam);
  }
  // single process, fused path: k_commit_step (+ loss stats / Adam factor from block 0),
  // then the fused deterministic reduction + TF Adam; no all-reduce point in between
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const float pairs = pair_count(s);
  const bool split = use_split(s);
  HIP_TRY(dispatch_step<true>(s, bt, state->params, ws, w, step_out(out), 10.f / pairs, nullptr,
                              st, split, state->beta_pow));
  hipLaunchKernelGGL(k_reduce_adam, dim3((GRAD_LEN + RED_P - 1) / RED_P), dim3(1024), 0, st,
                     ws + w.part, part_rows(s, split), state->params, state->adam_m,
                     state->adam_v, state->beta_pow, ws + w.aux, lr, 1.f / pairs,
                     out ? out->stats : nullptr, grad, split ? part_rows(s, split) : 0);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_forward(const hdg_shape* s, const hdg_batch* bt, const float* params, hdg_outputs* out,
                float* ce_sum, void* workspace, void* stream) {
  RESOLVE(s, path);
  if (int rc = check_batch(bt)) return rc;
  if (!params || !workspace) return fail(HDG_EINVAL, "NULL params/workspace");
  hipStream_t st = (hipStream_t)stream;
  if (path == HDG_PATH_GENERAL)
    return hdg::wide_run(s, bt, params, nullptr, out, ce_sum, workspace, false, st);
  if (is_hybrid(s, path))
    return hybrid_run(s, bt, params, nullptr, out, ce_sum, workspace, false, st, nullptr);
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const bool split = use_split(s);
  HIP_TRY(dispatch_step<false>(s, bt, params, ws, w, step_out(out), 0.f, nullptr, st, split));
  if (ce_sum) {
    hipLaunchKernelGGL(k_grad_reduce, dim3(1), dim3(1024), 0, st, ws + w.part,
                       part_rows(s, split), m2::NP, m2::NP + 1, GRAD_LEN, 0, ce_sum);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(fused_ehr(s, ws, w, params, out, st));
  return 0;
}

// ---- data parallelism over xGMI ------------------------------------------------
static_assert(sizeof(hipIpcMemHandle_t) == HDG_DP_HANDLE_BYTES, "IPC handle size");

size_t hdg_dp_mailbox_bytes(void) { return dpk::BYTES; }

// CRC-32C (Castagnoli, reflected 0x82F63B78), slicing by 8: the checksum of the TF V2
// checkpoint bundle's records (hdgnn.tfckpt; LevelDB / TF masked CRCs)
uint32_t hdg_crc32c(const void* data, size_t n, uint32_t crc) {
  // slicing-by-8 tables, built once (a C++11 function-local static: thread-safe init)
  struct Tab {
    uint32_t t[8][256];
    Tab() {
      for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        t[0][i] = c;
      }
      for (uint32_t i = 0; i < 256; ++i)
        for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFFu];
    }
  };
  static const Tab T;
  const auto& tab = T.t;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = crc ^ 0xFFFFFFFFu;
  for (; n >= 8; n -= 8, p += 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = tab[7][lo & 0xFFu] ^ tab[6][(lo >> 8) & 0xFFu] ^ tab[5][(lo >> 16) & 0xFFu] ^
        tab[4][lo >> 24] ^ tab[3][hi & 0xFFu] ^ tab[2][(hi >> 8) & 0xFFu] ^
        tab[1][(hi >> 16) & 0xFFu] ^ tab[0][hi >> 24];
  }
  for (; n; --n, ++p) c = tab[0][(c ^ *p) & 0xFFu] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

static uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

static int write_file(const char* path, const void* p, size_t n) {
  FILE* f = fopen(path, "wb");
  if (!f) return fail(HDG_EINVAL, "cannot open %s for writing", path);
  const size_t w = n ? fwrite(p, 1, n, f) : 0;
  const int rc = fclose(f);
  if (w != n || rc != 0) return fail(HDG_EINVAL, "short write to %s", path);
  return 0;
}

int hdg_bundle_write(const char* data_path, const char* index_path, const float* state,
                     int64_t n_state, const int32_t* gather, int64_t n_floats,
                     uint8_t* index_img, int64_t index_len, const int64_t* entries,
                     int32_t n_entries, const int64_t* blocks, int32_t n_blocks) {
  if (!data_path || !index_path || !state || n_state < 0 || !gather || n_floats < 0 ||
      !index_img || index_len < 48 || (n_entries && !entries) || (n_blocks && !blocks))
    return fail(HDG_EINVAL, "hdg_bundle_write: bad arguments");
  std::vector<float> blob((size_t)n_floats);
  for (int64_t i = 0; i < n_floats; ++i) {
    if (gather[i] < 0 || gather[i] >= n_state)
      return fail(HDG_EINVAL, "hdg_bundle_write: gather[%lld] = %d outside the %lld-float state",
                  (long long)i, (int)gather[i], (long long)n_state);
    blob[i] = state[gather[i]];
  }
  const uint8_t* bytes = reinterpret_cast<const uint8_t*>(blob.data());
  const int64_t nbytes = n_floats * 4;
  for (int32_t e = 0; e < n_entries; ++e) {        // entry proto field 6: masked CRC of bytes
    const int64_t off = entries[3 * e], size = entries[3 * e + 1], pos = entries[3 * e + 2];
    if (off < 0 || size < 0 || off + size > nbytes || pos < 0 || pos + 4 > index_len)
      return fail(HDG_EINVAL, "hdg_bundle_write: entry %d out of range", (int)e);
    const uint32_t c = mask_crc(hdg_crc32c(bytes + off, (size_t)size, 0));
    memcpy(index_img + pos, &c, 4);
  }
  for (int32_t b = 0; b < n_blocks; ++b) {         // block trailer: type byte + masked CRC
    const int64_t off = blocks[2 * b], len = blocks[2 * b + 1];
    if (off < 0 || len < 0 || off + len + 5 > index_len)
      return fail(HDG_EINVAL, "hdg_bundle_write: block %d out of range", (int)b);
    const uint32_t c = mask_crc(hdg_crc32c(index_img + off, (size_t)len + 1, 0));
    memcpy(index_img + off + len + 1, &c, 4);
  }
  // both files under temporary names first, then renamed data before index: a crash or a
  // full disk mid-save never leaves a new .index beside a stale or partial .data
  const std::string dtmp = std::string(data_path) + ".tmp", itmp = std::string(index_path) + ".tmp";
  int rc = write_file(dtmp.c_str(), bytes, (size_t)nbytes);
  if (!rc) rc = write_file(itmp.c_str(), index_img, (size_t)index_len);
  if (!rc && rename(dtmp.c_str(), data_path) != 0)
    rc = fail(HDG_EINVAL, "cannot rename %s to %s", dtmp.c_str(), data_path);
  if (!rc && rename(itmp.c_str(), index_path) != 0)
    rc = fail(HDG_EINVAL, "cannot rename %s to %s", itmp.c_str(), index_path);
  if (rc) {
    remove(dtmp.c_str());
    remove(itmp.c_str());
  }
  return rc;
}

// ---- background checkpoint writer -------------------------------------------------
// saver.save off the training thread: one native thread writes the queued bundles (and the
// small text files that go with them) in submission order, so the training loop's thread
// only copies the state into the job.  The first failure is kept for flush().
struct CkptJob {
  std::vector<float> state;                  // empty: no bundle in this job
  std::string data_path, index_path, removes, text_path, text;
  bool text_append = false;
};
struct hdg_ckpt_writer_s {
  std::vector<int32_t> gather;
  std::vector<uint8_t> image;
  std::vector<int64_t> entries, blocks;
  int64_t n_state = 0;
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<CkptJob> q;
  bool busy = false, stop = false;
  int err_code = 0;
  char err[512] = "";
  std::thread th;
};

static int ckpt_run(hdg_ckpt_writer_s* w, CkptJob& j) {
  if (!j.state.empty()) {
    std::vector<uint8_t> img = w->image;     // the CRCs are patched into a private copy
    if (int rc = hdg_bundle_write(j.data_path.c_str(), j.index_path.c_str(), j.state.data(),
                                  (int64_t)j.state.size(), w->gather.data(),
                                  (int64_t)w->gather.size(), img.data(), (int64_t)img.size(),
                                  w->entries.data(), (int32_t)(w->entries.size() / 3),
                                  w->blocks.data(), (int32_t)(w->blocks.size() / 2)))
      return rc;
  }
  size_t a = 0;                              // '\n'-separated paths: missing ones are fine
  while (a < j.removes.size()) {
    size_t e = j.removes.find('\n', a);
    if (e == std::string::npos) e = j.removes.size();
    if (e > a) remove(j.removes.substr(a, e - a).c_str());
    a = e + 1;
  }
  if (!j.text_path.empty()) {
    FILE* f = fopen(j.text_path.c_str(), j.text_append ? "ab" : "wb");
    if (!f) return fail(HDG_EINVAL, "cannot open %s for writing", j.text_path.c_str());
    const size_t n = j.text.size(), wr = n ? fwrite(j.text.data(), 1, n, f) : 0;
    if (fclose(f) != 0 || wr != n) return fail(HDG_EINVAL, "short write to %s", j.text_path.c_str());
  }
  return 0;
}

static void ckpt_loop(hdg_ckpt_writer_s* w) {
  std::unique_lock<std::mutex> lk(w->mu);
  for (;;) {
    w->cv.wait(lk, [&] { return w->stop || !w->q.empty(); });
    if (w->q.empty()) return;                // stop with nothing queued
    CkptJob j = std::move(w->q.front());
    w->q.pop_front();
    w->busy = true;
    lk.unlock();
    const int rc = ckpt_run(w, j);
    lk.lock();
    if (rc && !w->err_code) {
      w->err_code = rc;
      snprintf(w->err, sizeof(w->err), "%s", hdg::g_err);
    }
    w->busy = false;
    if (w->q.empty()) w->idle.notify_all();
  }
}

int hdg_ckpt_writer_create(const int32_t* gather, int64_t n_floats, int64_t n_state,
                           const uint8_t* index_img, int64_t index_len, const int64_t* entries,
                           int32_t n_entries, const int64_t* blocks, int32_t n_blocks,
                           void** writer) {
  if (!writer || !gather || n_floats < 0 || n_state < 0 || !index_img || index_len < 48 ||
      (n_entries && !entries) || (n_blocks && !blocks))
    return fail(HDG_EINVAL, "hdg_ckpt_writer_create: bad arguments");
  for (int64_t i = 0; i < n_floats; ++i)
    if (gather[i] < 0 || gather[i] >= n_state)
      return fail(HDG_EINVAL, "hdg_ckpt_writer_create: gather[%lld] outside the state",
                  (long long)i);
  auto* w = new hdg_ckpt_writer_s;
  w->gather.assign(gather, gather + n_floats);
  w->image.assign(index_img, index_img + index_len);
  w->entries.assign(entries, entries + 3 * (size_t)n_entries);
  w->blocks.assign(blocks, blocks + 2 * (size_t)n_blocks);
  w->n_state = n_state;
  w->th = std::thread(ckpt_loop, w);
  *writer = w;
  return 0;
}

int hdg_ckpt_writer_submit(void* writer, const float* state, const char* data_path,
                           const char* index_path, const char* removes, const char* text_path,
                           const char* text, int32_t text_append) {
  auto* w = static_cast<hdg_ckpt_writer_s*>(writer);
  if (!w || (state && (!data_path || !index_path)) || (text_path && !text))
    return fail(HDG_EINVAL, "hdg_ckpt_writer_submit: bad arguments");
  CkptJob j;
  if (state) {
    j.state.assign(state, state + w->n_state);
    j.data_path = data_path;
    j.index_path = index_path;
  }
  if (removes) j.removes = removes;
  if (text_path) {
    j.text_path = text_path;
    j.text = text;
    j.text_append = text_append != 0;
  }
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->q.push_back(std::move(j));
  }
  w->cv.notify_one();
  return 0;
}

int hdg_ckpt_writer_flush(void* writer) {
  auto* w = static_cast<hdg_ckpt_writer_s*>(writer);
  if (!w) return fail(HDG_EINVAL, "hdg_ckpt_writer_flush: NULL writer");
  std::unique_lock<std::mutex> lk(w->mu);
  w->idle.wait(lk, [&] { return w->q.empty() && !w->busy; });
  const int rc = w->err_code;
  if (rc) {
    snprintf(hdg::g_err, sizeof(hdg::g_err), "%s", w->err);
    w->err_code = 0;                         // reported once, as a future's exception is
  }
  return rc;
}

int hdg_ckpt_writer_poll(void* writer) {
  auto* w = static_cast<hdg_ckpt_writer_s*>(writer);
  if (!w) return fail(HDG_EINVAL, "hdg_ckpt_writer_poll: NULL writer");
  std::lock_guard<std::mutex> lk(w->mu);
  const int rc = w->err_code;
  if (rc) {
    snprintf(hdg::g_err, sizeof(hdg::g_err), "%s", w->err);
    w->err_code = 0;
  }
  return rc;
}

int hdg_ckpt_writer_destroy(void* writer) {
  auto* w = static_cast<hdg_ckpt_writer_s*>(writer);
  if (!w) return 0;
  const int rc = hdg_ckpt_writer_flush(w);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->stop = true;
  }
  w->cv.notify_all();
  w->th.join();
  delete w;
  return rc;
}

// stream-ordered copy and completion events for the training loop's host reads (the same
// HIP calls torch's copy_ / Event make, without the dispatcher on every epoch)
int hdg_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream));
  return 0;
}
int hdg_event_create(void** ev) {
  if (!ev) return fail(HDG_EINVAL, "NULL event pointer");
  HIP_TRY(hipEventCreateWithFlags((hipEvent_t*)ev, hipEventDisableTiming));
  return 0;
}
int hdg_event_record(void* ev, void* stream) {
  HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
  return 0;
}
int hdg_event_synchronize(void* ev) {
  HIP_TRY(hipEventSynchronize((hipEvent_t)ev));
  return 0;
}
int hdg_event_destroy(void* ev) {
  if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev));
  return 0;
}

int hdg_dp_mailbox_alloc(void** mailbox, void* handle) {
  if (!mailbox || !handle) return fail(HDG_EINVAL, "NULL mailbox/handle pointer");
  *mailbox = nullptr;
  // uncached: the peers' write-through words and this rank's polling loads meet in memory
  HIP_TRY(hipExtMallocWithFlags(mailbox, dpk::BYTES, hipDeviceMallocUncached));
  hipIpcMemHandle_t h;
  hipError_t e = hipMemset(*mailbox, 0, dpk::BYTES);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, *mailbox);
  if (e != hipSuccess) {
    (void)hipFree(*mailbox);
    *mailbox = nullptr;
    return fail((int)e, "mailbox setup: %s", hipGetErrorString(e));
  }
  memcpy(handle, &h, sizeof(h));
  return 0;
}

int hdg_dp_mailbox_open(const void* handle, void** mailbox) {
  if (!mailbox || !handle) return fail(HDG_EINVAL, "NULL mailbox/handle pointer");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  *mailbox = nullptr;
  HIP_TRY(hipIpcOpenMemHandle(mailbox, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

int hdg_dp_mailbox_close(void* mailbox) {
  HIP_TRY(hipIpcCloseMemHandle(mailbox));
  return 0;
}

int hdg_dp_mailbox_free(void* mailbox) {
  HIP_TRY(hipFree(mailbox));
  return 0;
}

}  // extern "C"

namespace {
int dp_args(const hdg_dp* dp, DpArgs& a) {
  if (!dp) return fail(HDG_EINVAL, "NULL hdg_dp");
  if (dp->world < 1 || dp->world > HDG_DP_MAX_WORLD || dp->rank < 0 || dp->rank >= dp->world)
    return fail(HDG_EINVAL, "hdg_dp: rank %d / world %d out of range (world <= %d)", dp->rank,
                dp->world, HDG_DP_MAX_WORLD);
  if (dp->flags & ~HDG_DP_SHARED) return fail(HDG_EINVAL, "hdg_dp: unknown flags 0x%x", dp->flags);
  memset(&a, 0, sizeof(a));
  for (int r = 0; r < dp->world; ++r) {
    if (!dp->mailbox[r]) return fail(HDG_EINVAL, "hdg_dp: mailbox of rank %d is NULL", r);
    a.box[r] = (uint32_t*)dp->mailbox[r];
  }
  a.rank = dp->rank;
  a.world = dp->world;
  a.wait = dp->wait_ticks ? dp->wait_ticks : dpk::WAIT_DEFAULT;
  return 0;
}
bool dp_shared(const hdg_dp* dp) { return (dp->flags & HDG_DP_SHARED) != 0; }
// blocks per rank of the shared-device tail: as many as keep the W - 1 waiting ranks'
// spinning blocks on at most half of the CUs (at least HDG_DP_SHARED_BLOCKS: 15 x 8 = 120
// <= 128 at HDG_DP_MAX_WORLD), at most one per slot group
unsigned dp_shared_grid(int n, int world) {
  const int groups = (n + RED_P - 1) / RED_P;
  const int cus = cu_count() > 0 ? cu_count() : 256;
  int g = cus / (2 * (world > 1 ? world - 1 : 1));
  if (g < HDG_DP_SHARED_BLOCKS) g = HDG_DP_SHARED_BLOCKS;
  return (unsigned)(groups < g ? groups : g);
}
float* dp_aux(const hdg_dp* dp) {
  return (float*)((char*)dp->mailbox[dp->rank] + dpk::OFF_AUX);
}
}  // namespace

extern "C" {

int hdg_dp_allreduce(const hdg_dp* dp, const float* in, float* out, int32_t n, uint32_t* status,
                     void* stream) {
  DpArgs a;
  if (int rc = dp_args(dp, a)) return rc;
  if (!in || !out || n < 1 || n > HDG_DP_MAX_LEN)
    return fail(HDG_EINVAL, "hdg_dp_allreduce: NULL buffer or n=%d outside [1, %d]", n,
                HDG_DP_MAX_LEN);
  if (dp_shared(dp))
    hipLaunchKernelGGL(k_dp_tail_shared<dpk::SUM>, dim3(dp_shared_grid(n, a.world)), dim3(DP_NT_LIGHT), 0,
                       (hipStream_t)stream, in, 0, n, out, nullptr, nullptr, nullptr, nullptr,
                       nullptr, 0.f, 0.f, nullptr, status, a);
  else
    hipLaunchKernelGGL(k_dp_tail<dpk::SUM>, dim3((n + RED_P - 1) / RED_P), dim3(DP_NT_LIGHT), 0,
                       (hipStream_t)stream, in, 1, 0, n, out, nullptr, nullptr, nullptr, nullptr,
                       nullptr, 0.f, 0.f, nullptr, status, 0, a);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_adam_dp(const hdg_shape* s, hdg_state* state, const float* grad_local, float* grad_out,
                float lr, float* stats, uint32_t* status, const hdg_dp* dp, void* stream) {
  RESOLVE(s, path);
  (void)path;
  DpArgs a;
  if (int rc = dp_args(dp, a)) return rc;
  if (!state || !state->params || !state->adam_m || !state->adam_v || !state->beta_pow ||
      !grad_local || !grad_out)
    return fail(HDG_EINVAL, "NULL state/grad pointer");
  const int np = hdg::param_offsets(s->variant).NP, glen = np + HDG_TRAILER;
  hipStream_t st = (hipStream_t)stream;
  float* aux = dp_aux(dp);
  hipLaunchKernelGGL(k_dp_aux, dim3(1), dim3(1024), 0, st, state->params, np, state->beta_pow,
                     aux);
  if (dp_shared(dp))
    hipLaunchKernelGGL(k_dp_tail_shared<dpk::GRAD>, dim3(dp_shared_grid(glen, a.world)), dim3(DP_NT_LIGHT),
                       0, st, grad_local, np, glen, grad_out, state->params, state->adam_m,
                       state->adam_v, state->beta_pow, aux, lr, 1.f / pair_count(s), stats,
                       status, a);
  else
    hipLaunchKernelGGL(k_dp_tail<dpk::GRAD>, dim3((glen + RED_P - 1) / RED_P), dim3(DP_NT_LIGHT),
                       0, st, grad_local, 1, np, glen, grad_out, state->params, state->adam_m,
                       state->adam_v, state->beta_pow, aux, lr, 1.f / pair_count(s), stats,
                       status, 0, a);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hdg_train_step_dp(const hdg_shape* s, const hdg_batch* bt, hdg_state* state, float lr,
                      hdg_outputs* out, float* grad, void* workspace, const hdg_dp* dp,
                      void* stream) {
  if (!state || !state->params || !state->adam_m || !state->adam_v || !state->beta_pow)
    return fail(HDG_EINVAL, "NULL state pointer");
  RESOLVE(s, path);
  if (int rc = check_batch(bt)) return rc;
  if (!grad || !workspace) return fail(HDG_EINVAL, "NULL grad/workspace");
  DpArgs a;
  if (int rc = dp_args(dp, a)) return rc;
  hipStream_t st = (hipStream_t)stream;
  uint32_t* status = out ? out->status : nullptr;
  float* stats = out ? out->stats : nullptr;
  if (path == HDG_PATH_GENERAL || is_hybrid(s, path) || dp_shared(dp)) {
    // the rank's own reduced gradient lands in the mailbox's local scratch (the tail
    // reads it while other blocks already write the world sums into grad).  Ranks that
    // share a device take this route on the fused path too: the partial rows are reduced
    // by the non-spinning k_grad_reduce, and only the light tail waits for the peers
    float* local = (float*)((char*)dp->mailbox[dp->rank] + dpk::OFF_GLOC);
    const int rc = path == HDG_PATH_GENERAL
        ? hdg::wide_run(s, bt, state->params, local, out, nullptr, workspace, true, st)
        : is_hybrid(s, path)
        ? hybrid_run(s, bt, state->params, local, out, nullptr, workspace, true, st, nullptr)
        : hdg_fwd_bwd(s, bt, state->params, local, out, workspace, stream);
    if (rc) return rc;
    return hdg_adam_dp(s, state, local, grad, lr, stats, status, dp, stream);
  }
  // fused path: k_commit_step (aux from block 0), then the reduction + exchange + Adam
  const Work w = work_layout(s);
  float* ws = (float*)workspace;
  const float pairs = pair_count(s);
  const bool split = use_split(s);
  HIP_TRY(dispatch_step<true>(s, bt, state->params, ws, w, step_out(out), 10.f / pairs, nullptr,
                              st, split, state->beta_pow));
  hipLaunchKernelGGL(k_dp_tail<dpk::PART>, dim3((GRAD_LEN + RED_P - 1) / RED_P), dim3(1024), 0,
                     st, ws + w.part, part_rows(s, split), m2::NP, GRAD_LEN, grad, state->params,
                     state->adam_m, state->adam_v, state->beta_pow, ws + w.aux, lr, 1.f / pairs,
                     stats, status, split ? part_rows(s, split) : 0, a);
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"
