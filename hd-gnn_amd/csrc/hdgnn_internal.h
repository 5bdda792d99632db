// hdgnn_internal.h -- declarations shared by the two engine paths of libhdgnn.so
// (not part of the public C ABI; see include/hdgnn.h).
//
//   fused path   hdgnn.hip  one 1024-thread block per commit, LDS-resident commit state;
//                           model_2 with ne <= 256, nc <= 160 (the benchmark shape)
//   general path wide.hip   any ne / nc, model variants 1-4, one phase per launch with
//                           many 256-thread blocks per commit, state in HBM
#ifndef HDGNN_INTERNAL_H
#define HDGNN_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "hdgnn.h"

namespace hdg {

constexpr int HS = 20;   // h_size = De_e = De_er (model_2.py:163, 192, 247, 306)

// ------------------------------------------------------------------------------
// Prepared batch, fused-path layout (hdg_prepare: once per uploaded batch, independent
// of the parameters).  Per commit, in 4-byte words:
//   xsrt[NE4]    x sorted ascending            perm[NE4]  node at sorted slot m
//   xu[NE4]      the nd distinct x values      cum[NE4+4] cum[q] = #nodes with x < xu[q]
//   pxd[NE4+4]   f64 pxd[q] = sum of x over nodes with x < xu[q]      meta[4] = {nd}
//   offr, offc   CSR offsets of the a = 1 neighbours of each node (rows of a, of a^T)
//   lists        u8 ids of the a = 1 row neighbours, laid out like the row x-lists
//                (node i at byte xoffr[i], zero-padded to a multiple of 4)
//   xoffr, xoffc offsets (in elements, multiples of 4) of each node's neighbour list in xl
//   xl           f32 x_j of the a = 1 neighbours j of each node, row lists then column
//                lists, each padded with NaN to a multiple of 4 (16-byte vector reads)
//   ks, kt       [Nc][Ne] u16 cross-graph counts (k_prep_counts)
//   ncst[Nc][2]  f32 count of relations binned to hunk c with a = 0 / a = 1
// The general path has its own per-commit layout (wide.hip, GenPrep): ks / kt / ncst as
// here, transposed class bits, and the sorted-x tables without the byte neighbour lists.
// ------------------------------------------------------------------------------
struct PrepLayout {
  int xsrt, perm, xu, cum, pxd, meta, offr, offc, ks, kt, ncst, lists, xoffr, xoffc, xl, words;
};

__host__ __device__ inline PrepLayout prep_layout(int Ne, int Nc) {
  PrepLayout L;
  const int NE4 = (Ne + 3) & ~3;
  const int kw = ((Nc * Ne + 1) / 2 + 3) & ~3;
  int o = 0;
  L.xsrt = o; o += NE4;
  L.perm = o; o += NE4;
  L.xu = o;   o += NE4;
  L.cum = o;  o += NE4 + 4;
  L.pxd = o;  o += 2 * (NE4 + 4);     // even word offset: 8-byte aligned
  L.meta = o; o += 4;                 // nd, nnz_r, nnz_c, byte offset of the column lists
  L.offr = o; o += NE4 + 4;           // CSR row offsets (a_ij = 1, j != i)
  L.offc = o; o += NE4 + 4;           // CSR column offsets (a_ji = 1)
  L.ks = o;   o += kw;
  L.kt = o;   o += kw;
  L.ncst = o; o += (2 * Nc + 3) & ~3;
  L.lists = o; o += (Ne * (Ne - 1) + 3 * Ne + 4 + 3) / 4;   // u8 row neighbour ids, padded
  L.xoffr = o; o += NE4 + 4;
  L.xoffc = o; o += NE4 + 4;
  o = (o + 3) & ~3;                   // 16-byte aligned
  L.xl = o;   o += 2 * Ne * (Ne - 1) + 6 * Ne + 8;   // f32 neighbour x-lists, NaN-padded
  L.words = (o + 63) & ~63;
  return L;
}

// Flat parameter offsets of one model variant (tf.global_variables order, SURVEY
// Appendix A); -1 for blocks the variant does not have.
struct Off {
  int E1_W1, E1_B1, E1_W5, E1_B5;            // phi_E_O1  mlp_entity_B1
  int E3_W1, E3_B1, E3_W2, E3_B2;            // phi_U_O1  mlp2_entity_B1
  int EE_W11, EE_W12, EE_B1, EE_W2, EE_B2;   // phi_E_R1  mlp_entityedge_B1 (model_4)
  int EC_W1, EC_B1, EC_W2, EC_B2;            // phi_U_R1  mlp2_entityedge_B1 (model_4)
  int H1_W1, H1_B1, H1_W2, H1_B2;            // mlp_hunk_B2
  int H2_W1, H2_B1, H2_W2, H2_B2;            // phi_U_R1(_1)  mlp_hunkedge_B2
  int TH1, TH2, NP;                          // map_conv thetas, parameter count
};

Off param_offsets(int variant);   // NP = -1 for an unknown variant

// general path (wide.hip)
// A single-process training step's TF-Adam tail run inside the general path's final
// reduction (kw_reduce_adam) instead of a separate k_adam_tf launch; state updated in place.
// The fused step kernel's per-block gradient rows (model_4 on the fused path): frows rows of
// fstride floats in the model_2 layout; slot p of the model_4 vector is row slot p, or
// p - f_shift from f_at on (past the entity-edge block); f_np = model_2's parameter count.
struct FusedRows {
  const float* fp;
  int frows, fstride, f_at, f_shift, f_np;
  const float* ffault;   // split mode: the rows' fault slots, contiguous (NULL: no check)
};
struct WideAdam {
  hdg_state* state;
  float lr, inv_pairs;
  float* stats;      // may be NULL
  FusedRows fused;   // fp = NULL: every gradient slot from the general path's rows
};
size_t wide_workspace_bytes(const hdg_shape* s);
size_t wide_prep_bytes(const hdg_shape* s);
void wide_prep_counts_layout(const hdg_shape* s, int64_t* stride, int64_t* ks, int64_t* kt,
                             int64_t* ncst);
int wide_prepare(const hdg_shape* s, const hdg_batch* bt, hipStream_t st);
// train: forward + backward -> grad[NP + 4] (slot NP = CE sum); !train: forward only,
// CE sum -> *ce_sum (may be NULL).  Outputs as in hdg_fwd_bwd.
// adam (train only, may be NULL): apply TF Adam to adam->state in the final reduction
int wide_run(const hdg_shape* s, const hdg_batch* bt, const float* params, float* grad,
             hdg_outputs* out, float* ce_sum, void* workspace, bool train, hipStream_t st,
             const WideAdam* adam = nullptr);
// model_4 on the fused path: the entity-edge stage on the general path's kernels around
// the fused step kernel.  wide_ee_fwd: EE first layer, node products, classifier over the
// mapped relations -> per-tile partial bins (wide_ncpart: u64 [B][wide_ncpart_tiles][Nc][2],
// 2^-32 fixed point) of n_c[2:4] of marshalling_B2 (model_4.py:95-97), which the step kernel
// sums;
// wide_ee_bwd: from dn (wide_dn, [B][Nc][4], written by the step kernel) the EE backward
// and the reduction of the EE parameters' gradient rows into grad[EE_W11 .. EC_B2 + 2).
// bt->prep, workspace: this path's layouts (wide_prep_bytes / wide_workspace_bytes).
float* wide_dn(const hdg_shape* s, void* workspace);
// bpow (a step ending in wide_ee_bwd with adam): the Adam factors' beta powers.
// wide_ee_bwd with adam: every parameter's TF-Adam update in its final reduction, the
// non-entity-edge gradients read from grad (the fused kernel's reduction wrote them).
int wide_ee_fwd(const hdg_shape* s, const hdg_batch* bt, const float* params, void* workspace,
                hipStream_t st, const float* bpow = nullptr);
const unsigned long long* wide_ncpart(const hdg_shape* s, void* workspace);
int wide_ncpart_tiles(const hdg_shape* s);
int wide_ee_bwd(const hdg_shape* s, const hdg_batch* bt, const float* params, void* workspace,
                float* grad, hipStream_t st, const WideAdam* adam = nullptr);

// loss_E_HR of a forward launch (model_2.py:122) from the complete hunk row / column sums
// G, H ([Nc][20] per commit at stride cs floats): out[0] = 0.001 l2_loss(C_edge_output)
hipError_t launch_ehr(const float* G, const float* Hh, size_t cs, int B, int Nc,
                      const float* params, int variant, float* out, hipStream_t st);

// the general path's one-sweep hunk pair sums (kh_tile<MODE>, hdgnn.hip: the fused kernel's
// pair tiles on HTR x HTC blocks of the pair grid); mode 0 relu sums, 1 MLP mask sums,
// 2 classifier mask sums (see hdgnn.hip).  All pointers are per batch (commit b at b * Nc *
// 20 floats, gam at b * Nc * Nc); rpart / cpart / ysp the block partials.
struct HTileArgs {
  int Nc;
  const float *rows, *cols;       // alpha / beta (modes 0, 1), sigma / tau (mode 2)
  const float *wrow, *wcol;       // dG / dH (mode 1)
  const float* gam;               // [B][Nc][Nc] (mode 2)
  const float* dl;                // delta (D + D_DLT) / eps (D + D_EPS): 20 floats
  const uint32_t* ybits;          // [B][Nc][ceil(Nc/32)]
  float *rpart, *cpart, *ysp;
};
hipError_t launch_hunk_tile(int mode, const HTileArgs& a, int B, hipStream_t st);
int hunk_tile_cols();             // HTC: columns per block
int hunk_tile_rows();             // HTR: rows per block

// fused path pieces the general path reuses (hdgnn.hip)
hipError_t launch_prep_maps(const hdg_shape* s, const hdg_batch* bt, int stride, int o_ks,
                            int o_kt, int o_ncst, hipStream_t st);
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Per-kernel timing hook (hdg_fwd_bwd_kernel_events): while a traced call runs, every
// launch site of the step records one event after its launch, so events[k] .. events[k+1]
// bracket the k-th kernel on the stream.  Thread-local and NULL outside a traced call.
struct KTrace {
  void* const* ev;
  int cap, n;
  const char** names;
};
extern thread_local KTrace* g_ktrace;
// the launch's error, then (traced calls only) the event after it
inline hipError_t kmark(const char* name, hipStream_t st) {
  const hipError_t e = hipGetLastError();
  KTrace* t = g_ktrace;
  if (e != hipSuccess || !t || t->n + 1 >= t->cap) return e;
  t->names[t->n++] = name;
  return hipEventRecord((hipEvent_t)t->ev[t->n], st);
}

// ------------------------------------------------------------------------------
// MFMA 16x16 fp32 tile (v_mfma_f32_16x16x4_f32) used by both paths
// ------------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));

// The same tile with strided operands: lane l supplies row r = l & 15 of A as
// pa[k * sa] and column r of B as pb[k * sb], k < K.  A row / column outside the matrix
// passes a pointer to a 0.f word with stride 0 (a row of ones: a 1.f word, stride 0), so
// the K loop carries no bounds logic: one LDS read and one address add per operand.
__device__ __forceinline__ f4v mfma_tile16_p(const float* pa, const int sa, const float* pb,
                                             const int sb, const int K, const int lane) {
  const int q = lane >> 4;
  const float* a = pa + q * sa;
  const float* b = pb + q * sb;
  const int sa4 = 4 * sa, sb4 = 4 * sb;
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  int k = 0;
  for (; k + 16 <= K; k += 16) {
    float av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      av[u] = a[u * sa4];
      bv[u] = b[u * sb4];
    }
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], c1, 0, 0, 0);
    a += 4 * sa4;
    b += 4 * sb4;
  }
  for (; k + 4 <= K; k += 4) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c0, 0, 0, 0);
    a += sa4;
    b += sb4;
  }
  if (k < K) {                       // K % 4 tail: entries k + q >= K are selected to zero
    const bool ok = k + q < K;       // (callers' arrays are padded, the read stays in LDS)
    const float av = ok ? a[0] : 0.f, bv = ok ? b[0] : 0.f;
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, c0, 0, 0, 0);
  }
  return c0 + c1;
}

}  // namespace hdg

#endif  // HDGNN_INTERNAL_H
