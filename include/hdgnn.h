/*
 * hdgnn.h -- C ABI of the MI355X-native HD-GNN training-step engine (libhdgnn.so).
 *
 * The reference has no FFI: its only boundary is Python -> TF1 C++ runtime at
 * sess.run().  These entry points are what that boundary would bind for the
 * north-star path, one per sess.run() the reference issues:
 *
 *   hdg_train_step   sess.run([C_edge_output2, loss_Hedge_mse, loss_map, theta, trainer],
 *                             feed_dict)                      model_2.py:369-383
 *                    = hdg_fwd_bwd + hdg_adam_tf (single process)
 *   hdg_fwd_bwd      forward + backward of train_loss (model_2.py:336) -> flat gradient
 *                    of the data term + CE sum; the DP all-reduce sits between this
 *                    and hdg_adam_tf
 *   hdg_adam_tf      AdamOptimizer(0.0003).minimize(train_loss) (model_2.py:337-338):
 *                    adds the loss_para / loss_map gradients, applies TF1 ApplyAdam
 *   hdg_forward      sess.run([loss_Hedge_mse, loss_map, C_edge_output2], feed_dict)
 *                    model_2.py:486-502 (test path, forward only)
 *
 * Conventions
 *   - every pointer is a caller-owned DEVICE pointer (the library never allocates);
 *     `stream` is a hipStream_t passed as void*; all work is enqueued on it, no host
 *     synchronisation happens inside any call (graph-capturable).
 *   - return 0 on success, HDG_EINVAL for a shape/argument error, or the hipError_t
 *     of a failed launch; hdg_last_error() gives a thread-local message.
 *   - parameters are one flat fp32 vector in tf.global_variables() order with TF
 *     (in,out) row-major weights (hdg_param_count()).
 *   - the library keeps no global mutable state apart from the thread-local error and
 *     memos of per-device queries (kernel attributes set, occupancy per kernel and LDS
 *     size): idempotent, the same answer for every caller.
 */
#ifndef HDGNN_H
#define HDGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDG_ABI_VERSION 9
#define HDG_EINVAL 1000

/* Per-launch problem shape (one rank's share of the commit batch). */
typedef struct hdg_shape {
    int32_t batch;      /* commits in this call (Mini_batch per rank)              */
    int32_t ne;         /* entity nodes per commit   (main.py --Ne, 2 <= ne <= 4096) */
    int32_t nc;         /* hunk nodes per commit     (main.py --Nc, 2 <= nc <= 2048) */
    int32_t variant;    /* model_<variant>.py: 1 HD-GNN/ES, 2 HD-GNN/S, 3 HD-GNN/E,
                           4 HD-GNN                                      */
    int32_t batch_global; /* commits summed by the CE mean across all ranks         */
    int32_t path;       /* HDG_PATH_AUTO / _FUSED / _GENERAL (see below)           */
    int32_t flags;      /* HDG_FLAG_* bits, 0 for the defaults                      */
} hdg_shape;
/* HDG_FLAG_NO_SPLIT: the fused path runs one block per commit even where split mode
 * (two co-resident blocks per commit, see hdg_workspace_bytes) would apply: what a
 * caller retries with after HDG_STATUS_XCH_TIMEOUT.  Same results up to fp32
 * re-association of the block-pair sums.                                              */
#define HDG_FLAG_NO_SPLIT 1
/* General path, hunk pair sums of the first hunk MLP layer (forward relu sums, backward mask
 * sums): a dense sweep of the pair grid, or per-unit sorted thresholds (a binary search per
 * node and unit plus the label pairs one by one) from nc >= HDG_HUNK_SORTED_MIN_NC; these
 * flags force one form (same results up to fp32 re-association; the layout of
 * hdg_workspace_bytes follows the choice, so keep the flags fixed for a workspace).      */
#define HDG_FLAG_HUNK_DENSE 2
#define HDG_FLAG_HUNK_SORTED 4
/* HDG_FLAG_HUNK_TILED: the hunk pair passes (relu sums, MLP and classifier mask sums) as
 * one sweep over blocks of the pair grid giving row and column sums together (the fused
 * kernel's pair tiles), instead of a row pass and a column pass over every pair.        */
#define HDG_FLAG_HUNK_TILED 8
/* HDG_FLAG_HUNK_GROUP (ABI 9): the sorted form's per-node passes as one block per unit group
 * (their shape for nc > 512) at any nc; below that the default is one block for all 20 units,
 * which sums each node's label walk in two halves -- the two shapes differ by fp32
 * re-association only (a diagnostic / test flag).                                         */
#define HDG_FLAG_HUNK_GROUP 16
/* Without a form flag the general path picks by nc: tiled from HDG_HUNK_TILED_MIN_NC, sorted
 * from HDG_HUNK_SORTED_MIN_NC below that, dense otherwise (the measured crossovers at the
 * default 10% label density).                                              */
#define HDG_HUNK_SORTED_MIN_NC 384
#define HDG_HUNK_TILED_MIN_NC 1024

/* Engine paths.  FUSED: one block per commit with the commit's state in LDS; model_2
 * and model_4 with ne <= 256, nc <= 160 (the benchmark shapes; model_4's entity-edge
 * stage runs on the GENERAL path's kernels around the fused step kernel, so its prepared
 * tables and workspace hold both paths' parts).  GENERAL: one launch per phase, many
 * blocks per commit, state in HBM; every variant and shape.  AUTO picks FUSED when it
 * applies.  hdg_prep_bytes / hdg_workspace_bytes depend on the path. */
#define HDG_PATH_AUTO 0
#define HDG_PATH_FUSED 1
#define HDG_PATH_GENERAL 2

/* One batch of commits in compact device form (replaces the 12-tuple feed of
 * utils2.read_data, utils2.py:248-253, bit-exactly).       */
typedef struct hdg_batch {
    const float*    x;      /* [B][ne]     node attribute = diag(CAdjs)  (E_node_train)   */
    const uint32_t* abits;  /* [B][ne][ceil(ne/32)] entity class bits: bit j of row i =
                               (E_edge class of relation (i,j) == 1); diagonal bits 0     */
    const uint32_t* ybits;  /* [B][nc][ceil(nc/32)] hunk class bits (C_edge), diag 0      */
    const int32_t*  hid;    /* [B][ne] Esc/Etc hunk row of index line i' (-1 = none)      */
    const int32_t*  nlen;   /* [B] n = len(readlines()[:Ne]) of the commit's index file   */
    void*           prep;   /* hdg_prep_bytes(shape) of device scratch, filled once per
                               uploaded batch by hdg_prepare (sorted x, transposed bits,
                               cross-graph count matrices, per-node neighbour id lists);
                               read by every step after                                 */
} hdg_batch;

/* Adam / parameter state (all device, fp32). */
typedef struct hdg_state {
    float* params;       /* [P] */
    float* adam_m;       /* [P] */
    float* adam_v;       /* [P] */
    float* beta_pow;     /* [2] beta1^t, beta2^t (TF beta1_power/beta2_power vars) */
} hdg_state;

/* Per-step outputs (device). Any pointer may be NULL to skip that output. */
typedef struct hdg_outputs {
    float* probs;        /* [B][2][nc(nc-1)]  C_edge_output2        */
    float* logits;       /* [B][2][nc(nc-1)]  C_edge_output2_logits */
    float* stats;        /* [8] ce (loss_Hedge_mse), loss_map, loss_para, train_loss
                            (pre-update values, as sess.run returns them), then the
                            step's gradient trailer slots HDG_TR_COUNT..HDG_TR_FAULT
                            (top_ACC count parts, fault count): a training loop points
                            each step at its own row and reads a whole epoch at once  */
    uint32_t* status;    /* [1] sticky device status word: the library ORs HDG_STATUS_*
                            bits into it (write-through store) and never clears it; the
                            caller zeroes it and reads it whenever it synchronises     */
    float* ehr;          /* [1] loss_E_HR = 0.001 l2_loss(C_edge_output) of the call's
                            commits (model_2.py:122; computed by the reference graph but
                            fetched by neither of its sess.run calls): written by
                            hdg_forward only, ignored by the training entry points      */
} hdg_outputs;

/* Status bits (hdg_outputs.status).  HDG_STATUS_XCH_TIMEOUT: in the fused path's split
 * mode a block waited ~20 ms for its partner block's exchange words and gave up (the pair
 * was not co-resident: another process holding CUs, CU masking).  The launch's CE sum
 * is NaN; a forward-only launch also writes NaN over the timed-out block's probs / logits
 * rows; a training launch's gradient trailer carries the fault count (HDG_TR_FAULT) and
 * the Adam update of that step is skipped on every rank (parameters, moments and beta
 * powers unchanged).  Outputs of a launch with this bit set are void.                  */
#define HDG_STATUS_XCH_TIMEOUT 1u

/* Gradient trailer: hdg_fwd_bwd's grad buffer is [param_count + HDG_TRAILER] floats.
 * Every slot sums exactly under a float all-reduce (SUM) over up to 256 ranks.          */
#define HDG_TRAILER 8
#define HDG_TR_CE 0      /* CE sum over this call's relations                              */
#define HDG_TR_COUNT 1   /* slots 1..3: number of relations whose argmax prediction equals
                            the label (EvaluationFuncs.top_ACC numerator, np.argmax tie
                            rule), as three 16-bit parts: count = s1 + s2 2^16 + s3 2^32  */
#define HDG_TR_FAULT 4   /* blocks whose pair exchange timed out (0 = clean step)          */

int         hdg_version(void);
const char* hdg_last_error(void);
/* the path AUTO resolves to for this shape (HDG_PATH_FUSED / _GENERAL), or -1 */
int         hdg_resolve_path(const hdg_shape* shape);
/* flat parameter count of model_<variant> (SURVEY Appendix A order), or -1 (message in
 * hdg_last_error) for a variant outside 1..4                                         */
int         hdg_param_count(int32_t variant);
/* length of the gradient buffer hdg_fwd_bwd fills: param_count + HDG_TRAILER (the
 * trailer slots above); all-reduce the whole buffer.                                */
int         hdg_grad_len(int32_t variant);
/* Scratch the library carves per call (parked node rows, partial gradient rows, the
 * block-pair inboxes and per-commit launch epochs of the fused path's split mode).  Keep
 * it per shape across calls; its initial content does not matter (exchange tags derive
 * from the epoch word and differ from the word's own bit pattern, everything else is
 * written before it is read).  Split mode (two blocks per commit) runs whenever
 * 2 * batch <= the device's CU count and one 1024-thread block of the step kernel fits
 * a CU; HDG_FUSED_SPLIT=0 forces one block per commit.  The two blocks of a pair must
 * run at the same time: plain launches do not guarantee it, so a pair that cannot meet
 * is detected (HDG_STATUS_XCH_TIMEOUT) instead of producing silent garbage.          */
size_t      hdg_workspace_bytes(const hdg_shape* shape);
/* bytes of batch->prep for this shape (0 on a shape error).  It depends on the path the
 * shape resolves to (fused, fused + entity-edge, general), never on the flags: prepare a
 * batch with a shape that resolves to the same path as the steps that read it.      */
size_t      hdg_prep_bytes(const hdg_shape* shape);
/* Where hdg_prepare puts the cross-graph count tables of commit b inside batch->prep
 * (4-byte words from prep + b * stride_words): K_s at ks, K_t at kt (u16 [Nc][Ne]),
 * class counts at ncst (f32 [Nc][2]).  K_s = (Esc + Etc) . Es^T and K_t = (Esc + Etc) .
 * Et^T of utils2.py:111-137 (the marshalling_B2 maps, model_2.py:146-150), so tests can
 * check the index bookkeeping bit-exactly.  0, or an error code on a shape error.    */
int         hdg_prep_counts_layout(const hdg_shape* shape, int64_t* stride_words,
                                   int64_t* ks, int64_t* kt, int64_t* ncst);

/* Build batch->prep from x / abits / hid / nlen (the parameter-independent per-commit
 * tables the step kernel reads).  Call once after uploading a batch, before any step;
 * re-call whenever the batch contents change.  Replaces nothing in the reference: it is
 * the device-side half of the feed_dict marshalling (utils2.py:111-137, 248-253).    */
int hdg_prepare(const hdg_shape* shape, const hdg_batch* batch, void* stream);
/* Upload helper: a (batch, n, n) u8 class grid on the device (class of relation (i, j),
 * 0 or 1: the E_edge / C_edge one-hots of utils2.py:82, 105) -> the (batch, n,
 * ceil(n/32)) u32 bit rows hdg_batch.abits / ybits hold (bit j of row i = class 1,
 * diagonal cleared).  Lets a caller ship the compact grids and pack them on the GPU. */
int hdg_pack_classes(const uint8_t* cls, int32_t batch, int32_t n, uint32_t* bits,
                     void* stream);

int hdg_fwd_bwd(const hdg_shape* shape, const hdg_batch* batch, const float* params,
                float* grad, hdg_outputs* out, void* workspace, void* stream);

/* hdg_fwd_bwd with hipEvent_t events[3] recorded on `stream` before k_commit_step,
 * before k_grad_reduce and after it (per-kernel timing for bench.py; may be NULL). */
int hdg_fwd_bwd_events(const hdg_shape* shape, const hdg_batch* batch, const float* params,
                       float* grad, hdg_outputs* out, void* workspace, void* stream,
                       void* const* events);

/* hdg_fwd_bwd with per-kernel timing of every engine path (bench.py's roofline): events
 * [n_events] hipEvent_t; events[0] is recorded on `stream` before the first launch and
 * events[k + 1] right after the k-th kernel launch, whose name goes to names[k] (static
 * strings).  *n_kernels = the kernels bracketed (at most n_events - 1; later launches run
 * untimed).  Replaces nothing in the reference (its only clock is time.time(),
 * model_2.py:358, 423-424).                                                          */
int hdg_fwd_bwd_kernel_events(const hdg_shape* shape, const hdg_batch* batch,
                              const float* params, float* grad, hdg_outputs* out,
                              void* workspace, void* stream, void* const* events,
                              int32_t n_events, const char** names, int32_t* n_kernels);

/* Diagnostic: run k_commit_step alone with s_memrealtime (100 MHz) stamps at every
 * phase barrier, stamps[2B][32] (device; row = the block's partial-gradient row, 2b + h
 * in split mode).  Overwrites the workspace.                                        */
int hdg_debug_step_stamps(const hdg_shape* shape, const hdg_batch* batch, const float* params,
                         void* workspace, unsigned long long* stamps, void* stream);

/* TF ApplyAdam from an (all-reduced) gradient buffer; skips the whole update (parameters,
 * moments, beta powers) when grad[P + HDG_TR_FAULT] != 0.                            */
int hdg_adam_tf(const hdg_shape* shape, hdg_state* state, const float* grad,
                float lr, float* stats, void* stream);

int hdg_train_step(const hdg_shape* shape, const hdg_batch* batch, hdg_state* state,
                   float lr, hdg_outputs* out, float* grad, void* workspace, void* stream);

int hdg_forward(const hdg_shape* shape, const hdg_batch* batch, const float* params,
                hdg_outputs* out, float* ce_sum, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------
 * Data parallelism over xGMI (one all-reduce of the flat gradient per step).
 *
 * Instead of an RCCL call between hdg_fwd_bwd and hdg_adam_tf, the step's reduction
 * kernel exchanges the gradient itself: every rank owns a MAILBOX (uncached device
 * memory, hdg_dp_mailbox_alloc) that every other rank of the node maps through HIP IPC
 * (hdg_dp_mailbox_open on the 64-byte handle, exchanged by the caller, e.g. with
 * torch.distributed.all_gather).  Each block of the tail kernel writes its gradient
 * slots as tagged words straight into every peer's mailbox over xGMI (one hop), polls
 * its own mailbox for the peers' words, sums the world's values in rank order (the same
 * bits on every rank: replicas stay bitwise equal) and applies TF Adam -- one kernel, no
 * collective launch.  A peer that does not arrive within wait_ticks fails the launch
 * loudly, but only where the wait happened: each tail block waits for the peers' words of
 * ITS OWN slots, and a block that times out sets HDG_STATUS_DP_TIMEOUT in this rank's
 * status word, writes a NaN loss and skips the update of its slots.  The other blocks of
 * the same rank (block 0's beta-power update included) and every peer that did receive
 * the words still apply the step, so after a timeout the parameters are partly updated
 * and the ranks disagree: DP_TIMEOUT is unrecoverable -- no retry; restore every rank
 * from a checkpoint.  (The split-mode pair timeout, HDG_STATUS_XCH_TIMEOUT, is different:
 * its step is skipped whole and a one-block retry is exact.)  The deadline counts from
 * the moment each block starts waiting, so host-side skew between ranks (data loading,
 * rank-0 file writes) counts against it: callers barrier the ranks before the first step
 * and after rank-only host work (graph2graph.train does).  All ranks must issue the same
 * sequence of hdg_*_dp calls (per-block launch counters in the mailbox tag the words).
 * The mailbox calls are the one place the library allocates device memory (IPC needs an
 * allocation of its own); everything else stays caller-owned.
 * --------------------------------------------------------------------------------- */
#define HDG_DP_MAX_WORLD 16
#define HDG_DP_HANDLE_BYTES 64
#define HDG_DP_MAX_LEN 3152          /* longest vector hdg_dp_allreduce accepts          */
#define HDG_STATUS_DP_TIMEOUT 2u     /* a peer's gradient words never arrived            */

typedef struct hdg_dp {
    int32_t  rank;        /* this process's rank, 0 <= rank < world                      */
    int32_t  world;       /* ranks on this node, 1 <= world <= HDG_DP_MAX_WORLD          */
    uint64_t wait_ticks;  /* 100 MHz ticks a block waits for a peer (0: 10 s)            */
    void*    mailbox[HDG_DP_MAX_WORLD];  /* rank r's mailbox as mapped in this process   */
    int32_t  flags;       /* HDG_DP_* bits (ABI 9), 0 for one rank per device            */
    int32_t  reserved;    /* 0                                                            */
} hdg_dp;
/* HDG_DP_SHARED: several ranks share one device (a rehearsal of the node's DP step on a
 * box with fewer GPUs).  A waiting tail block spins on a CU; with one rank per device
 * nothing else needs that CU, but a peer rank on the SAME device still has to place its
 * step kernel, whose 1024-thread blocks each take a whole CU (all VGPRs, up to all of the
 * LDS).  The tails of W-1 waiting ranks must therefore never cover every CU: with this
 * flag every exchange runs as G light blocks per rank that loop over the slot groups (all
 * of a block's words sent first, then its groups received in order), G chosen so that the
 * W-1 waiting ranks hold at most half of the device's CUs (G >= HDG_DP_SHARED_BLOCKS:
 * (HDG_DP_MAX_WORLD - 1) * 8 = 120 <= 128), and the fused path reduces its partial rows
 * with the non-spinning k_grad_reduce before the exchange (hdg_fwd_bwd -> hdg_adam_dp)
 * instead of inside the spinning tail.  Same bits as the one-rank-per-device calls.    */
#define HDG_DP_SHARED 1
#define HDG_DP_SHARED_BLOCKS 8

size_t hdg_dp_mailbox_bytes(void);
/* Host utility: CRC-32C (Castagnoli) of n bytes, continuing from crc (0 to start) -- the
 * record checksum of the TF V2 checkpoint bundles graph2graph.saver writes.          */
uint32_t hdg_crc32c(const void* data, size_t n, uint32_t crc);
/* Host utility: write one TF V2 checkpoint bundle of float32 tensors from a prebuilt
 * template (hdgnn.tfckpt.BundleTemplate; replaces the Python encoder of saver.save,
 * model_2.py:427-437, so the caller's thread runs it without holding the GIL):
 *   data file  = state[gather[i]] for i < n_floats (the tensors' bytes, sorted by name;
 *                every gather index is checked against the n_state floats of state)
 *   index file = index_img with each entry's masked CRC-32C of its bytes written at
 *                entries[3e + 2] (the tensor spans [entries[3e], +entries[3e + 1]) bytes of
 *                the data file), then each block's trailer CRC (blocks[2b] offset,
 *                blocks[2b + 1] length; type byte at offset + length) -- index_img is
 *                modified in place.  Both files are written under "<path>.tmp" and renamed
 *                into place, data before index.  0, or HDG_EINVAL (hdg_last_error).    */
int hdg_bundle_write(const char* data_path, const char* index_path, const float* state,
                     int64_t n_state, const int32_t* gather, int64_t n_floats,
                     uint8_t* index_img, int64_t index_len, const int64_t* entries,
                     int32_t n_entries, const int64_t* blocks, int32_t n_blocks);
/* Host utility: background checkpoint writer (saver.save off the training thread).  One
 * native thread runs the submitted jobs in order; a job writes a bundle of `state` exactly
 * as hdg_bundle_write does with the writer's template (gather / index image / entries /
 * blocks, copied at create), then removes the '\n'-separated `removes` paths (bundles that
 * fell out of max_to_keep; missing files are fine), then writes `text` to `text_path`
 * (appended when text_append != 0, else replacing it: the 'checkpoint' state file, a
 * result line).  NULL state / removes / text_path skip that part.  submit copies
 * everything it is given (n_state floats of state) and returns at once; flush waits for
 * the queue and returns the first failure since the last flush (HDG_EINVAL, message in
 * hdg_last_error); destroy flushes, stops the thread and frees the writer.              */
int hdg_ckpt_writer_create(const int32_t* gather, int64_t n_floats, int64_t n_state,
                           const uint8_t* index_img, int64_t index_len, const int64_t* entries,
                           int32_t n_entries, const int64_t* blocks, int32_t n_blocks,
                           void** writer);
int hdg_ckpt_writer_submit(void* writer, const float* state, const char* data_path,
                           const char* index_path, const char* removes, const char* text_path,
                           const char* text, int32_t text_append);
int hdg_ckpt_writer_flush(void* writer);
/* the first failure since the last flush / poll without waiting for the queue (ABI 9): 0 or
 * the failed job's code (message in hdg_last_error), reported once.  A job whose bundle
 * write fails skips its removals and text, so the caller re-books its keep-list.        */
int hdg_ckpt_writer_poll(void* writer);
int hdg_ckpt_writer_destroy(void* writer);
/* Host utility: hipMemcpyAsync (kind default) and completion events without timing, for
 * the training loop's stream-ordered reads into pinned host memory.                     */
int hdg_memcpy_async(void* dst, const void* src, size_t bytes, void* stream);
int hdg_event_create(void** event);
int hdg_event_record(void* event, void* stream);
int hdg_event_synchronize(void* event);
int hdg_event_destroy(void* event);
/* allocate + zero this rank's mailbox on the current device; handle: 64 bytes out */
int hdg_dp_mailbox_alloc(void** mailbox, void* handle);
/* map a peer's mailbox (its handle) into this process; close / free undo the calls */
int hdg_dp_mailbox_open(const void* handle, void** mailbox);
int hdg_dp_mailbox_close(void* mailbox);
int hdg_dp_mailbox_free(void* mailbox);

/* One data-parallel training step: hdg_fwd_bwd -> xGMI all-reduce -> TF Adam with the
 * exchange inside the reduction kernel.  grad receives the world-summed gradient +
 * trailer (as hdg_fwd_bwd + all_reduce would leave it); out->stats the world's loss.   */
int hdg_train_step_dp(const hdg_shape* shape, const hdg_batch* batch, hdg_state* state,
                      float lr, hdg_outputs* out, float* grad, void* workspace,
                      const hdg_dp* dp, void* stream);
/* xGMI all-reduce of a local gradient (hdg_fwd_bwd's buffer) fused with TF Adam:
 * grad_out = sum over ranks of grad_local (must not overlap), then hdg_adam_tf's update. */
int hdg_adam_dp(const hdg_shape* shape, hdg_state* state, const float* grad_local,
                float* grad_out, float lr, float* stats, uint32_t* status, const hdg_dp* dp,
                void* stream);
/* out[i] = sum over ranks (rank order) of in[i], n <= HDG_DP_MAX_LEN, in / out disjoint. */
int hdg_dp_allreduce(const hdg_dp* dp, const float* in, float* out, int32_t n,
                     uint32_t* status, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HDGNN_H */
