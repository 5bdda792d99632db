"""ctypes binding of libhdgnn.so (include/hdgnn.h).

The library is built in-tree (hd-gnn_amd/csrc/libhdgnn.so, see build.py).  There
is deliberately no fallback: if the shared object is missing or fails to load,
every entry point raises.  torch is imported first so that the process uses
torch's HIP runtime (same SONAME libamdhip64.so.7) for both.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's libamdhip64 before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "csrc", "libhdgnn.so")


class Shape(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("ne", ctypes.c_int32), ("nc", ctypes.c_int32),
                ("variant", ctypes.c_int32), ("batch_global", ctypes.c_int32),
                ("path", ctypes.c_int32), ("flags", ctypes.c_int32)]


PATH_AUTO, PATH_FUSED, PATH_GENERAL = 0, 1, 2
FLAG_NO_SPLIT, FLAG_HUNK_DENSE, FLAG_HUNK_SORTED, FLAG_HUNK_TILED = 1, 2, 4, 8
FLAG_HUNK_GROUP = 16
# the general path's automatic hunk pair-sum form (include/hdgnn.h): tiled from nc >= 1024,
# sorted from nc >= 384 below that, dense otherwise
HUNK_SORTED_MIN_NC, HUNK_TILED_MIN_NC = 384, 1024
STATS_LEN = 8          # hdg_outputs.stats: ce, loss_map, loss_para, train_loss, count x3, fault


class Batch(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("abits", ctypes.c_void_p), ("ybits", ctypes.c_void_p),
                ("hid", ctypes.c_void_p), ("nlen", ctypes.c_void_p), ("prep", ctypes.c_void_p)]


class State(ctypes.Structure):
    _fields_ = [("params", ctypes.c_void_p), ("adam_m", ctypes.c_void_p),
                ("adam_v", ctypes.c_void_p), ("beta_pow", ctypes.c_void_p)]


class Outputs(ctypes.Structure):
    _fields_ = [("probs", ctypes.c_void_p), ("logits", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("ehr", ctypes.c_void_p)]


class Dp(ctypes.Structure):
    """hdg_dp: this rank's view of the node's xGMI mailboxes (include/hdgnn.h)."""
    _fields_ = [("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("wait_ticks", ctypes.c_uint64), ("mailbox", ctypes.c_void_p * 16),
                ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32)]


DP_MAX_WORLD, DP_HANDLE_BYTES, DP_MAX_LEN = 16, 64, 3152
DP_SHARED, DP_SHARED_BLOCKS = 1, 8      # hdg_dp.flags: ranks share a device (include/hdgnn.h)

ABI_VERSION = 9
# gradient trailer (include/hdgnn.h): grad = [P parameter gradients | TRAILER slots]
TRAILER, TR_CE, TR_COUNT, TR_FAULT = 8, 0, 1, 4
STATUS_XCH_TIMEOUT, STATUS_DP_TIMEOUT = 1, 2


def trailer_count(tr):
    """Correct-prediction count from the trailer's three 16-bit parts (slots 1..3)."""
    return (int(round(float(tr[TR_COUNT]))) + (int(round(float(tr[TR_COUNT + 1]))) << 16)
            + (int(round(float(tr[TR_COUNT + 2]))) << 32))


EXPORTS = ["hdg_version", "hdg_last_error", "hdg_resolve_path", "hdg_param_count", "hdg_grad_len",
           "hdg_workspace_bytes", "hdg_prep_bytes", "hdg_prepare", "hdg_fwd_bwd",
           "hdg_fwd_bwd_events", "hdg_adam_tf", "hdg_train_step", "hdg_forward",
           "hdg_debug_step_stamps", "hdg_prep_counts_layout", "hdg_dp_mailbox_bytes",
           "hdg_dp_mailbox_alloc", "hdg_dp_mailbox_open", "hdg_dp_mailbox_close",
           "hdg_dp_mailbox_free", "hdg_train_step_dp", "hdg_adam_dp", "hdg_dp_allreduce",
           "hdg_pack_classes", "hdg_crc32c", "hdg_fwd_bwd_kernel_events",
           "hdg_bundle_write", "hdg_ckpt_writer_create", "hdg_ckpt_writer_submit",
           "hdg_ckpt_writer_flush", "hdg_ckpt_writer_poll", "hdg_ckpt_writer_destroy", "hdg_memcpy_async",
           "hdg_event_create", "hdg_event_record", "hdg_event_synchronize", "hdg_event_destroy"]

_lib = None


def load(path=None):
    """Load (once) and type the library.  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    # HDG_LIB_PATH: an alternative build of the same library (diagnostic ablation builds)
    path = path or os.environ.get("HDG_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError("libhdgnn.so is not built (%s); run __graft_entry__.build() or "
                           "python hd-gnn_amd/hdgnn/build.py" % path)
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    vp, f32, i32 = ctypes.c_void_p, ctypes.c_float, ctypes.c_int32
    lib.hdg_version.restype = ctypes.c_int
    lib.hdg_last_error.restype = ctypes.c_char_p
    lib.hdg_resolve_path.argtypes = [P(Shape)]
    lib.hdg_param_count.argtypes = [i32]
    lib.hdg_grad_len.argtypes = [i32]
    lib.hdg_workspace_bytes.argtypes = [P(Shape)]
    lib.hdg_workspace_bytes.restype = ctypes.c_size_t
    lib.hdg_prep_bytes.argtypes = [P(Shape)]
    lib.hdg_prep_bytes.restype = ctypes.c_size_t
    lib.hdg_prep_counts_layout.argtypes = [P(Shape)] + [P(ctypes.c_int64)] * 4
    lib.hdg_prep_counts_layout.restype = ctypes.c_int
    lib.hdg_prepare.argtypes = [P(Shape), P(Batch), vp]
    lib.hdg_pack_classes.argtypes = [vp, i32, i32, vp, vp]
    lib.hdg_fwd_bwd.argtypes = [P(Shape), P(Batch), vp, vp, P(Outputs), vp, vp]
    lib.hdg_fwd_bwd_events.argtypes = [P(Shape), P(Batch), vp, vp, P(Outputs), vp, vp, vp]
    lib.hdg_fwd_bwd_kernel_events.argtypes = [P(Shape), P(Batch), vp, vp, P(Outputs), vp, vp,
                                              vp, i32, P(ctypes.c_char_p), P(i32)]
    lib.hdg_debug_step_stamps.argtypes = [P(Shape), P(Batch), vp, vp, vp, vp]
    lib.hdg_adam_tf.argtypes = [P(Shape), P(State), vp, f32, vp, vp]
    lib.hdg_train_step.argtypes = [P(Shape), P(Batch), P(State), f32, P(Outputs), vp, vp, vp]
    lib.hdg_forward.argtypes = [P(Shape), P(Batch), vp, P(Outputs), vp, vp, vp]
    lib.hdg_dp_mailbox_bytes.restype = ctypes.c_size_t
    lib.hdg_dp_mailbox_alloc.argtypes = [P(vp), vp]
    lib.hdg_dp_mailbox_open.argtypes = [vp, P(vp)]
    lib.hdg_dp_mailbox_close.argtypes = [vp]
    lib.hdg_dp_mailbox_free.argtypes = [vp]
    lib.hdg_train_step_dp.argtypes = [P(Shape), P(Batch), P(State), f32, P(Outputs), vp, vp,
                                      P(Dp), vp]
    lib.hdg_adam_dp.argtypes = [P(Shape), P(State), vp, vp, f32, vp, vp, P(Dp), vp]
    lib.hdg_dp_allreduce.argtypes = [P(Dp), vp, vp, i32, vp, vp]
    lib.hdg_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
    lib.hdg_crc32c.restype = ctypes.c_uint32
    lib.hdg_bundle_write.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, ctypes.c_int64, vp,
                                     ctypes.c_int64, vp, ctypes.c_int64, vp, i32, vp, i32]
    cp = ctypes.c_char_p
    lib.hdg_ckpt_writer_create.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int64,
                                           vp, i32, vp, i32, P(vp)]
    lib.hdg_ckpt_writer_submit.argtypes = [vp, vp, cp, cp, cp, cp, cp, i32]
    lib.hdg_ckpt_writer_flush.argtypes = [vp]
    lib.hdg_ckpt_writer_poll.argtypes = [vp]
    lib.hdg_ckpt_writer_destroy.argtypes = [vp]
    lib.hdg_memcpy_async.argtypes = [vp, vp, ctypes.c_size_t, vp]
    lib.hdg_event_create.argtypes = [P(vp)]
    lib.hdg_event_record.argtypes = [vp, vp]
    lib.hdg_event_synchronize.argtypes = [vp]
    lib.hdg_event_destroy.argtypes = [vp]
    for name in EXPORTS:
        getattr(lib, name)
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = load().hdg_last_error().decode(errors="replace")
        raise RuntimeError("libhdgnn error %d: %s" % (rc, msg))
    return rc


class HipEvents:
    """hipEvent_t handles from the HIP runtime torch already loaded (for per-kernel timing
    on the stream the kernels run on; torch.cuda.Event only sees torch's own stream API)."""

    def __init__(self, n):
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        self.rt.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.rt.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                                ctypes.c_void_p]
        self.rt.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        self.rt.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = (ctypes.c_void_p * n)()
        for i in range(n):
            h = ctypes.c_void_p()
            if self.rt.hipEventCreate(ctypes.byref(h)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev[i] = h
        self.n = n

    def elapsed_ms(self, a, b):
        self.rt.hipEventSynchronize(self.ev[b])
        out = ctypes.c_float()
        if self.rt.hipEventElapsedTime(ctypes.byref(out), self.ev[a], self.ev[b]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return out.value

    def __del__(self):
        try:
            for i in range(self.n):
                self.rt.hipEventDestroy(self.ev[i])
        except Exception:
            pass
