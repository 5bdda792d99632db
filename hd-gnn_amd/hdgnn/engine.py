"""Device-side step runner over libhdgnn.so.

Owns the fp32 parameter vector, TF-Adam state, gradient buffer, workspace and
per-step outputs on one GPU.  One training step = hdg_fwd_bwd -> (all-reduce of
the flat gradient + CE-sum trailer when distributed) -> hdg_adam_tf, all enqueued
on torch's current stream (so a torch.cuda.CUDAGraph can capture it).  The
all-reduce is the in-kernel xGMI exchange (hdgnn/xgmi.py, hdg_train_step_dp) when
every rank is on this node, else torch.distributed (RCCL); HDG_DP_ALLREDUCE or the
`allreduce` argument ("auto" | "xgmi" | "rccl") overrides the choice.
"""
import ctypes
import os
import warnings

import numpy as np
import torch

from . import _lib
from .layout import n_params, state_offsets


class Engine:
    def __init__(self, ne, nc, batch, variant=2, device="cuda", batch_global=None, lr=3e-4,
                 process_group=None, path=_lib.PATH_AUTO, allreduce=None, flags=0,
                 dp_shared=None):
        """variant: model_<variant>.py (1 HD-GNN/ES, 2 HD-GNN/S, 3 HD-GNN/E, 4 HD-GNN).
        path: PATH_AUTO (fused kernel when it applies, else the general path),
        PATH_FUSED or PATH_GENERAL (include/hdgnn.h).  flags: HDG_FLAG_* bits
        (FLAG_HUNK_DENSE / FLAG_HUNK_SORTED force the general path's hunk-sum form).
        dp_shared: the xGMI ranks share devices (HDG_DP_SHARED); None detects it."""
        self.lib = _lib.load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("Engine needs a HIP device (got %s)" % self.device)
        if self.device.index is None:          # "cuda" -> the current device, explicitly,
            self.device = torch.device("cuda", torch.cuda.current_device())  # as tensors report
        self.ne, self.nc, self.batch, self.variant = ne, nc, batch, variant
        self.batch_global = batch_global or batch
        self.lr = lr
        self.pg = process_group
        self.shape = _lib.Shape(batch, ne, nc, variant, self.batch_global, path, flags)
        self.path = self.lib.hdg_resolve_path(ctypes.byref(self.shape))
        if self.path < 0:
            raise ValueError(self.lib.hdg_last_error().decode())
        self.np = self.lib.hdg_param_count(variant)
        assert self.np == n_params(variant)
        self.glen = self.lib.hdg_grad_len(variant)
        wsb = self.lib.hdg_workspace_bytes(ctypes.byref(self.shape))
        if wsb == 0:
            raise RuntimeError(self.lib.hdg_last_error().decode())
        dev = self.device
        f32 = torch.float32
        self.workspace = torch.zeros(wsb // 4, dtype=f32, device=dev)   # block-pair inboxes start at 0
        # the training state as one flat buffer [params | adam_m | adam_v | beta_pow]: one
        # copy snapshots, restores or reads it (the checkpoint's host copy)
        # (each slice 64-byte aligned, layout.state_offsets; the pads stay zero)
        P, so = self.np, state_offsets(variant)
        self.state = torch.zeros(so["len"], dtype=f32, device=dev)
        self.params, self.m, self.v, self.beta_pow = (
            self.state[:P], self.state[so["m"]:so["m"] + P], self.state[so["v"]:so["v"] + P],
            self.state[so["beta_pow"]:so["beta_pow"] + 2])
        for t in (self.params, self.m, self.v, self.beta_pow):
            assert t.data_ptr() % 64 == 0, "training-state slice not 64-byte aligned"
        self.beta_pow.copy_(torch.tensor([0.9, 0.999]))
        self.grad = torch.zeros(self.glen, dtype=f32, device=dev)
        # ce, loss_map, loss_para, train_loss, count parts (3), fault count (hdg_outputs.stats)
        self.stats = torch.zeros(_lib.STATS_LEN, dtype=f32, device=dev)
        # sticky status word (HDG_STATUS_* bits); check_status() reads it
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ce_sum = torch.zeros(1, dtype=f32, device=dev)
        self.ehr = torch.zeros(1, dtype=f32, device=dev)     # loss_E_HR of the last forward
        pc = nc * (nc - 1)
        self.probs = torch.zeros(batch, 2, pc, dtype=f32, device=dev)
        self.logits = torch.zeros(batch, 2, pc, dtype=f32, device=dev)
        self._state = _lib.State(self.params.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                 self.beta_pow.data_ptr())
        st = self.status.data_ptr()
        self._out = _lib.Outputs(self.probs.data_ptr(), self.logits.data_ptr(),
                                 self.stats.data_ptr(), st, self.ehr.data_ptr())
        # a training sess.run fetches C_edge_output2 (the probabilities), not the logits
        self._out_train = _lib.Outputs(self.probs.data_ptr(), None, self.stats.data_ptr(), st,
                                       None)
        self._out_none = _lib.Outputs(None, None, None, st, None)   # status only
        # data parallelism: which all-reduce joins the ranks' gradients
        self.xgmi, self.allreduce_kind, self.allreduce_selftest = None, None, None
        if self._distributed():
            mode = allreduce or os.environ.get("HDG_DP_ALLREDUCE", "auto")
            if mode not in ("auto", "xgmi", "rccl"):
                raise ValueError("allreduce must be auto, xgmi or rccl (got %r)" % mode)
            if mode != "rccl":
                from .xgmi import XgmiGroup
                self.xgmi = XgmiGroup.create(self.lib, self.pg or torch.distributed.group.WORLD,
                                             dev, required=mode == "xgmi", shared=dp_shared)
                self.allreduce_selftest = XgmiGroup.verdict
            else:
                self.allreduce_selftest = "xGMI not tried (HDG_DP_ALLREDUCE=rccl)"
            self.allreduce_kind = "xgmi" if self.xgmi else "rccl"
        # hdg_fwd_bwd's own (local) gradient: the xGMI tail reads it while writing the
        # world sum into self.grad, so the two must not overlap
        self.grad_local = (torch.zeros(self.glen, dtype=f32, device=dev) if self.xgmi
                           else self.grad)

    # ---- parameters ---------------------------------------------------------
    def set_params(self, flat):
        flat = np.asarray(flat, np.float32).reshape(-1)
        assert flat.size == self.np
        self.params.copy_(torch.from_numpy(flat))
        self.m.zero_()
        self.v.zero_()
        self.beta_pow.copy_(torch.tensor([0.9, 0.999]))

    def get_params(self):
        return self.params.detach().cpu().numpy().copy()

    # ---- steps --------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def upload(self, cb):
        """Host CommitBatch -> DeviceBatch prepared for this engine's path."""
        return cb.to_device(self.device, self.variant, self.path)

    def _check(self, dbatch):
        assert dbatch.B == self.batch and dbatch.Ne == self.ne and dbatch.Nc == self.nc
        if dbatch.path != self.path or getattr(dbatch, "variant", self.variant) != self.variant:
            raise ValueError("batch prepared for model_%s path %d, engine runs model_%d path %d "
                             "(use Engine.upload)" % (getattr(dbatch, "variant", "?"), dbatch.path,
                                                      self.variant, self.path))

    def _outputs(self, outputs, logits, stats=None):
        if not outputs:
            return self._out_none
        out = self._out if logits else self._out_train
        if stats is None:
            return out
        # a caller-provided stats row (a training loop's per-step row of an epoch buffer)
        assert stats.device == self.device and stats.dtype == torch.float32 and \
            stats.is_contiguous() and stats.numel() >= _lib.STATS_LEN
        return _lib.Outputs(out.probs, out.logits, stats.data_ptr(), out.status, out.ehr)

    # ---- split mode (fused path: two co-resident blocks per commit) -------------------
    @property
    def split(self):
        """False once set_split(False) forced one block per commit (HDG_FLAG_NO_SPLIT)."""
        return not (self.shape.flags & _lib.FLAG_NO_SPLIT)

    def set_split(self, on):
        self.shape.flags = (self.shape.flags & ~_lib.FLAG_NO_SPLIT) | (0 if on else
                                                                       _lib.FLAG_NO_SPLIT)

    def snapshot(self):
        """A device copy of the training state (parameters, Adam moments, beta powers)."""
        return self.state.clone()

    def restore(self, snap):
        """Set the training state from a snapshot() (device) or a host copy of self.state."""
        if isinstance(snap, np.ndarray):
            snap = torch.from_numpy(np.ascontiguousarray(snap, np.float32))
        self.state.copy_(snap)

    def split_fault_retry(self):
        """After a step whose block-pair exchange timed out (HDG_STATUS_XCH_TIMEOUT; its
        update was skipped on every rank, the fault count travels in the all-reduced
        gradient trailer): switch to one block per commit for the rest of the run and
        clear the status, so the caller re-runs the step.  Returns False when already in
        one-block mode (the fault is then not a residency problem)."""
        if not self.split:
            return False
        warnings.warn("libhdgnn: a split-mode block-pair exchange timed out (the two blocks "
                      "of a commit were not co-resident); re-running in one-block-per-commit "
                      "mode for the rest of this run", RuntimeWarning, stacklevel=2)
        self.set_split(False)
        self.clear_status()
        return True

    def train_step_checked(self, dbatch, outputs=True, logits=False, stats=None):
        """train_step that survives a split-mode pair timeout: on a faulted step (read from
        the gradient trailer, identical on every rank) the state is restored and the step
        re-run with one block per commit.

        A per-step diagnostic / test helper, not a loop body: it snapshots the whole state
        and synchronises with the device on every call.  Training loops use the epoch-buffer
        pattern of graph2graph.train (every step's stats into its own device row, one read
        per epoch, the retry decided from those rows)."""
        snap = self.snapshot() if self.split else None
        self.train_step(dbatch, outputs, logits, stats)
        fault = float(self.grad[self.np + _lib.TR_FAULT].item())
        if fault != 0.0 and snap is not None and self.split_fault_retry():
            self.restore(snap)
            self.train_step(dbatch, outputs, logits, stats)
            fault = float(self.grad[self.np + _lib.TR_FAULT].item())
        if fault != 0.0 or int(self.status.item()):
            self.check_status()

    # ---- status / trailer -----------------------------------------------------
    def check_status(self):
        """Raise if any launch since the last clear_status() failed on the device (the
        sticky status word, include/hdgnn.h).  Synchronises with the device."""
        st = int(self.status.item())
        if st & _lib.STATUS_DP_TIMEOUT:
            raise RuntimeError(
                "libhdgnn: a peer rank's gradient words did not arrive over xGMI in time (a "
                "rank stopped or issued a different sequence of steps); that step's loss is "
                "NaN and its update was skipped on the waiting blocks.")
        if st & _lib.STATUS_XCH_TIMEOUT:
            raise RuntimeError(
                "libhdgnn: a block-pair exchange of the fused split path timed out (the two "
                "blocks of a commit were not resident together: another process holding "
                "CUs?); that step's outputs are NaN and its Adam update was skipped. "
                "HDG_FUSED_SPLIT=0 runs one block per commit.")
        if st:
            raise RuntimeError("libhdgnn: device status 0x%x" % st)

    def clear_status(self):
        self.status.zero_()

    def correct_count(self, trailer=None):
        """top_ACC numerator of the last fwd_bwd / train step (summed over ranks when the
        gradient was all-reduced) from the gradient trailer."""
        tr = (self.grad[self.np:] if trailer is None else trailer)
        return _lib.trailer_count(tr.cpu().numpy() if hasattr(tr, "cpu") else tr)

    def fwd_bwd(self, dbatch, outputs=True, logits=True):
        self._reduced = False
        self._check(dbatch)
        b = dbatch.struct()
        out = self._outputs(outputs, logits)
        _lib.check(self.lib.hdg_fwd_bwd(ctypes.byref(self.shape), ctypes.byref(b),
                                        ctypes.c_void_p(self.params.data_ptr()),
                                        ctypes.c_void_p(self.grad_local.data_ptr()),
                                        ctypes.byref(out),
                                        ctypes.c_void_p(self.workspace.data_ptr()),
                                        self._stream()))

    def allreduce(self):
        """All-reduce the flat gradient: RCCL in place on self.grad; xGMI from the local
        gradient fwd_bwd wrote (grad_local) into self.grad (hdg_dp_allreduce).  Either way
        self.grad then holds the world sum, and adam() applies TF Adam to it."""
        if not self._distributed():
            return
        if self.xgmi:
            _lib.check(self.lib.hdg_dp_allreduce(ctypes.byref(self.xgmi.dp),
                                                 ctypes.c_void_p(self.grad_local.data_ptr()),
                                                 ctypes.c_void_p(self.grad.data_ptr()),
                                                 ctypes.c_int32(self.glen),
                                                 ctypes.c_void_p(self.status.data_ptr()),
                                                 self._stream()))
            self._reduced = True
            return
        torch.distributed.all_reduce(self.grad, group=self.pg)

    def adam(self):
        """TF Adam on the world gradient.  xGMI: when allreduce() already summed it into
        self.grad, a local update of that sum (every rank holds the same bits); otherwise
        the exchange and the update in one kernel (hdg_adam_dp, from grad_local)."""
        if self.xgmi and not getattr(self, "_reduced", False):
            _lib.check(self.lib.hdg_adam_dp(ctypes.byref(self.shape), ctypes.byref(self._state),
                                            ctypes.c_void_p(self.grad_local.data_ptr()),
                                            ctypes.c_void_p(self.grad.data_ptr()),
                                            ctypes.c_float(self.lr),
                                            ctypes.c_void_p(self.stats.data_ptr()),
                                            ctypes.c_void_p(self.status.data_ptr()),
                                            ctypes.byref(self.xgmi.dp), self._stream()))
            return
        self._reduced = False
        _lib.check(self.lib.hdg_adam_tf(ctypes.byref(self.shape), ctypes.byref(self._state),
                                        ctypes.c_void_p(self.grad.data_ptr()),
                                        ctypes.c_float(self.lr),
                                        ctypes.c_void_p(self.stats.data_ptr()), self._stream()))

    def _distributed(self):
        return self.pg is not None or (torch.distributed.is_available()
                                       and torch.distributed.is_initialized()
                                       and torch.distributed.get_world_size() > 1)

    def train_step(self, dbatch, outputs=True, logits=False, stats=None):
        """sess.run([C_edge_output2, loss_Hedge_mse, loss_map, theta, trainer]) equivalent:
        outputs land in self.probs / self.stats (pre-update), params updated in place;
        self.logits only with logits=True (the reference's training run does not fetch them);
        stats: a device row of >= 8 floats for this step's hdg_outputs.stats instead of
        self.stats (so a loop can keep every step's values and read them once).
        Single process: hdg_train_step (step kernel + fused reduce/Adam).  Data parallel
        over xGMI: hdg_train_step_dp (the same two kernels, the exchange inside the second).
        Over RCCL: hdg_fwd_bwd -> all-reduce of the flat gradient -> hdg_adam_tf."""
        if self.xgmi:
            self._check(dbatch)
            b = dbatch.struct()
            out = self._outputs(outputs, logits, stats)
            _lib.check(self.lib.hdg_train_step_dp(ctypes.byref(self.shape), ctypes.byref(b),
                                                  ctypes.byref(self._state),
                                                  ctypes.c_float(self.lr), ctypes.byref(out),
                                                  ctypes.c_void_p(self.grad.data_ptr()),
                                                  ctypes.c_void_p(self.workspace.data_ptr()),
                                                  ctypes.byref(self.xgmi.dp), self._stream()))
            return
        if self._distributed():
            self.fwd_bwd(dbatch, outputs, logits)
            self.allreduce()
            self.adam()
            if stats is not None:
                stats[:_lib.STATS_LEN].copy_(self.stats)
            return
        self._check(dbatch)
        b = dbatch.struct()
        out = self._outputs(outputs, logits, stats)
        _lib.check(self.lib.hdg_train_step(ctypes.byref(self.shape), ctypes.byref(b),
                                           ctypes.byref(self._state), ctypes.c_float(self.lr),
                                           ctypes.byref(out),
                                           ctypes.c_void_p(self.grad.data_ptr()),
                                           ctypes.c_void_p(self.workspace.data_ptr()),
                                           self._stream()))

    def step_call(self, dbatch, stats=None, logits=False):
        """A zero-argument callable that enqueues train_step(dbatch, logits=logits,
        stats=stats) on the current stream, its ctypes arguments built once (a training
        loop's per-step host cost).  Single process only; data parallel: train_step itself."""
        if self.xgmi or self._distributed():
            return lambda: self.train_step(dbatch, True, logits, stats)
        self._check(dbatch)
        b = dbatch.struct()
        out = self._outputs(True, logits, stats)
        fn, check = self.lib.hdg_train_step, _lib.check
        args = (ctypes.byref(self.shape), ctypes.byref(b), ctypes.byref(self._state),
                ctypes.c_float(self.lr), ctypes.byref(out),
                ctypes.c_void_p(self.grad.data_ptr()),
                ctypes.c_void_p(self.workspace.data_ptr()), self._stream())

        def call():
            check(fn(*args))
        return call

    # ---- HIP graph of one training step ----------------------------------------
    def capture(self, dbatch, outputs=True, logits=False, steps=1):
        """Capture `steps` consecutive train_step(dbatch) calls (fwd_bwd [+ RCCL all-reduce]
        + Adam each) into one HIP graph; replay() then runs that many training steps with a
        single launch (no per-step graph launch gap).  dbatch must stay alive."""
        saved = self.snapshot()
        self.train_step(dbatch, outputs, logits)  # warm: attributes set, RCCL comm built
        self.restore(saved)                       # the warm-up step leaves no trace
        torch.cuda.synchronize(self.device)
        self._graph_batch = dbatch
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                self.train_step(dbatch, outputs, logits)
        torch.cuda.synchronize(self.device)
        self._graph = g
        self.graph_steps = steps
        return g

    def replay(self):
        self._graph.replay()

    def forward(self, dbatch):
        """sess.run([loss_Hedge_mse, loss_map, C_edge_output2]) equivalent (test path);
        also fills self.ehr with the batch's loss_E_HR (model_2.py:122)."""
        self._check(dbatch)
        b = dbatch.struct()
        _lib.check(self.lib.hdg_forward(ctypes.byref(self.shape), ctypes.byref(b),
                                        ctypes.c_void_p(self.params.data_ptr()),
                                        ctypes.byref(self._out),
                                        ctypes.c_void_p(self.ce_sum.data_ptr()),
                                        ctypes.c_void_p(self.workspace.data_ptr()),
                                        self._stream()))
        return self.probs, self.logits, self.ce_sum
