"""xGMI mailboxes for the data-parallel gradient all-reduce (include/hdgnn.h hdg_*_dp).

SURVEY 8(e): the step's only coupling between ranks is one all-reduce of the flat fp32
gradient (2131 floats for model_2).  At that size the collective is pure latency, so
instead of an RCCL call between two kernels the step's reduction kernel exchanges the
gradient itself: every rank allocates a mailbox of uncached device memory, the 64-byte
HIP IPC handles are all-gathered once over the process group, every rank maps every
peer's mailbox, and from then on each step's tail kernel writes its gradient slots
straight into all peers' mailboxes over xGMI and sums the world's values in rank order
(the same bits on every rank).

`XgmiGroup.create` decides ONCE, consistently on every rank (all-reduce MIN of each
rank's verdict), whether the node can run it: single host, world <= 16, mailbox
allocated, every peer handle opened, and a self-test all-reduce through the mailboxes
returns the exact sums.  Otherwise it returns None (auto mode: the caller all-reduces
through torch.distributed / RCCL) or raises (mode "xgmi").
"""
import contextlib
import ctypes
import os
import socket
import sys

import numpy as np
import torch

from . import _lib

TICKS_PER_S = 100_000_000           # s_memrealtime
SELFTEST_WAIT_S = 5.0


def device_identity(device):
    """A string naming the physical GPU behind `device`: its UUID and PCI location as torch
    reports them (every one available, so a runtime that leaves the UUID blank or equal on
    all GPUs still tells them apart by bus), else its index: equal for two ranks on the
    same GPU.  A CPU device (the set-up protocol's tests) names the process: never shared."""
    device = torch.device(device)
    if device.type != "cuda":
        return "%s:pid%d" % (device.type, os.getpid())
    p = torch.cuda.get_device_properties(device)
    parts = ["%s=%s" % (a, getattr(p, a)) for a in ("uuid", "pci_domain_id", "pci_bus_id",
                                                    "pci_device_id")
             if getattr(p, a, None) is not None and str(getattr(p, a))]
    return ";".join(parts) if parts else "index:%d" % device.index


class XgmiGroup:
    # the last create()'s outcome on this rank: "passed: ..." or why it gave up
    verdict = None

    def __init__(self, lib, rank, world, own, peers, device):
        self.lib, self.rank, self.world, self.device = lib, rank, world, device
        self._own, self._peers = own, peers          # c_void_p; {rank: c_void_p} opened
        self.dp = _lib.Dp()
        self.dp.rank, self.dp.world = rank, world
        for r in range(world):
            self.dp.mailbox[r] = own.value if r == rank else peers[r].value

    # ------------------------------------------------------------------ setup
    @classmethod
    def create(cls, lib, pg, device, required=False, wait_s=10.0, shared=None):
        """shared: the ranks share devices (hdg_dp.flags HDG_DP_SHARED: light capped tails
        that cannot starve a peer's step kernel of CUs); None = detect it from the ranks'
        device identities (one GPU box: every rank on device 0)."""
        dist = torch.distributed
        world, rank = dist.get_world_size(pg), dist.get_rank(pg)
        tdev = device if dist.get_backend(pg) == "nccl" else torch.device("cpu")
        if shared is None:
            devs = [None] * world
            dist.all_gather_object(devs, (socket.gethostname(), device_identity(device)),
                                   group=pg)
            shared = len(set(devs)) < world

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg)
            return bool(t.item())

        def give_up(why):
            cls.verdict = why
            if required:
                raise RuntimeError("xGMI all-reduce unavailable: %s" % why)
            return None

        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname(), group=pg)
        if not agree(world <= _lib.DP_MAX_WORLD and len(set(hosts)) == 1):
            return give_up("ranks span several hosts or world > %d" % _lib.DP_MAX_WORLD)
        dctx = torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()
        with dctx:
            own = ctypes.c_void_p()
            h = (ctypes.c_ubyte * _lib.DP_HANDLE_BYTES)()
            ok = lib.hdg_dp_mailbox_alloc(ctypes.byref(own), h) == 0
            err = "" if ok else lib.hdg_last_error().decode(errors="replace")
            mine = torch.tensor(np.frombuffer(bytes(h), np.uint8).copy(), device=tdev)
            allh = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(allh, mine, group=pg)
            if not agree(ok):
                if own.value:
                    lib.hdg_dp_mailbox_free(own)
                return give_up("mailbox allocation failed (%s)" % err)
            peers = {}
            for r in range(world):
                if r == rank:
                    continue
                p = ctypes.c_void_p()
                hb = (ctypes.c_ubyte * _lib.DP_HANDLE_BYTES).from_buffer_copy(
                    allh[r].cpu().numpy().tobytes())
                if lib.hdg_dp_mailbox_open(hb, ctypes.byref(p)) != 0:
                    ok = False
                    err = lib.hdg_last_error().decode(errors="replace")
                    break
                peers[r] = p
            grp = cls(lib, rank, world, own, peers, device) if ok else None
            if grp:
                grp.dp.flags = _lib.DP_SHARED if shared else 0
            if not agree(ok):
                if grp:
                    grp.close()
                else:
                    for p in peers.values():
                        lib.hdg_dp_mailbox_close(p)
                    lib.hdg_dp_mailbox_free(own)
                return give_up("opening a peer mailbox failed (%s)" % err)
            why = grp.selftest()
            if not agree(why is None):
                grp.close()
                return give_up("self-test failed on some rank (%s)" % (why or "peer"))
            grp.dp.wait_ticks = int(wait_s * TICKS_PER_S)
            cls.verdict = ("passed: exact rank-order sums of %d floats over %d ranks through "
                           "the mailboxes%s" % (_lib.DP_MAX_LEN, world,
                                                " (ranks share a device: light tails, the "
                                                "waiting ranks on at most half the CUs)"
                                                if shared else ""))
            return grp

    def selftest(self, n=_lib.DP_MAX_LEN):
        """All-reduce rank-dependent integers through the mailboxes; None if the sums are
        exact and no peer timed out, else a reason."""
        saved = self.dp.wait_ticks
        self.dp.wait_ticks = int(SELFTEST_WAIT_S * TICKS_PER_S)
        try:
            base = torch.arange(n, dtype=torch.float32, device=self.device) % 1021
            x = base * (self.rank + 1) + self.rank
            out = torch.full_like(x, float("nan"))
            status = torch.zeros(1, dtype=torch.int32, device=self.device)
            self.allreduce(x, out, status)
            torch.cuda.synchronize(self.device)
            w = self.world
            want = base * (w * (w + 1) // 2) + w * (w - 1) // 2
            if int(status.item()) & _lib.STATUS_DP_TIMEOUT:
                return "a peer's words did not arrive"
            if not torch.equal(out, want):
                return "wrong sums (max err %g)" % float((out - want).abs().max())
            return None
        finally:
            self.dp.wait_ticks = saved

    # ------------------------------------------------------------------ calls
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def allreduce(self, x, out, status=None):
        """out = sum over ranks of x (fp32, contiguous, numel <= DP_MAX_LEN)."""
        assert x.dtype == torch.float32 and x.is_contiguous() and out.numel() >= x.numel()
        _lib.check(self.lib.hdg_dp_allreduce(ctypes.byref(self.dp), ctypes.c_void_p(x.data_ptr()),
                                             ctypes.c_void_p(out.data_ptr()), x.numel(),
                                             ctypes.c_void_p(status.data_ptr() if status is not None
                                                             else None),
                                             self._stream()))

    def close(self):
        if self._own is None:
            return
        try:
            torch.cuda.synchronize(self.device)
        except Exception:
            pass
        for p in self._peers.values():
            self.lib.hdg_dp_mailbox_close(p)
        self.lib.hdg_dp_mailbox_free(self._own)
        self._own, self._peers = None, {}

    def __del__(self):
        if sys.is_finalizing():      # the process exit releases the mappings
            return
        try:
            self.close()
        except Exception:
            pass
