"""Diagnostic: per-phase wall time of k_commit_step from s_memrealtime stamps (100 MHz)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hd-gnn_amd"))
from hdgnn import _lib, layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

# python tools/mid_phases.py [ne nc [B]]  (default glide 200 74 100)
ne = int(sys.argv[1]) if len(sys.argv) > 2 else 200
nc = int(sys.argv[2]) if len(sys.argv) > 2 else 74
B = int(sys.argv[3]) if len(sys.argv) > 3 else 100
cb = synth_commits(B, ne, nc, 1)
db = cb.to_device()
eng = Engine(ne, nc, B)
eng.set_params(layout.init_flat(0))
for _ in range(3):
    eng.train_step(db)
# one row of 32 phase stamps per block (split: 2 per commit), then [2B][16 waves][8] wave stamps
st = torch.zeros(2 * B * 32 + 2 * B * 16 * 8, dtype=torch.int64, device="cuda")
for _ in range(3):
    _lib.check(eng.lib.hdg_debug_step_stamps(ctypes.byref(eng.shape), ctypes.byref(db.struct()),
                                            ctypes.c_void_p(eng.params.data_ptr()),
                                            ctypes.c_void_p(eng.workspace.data_ptr()),
                                            ctypes.c_void_p(st.data_ptr()), eng._stream()))
torch.cuda.synchronize()
allst = st.cpu().numpy().astype(np.int64)
nblk = 2 * B if allst[B * 32] > 0 or allst[(2 * B - 1) * 32] > 0 else B
s = allst[:2 * B * 32].reshape(2 * B, 32)
wst = allst[nblk * 32: nblk * 32 + nblk * 128].reshape(nblk, 16, 8)
s = s[:nblk]
n = int((s[0] > 0).sum())
d = np.diff(s[:, :n], axis=1) * 10e-3   # us
med = np.median(d, axis=0)
for i, v in enumerate(med):
    print("phase %2d->%2d  %8.2f us" % (i, i + 1, v))
print("total (median block) %.1f us; block span max %.1f us" % (np.median(d.sum(1)), d.sum(1).max()))
t0 = s[:, 0] - s[:, 0].min()
print("block start skew: median %.2f us, max %.2f us; first start -> last end %.1f us" % (
    np.median(t0) * 10e-3, t0.max() * 10e-3, (s[:, n - 1].max() - s[:, 0].min()) * 10e-3))

# per-wave stamps: (slot, phase stamp it is measured from, label)
WAVE = [(5, 0, "stage staged (from kernel start)"), (0, 1, "E1 done (from E1 start)"), (1, 8, "M7 loop done (from M7 start)"),
        (3, 19, "scan start (from M13 start)"), (4, 19, "scans done (from M13 start)"),
        (2, 21, "E2 done (from E2 start)")]
for slot, ph, label in WAVE:
    if wst[:, :, slot].max() == 0:
        continue
    rel = (wst[:, :, slot] - s[:, ph:ph + 1]) * 10e-3
    print("%-32s per wave (median over blocks, us): %s" % (
        label, " ".join("%.2f" % v for v in np.median(rel, axis=0))))
