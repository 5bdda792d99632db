"""Diagnostic: per-wave phase times of one general-path kernel from WSTAMP stamps.

Build a timing library (the kernel id selects which kernel stamps, see wide.hip WSTAMP):
    HDG_HIPCC_FLAGS=-DHDG_WSTAMP=2 python -c "import sys; sys.path.insert(0,'hd-gnn_amd');
        from hdgnn import build; build.build(out='hd-gnn_amd/csrc/ws_2.so')"
then on the GPU box:
    HDG_LIB_PATH=$PWD/hd-gnn_amd/csrc/ws_2.so python tools/wstamp.py <slots> [--ne N --nc N
        --batch B --variant V --hunk dense|sorted|tiled]
Prints, per stamp interval, the median / p90 / max over waves (us), the kernel span (first
stamp 0 -> last final stamp) and the spread of wave start times.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hd-gnn_amd"))
from hdgnn import _lib, layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("slots", type=int)
ap.add_argument("--ne", type=int, default=1024)
ap.add_argument("--nc", type=int, default=512)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--variant", type=int, default=2)
ap.add_argument("--hunk", default="sorted")
ap.add_argument("--path", type=int, default=2, help="0 auto, 1 fused (model_4: hybrid), 2 general")
ap.add_argument("--groups", type=int, default=1,
                help="report the stamped waves as this many contiguous groups (grid z slices)")
a = ap.parse_args()
flags = {"dense": _lib.FLAG_HUNK_DENSE, "sorted": _lib.FLAG_HUNK_SORTED,
         "tiled": _lib.FLAG_HUNK_TILED}[a.hunk]
eng = Engine(a.ne, a.nc, a.batch, variant=a.variant, path=a.path, flags=flags)
eng.set_params(layout.init_flat(0, a.variant))
db = eng.upload(synth_commits(a.batch, a.ne, a.nc, 1))
N = 1 << 22
st = torch.zeros(N * 8, dtype=torch.int64, device="cuda")
lib = eng.lib
lib.hdg_wstamp_set.argtypes = [ctypes.c_void_p]
assert lib.hdg_wstamp_set(ctypes.c_void_p(st.data_ptr())) == 0, "not a WSTAMP build"
for _ in range(3):
    eng.fwd_bwd(db)
torch.cuda.synchronize()
lib.hdg_wstamp_set(ctypes.c_void_p(0))
s_all = st.view(N, 8).cpu().numpy()[:, :a.slots].astype(np.int64)
s_all = s_all[s_all[:, 0] > 0]
for gi, s in enumerate(np.array_split(s_all, a.groups)):
    if a.groups > 1:
        print("-- group %d of %d" % (gi, a.groups))
    done = (s > 0).all(1)
    print("waves stamped %d (complete %d)" % (len(s), int(done.sum())))
    s = s[done]
    d = np.diff(s, axis=1) * 1e-2               # 100 MHz ticks -> us
    for i in range(a.slots - 1):
        print("stamp %d->%d  median %7.2f  p90 %7.2f  max %7.2f us" % (
            i, i + 1, np.median(d[:, i]), np.percentile(d[:, i], 90), d[:, i].max()))
    tot = (s[:, -1] - s[:, 0]) * 1e-2
    print("per wave total: median %.2f p90 %.2f max %.2f us" % (
        np.median(tot), np.percentile(tot, 90), tot.max()))
    t0 = (s[:, 0] - s_all[:, 0].min()) * 1e-2
    print("wave starts: p10 %.2f median %.2f p90 %.2f max %.2f us; span %.2f us" % (
        np.percentile(t0, 10), np.median(t0), np.percentile(t0, 90), t0.max(),
        (s[:, -1].max() - s_all[:, 0].min()) * 1e-2))
