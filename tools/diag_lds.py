"""Diagnostic: poison every CU's LDS, then run one step per engine path; a changed or
non-finite gradient means a kernel reads LDS it never wrote."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
from hdgnn import layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

P = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "liblds_poison.so"))
P.lds_poison.argtypes = [ctypes.c_float, ctypes.c_void_p]
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for (B, ne, nc) in ((4, 60, 21), (100, 200, 74), (3, 7, 5)):
    cb = synth_commits(B, ne, nc, 8)
    for v, path in ((2, 1), (2, 2), (4, 2)):
        e = Engine(ne, nc, B, variant=v, path=path)
        e.set_params(layout.init_flat(5, v))
        db = e.upload(cb)
        P.lds_poison(0.0, st())
        e.fwd_bwd(db)
        g0 = e.grad.clone()
        for val in (float("nan"), 1e30, -1e30, float("inf")):
            P.lds_poison(val, st())
            e.fwd_bwd(db)
            torch.cuda.synchronize()
            nb = int((~torch.isfinite(e.grad)).sum())
            same = torch.equal(e.grad, g0)
            print("B=%d ne=%d nc=%d v=%d path=%d poison=%g: non-finite %d bitwise-same %s" % (
                B, ne, nc, v, path, val, nb, same), flush=True)
            if nb or not same:
                bad = ((e.grad != g0) | ~torch.isfinite(e.grad)).nonzero().flatten().tolist()
                print("   differing params:", bad[:12], "...", len(bad))
