"""Diagnostic: fill an engine's workspace / outputs with large finite garbage before each
step; a non-finite or changed gradient means a kernel reads memory it never wrote."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hd-gnn_amd"))
from hdgnn import layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

B, ne, nc = 4, 60, 21
cb = synth_commits(B, ne, nc, 8)
for v, path in ((2, 1), (2, 2), (4, 2), (1, 2)):
    ref = Engine(ne, nc, B, variant=v, path=path)
    ref.set_params(layout.init_flat(5, v))
    db = ref.upload(cb)
    ref.workspace.zero_()
    ref.fwd_bwd(db)
    g0 = ref.grad.clone()
    for fill in (1e30, -1e30, 3.0e38, 7.0):
        e = Engine(ne, nc, B, variant=v, path=path)
        e.set_params(layout.init_flat(5, v))
        e.workspace.fill_(fill)
        e.grad.fill_(fill)
        e.probs.fill_(fill)
        e.fwd_bwd(db)
        torch.cuda.synchronize()
        g = e.grad
        nb = (~torch.isfinite(g)).nonzero().flatten().tolist()
        diff = (g - g0).abs().max().item() if not nb else float("nan")
        print("v=%d path=%d fill=%g: non-finite %d %s  max|g-g0| %.3g" % (v, path, fill, len(nb), nb[:10], diff), flush=True)
