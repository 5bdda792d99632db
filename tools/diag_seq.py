"""Diagnostic: run some general-path model_4 work first (argv[1]: train / fwd / both / none,
argv[2]: B,ne,nc), then a fused model_2 hdg_fwd_bwd at (4, 60, 21); report non-finite grads."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hd-gnn_amd"))
from hdgnn import layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

what = sys.argv[1]
B0, ne0, nc0 = (int(t) for t in sys.argv[2].split(","))
v0 = int(sys.argv[3]) if len(sys.argv) > 3 else 4
pre = Engine(ne0, nc0, B0, variant=v0, path=2)
pre.set_params(layout.init_flat(7, v0))
dpre = pre.upload(synth_commits(B0, ne0, nc0, 3))
if what in ("train", "both"):
    pre.train_step(dpre)
if what in ("fwd", "both"):
    pre.forward(dpre)
torch.cuda.synchronize()
del pre, dpre
e = Engine(60, 21, 4, variant=2)
e.set_params(layout.init_flat(5, 2))
db = e.upload(synth_commits(4, 60, 21, 8))
e.fwd_bwd(db)
torch.cuda.synchronize()
print("%s %s v%d -> fused fwd_bwd non-finite grads: %d" % (
    what, sys.argv[2], v0, int((~torch.isfinite(e.grad)).sum())), flush=True)
