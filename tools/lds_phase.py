"""Counter-attribution driver (tools/lds_phases.sh): a few eager fwd_bwd launches of the
glide step (model_2 fused, B=100, split) with fixed parameters, so a rocprofv3 --pmc run
of a HDG_STOP_AFTER build counts the kernel's work up to that phase boundary only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
import torch  # noqa: E402

from hdgnn import layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import seed_for, synth_commits  # noqa: E402

ne, nc, B = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (200, 74, 100)))
cb = synth_commits(B, ne, nc, seed_for(1, 0))
eng = Engine(ne, nc, B)
eng.set_params(layout.init_flat(0, 2))
db = eng.upload(cb)
for _ in range(6):
    eng.fwd_bwd(db)
torch.cuda.synchronize()
print("ok")
