"""Diagnostic: does an eager RCCL all_reduce issued after a graph-captured one (same
communicator, world 1) change the buffer?  Memory is dirtied first, like a long session."""
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hd-gnn_amd"))
from hdgnn import layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
pg = dist.group.WORLD
junk = [torch.randn(1 << 22, device="cuda") * 1e30 for _ in range(16)]
del junk
B, ne, nc, v = 4, 60, 21, 2
cb = synth_commits(B, ne, nc, 8)
flat = layout.init_flat(5, v)
dp = Engine(ne, nc, B, variant=v, process_group=pg)
dg = Engine(ne, nc, B, variant=v, process_group=pg)
for e in (dp, dg):
    e.set_params(flat)
db = dp.upload(cb)
for capture in (False, True):
    if capture:
        dg.capture(db)
        print("captured", flush=True)
    for it in range(3):
        dp.fwd_bwd(db)
        torch.cuda.synchronize()
        g1 = dp.grad.clone()
        dp.allreduce()
        torch.cuda.synchronize()
        g2 = dp.grad.clone()
        print("capture=%s it=%d grad finite before %s after %s  changed by allreduce: %s" % (
            capture, it, bool(torch.isfinite(g1).all()), bool(torch.isfinite(g2).all()),
            not torch.equal(g1, g2)), flush=True)
        dp.adam()
        if capture:
            dg.replay()
        torch.cuda.synchronize()
dist.destroy_process_group()
