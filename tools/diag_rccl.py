"""Diagnostic: eager DP step (fwd_bwd -> RCCL all_reduce -> adam) on world 1; checks for
non-finite values after every stage, with and without host syncs in between."""
import os
import socket
import sys

import numpy as np
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
B, ne, nc, v = 4, 60, 21, 2
cb = synth_commits(B, ne, nc, 8)
flat = layout.init_flat(5, v)


def bad(t):
    t = t.detach().float().cpu().numpy()
    return int((~np.isfinite(t)).sum()), (np.nonzero(~np.isfinite(t))[0][:8].tolist())


poison = os.environ.get("POISON", "1") == "1"
for sync in (True, False):
    if poison:   # recycled allocator blocks full of NaN: exposes reads of unwritten memory
        junk = [torch.full((1 << 24,), float("nan"), device="cuda") for _ in range(8)]
        del junk
    e = Engine(ne, nc, B, variant=v, process_group=pg)
    e.set_params(flat)
    db = e.upload(cb)
    for it in range(4):
        e.grad.fill_(12345.0)
        e.fwd_bwd(db)
        if sync:
            torch.cuda.synchronize()
            print("sync=%s it=%d after fwd_bwd grad bad %s" % (sync, it, bad(e.grad)))
        e.allreduce()
        if sync:
            torch.cuda.synchronize()
            print("sync=%s it=%d after allreduce grad bad %s" % (sync, it, bad(e.grad)))
        e.adam()
        torch.cuda.synchronize()
        print("sync=%s it=%d after adam params bad %s m bad %s v bad %s" % (
            sync, it, bad(e.params), bad(e.m), bad(e.v)), flush=True)
for pv, path in ((2, 1), (2, 2), (4, 2)):
    for mode in ("train_step", "fwd_bwd+adam"):
        junk = [torch.full((1 << 24,), float("nan"), device="cuda") for _ in range(8)]
        del junk
        e = Engine(ne, nc, B, variant=pv, path=path, process_group=None if mode == "train_step" else pg)
        e.set_params(layout.init_flat(5, pv))
        db = e.upload(cb)
        for it in range(3):
            e.train_step(db)
        torch.cuda.synchronize()
        print("poisoned v=%d path=%d %s: params bad %s grad bad %s probs bad %s" % (
            pv, path, mode, bad(e.params), bad(e.grad), bad(e.probs)), flush=True)
dist.destroy_process_group()
