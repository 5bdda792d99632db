"""Per-epoch cost parts of graph2graph.train at glide B=100 (GPU box): the step with its
one stats read, the split-mode snapshot, the state's host copy and the bundle write.
    python tools/e2e_parts.py"""
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hd-gnn_amd"))
from hdgnn import _lib, tfckpt  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.model import Saver  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402


def timed(f, n=50):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main():
    dev = torch.device("cuda:0")
    B, ne, nc = 100, 200, 74
    cb = synth_commits(B, ne, nc, 20250308)
    eng = Engine(ne, nc, B, variant=2, device=dev)
    db = eng.upload(cb)
    es = torch.zeros(1, _lib.STATS_LEN, dtype=torch.float32, device=dev)
    sv = Saver(type("M", (), {"engine": eng, "variant": 2})())
    d = tempfile.mkdtemp()
    st = sv._host_state()
    parts = {
        "train_step": timed(lambda: eng.train_step(db, logits=False, stats=es[0])),
        "train_step+stats_read": timed(lambda: (eng.train_step(db, logits=False, stats=es[0]),
                                                es.cpu())),
        "snapshot": timed(lambda: eng.snapshot()),
        "host_state": timed(lambda: sv._host_state()),
        "bundle_write": timed(lambda: sv._write(os.path.join(d, "g2g.model-1"), st)),
    }
    print({k: round(v, 4) for k, v in parts.items()})


if __name__ == "__main__":
    main()
