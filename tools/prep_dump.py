"""Dump the prepared tables (hdg_prepare's `prep` buffer, zero-initialised) of a fixed set
of batches: run once per library build (HDG_LIB_PATH) and compare the dumps bytewise.
    python tools/prep_dump.py OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))

import torch  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

CASES = [  # (B, Ne, Nc, variant, path, seed)
    (3, 24, 10, 2, 1, 1), (3, 24, 10, 2, 2, 2), (8, 200, 74, 2, 1, 3), (8, 200, 74, 4, 2, 4),
    (6, 250, 150, 2, 1, 5), (4, 250, 150, 4, 2, 6), (2, 1024, 512, 2, 2, 7),
    (3, 300, 33, 1, 2, 8), (4, 64, 64, 2, 1, 9),
]


def edge(cb, seed):
    """n in {0, 1, 2, Ne} on the first commits, one commit with every node mapped."""
    rng = np.random.default_rng(seed)
    ne, nc = cb.x.shape[1], cb.y.shape[1]
    B = cb.x.shape[0]
    for i, n in enumerate([0, 1, 2, ne][:B - 1]):
        cb.nlen[i] = n
    cb.nlen[-1] = ne
    cb.hid[-1] = rng.integers(0, nc, ne)          # every node mapped (dense hid)
    return cb


def main(out):
    res = {}
    for (B, ne, nc, v, path, seed) in CASES:
        cb = edge(synth_commits(B, ne, nc, seed), seed)
        db = cb.to_device("cuda:0", v, path)
        torch.cuda.synchronize()
        res["%d_%d_%d_%d_%d" % (B, ne, nc, v, path)] = db.prep.cpu().numpy()
    np.savez(out, **res)
    print("dumped", len(res), "cases to", out)


if __name__ == "__main__":
    main(sys.argv[1])
