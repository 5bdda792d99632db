"""Synthetic glide-shaped commits; the dataset (Adjset/glide.zip) is absent.

Per commit, numpy PCG64 seeded with 20250301 + 1000*config_idx + rank:
  * entity adjacency: off-diagonal Bernoulli(0.05); diagonal node attribute = integer 0..9
  * hunk adjacency (labels): symmetric Bernoulli(0.10)
  * index file: n ~ U{ceil(Ne/2)..ceil(3Ne/2)} lines, truncated to Ne (utils2.py:121);
    each line 'null' w.p. 0.2, else hunk id ~ U{0..floor(1.25 Nc)}; ids >= Nc dropped

Data-dependence knobs (bench.py --edensity/--hdensity/--xkind; the defaults are the
generator above): entity density, hunk (label) density, and the attribute kind -- "int10"
integers 0..9, or "real": Ne distinct signed reals per commit (the sorted-x entity sums
then see nd = Ne distinct values, their worst case).
"""
import math

import numpy as np

from .data import CommitBatch

SEED_BASE = 20250301


def seed_for(config_idx=0, rank=0):
    return SEED_BASE + 1000 * config_idx + rank


XKINDS = ("int10", "real")


def synth_commits(B, ne, nc, seed=SEED_BASE, edensity=0.05, hdensity=0.10, xkind="int10"):
    if xkind not in XKINDS:
        raise ValueError("xkind must be one of %s" % (XKINDS,))
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 10, (B, ne)).astype(np.float32)
    a = (rng.random((B, ne, ne)) < edensity).astype(np.uint8)
    idx = np.arange(ne)
    a[:, idx, idx] = 0
    u = rng.random((B, nc, nc)) < hdensity
    up = np.triu(u, 1)
    y = (up | up.transpose(0, 2, 1)).astype(np.uint8)
    lo, hi = math.ceil(ne / 2), math.ceil(3 * ne / 2)
    n = rng.integers(lo, hi + 1, B)
    nlen = np.minimum(n, ne).astype(np.int32)
    null = rng.random((B, ne)) < 0.2
    ids = rng.integers(0, int(1.25 * nc) + 1, (B, ne))
    hid = np.where(null | (ids >= nc), -1, ids).astype(np.int32)
    hid[np.arange(ne)[None, :] >= nlen[:, None]] = -1
    if xkind == "real":        # drawn after the default stream: a, y, hid are unchanged
        x = (rng.standard_normal((B, ne)) * 4).astype(np.float32)
    return CommitBatch(x, a, y, hid, nlen)
