"""Commit batches in compact form, and the bit-exact adapter from utils2's 12-tuple.

utils2.read_data (utils2.py:11-253) stays the reference loader.  Its 12 dense
arrays (~9 GB at glide step 2) encode, per commit, only:
    x    = E_node[:, 0, :]                      node attributes (float64 -> fed as f32)
    a    = class of E_edge per relation         (one-hot over Dr=2)
    y    = class of C_edge per relation
    n, hid : Esc/Etc = hunk rows of the first n index lines, enumerated with the
             n-grid relation counter (utils2.py:123-137)
plus Es/Et/Cs/Ct, which are the canonical complete-digraph incidences for every
commit.  compact_from_read_data() extracts exactly that and VERIFIES the rest, so
a feed that is not of this form is rejected instead of silently mis-read.
"""
import ctypes
from dataclasses import dataclass

import numpy as np


def pair_index(n):
    """(I, J) of relation r on an n-node complete digraph, row-major, j != i
    (the order utils2 fills Es/Et, Cs/Ct and Esc/Etc)."""
    if n < 2:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    r = np.arange(n * (n - 1), dtype=np.int64)
    i = r // (n - 1)
    jj = r % (n - 1)
    return i, jj + (jj >= i)


def pack_bits(cls):
    """(B, N, N) class array -> (B, N, ceil(N/32)) uint32, bit j of row i = (cls[i,j]==1),
    diagonal cleared (relations never include i == j)."""
    cls = np.asarray(cls)
    B, N, _ = cls.shape
    W = (N + 31) // 32
    m = (cls == 1)
    m = m & ~np.eye(N, dtype=bool)[None]
    pad = np.zeros((B, N, W * 32), bool)
    pad[:, :, :N] = m
    by = np.packbits(pad, axis=-1, bitorder="little")          # (B, N, 4W) bytes
    return np.ascontiguousarray(by).view("<u4").reshape(B, N, W)


def onehot_relations(cls):
    """(B, N, N) classes -> (B, 2, N(N-1)) float32 one-hot over relations in utils2's order:
    the C_edge / E_edge arrays the reference feeds and scores (utils2.py:86-106)."""
    cls = np.asarray(cls)
    I, J = pair_index(cls.shape[1])
    c = cls[:, I, J]
    return np.stack([(c == 0), (c == 1)], 1).astype(np.float32)


@dataclass
class CommitBatch:
    """Host-side compact commits.  x f32 (B,Ne); a, y u8 class grids; hid i32 (B,Ne);
    nlen i32 (B,)."""
    x: np.ndarray
    a: np.ndarray
    y: np.ndarray
    hid: np.ndarray
    nlen: np.ndarray

    @property
    def B(self):
        return self.x.shape[0]

    @property
    def Ne(self):
        return self.x.shape[1]

    @property
    def Nc(self):
        return self.y.shape[1]

    def slice(self, lo, hi):
        return CommitBatch(self.x[lo:hi], self.a[lo:hi], self.y[lo:hi], self.hid[lo:hi],
                           self.nlen[lo:hi])

    def with_maps(self, maps):
        """Reference quirk (model_2.py:376-381, 495-500): Es..Etc are always fed as
        [:Mini_batch], so position k of every batch uses commit k's hunk maps."""
        return CommitBatch(self.x, self.a, self.y, maps.hid[:self.B], maps.nlen[:self.B])

    def validate(self):
        B, Ne = self.x.shape
        Nc = self.y.shape[1]
        assert self.a.shape == (B, Ne, Ne) and self.y.shape == (B, Nc, Nc)
        assert self.hid.shape == (B, Ne) and self.nlen.shape == (B,)
        for m in (self.a, self.y):         # classes in {0, 1}
            if not m.size:
                continue
            if m.dtype.kind in "uib":      # integer grids: two reductions, no np.isin
                bad = m.max() > 1 or (m.dtype.kind == "i" and m.min() < 0)
            else:                          # float grids: exact membership (0.5, NaN fail)
                bad = not ((m == 0) | (m == 1)).all()
            if bad:
                raise ValueError("edge classes must be 0/1")
        if np.any(self.hid < -1) or np.any(self.hid >= Nc):
            raise ValueError("hid entries must be in [-1, Nc)")
        if np.any(self.nlen < 0) or np.any(self.nlen > Ne):
            raise ValueError("nlen must be in [0, Ne]")
        return self

    def to_device(self, device="cuda", variant=2, path=0):
        """Upload + hdg_prepare.  The prepared tables depend on the engine path the
        (variant, path) pair resolves to, so pass the Engine's."""
        return DeviceBatch.from_host(self, device, variant, path)


class DeviceBatch:
    """The hdg_batch struct's device arrays (include/hdgnn.h), prepared on upload:
    hdg_prepare builds the per-commit sort / transposed-bit / count tables in `prep`."""

    def __init__(self, x, abits, ybits, hid, nlen, Ne, Nc, variant=2, path=0):
        import torch
        from . import _lib
        self.x, self.abits, self.ybits, self.hid, self.nlen = x, abits, ybits, hid, nlen
        self.B, self.Ne, self.Nc, self.variant = x.shape[0], Ne, Nc, variant
        lib = _lib.load()
        shape = _lib.Shape(self.B, Ne, Nc, variant, self.B, path)
        self.path = lib.hdg_resolve_path(ctypes.byref(shape))   # prep layout is per path
        if self.path < 0:
            raise ValueError(lib.hdg_last_error().decode())
        nbytes = lib.hdg_prep_bytes(ctypes.byref(shape))
        if nbytes == 0:
            raise ValueError(lib.hdg_last_error().decode())
        # zeroed: words no table covers (padding) are deterministic, so two preparations
        # of one batch compare bytewise (tools/prep_dump.py)
        self.prep = torch.zeros(nbytes // 4, dtype=torch.int32, device=x.device)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(lib.hdg_prepare(ctypes.byref(shape), ctypes.byref(self.struct()),
                                   ctypes.c_void_p(stream)))

    @classmethod
    def from_host(cls, cb, device="cuda", variant=2, path=0):
        """Upload: the compact u8 class grids travel as they are (through pinned staging
        buffers, asynchronously) and are packed into bit rows on the GPU
        (hdg_pack_classes); then hdg_prepare.  No host-side bit packing."""
        import torch
        from . import _lib
        cb.validate()
        device = torch.device(device)

        def up(arr, dt):
            host = torch.from_numpy(np.ascontiguousarray(arr))
            if host.dtype != dt:
                host = host.to(dt)
            staged = torch.empty(host.shape, dtype=dt, pin_memory=True)
            staged.copy_(host)
            return staged.to(device, non_blocking=True)

        lib = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)

        def bits(grid):
            g = up(grid, torch.uint8)
            B, N = grid.shape[0], grid.shape[1]
            out = torch.empty((B, N, (N + 31) // 32), dtype=torch.int32, device=device)
            _lib.check(lib.hdg_pack_classes(ctypes.c_void_p(g.data_ptr()), B, N,
                                            ctypes.c_void_p(out.data_ptr()), stream))
            return out                      # g's memory is reused in stream order only

        return cls(up(cb.x, torch.float32), bits(cb.a), bits(cb.y), up(cb.hid, torch.int32),
                   up(cb.nlen, torch.int32), cb.Ne, cb.Nc, variant, path)

    def struct(self):
        from ._lib import Batch
        prep = getattr(self, "prep", None)
        return Batch(self.x.data_ptr(), self.abits.data_ptr(), self.ybits.data_ptr(),
                     self.hid.data_ptr(), self.nlen.data_ptr(),
                     prep.data_ptr() if prep is not None else None)


# ----------------------------------------------------------------------------
# adapter from utils2.read_data's 12-tuple
# ----------------------------------------------------------------------------
def _classes(onehot, what):
    """(B, 2, R) one-hot -> (B, R) class, verifying exactly one 1 per relation."""
    oh = np.asarray(onehot)
    if oh.ndim != 3 or oh.shape[1] != 2:
        raise ValueError("%s must be (B, 2, R)" % what)
    if not (np.all((oh == 0) | (oh == 1)) and np.all(oh.sum(1) == 1)):
        raise ValueError("%s is not one-hot over Dr=2" % what)
    return oh[:, 1, :].astype(np.uint8)


def _grid(cls_rel, n):
    I, J = pair_index(n)
    out = np.zeros((cls_rel.shape[0], n, n), np.uint8)
    out[:, I, J] = cls_rel
    return out


def _check_incidence(M, n, src, what):
    I, J = pair_index(n)
    idx = I if src else J
    M = np.asarray(M)
    if M.shape[1:] != (n, len(I)):
        raise ValueError("%s has shape %s, expected (*, %d, %d)" % (what, M.shape, n, len(I)))
    exp = np.zeros((n, len(I)), M.dtype)
    exp[idx, np.arange(len(I))] = 1
    if not np.all(M == exp[None]):
        raise ValueError("%s is not the canonical complete-graph incidence" % what)


def _rel_rows(M, what):
    """(B, Nc, R) 0/1 -> (B, R) row of the single 1 per column, -1 when empty."""
    M = np.asarray(M)
    s = M.sum(1)
    if not (np.all((M == 0) | (M == 1)) and np.all(s <= 1)):
        raise ValueError("%s columns must hold at most one 1" % what)
    out = M.argmax(1).astype(np.int64)
    out[s == 0] = -1
    return out


def factorize_maps(s, t, ne):
    """Per-relation hunk rows (s_r, t_r) of one commit -> (n, hid) such that
    s_r = hid[i'(r)], t_r = hid[j'(r)] for r < n(n-1) on the n-grid and -1 beyond
    (utils2.py:121-137).  Raises if no such (n, hid) exists."""
    s = np.asarray(s)
    t = np.asarray(t)
    nz = np.nonzero((s >= 0) | (t >= 0))[0]
    if len(nz) == 0:
        return ne, np.full(ne, -1, np.int32)
    rmax = int(nz.max())
    n_min = 2
    while n_min * (n_min - 1) <= rmax:
        n_min += 1
    for n in [ne] + list(range(n_min, ne)):
        if n * (n - 1) <= rmax:
            continue
        I, J = pair_index(n)
        hid = np.full(ne, -1, np.int64)
        hid[I[::-1]] = s[:len(I)][::-1]       # any relation of row i' carries hid[i']
        es = np.full_like(s, -1)
        et = np.full_like(t, -1)
        es[:len(I)] = hid[I]
        et[:len(I)] = hid[J]
        if np.array_equal(es, s) and np.array_equal(et, t):
            return n, hid.astype(np.int32)
    raise ValueError("Esc/Etc maps are not of the utils2 index-line form")


def compact_from_read_data(tup, ne, nc, mini_batch=None):
    """utils2.read_data 12-tuple -> (train CommitBatch, test CommitBatch, maps CommitBatch).

    maps holds the hunk maps of the first `mini_batch` commits (the rows the
    reference feeds for every batch).  Bit-exact: see tests/test_data.py."""
    (E_node_train, E_node_test, E_edge_train, E_edge_test, C_edge_train, C_edge_test,
     Es, Et, Cs, Ct, Esc, Etc) = tup
    mb = mini_batch or len(E_node_train)
    for M, n, src, what in ((Es[:mb], ne, True, "Es"), (Et[:mb], ne, False, "Et"),
                            (Cs[:mb], nc, True, "Cs"), (Ct[:mb], nc, False, "Ct")):
        _check_incidence(M, n, src, what)

    def part(E_node, E_edge, C_edge):
        x = np.asarray(E_node)[:, 0, :].astype(np.float32)     # TF feed casts f64 -> f32
        a = _grid(_classes(E_edge, "E_edge"), ne)
        y = _grid(_classes(C_edge, "C_edge"), nc)
        B = x.shape[0]
        return CommitBatch(x, a, y, np.full((B, ne), -1, np.int32), np.zeros(B, np.int32))

    train = part(E_node_train, E_edge_train, C_edge_train)
    test = part(E_node_test, E_edge_test, C_edge_test)
    s = _rel_rows(Esc[:mb], "Esc")
    t = _rel_rows(Etc[:mb], "Etc")
    hid = np.zeros((mb, ne), np.int32)
    nlen = np.zeros(mb, np.int32)
    for k in range(mb):
        nlen[k], hid[k] = factorize_maps(s[k], t[k], ne)
    maps = CommitBatch(train.x[:mb], train.a[:mb], train.y[:mb], hid, nlen)
    return train, test, maps
