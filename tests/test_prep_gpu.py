"""hdg_prepare's cross-graph count tables against the oracle's relation maps, bit-exact.

K_s[c][I] = #{relations r in Ne-row I : s_r = c} + #{... : t_r = c}, K_t over Ne-columns,
ncst[c][a] = the same counts split by the relation's class a (utils2.py:111-137, the
marshalling_B2 maps of model_2.py:146-150; s_r, t_r walk the n-grid: oracle.model_ref.
relation_maps).  Cases: n in {0, 1, 2, Ne}, unmapped nodes, every node mapped, both
engine paths, the stress shape."""
import ctypes

import numpy as np
import pytest

from hdgnn import _lib
from hdgnn.synth import synth_commits
from oracle import model_ref

pytestmark = pytest.mark.gpu


def expected_counts(cb):
    B, ne = cb.x.shape
    nc = cb.y.shape[1]
    s, t = model_ref.relation_maps(cb.hid, cb.nlen, ne, nc)
    I, J = model_ref.pair_index(ne)
    ks = np.zeros((B, nc, ne), np.int64)
    kt = np.zeros((B, nc, ne), np.int64)
    ncst = np.zeros((B, nc, 2), np.int64)
    for b in range(B):
        a = cb.a[b, I, J].astype(np.int64)
        for h in (s[b], t[b]):
            m = h >= 0
            np.add.at(ks[b], (h[m], I[m]), 1)
            np.add.at(kt[b], (h[m], J[m]), 1)
            np.add.at(ncst[b], (h[m], a[m]), 1)
    return ks, kt, ncst


def device_counts(db, ne, nc, variant, path):
    lib = _lib.load()
    sh = _lib.Shape(db.B, ne, nc, variant, db.B, path)
    st, ks, kt, nco = (ctypes.c_int64() for _ in range(4))
    _lib.check(lib.hdg_prep_counts_layout(ctypes.byref(sh), ctypes.byref(st), ctypes.byref(ks),
                                          ctypes.byref(kt), ctypes.byref(nco)))
    words = db.prep.cpu().numpy().view(np.uint32)[:db.B * st.value].reshape(db.B, st.value)
    u16 = lambda o: words[:, o:o + (nc * ne + 1) // 2].copy().view(np.uint16)[:, :nc * ne]
    return (u16(ks.value).reshape(db.B, nc, ne), u16(kt.value).reshape(db.B, nc, ne),
            words[:, nco.value:nco.value + 2 * nc].copy().view(np.float32).reshape(db.B, nc, 2))


@pytest.mark.parametrize("B,ne,nc,variant,path", [
    (5, 24, 10, 2, _lib.PATH_FUSED), (5, 24, 10, 2, _lib.PATH_GENERAL),
    (6, 200, 74, 2, _lib.PATH_FUSED), (6, 200, 74, 4, _lib.PATH_GENERAL),
    (5, 250, 150, 2, _lib.PATH_FUSED), (5, 300, 33, 1, _lib.PATH_GENERAL),
    (2, 1024, 512, 2, _lib.PATH_GENERAL)])
def test_count_tables_bit_exact(B, ne, nc, variant, path):
    cb = synth_commits(B, ne, nc, 11 + ne + nc)
    for i, n in enumerate([0, 1, 2, ne][:B - 1]):
        cb.nlen[i] = n
    cb.nlen[-1] = ne
    cb.hid[-1] = np.random.default_rng(ne).integers(0, nc, ne)   # every node mapped
    db = cb.to_device("cuda:0", variant, path)
    ks, kt, ncst = device_counts(db, ne, nc, variant, path)
    eks, ekt, encst = expected_counts(cb)
    np.testing.assert_array_equal(ks, eks)
    np.testing.assert_array_equal(kt, ekt)
    np.testing.assert_array_equal(ncst, encst.astype(np.float32))


@pytest.mark.parametrize("B,ne,nc,variant", [
    (3, 24, 10, 2), (3, 37, 12, 4), (4, 200, 74, 4), (2, 1024, 512, 2), (3, 5, 3, 2)])
def test_neighbour_lists_bit_exact(B, ne, nc, variant):
    """The general path's per-node neighbour id lists (wide.hip kw_prep_lists: side 0 the
    j != i with a_ij = 1, side 1 the j with a_ji = 1, ascending, padded to 4 with the
    sentinel ne) against the adjacency, including a full and an empty commit."""
    cb = synth_commits(B, ne, nc, 5 + ne)
    cb.a[0] = 1                      # full adjacency, diagonal included (lists skip j == i)
    cb.a[1] = 0
    db = cb.to_device("cuda:0", variant, _lib.PATH_GENERAL)
    lib = _lib.load()
    sh = _lib.Shape(B, ne, nc, variant, B, _lib.PATH_GENERAL)
    st, ks, kt, nco = (ctypes.c_int64() for _ in range(4))
    _lib.check(lib.hdg_prep_counts_layout(ctypes.byref(sh), ctypes.byref(st), ctypes.byref(ks),
                                          ctypes.byref(kt), ctypes.byref(nco)))
    we, wc, ls = (ne + 31) // 32, (nc + 31) // 32, (ne + 3) & ~3
    c0 = (B * st.value + B * ne * we + B * nc * wc + 3) & ~3
    i0 = c0 + ((2 * B * ne + 3) & ~3)
    words = db.prep.cpu().numpy().view(np.uint32)
    assert words.size >= i0 + B * ne * ls
    cnt = words[c0:c0 + 2 * B * ne].reshape(2, B, ne)
    ids = words[i0:i0 + B * ne * ls].copy().view(np.uint16).reshape(2, B, ne, ls)
    for side, adj in ((0, cb.a), (1, cb.a.transpose(0, 2, 1))):
        for b in range(B):
            for i in range(ne):
                exp = np.flatnonzero(adj[b, i])
                exp = exp[exp != i]
                n = len(exp)
                assert cnt[side, b, i] == n, (side, b, i)
                np.testing.assert_array_equal(ids[side, b, i, :n], exp)
                assert (ids[side, b, i, n:(n + 3) & ~3] == ne).all()


@pytest.mark.parametrize("B,n", [(3, 7), (2, 33), (4, 200), (1, 1100)])
def test_pack_classes_matches_host(B, n):
    """hdg_pack_classes (the upload's device-side bit packing) == data.pack_bits."""
    import ctypes
    import torch
    from hdgnn import _lib
    from hdgnn.data import pack_bits
    rng = np.random.default_rng(n)
    grid = (rng.random((B, n, n)) < 0.3).astype(np.uint8)
    g = torch.from_numpy(grid).cuda()
    out = torch.full((B, n, (n + 31) // 32), -1, dtype=torch.int32, device="cuda")
    lib = _lib.load()
    _lib.check(lib.hdg_pack_classes(ctypes.c_void_p(g.data_ptr()), B, n,
                                    ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), pack_bits(grid))
