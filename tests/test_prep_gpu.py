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
