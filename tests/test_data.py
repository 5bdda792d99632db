"""Adapter from utils2's 12-tuple to the compact device form: bit-exact against the
reference loader's golden output and the oracle's bookkeeping restatement."""
import json
import os

import numpy as np
import pytest

from hdgnn import data, layout
from hdgnn.synth import synth_commits
from oracle import layout as olayout
from oracle import loader_ref


def _golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "loader_tiny.npz"))
    with open(os.path.join(golden_dir, "loader_tiny.json")) as f:
        return z, json.load(f)


NAMES = ["E_node_train", "E_node_test", "E_edge_train", "E_edge_test", "C_edge_train",
         "C_edge_test", "Es_data", "Et_data", "Cs_label", "Ct_label", "Esc_data", "Etc_data"]


@pytest.mark.parametrize("mini_batch", [50, 7])
def test_adapter_matches_reference_loader(golden_dir, mini_batch):
    z, meta = _golden(golden_dir)
    ne, nc = meta["Ne"], meta["Nc"]
    tup = tuple(z[n] for n in NAMES)
    train, test, maps = data.compact_from_read_data(tup, ne, nc, mini_batch)
    x, a, y, hid, nlen = loader_ref.compact_from_raw(z["CAdjs"], z["CHunkAdjs"],
                                                     meta["index_lines"], meta["hunkmaps"], ne, nc)
    np.testing.assert_array_equal(train.x, x[:50].astype(np.float32))
    np.testing.assert_array_equal(test.x, x[50:].astype(np.float32))
    np.testing.assert_array_equal(train.a * (1 - np.eye(ne, dtype=np.uint8)), a[:50])
    np.testing.assert_array_equal(test.y * (1 - np.eye(nc, dtype=np.uint8)), y[50:])
    # hunk maps: the factorised (n, hid) reproduce Esc/Etc exactly
    from oracle.model_ref import relation_maps
    s_ref, t_ref = relation_maps(hid[:mini_batch], nlen[:mini_batch], ne, nc)
    s_got, t_got = relation_maps(maps.hid, maps.nlen, ne, nc)
    np.testing.assert_array_equal(s_got, s_ref)
    np.testing.assert_array_equal(t_got, t_ref)
    # and against the reference's own dense arrays
    s_z = np.where(z["Esc_data"][:mini_batch].sum(1) > 0, z["Esc_data"][:mini_batch].argmax(1), -1)
    np.testing.assert_array_equal(s_got, s_z)


def test_adapter_rejects_non_canonical_incidence(golden_dir):
    z, meta = _golden(golden_dir)
    tup = [z[n].copy() for n in NAMES]
    tup[6][0, 0, 0] = 0.0     # break Es
    with pytest.raises(ValueError):
        data.compact_from_read_data(tuple(tup), meta["Ne"], meta["Nc"], 50)


def test_pack_bits_roundtrip():
    cb = synth_commits(3, 70, 33, 0)
    bits = data.pack_bits(cb.a)
    assert bits.shape == (3, 70, 3) and bits.dtype == np.uint32
    un = np.zeros_like(cb.a)
    for j in range(70):
        un[:, :, j] = (bits[:, :, j // 32] >> (j % 32)) & 1
    np.testing.assert_array_equal(un, cb.a * (1 - np.eye(70, dtype=np.uint8)))


def test_factorize_roundtrip_random():
    rng = np.random.default_rng(0)
    from oracle.model_ref import relation_maps
    for _ in range(50):
        ne, nc = int(rng.integers(2, 12)), int(rng.integers(2, 6))
        n = int(rng.integers(0, ne + 1))
        hid = rng.integers(-1, nc, ne).astype(np.int32)
        hid[n:] = -1
        s, t = relation_maps(hid[None], np.array([n]), ne, nc)
        n2, hid2 = data.factorize_maps(s[0], t[0], ne)
        s2, t2 = relation_maps(hid2[None], np.array([n2]), ne, nc)
        np.testing.assert_array_equal(s2, s)
        np.testing.assert_array_equal(t2, t)


def test_synth_shapes_and_ranges():
    cb = synth_commits(10, 200, 74, 20250301)
    cb.validate()
    assert cb.x.dtype == np.float32 and cb.x.min() >= 0 and cb.x.max() <= 9
    assert np.all(cb.y == cb.y.transpose(0, 2, 1))
    assert 0.02 < cb.a.mean() < 0.08
    assert np.all(cb.nlen <= 200) and np.all(cb.nlen >= 100)


@pytest.mark.parametrize("bad", [0.5, np.nan, 2.0, -1.0])
def test_validate_float_grids_exact_membership(bad):
    """Float class grids must hold exactly 0/1: a value the u8 upload would truncate to
    class 0 (0.5, NaN) is rejected, not silently reclassified."""
    cb = synth_commits(2, 20, 9, 1)
    for name in ("a", "y"):
        f = data.CommitBatch(cb.x, cb.a.astype(np.float32), cb.y.astype(np.float32),
                             cb.hid, cb.nlen)
        f.validate()                                   # exact 0/1 floats pass
        getattr(f, name)[1, 3, 4] = bad
        with pytest.raises(ValueError):
            f.validate()
    i = data.CommitBatch(cb.x, cb.a.astype(np.int8), cb.y, cb.hid, cb.nlen)
    i.validate()
    i.a[0, 1, 2] = -1
    with pytest.raises(ValueError):
        i.validate()


def test_layouts_agree():
    assert layout.n_params(2) == olayout.n_params(2) == 2127
    eng = [(n.split(":")[0], s) for n, s in layout.specs(2)]
    assert eng == olayout.specs(2)
