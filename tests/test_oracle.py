"""Oracle pinning: loader bookkeeping vs the reference utils2 goldens, and the
pair-explicit model restatement vs the literal incidence restatement."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import layout, literal, loader_ref, model_ref


def _golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "loader_tiny.npz"))
    with open(os.path.join(golden_dir, "loader_tiny.json")) as f:
        meta = json.load(f)
    return z, meta


def test_param_counts_match_survey():
    # model_1 1146, model_2 2127, model_3 2148, model_4 3129
    assert [layout.n_params(v) for v in (1, 2, 3, 4)] == [1146, 2127, 2148, 3129]
    assert len(layout.specs(2)) == 18 and len(layout.specs(4)) == 27


def test_loader_restatement_matches_reference_goldens(golden_dir):
    z, meta = _golden(golden_dir)
    ne, nc = meta["Ne"], meta["Nc"]
    x, a, y, hid, nlen = loader_ref.compact_from_raw(
        z["CAdjs"], z["CHunkAdjs"], meta["index_lines"], meta["hunkmaps"], ne, nc)
    dense = literal.build_dense(x, a, y, hid, nlen, dtype=torch.float64)
    half = x.shape[0] // 2
    # node attributes (float64, exact)
    assert np.array_equal(dense["E_node"][:half].numpy(), z["E_node_train"])
    assert np.array_equal(dense["E_node"][half:].numpy(), z["E_node_test"])
    for ours, ref in (("E_edge", "E_edge"), ("C_edge", "C_edge")):
        assert np.array_equal(dense[ours][:half].numpy(), z[ref + "_train"])
        assert np.array_equal(dense[ours][half:].numpy(), z[ref + "_test"])
    for ours, ref in (("Es", "Es_data"), ("Et", "Et_data"), ("Cs", "Cs_label"),
                      ("Ct", "Ct_label"), ("Esc", "Esc_data"), ("Etc", "Etc_data")):
        assert np.array_equal(dense[ours].numpy(), z[ref]), ours


def test_loader_goldens_cover_edge_cases(golden_dir):
    z, meta = _golden(golden_dir)
    ne = meta["Ne"]
    lens = {len(l) for l in meta["index_lines"]}
    assert min(lens) < ne and max(lens) > ne          # n < Ne and truncation
    assert any("null" in l for l in meta["index_lines"])
    assert any(v < 0 for m in meta["hunkmaps"] for v in m.values())
    assert any(v >= meta["Nc"] for m in meta["hunkmaps"] for v in m.values())
    assert (z["CAdjs"] == -1).any()


def _rand_case(seed, B=3, ne=7, nc=5):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 10, (B, ne)).astype(np.float64)
    a = (rng.random((B, ne, ne)) < 0.3).astype(np.int8)
    y = (rng.random((B, nc, nc)) < 0.35).astype(np.int8)
    nlen = rng.integers(2, ne + 1, B).astype(np.int32)
    hid = rng.integers(-1, nc + 2, (B, ne)).astype(np.int32)
    hid[hid >= nc] = -1
    return x, a, y, hid, nlen


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pair_explicit_equals_literal(seed):
    x, a, y, hid, nlen = _rand_case(seed)
    params = model_ref.init_params(seed)
    B, ne = x.shape
    nc = y.shape[1]
    P1 = model_ref.to_torch_params(params)
    out1 = model_ref.forward(P1, x, a, y, hid, nlen)
    out1["total"].backward()
    P2 = model_ref.to_torch_params(params)
    D = literal.build_dense(x, a, y, hid, nlen, dtype=torch.float64)
    out2 = literal.forward(P2, D, B, ne, nc)
    out2["total"].backward()
    np.testing.assert_allclose(out1["logits"].detach().numpy(),
                               out2["logits"].transpose(1, 2).detach().numpy(),
                               rtol=1e-12, atol=1e-12)
    for k in ("ce", "loss_map", "loss_para", "total"):
        np.testing.assert_allclose(float(out1[k]), float(out2[k]), rtol=1e-12)
    for k in P1:
        np.testing.assert_allclose(P1[k].grad.numpy(), P2[k].grad.numpy(),
                                   rtol=1e-10, atol=1e-12)


def test_tf_adam_first_step_is_signed_lr():
    # TF Adam first step: lr_t * m/sqrt(v) = lr*sqrt(1-b2)/(1-b1) * (1-b1)|g|/(sqrt(1-b2)|g|)
    # = lr * sign(g)  (up to eps)
    opt = model_ref.AdamTF(3)
    th = np.zeros(3)
    g = np.array([2.0, -0.5, 1e-3])
    th = opt.step(th, g)
    np.testing.assert_allclose(th, -3e-4 * np.sign(g), rtol=1e-3)
