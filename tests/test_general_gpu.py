"""General engine path (csrc/wide.hip) vs the CPU oracle, every model variant.  GPU only.

Variants: 1 model_1 HD-GNN/ES (hunk stage on B_1), 2 model_2 HD-GNN/S,
3 model_3 HD-GNN/E (entity-edge stage computed, unused), 4 model_4 HD-GNN (entity-edge
probabilities replace E_edge in B_2).  Tolerances, set at about 4x the worst error any
case here reached (profiles/r03/parity_summary.txt):
  logits  2e-5 |ref| + 2e-6 max(1, max|ref|)   (worst 8.7e-7 max|ref| in round 4; 3.3e-6 with
          the dense form at Nc = 2048, which the automatic choice no longer runs)
  probs = softmax(logits) to 1e-6; CE rel 1e-5
  gradients  8e-5 |ref| + 8e-6 max|ref| per variable (worst 2.45e-5 |ref| on the largest
          element at the 4096-node shape; <= 3.5e-6 max|ref| at glide)
  weights after TF-Adam atol 2e-6.
"""
import numpy as np
import pytest
import torch

from hdgnn import _lib, layout
from hdgnn.data import CommitBatch
from hdgnn.synth import synth_commits
from oracle import layout as olayout
from oracle import model_ref
from tests import _errlog

pytestmark = pytest.mark.gpu

GEN = _lib.PATH_GENERAL
LOGIT_RTOL, LOGIT_ATOL = 2e-5, 2e-6       # x |ref|, x max(1, max|ref|) of the commit
GRAD_RTOL, GRAD_ATOL = 8e-5, 8e-6         # x |ref|, x max|ref| of the variable


def _keys(v):
    return [k for k, _, _ in olayout.keyed_specs(v)]


def _engine(B, ne, nc, v, path=GEN, flags=0):
    from hdgnn.engine import Engine
    return Engine(ne, nc, B, variant=v, path=path, flags=flags)


def _oracle(flat, cb, v):
    params = model_ref.unflatten(np.asarray(flat, np.float64), v)
    out, grads = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                          cb.nlen, variant=v)
    return out, np.concatenate([grads[k].reshape(-1) for k in _keys(v)])


def _reg_grad(flat):
    """loss_para + 0.1 loss_map gradients (model_2.py:123-130, 326-333); thetas last."""
    g = 0.001 * flat.astype(np.float64)
    n = len(flat)
    for off in (n - 4, n - 2):
        th = flat[off:off + 2].astype(np.float64)
        g[off:off + 2] += 0.001 * th / np.linalg.norm(th)
    return g


def _check_outputs(logits, probs, out):
    ref = out["logits"].transpose(0, 2, 1)
    scale = np.maximum(1.0, np.abs(ref).reshape(ref.shape[0], -1).max(1))[:, None, None]
    tol = LOGIT_RTOL * np.abs(ref) + LOGIT_ATOL * scale
    err = np.abs(logits - ref)
    _errlog.record("logits", (err / scale).max(), (err / tol).max())
    assert np.all(err <= tol), "logits: max err %.3g" % err.max()
    sm = np.exp(logits - logits.max(1, keepdims=True))
    sm /= sm.sum(1, keepdims=True)
    np.testing.assert_allclose(probs, sm, atol=1e-6)


def _grad_close(g_eng, g_ref, v):
    bad = []
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        a, r = g_eng[o:o + n], g_ref[o:o + n]
        scale = max(np.abs(r).max(), 1e-12)
        tol = GRAD_RTOL * np.abs(r) + GRAD_ATOL * scale + 1e-9
        err = np.abs(a - r)
        _errlog.record("grad:" + name, err.max() / scale, (err / tol).max())
        if not np.all(err <= tol):
            bad.append("%s: max err %.3g, scale %.3g, %d/%d bad" % (
                name, np.nanmax(err) if np.isfinite(err).any() else np.nan, scale,
                int((~(err <= tol)).sum()), n))
    assert not bad, "gradient mismatch:\n  " + "\n  ".join(bad)


def _run_and_check(cb, v, seed, path=GEN, flags=0):
    B, ne, nc = cb.B, cb.Ne, cb.Nc
    flat = layout.init_flat(seed, v)
    eng = _engine(B, ne, nc, v, path, flags)
    eng.set_params(flat)
    db = eng.upload(cb)
    eng.fwd_bwd(db)
    torch.cuda.synchronize()
    out, g_ref = _oracle(flat, cb, v)
    _check_outputs(eng.logits.cpu().numpy(), eng.probs.cpu().numpy(), out)
    g = eng.grad.cpu().numpy().astype(np.float64)
    np_ = len(flat)
    _grad_close(g[:np_] + _reg_grad(flat), g_ref, v)
    np.testing.assert_allclose(g[np_] / (B * nc * (nc - 1)), float(out["ce"]), rtol=1e-5)
    probs, logits, ce_sum = eng.forward(db)          # test path (forward only)
    torch.cuda.synchronize()
    _check_outputs(logits.cpu().numpy(), probs.cpu().numpy(), out)
    np.testing.assert_allclose(ce_sum.item() / (B * nc * (nc - 1)), float(out["ce"]), rtol=1e-5)
    np.testing.assert_allclose(eng.ehr.item(), float(out["loss_E_HR"]), rtol=1e-4)
    return eng


SHAPES = [
    (3, 7, 5, 0),       # tiny
    (2, 37, 19, 1),     # ragged
    (2, 64, 64, 2),     # exactly one tile
    (2, 65, 70, 3),     # one past a tile on both graphs
    (2, 200, 74, 4),    # glide step 2 (BASELINE config 1/2)
    (1, 250, 114, 5),   # step=3 shapes (BASELINE config 3)
]


@pytest.mark.parametrize("v", [1, 2, 3, 4])
@pytest.mark.parametrize("B,ne,nc,seed", SHAPES)
def test_variant_matches_oracle(v, B, ne, nc, seed):
    _run_and_check(synth_commits(B, ne, nc, seed), v, seed)


FUS = _lib.PATH_FUSED


@pytest.mark.parametrize("B,ne,nc,seed", SHAPES + [(1, 256, 160, 6), (2, 120, 100, 8)])
def test_model2_fused_path_matches_oracle(B, ne, nc, seed):
    """the fused path over every tile width of its hunk passes (NC16 = 16 .. 160)"""
    _run_and_check(synth_commits(B, ne, nc, seed), 2, seed, FUS)


@pytest.mark.parametrize("B,ne,nc,seed", SHAPES + [(1, 256, 160, 6)])
def test_model4_fused_path_matches_oracle(B, ne, nc, seed):
    """model_4 on the fused path: the entity-edge stage on the general kernels around the
    fused step kernel (class part of n_c in, dn out), up to the fused engine's limits."""
    _run_and_check(synth_commits(B, ne, nc, seed), 4, seed, FUS)


def test_model4_fused_equals_general():
    B, ne, nc, v = 3, 200, 74, 4
    cb = synth_commits(B, ne, nc, 13)
    flat = layout.init_flat(2, v)
    outs = []
    for path in (FUS, GEN):
        eng = _engine(B, ne, nc, v, path)
        assert eng.path == path
        eng.set_params(flat)
        eng.fwd_bwd(eng.upload(cb))
        torch.cuda.synchronize()
        outs.append((eng.logits.cpu().numpy().astype(np.float64),
                     eng.grad.cpu().numpy().astype(np.float64)))
    (l1, g1), (l2, g2) = outs
    scale = np.maximum(1.0, np.abs(l1).max())
    assert np.abs(l1 - l2).max() <= 1e-4 * scale
    np_ = layout.n_params(v)
    _grad_close(g2[:np_], g1[:np_], v)
    assert _lib.trailer_count(g1[np_:]) == _lib.trailer_count(g2[np_:])


@pytest.mark.parametrize("v", [2, 4])
def test_stress_shape_matches_oracle(v):
    """BASELINE config 5 shapes (Ne=1024, Nc=512): beyond the fused kernel's LDS budget."""
    _run_and_check(synth_commits(1, 1024, 512, 9), v, 9)


@pytest.mark.parametrize("ne", [401, 600])
def test_ee_gamma_table_mode_matches_oracle(ne):
    """kw_ee_fwd's gam-only LDS table (Ne past the two-table limit 400, while the table
    fits the LDS; Ne = 1024 is covered by the stress shape), ragged node counts."""
    _run_and_check(synth_commits(2, ne, 50, 21), 4, 21)


def test_general_equals_fused_model2():
    B, ne, nc = 4, 200, 74
    cb = synth_commits(B, ne, nc, 12)
    flat = layout.init_flat(2)
    outs = []
    for path in (_lib.PATH_FUSED, GEN):
        eng = _engine(B, ne, nc, 2, path)
        eng.set_params(flat)
        eng.fwd_bwd(eng.upload(cb))
        torch.cuda.synchronize()
        outs.append((eng.logits.cpu().numpy().astype(np.float64),
                     eng.grad.cpu().numpy().astype(np.float64)))
    (l1, g1), (l2, g2) = outs
    scale = np.maximum(1.0, np.abs(l1).max())
    assert np.abs(l1 - l2).max() <= 1e-4 * scale
    _grad_close(g2[:2127], g1[:2127], 2)


EDGE = {
    "no_index_lines": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid * 0 - 1, cb.nlen * 0),
    "one_index_line": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid, cb.nlen * 0 + 1),
    "two_index_lines": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid, cb.nlen * 0 + 2),
    "full_index_file": lambda cb: CommitBatch(cb.x, cb.a, cb.y, np.abs(cb.hid) % cb.Nc,
                                              cb.nlen * 0 + cb.Ne),
    "all_lines_one_hunk": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid * 0, cb.nlen * 0 + cb.Ne),
    "empty_adjacency": lambda cb: CommitBatch(cb.x, 0 * cb.a, 0 * cb.y, cb.hid, cb.nlen),
    "full_adjacency": lambda cb: CommitBatch(cb.x, 1 - np.eye(cb.Ne, dtype=np.uint8)[None] + 0 * cb.a,
                                             1 - np.eye(cb.Nc, dtype=np.uint8)[None] + 0 * cb.y,
                                             cb.hid, cb.nlen),
    "float_attributes": lambda cb: CommitBatch(
        (np.random.default_rng(3).standard_normal(cb.x.shape) * 4).astype(np.float32),
        cb.a, cb.y, cb.hid, cb.nlen),
}


@pytest.mark.parametrize("path", [GEN, FUS])
@pytest.mark.parametrize("case", sorted(EDGE))
def test_model4_edge_cases(case, path):
    cb = EDGE[case](synth_commits(2, 70, 13, 7))
    _run_and_check(cb, 4, 7, path)


@pytest.mark.parametrize("path", [GEN, FUS])
def test_model4_train_steps_match_oracle_adam(path):
    B, ne, nc, seed, v = 2, 45, 17, 5, 4
    cb = synth_commits(B, ne, nc, seed)
    flat = layout.init_flat(seed, v)
    eng = _engine(B, ne, nc, v, path)
    eng.set_params(flat)
    db = eng.upload(cb)
    theta = flat.astype(np.float64)
    opt = model_ref.AdamTF(len(flat))
    for _ in range(3):
        eng.train_step(db)
        torch.cuda.synchronize()
        out, g_ref = _oracle(theta.astype(np.float32), cb, v)
        stats = eng.stats.cpu().numpy()
        for i, k in enumerate(("ce", "loss_map", "loss_para", "total")):
            np.testing.assert_allclose(stats[i], float(out[k]), rtol=1e-5)
        theta = opt.step(theta, g_ref)
        np.testing.assert_allclose(eng.get_params(), theta, rtol=0, atol=2e-6)


def test_general_deterministic_bitwise():
    cb = synth_commits(3, 200, 74, 11)
    eng = _engine(3, 200, 74, 4)
    eng.set_params(layout.init_flat(1, 4))
    db = eng.upload(cb)
    eng.fwd_bwd(db)
    g1, p1 = eng.grad.clone(), eng.probs.clone()
    eng.fwd_bwd(db)
    assert torch.equal(g1, eng.grad) and torch.equal(p1, eng.probs)


@pytest.mark.parametrize("path", [GEN, FUS])
def test_general_graph_replay_equals_eager(path):
    B, ne, nc, v = 3, 50, 30, 4
    cb = synth_commits(B, ne, nc, 4)
    flat = layout.init_flat(3, v)
    e1, e2 = _engine(B, ne, nc, v, path), _engine(B, ne, nc, v, path)
    e1.set_params(flat)
    e2.set_params(flat)
    db = e1.upload(cb)
    e2.capture(db)
    for _ in range(3):
        e1.train_step(db)
        e2.replay()
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.probs, e2.probs)


@pytest.mark.parametrize("v,path", [(2, _lib.PATH_FUSED), (2, GEN), (4, GEN), (4, _lib.PATH_FUSED),
                                    (1, GEN)])
def test_workspace_garbage_does_not_leak(v, path):
    """Every workspace word a step reads it wrote first: prefilling the caller's workspace,
    gradient and outputs with NaN / Inf / huge values must not change one bit (a kernel that
    masks an unwritten value by multiplying with 0 turns NaN garbage into NaN output)."""
    B, ne, nc = 3, 60, 21
    cb = synth_commits(B, ne, nc, 8)
    ref = _engine(B, ne, nc, v, path)
    ref.set_params(layout.init_flat(5, v))
    db = ref.upload(cb)
    ref.workspace.zero_()
    ref.fwd_bwd(db)
    g0, p0 = ref.grad.clone(), ref.probs.clone()
    for fill in (float("nan"), float("inf"), -float("inf"), 1e30, -3e38):
        e = _engine(B, ne, nc, v, path)
        e.set_params(layout.init_flat(5, v))
        for t in (e.workspace, e.grad, e.probs, e.logits):
            t.fill_(fill)
        e.fwd_bwd(db)
        torch.cuda.synchronize()
        assert torch.equal(e.grad, g0) and torch.equal(e.probs, p0), "fill %g" % fill


@pytest.mark.parametrize("v,path", [(2, _lib.PATH_FUSED), (2, GEN), (4, GEN), (4, _lib.PATH_FUSED)])
def test_on_device_correct_count(v, path):
    """Gradient trailer count slots = EvaluationFuncs.top_ACC numerator on the returned probs
    (np.argmax tie rule), exactly; forward-only leaves the CE slot intact."""
    from hdgnn import metrics
    from hdgnn.data import onehot_relations
    B, ne, nc = 5, 70, 33
    cb = synth_commits(B, ne, nc, 2)
    eng = _engine(B, ne, nc, v, path)
    eng.set_params(layout.init_flat(1, v))
    eng.fwd_bwd(eng.upload(cb))
    torch.cuda.synchronize()
    want = metrics.top_acc_count(onehot_relations(cb.y), eng.probs.cpu().numpy())
    assert eng.correct_count() == want


@pytest.mark.parametrize("v", [2, 4])
def test_max_shape_matches_oracle(v):
    """The general path's upper limit Ne = 4096 (largest dynamic LDS of the entity and
    entity-edge kernels, 13-word neighbour lists of 4096 ids, a^T tiles of 128 words)."""
    _run_and_check(synth_commits(1, 4096, 40, 3), v, 3)


@pytest.mark.parametrize("v", [1, 4])
def test_max_classes_matches_oracle(v):
    """The general path's class limit Nc = 2048 (hunk pair passes over 2048 x 2047
    relations, 64-word y rows, u16 count tables)."""
    _run_and_check(synth_commits(1, 40, 2048, 4), v, 4)


SORTED, DENSE, TILED = _lib.FLAG_HUNK_SORTED, _lib.FLAG_HUNK_DENSE, _lib.FLAG_HUNK_TILED
FORMS = pytest.mark.parametrize("form", [SORTED, TILED], ids=["sorted", "tiled"])


@FORMS
@pytest.mark.parametrize("v", [1, 2, 4])
@pytest.mark.parametrize("B,ne,nc,seed", SHAPES + [(1, 90, 300, 10), (1, 40, 257, 11)])
def test_hunk_forms_match_oracle(form, v, B, ne, nc, seed):
    """The general path's other two forms of the hunk pair sums against the oracle at every
    tile boundary: sorted thresholds (kw_hunk_sort / _fwd_s / _wsum / _mlpb_s) and the
    one-sweep tiles (kh_tile<0..2> + kw_hunk_fin*: 64-column x 256-row blocks, so Nc = 65,
    257, 300 cross both block edges)."""
    _run_and_check(synth_commits(B, ne, nc, seed), v, seed, GEN, form)


@FORMS
@pytest.mark.parametrize("case", ["empty_adjacency", "full_adjacency", "float_attributes",
                                  "all_lines_one_hunk"])
def test_hunk_forms_edge_cases(form, case):
    """No label pairs, every pair labelled (the correction walk over all Nc - 1 bits, ties
    of equal alpha / beta values across nodes), real-valued attributes."""
    _run_and_check(EDGE[case](synth_commits(2, 70, 13, 7)), 2, 7, GEN, form)
    _run_and_check(EDGE[case](synth_commits(1, 40, 300, 7)), 2, 7, GEN, form)


@FORMS
@pytest.mark.parametrize("nc", [300, 512, 1024])
def test_hunk_forms_equal_dense(form, nc):
    """The forms of the general path agree far inside the oracle tolerance (the default
    picks one by Nc, include/hdgnn.h)."""
    B, ne, v = 1, 64, 2
    cb = synth_commits(B, ne, nc, 21)
    flat = layout.init_flat(4, v)
    outs = []
    for fl in (DENSE, form):
        eng = _engine(B, ne, nc, v, GEN, fl)
        eng.set_params(flat)
        eng.fwd_bwd(eng.upload(cb))
        torch.cuda.synchronize()
        outs.append((eng.logits.cpu().numpy().astype(np.float64),
                     eng.grad.cpu().numpy().astype(np.float64)))
    (l1, g1), (l2, g2) = outs
    scale = np.maximum(1.0, np.abs(l1).max())
    assert np.abs(l1 - l2).max() <= 2e-6 * scale
    np_ = layout.n_params(v)
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        a, r = g2[o:o + n], g1[o:o + n]
        assert np.abs(a - r).max() <= 1e-5 * max(np.abs(r).max(), 1e-12), name
    assert _lib.trailer_count(g1[np_:]) == _lib.trailer_count(g2[np_:])


@FORMS
def test_hunk_forms_deterministic_and_garbage_free(form):
    B, ne, nc, v = 2, 60, 290, 2
    cb = synth_commits(B, ne, nc, 8)
    flat = layout.init_flat(5, v)
    ref = _engine(B, ne, nc, v, GEN, form)
    ref.set_params(flat)
    db = ref.upload(cb)
    ref.fwd_bwd(db)
    g1, p1 = ref.grad.clone(), ref.probs.clone()
    ref.fwd_bwd(db)
    assert torch.equal(g1, ref.grad) and torch.equal(p1, ref.probs)
    dirty = _engine(B, ne, nc, v, GEN, form)
    dirty.set_params(flat)
    dirty.workspace.fill_(float("nan"))
    dirty.grad.fill_(float("inf"))
    dirty.fwd_bwd(dirty.upload(cb))
    torch.cuda.synchronize()
    assert torch.equal(g1, dirty.grad) and torch.equal(p1, dirty.probs)


@pytest.mark.parametrize("nc", [130, 300, 512])
@pytest.mark.parametrize("v", [2, 4])
def test_sorted_all_unit_vs_group_shape(nc, v):
    """The sorted form's two block shapes at an Nc both handle (the all-unit kernels
    kw_hunk_fwd_s / kw_hunk_mlpb_s, the default up to Nc 512, sum a node's label walk in two
    halves: dense + (half 0 + half 1); the group kernels _g, forced by FLAG_HUNK_GROUP, in one
    chain: dense + all).  They differ by fp32 re-association only: logits within 2e-6 of the
    commit's max |logit|, each variable's gradient within 1e-5 of its max |g|, the same
    top_ACC count -- and both match the oracle."""
    B, ne = 2, 64
    cb = synth_commits(B, ne, nc, 31)
    flat = layout.init_flat(6, v)
    outs = []
    for fl in (SORTED, SORTED | _lib.FLAG_HUNK_GROUP):
        eng = _engine(B, ne, nc, v, GEN, fl)
        eng.set_params(flat)
        eng.fwd_bwd(eng.upload(cb))
        torch.cuda.synchronize()
        outs.append((eng.logits.cpu().numpy().astype(np.float64),
                     eng.grad.cpu().numpy().astype(np.float64)))
    (l1, g1), (l2, g2) = outs
    scale = np.maximum(1.0, np.abs(l1).max())
    d = np.abs(l1 - l2).max()
    _errlog.record("logits:all_vs_group", d / scale, d / (2e-6 * scale))
    assert d <= 2e-6 * scale
    np_ = layout.n_params(v)
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        a, r = g2[o:o + n], g1[o:o + n]
        sc = max(np.abs(r).max(), 1e-12)
        e = np.abs(a - r).max()
        _errlog.record("grad_all_vs_group:" + name, e / sc, e / (1e-5 * sc))
        assert e <= 1e-5 * sc, name
    assert _lib.trailer_count(g1[np_:]) == _lib.trailer_count(g2[np_:])
    out, g_ref = _oracle(flat, cb, v)
    _grad_close(g2[:np_] + _reg_grad(flat), g_ref, v)
