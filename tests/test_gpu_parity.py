"""HIP engine (via the C ABI) vs the CPU oracle.  Runs on the MI355X box only.

Tolerances (fp32 engine vs float64 oracle; SURVEY 8(d) made scale-aware):
  Set at about 4-6x the worst error any case here reached (profiles/r03/parity_summary.txt):
  logits   |d| <= 1.5e-5 |ref| + 1.5e-6 * max(1, max_commit |ref|)   -- untrained random-init
           logits reach |z| ~ 3e3 at glide sizes, where a fixed 1e-5 is below fp32 resolution
           (worst 7.9e-7 max|ref|)
  probs    == softmax(engine logits) to 1e-6, and vs oracle |d| <= 0.5 * logit tolerance
  CE, loss_map, loss_para, train_loss: rel 1e-5
  gradients rtol 1.5e-4, atol 3e-6 * max|ref| of the variable (SURVEY 8(d) says atol 1e-6;
           the scale-relative form because the variables' gradients span 1e-4 .. 1e1.
           Achieved: <= 2.9e-6 * max|ref| over every case here)
  weights after TF-Adam steps: atol 2e-6 (lr 3e-4 per step)
"""
import numpy as np
import pytest
import torch

from hdgnn import layout
from hdgnn.data import CommitBatch
from hdgnn.synth import synth_commits
from oracle import model_ref
from tests import _errlog

pytestmark = pytest.mark.gpu

KEYS = [k for k, _, _ in __import__("oracle.layout", fromlist=["keyed_specs"]).keyed_specs(2)]


@pytest.fixture(params=["1", "0"], ids=["split", "one_block"])
def split_mode(request, monkeypatch):
    """HDG_FUSED_SPLIT: "1" two blocks per commit (hunk rows split by parity, block-pair
    exchanges; the default whenever 2 B <= CUs), "0" one block per commit."""
    monkeypatch.setenv("HDG_FUSED_SPLIT", request.param)
    return request.param


def _engine(B, ne, nc):
    from hdgnn.engine import Engine
    return Engine(ne, nc, B)


def _oracle(params_flat, cb, steps=0):
    params = model_ref.unflatten(params_flat.astype(np.float64))
    out, grads = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y,
                                          cb.hid, cb.nlen)
    return out, np.concatenate([grads[k].reshape(-1) for k in KEYS])


def _reg_grad(flat):
    g = 0.001 * flat.astype(np.float64)
    for off in (2123, 2125):
        th = flat[off:off + 2].astype(np.float64)
        g[off:off + 2] += 0.001 * th / np.linalg.norm(th)
    return g


def _logit_tol(ref):
    scale = np.maximum(1.0, np.abs(ref).reshape(ref.shape[0], -1).max(1))[:, None, None]
    return 1.5e-5 * np.abs(ref) + 1.5e-6 * scale


def _check_outputs(logits, probs, out):
    ref_l = out["logits"].transpose(0, 2, 1)            # (B, 2, Pc) like TF
    tol = _logit_tol(ref_l)
    err = np.abs(logits - ref_l)
    scale = np.maximum(1.0, np.abs(ref_l).reshape(ref_l.shape[0], -1).max(1))[:, None, None]
    _errlog.record("logits", (err / scale).max(), (err / tol).max())
    assert np.all(err <= tol), "logits: max err %.3g (tol %.3g)" % (err.max(), tol[err > tol].min())
    sm = np.exp(logits - logits.max(1, keepdims=True))
    sm /= sm.sum(1, keepdims=True)
    np.testing.assert_allclose(probs, sm, atol=1e-6)
    ref_p = out["probs"].transpose(0, 2, 1)
    perr = np.abs(probs - ref_p)
    assert np.all(perr <= 0.5 * tol + 1e-6), "probs: max err %.3g" % perr.max()


def _grad_close(g_eng, g_ref, rtol=1.5e-4, atol_rel=3e-6):
    bad = []
    for name, (o, shape) in layout.offsets(2).items():
        n = int(np.prod(shape))
        a, r = g_eng[o:o + n], g_ref[o:o + n]
        scale = max(np.abs(r).max(), 1e-12)
        tol = rtol * np.abs(r) + atol_rel * scale + 1e-9
        err = np.abs(a - r)
        _errlog.record("grad:" + name, err.max() / scale, (err / tol).max())
        if not np.all(err <= tol):       # NaN fails too
            bad.append("%s: max err %.3g, scale %.3g, %d/%d bad" % (
                name, np.nanmax(err) if np.isfinite(err).any() else np.nan, scale,
                int((~(err <= tol)).sum()), n))
    assert not bad, "gradient mismatch:\n  " + "\n  ".join(bad)


CASES = [
    # (B, Ne, Nc, seed) -- tiny, ragged (not multiples of 16/32), glide-shaped
    (3, 7, 5, 0),
    (4, 37, 19, 1),
    (2, 200, 74, 2),
    (1, 33, 17, 3),
    (2, 250, 150, 4),     # s5 shapes (BASELINE config 4), largest hunk tile
    (1, 256, 160, 5),     # engine limits
]


@pytest.mark.parametrize("B,ne,nc,seed", CASES)
def test_forward_matches_oracle(B, ne, nc, seed, split_mode):
    cb = synth_commits(B, ne, nc, seed)
    flat = layout.init_flat(seed)
    eng = _engine(B, ne, nc)
    eng.set_params(flat)
    probs, logits, ce_sum = eng.forward(cb.to_device())
    torch.cuda.synchronize()
    out, _ = _oracle(flat, cb)
    _check_outputs(logits.cpu().numpy(), probs.cpu().numpy(), out)
    ce = ce_sum.item() / (B * nc * (nc - 1))
    np.testing.assert_allclose(ce, float(out["ce"]), rtol=1e-5)
    # loss_E_HR (model_2.py:122) of the forward launch; sums of squares in f64
    np.testing.assert_allclose(eng.ehr.item(), float(out["loss_E_HR"]), rtol=1e-4)


@pytest.mark.parametrize("B,ne,nc,seed", CASES)
def test_gradients_match_oracle(B, ne, nc, seed, split_mode):
    cb = synth_commits(B, ne, nc, seed)
    flat = layout.init_flat(seed + 10)
    eng = _engine(B, ne, nc)
    eng.set_params(flat)
    eng.fwd_bwd(cb.to_device())
    torch.cuda.synchronize()
    g = eng.grad.cpu().numpy().astype(np.float64)
    out, g_ref = _oracle(flat, cb)
    g_eng = g[:2127] + _reg_grad(flat)
    _grad_close(g_eng, g_ref)
    np.testing.assert_allclose(g[2127] / (B * nc * (nc - 1)), float(out["ce"]), rtol=1e-5)


def test_train_steps_match_oracle_adam():
    B, ne, nc, seed = 3, 23, 11, 5
    cb = synth_commits(B, ne, nc, seed)
    flat = layout.init_flat(seed)
    eng = _engine(B, ne, nc)
    eng.set_params(flat)
    db = cb.to_device()
    theta = flat.astype(np.float64)
    opt = model_ref.AdamTF(2127)
    for step in range(3):
        eng.train_step(db)
        torch.cuda.synchronize()
        out, g_ref = _oracle(theta.astype(np.float32), cb)
        stats = eng.stats.cpu().numpy()
        np.testing.assert_allclose(stats[0], float(out["ce"]), rtol=1e-5)
        np.testing.assert_allclose(stats[1], float(out["loss_map"]), rtol=1e-5)
        np.testing.assert_allclose(stats[2], float(out["loss_para"]), rtol=1e-5)
        np.testing.assert_allclose(stats[3], float(out["total"]), rtol=1e-5)
        theta = opt.step(theta, g_ref)
        np.testing.assert_allclose(eng.get_params(), theta, rtol=0, atol=2e-6)


EDGE = {
    "empty_adjacency": lambda cb: CommitBatch(cb.x, 0 * cb.a, 0 * cb.y, cb.hid, cb.nlen),
    "full_adjacency": lambda cb: CommitBatch(cb.x, 1 - np.eye(cb.Ne, dtype=np.uint8)[None] + 0 * cb.a,
                                             1 - np.eye(cb.Nc, dtype=np.uint8)[None] + 0 * cb.y,
                                             cb.hid, cb.nlen),
    "no_index_lines": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid * 0 - 1, cb.nlen * 0),
    "one_index_line": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid, cb.nlen * 0 + 1),
    "all_lines_one_hunk": lambda cb: CommitBatch(cb.x, cb.a, cb.y, cb.hid * 0, cb.nlen * 0 + cb.Ne),
    "zero_attributes": lambda cb: CommitBatch(cb.x * 0, cb.a, cb.y, cb.hid, cb.nlen),
    # real-valued, signed, all-distinct attributes (the sorted-x entity sums see nd = Ne)
    "float_attributes": lambda cb: CommitBatch(
        (np.random.default_rng(3).standard_normal(cb.x.shape) * 4).astype(np.float32),
        cb.a, cb.y, cb.hid, cb.nlen),
    "dense_entity_rows": lambda cb: CommitBatch(
        cb.x, ((np.random.default_rng(4).random(cb.a.shape) < 0.6)
               & ~np.eye(cb.Ne, dtype=bool)[None]).astype(np.uint8), cb.y, cb.hid, cb.nlen),
}


@pytest.mark.parametrize("case", sorted(EDGE))
def test_edge_cases(case, split_mode):
    B, ne, nc, seed = 2, 21, 9, 7
    cb = EDGE[case](synth_commits(B, ne, nc, seed))
    flat = layout.init_flat(seed)
    eng = _engine(B, ne, nc)
    eng.set_params(flat)
    eng.fwd_bwd(cb.to_device())
    torch.cuda.synchronize()
    out, g_ref = _oracle(flat, cb)
    _check_outputs(eng.logits.cpu().numpy(), eng.probs.cpu().numpy(), out)
    _grad_close(eng.grad.cpu().numpy()[:2127].astype(np.float64) + _reg_grad(flat), g_ref)


def test_deterministic_bitwise():
    B, ne, nc = 8, 200, 74
    cb = synth_commits(B, ne, nc, 11)
    eng = _engine(B, ne, nc)
    eng.set_params(layout.init_flat(1))
    db = cb.to_device()
    eng.fwd_bwd(db)
    g1 = eng.grad.clone()
    p1 = eng.probs.clone()
    eng.fwd_bwd(db)
    assert torch.equal(g1, eng.grad) and torch.equal(p1, eng.probs)


def test_full_size_properties():
    """BASELINE config 2 (glide, B=100, the bench's split grid of 200 blocks): probabilities
    normalised, CE equals the mean -log p_label of the returned probabilities, a few
    commits' outputs match the oracle, and the full batch's gradient and one TF-Adam step
    match the oracle's (summed over chunks of 10 commits; tests/test_fullsize_gpu.py)."""
    B, ne, nc = 100, 200, 74
    cb = synth_commits(B, ne, nc, 20250301)
    eng = _engine(B, ne, nc)
    flat = layout.init_flat(0)
    eng.set_params(flat)
    eng.train_step(cb.to_device(), logits=True)
    torch.cuda.synchronize()
    probs = eng.probs.cpu().numpy()
    logits = eng.logits.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-6)
    from hdgnn.data import pair_index
    I, J = pair_index(nc)
    lab = cb.y[:, I, J]
    lse = np.logaddexp(logits[:, 0], logits[:, 1])         # CE from the returned logits
    ce = (lse - np.where(lab == 1, logits[:, 1], logits[:, 0])).mean()
    np.testing.assert_allclose(eng.stats[0].item(), ce, rtol=1e-5)
    sub = cb.slice(0, 3)
    out, _ = _oracle(flat, sub)
    _check_outputs(eng.logits.cpu().numpy()[:3], probs[:3], out)
    from tests.test_fullsize_gpu import check_full_batch_vs_oracle
    assert eng.split                           # 2B <= CUs: the bench's grid
    check_full_batch_vs_oracle(eng, cb.to_device(), cb, flat, 2)


def test_shape_errors_are_reported():
    from hdgnn import _lib
    from hdgnn.engine import Engine
    with pytest.raises(ValueError):
        Engine(300, 74, 4, path=_lib.PATH_FUSED)    # ne > 256 on the fused kernel
    with pytest.raises(ValueError):
        Engine(5000, 74, 4)                          # beyond every path


def test_graph_replay_equals_eager():
    B, ne, nc = 6, 50, 30
    cb = synth_commits(B, ne, nc, 4)
    flat = layout.init_flat(3)
    e1, e2 = _engine(B, ne, nc), _engine(B, ne, nc)
    e1.set_params(flat)
    e2.set_params(flat)
    db = cb.to_device()
    e2.capture(db)
    for _ in range(3):
        e1.train_step(db)
        e2.replay()
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.stats, e2.stats)
    assert torch.equal(e1.probs, e2.probs)


def test_multi_step_graph_equals_eager():
    """bench.py captures several training steps per HIP graph: one replay of a 3-step
    graph == 3 eager steps, bitwise (params, Adam state, last step's outputs)."""
    B, ne, nc = 6, 50, 30
    cb = synth_commits(B, ne, nc, 5)
    flat = layout.init_flat(4)
    e1, e2 = _engine(B, ne, nc), _engine(B, ne, nc)
    e1.set_params(flat)
    e2.set_params(flat)
    db = cb.to_device()
    e2.capture(db, steps=3)
    for _ in range(2):
        for _ in range(3):
            e1.train_step(db)
        e2.replay()
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.m, e2.m)
    assert torch.equal(e1.v, e2.v) and torch.equal(e1.beta_pow, e2.beta_pow)
    assert torch.equal(e1.stats, e2.stats) and torch.equal(e1.probs, e2.probs)
