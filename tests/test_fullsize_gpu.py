"""Full-size checks of every BASELINE workload's bench batch,
where co-residency, grid-size and tile-count bugs would show: the exact grids bench.py
launches, checked through size-independent properties plus the oracle on a few commits.

Per workload (variant x Ne x Nc x batch per GPU, the engine path bench.py picks):
  * probabilities normalised (softmax over the two classes) to 1e-6;
  * CE (stats[0]) equals mean -log p_label computed from the returned logits (rel 1e-5);
  * the first three commits' logits / probs vs the float64 oracle, forward of those
    commits alone (the forward is per commit), test_general_gpu.py's tolerances;
  * bitwise determinism of fwd_bwd (gradient and probabilities) on the full grid;
  * the data-parallel decomposition at full size: the two halves of the batch, each with
    the CE normalised by the whole batch, sum to the full batch's gradient (8e-5 |g| +
    8e-6 max|g| per variable: fp32 reduction order differs between the grids);
  * the full batch's gradient against the float64 oracle's, the oracle run over chunks of
    commits (its CE mean re-weighted by chunk / B and summed: the DP decomposition of
    tests/test_dp.py) at test_gpu_parity.py's gradient tolerances, and one TF-Adam step's
    weights at atol 2e-6 -- the whole grid the bench launches (split mode, 2B blocks, every
    block-pair exchange and the 2B-row reduction), not a few commits.
Reference shapes: main.py:11-15 (steps 2 / 3 / 5), SURVEY 8(d) stress; gradient and
update: model_2.py:115-130, 336-338.
"""
import numpy as np
import pytest
import torch

from hdgnn import _lib, layout
from hdgnn.data import pair_index
from hdgnn.synth import synth_commits
from oracle import model_ref
from tests import _errlog
from tests.test_general_gpu import _check_outputs, _oracle, _reg_grad

GRAD_RTOL, GRAD_ATOL = 1.5e-4, 3e-6      # test_gpu_parity.py: x |ref|, x max|ref| per variable


def oracle_batch_grad(flat, cb, v, chunk):
    """The float64 oracle's gradient of the whole batch's train_loss (model_2.py:336),
    computed over chunks of `chunk` commits: each chunk's data gradient (its gradient minus
    the parameter-only loss_para / loss_map terms) weighted by its share of the batch, plus
    those terms once.  Returns (gradient, CE of the batch)."""
    B = cb.B
    reg = _reg_grad(flat)
    g, ce = np.zeros(len(flat)), 0.0
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        out, gc = _oracle(flat, cb.slice(lo, hi), v)
        g += (gc - reg) * ((hi - lo) / B)
        ce += float(out["ce"]) * ((hi - lo) / B)
    return g + reg, ce


def grad_close(g_eng, g_ref, v, what):
    bad = []
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        a, r = g_eng[o:o + n], g_ref[o:o + n]
        scale = max(np.abs(r).max(), 1e-12)
        tol = GRAD_RTOL * np.abs(r) + GRAD_ATOL * scale + 1e-9
        err = np.abs(a - r)
        _errlog.record("%s:%s" % (what, name), err.max() / scale, (err / tol).max())
        if not np.all(err <= tol):
            bad.append("%s: max err %.3g, scale %.3g, %d/%d bad" % (
                name, np.nanmax(err) if np.isfinite(err).any() else np.nan, scale,
                int((~(err <= tol)).sum()), n))
    assert not bad, "%s mismatch:\n  " % what + "\n  ".join(bad)


def check_full_batch_vs_oracle(eng, db, cb, flat, v, chunk=10):
    """eng (parameters = flat) on the full batch: fwd_bwd's gradient and one training step's
    weights against the oracle.  Leaves eng's parameters updated by one step."""
    B, nc = cb.B, cb.Nc
    eng.set_params(flat)
    eng.fwd_bwd(db)
    torch.cuda.synchronize()
    eng.check_status()
    g = eng.grad.cpu().numpy().astype(np.float64)
    P = len(flat)
    g_ref, ce_ref = oracle_batch_grad(flat, cb, v, chunk)
    grad_close(g[:P] + _reg_grad(flat), g_ref, v, "fullgrad")
    np.testing.assert_allclose(g[P] / (B * nc * (nc - 1)), ce_ref, rtol=1e-5)
    eng.set_params(flat)                      # Adam moments and beta powers reset too
    eng.train_step(db)
    torch.cuda.synchronize()
    eng.check_status()
    want = model_ref.AdamTF(P).step(flat.astype(np.float64), g_ref)
    err = np.abs(eng.get_params() - want)
    _errlog.record("weights@1:full", err.max(), err.max() / 2e-6)
    np.testing.assert_allclose(eng.get_params(), want, rtol=0, atol=2e-6)
    np.testing.assert_allclose(eng.stats[0].item(), ce_ref, rtol=1e-5)

pytestmark = pytest.mark.gpu

WORKLOADS = [
    # (variant, Ne, Nc, batch per GPU, expected path)
    (4, 200, 74, 100, _lib.PATH_FUSED),       # glide, full HD-GNN (model_2 is in test_gpu_parity)
    (2, 250, 114, 100, _lib.PATH_FUSED),      # config 3 shapes
    (4, 250, 114, 100, _lib.PATH_FUSED),
    (2, 250, 150, 100, _lib.PATH_FUSED),      # config 4, one GPU's shard
    (4, 250, 150, 100, _lib.PATH_FUSED),
    (2, 1024, 512, 32, _lib.PATH_GENERAL),    # config 5 (stress), one GPU's shard
    (4, 1024, 512, 32, _lib.PATH_GENERAL),
]


def _ids(w):
    return "m%d_%dx%d_B%d" % w[:4]


@pytest.mark.parametrize("w", WORKLOADS, ids=_ids)
def test_full_size_workload(w):
    from hdgnn.engine import Engine
    v, ne, nc, B, path = w
    cb = synth_commits(B, ne, nc, 20250301 + ne + nc)
    flat = layout.init_flat(1, v)
    eng = Engine(ne, nc, B, variant=v)
    assert eng.path == path
    if path == _lib.PATH_FUSED:
        assert eng.split                      # 2B <= CUs: the bench's split mode
    eng.set_params(flat)
    db = eng.upload(cb)
    eng.train_step(db, logits=True)
    torch.cuda.synchronize()
    eng.check_status()
    probs = eng.probs.cpu().numpy()
    logits = eng.logits.cpu().numpy().astype(np.float64)
    assert np.isfinite(logits).all()
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-6)
    I, J = pair_index(nc)
    lab = cb.y[:, I, J]
    lse = np.logaddexp(logits[:, 0], logits[:, 1])
    ce = (lse - np.where(lab == 1, logits[:, 1], logits[:, 0])).mean()
    np.testing.assert_allclose(eng.stats[0].item(), ce, rtol=1e-5)
    out, _ = _oracle(flat, cb.slice(0, 3), v)
    _check_outputs(eng.logits.cpu().numpy()[:3], probs[:3], out)

    # bitwise determinism of the full grid (parameters reset: train_step updated them)
    eng.set_params(flat)
    eng.fwd_bwd(db)
    g1, p1 = eng.grad.clone(), eng.probs.clone()
    eng.fwd_bwd(db)
    torch.cuda.synchronize()
    assert torch.equal(g1, eng.grad) and torch.equal(p1, eng.probs)

    # the batch's two halves (CE normalised by the whole batch) sum to its gradient
    h = B // 2
    gsum = np.zeros(eng.glen, np.float64)
    for lo, hi in ((0, h), (h, B)):
        e = Engine(ne, nc, hi - lo, variant=v, batch_global=B)
        e.set_params(flat)
        e.fwd_bwd(e.upload(cb.slice(lo, hi)))
        torch.cuda.synchronize()
        e.check_status()
        gsum += e.grad.cpu().numpy().astype(np.float64)
    g = g1.cpu().numpy().astype(np.float64)
    P = len(flat)
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        a, r = gsum[o:o + n], g[o:o + n]
        tol = 8e-5 * np.abs(r) + 8e-6 * max(np.abs(r).max(), 1e-12) + 1e-9
        assert np.all(np.abs(a - r) <= tol), "%s: max err %.3g" % (name, np.abs(a - r).max())
    np.testing.assert_allclose(gsum[P], g[P], rtol=1e-5)          # CE sum trailer

    # the full grid's gradient and one TF-Adam step against the float64 oracle
    check_full_batch_vs_oracle(eng, db, cb, flat, v, chunk=10 if ne <= 256 else 4)
