"""50-step TF-Adam trajectories at the glide shape vs the CPU oracle.  GPU only.

SURVEY 8(d): "weights after 50 steps: rtol 1e-3".  The engine trains B=2 glide commits
(Ne=200, Nc=74, the BASELINE config-1 shape) for 50 steps of hdg_train_step (step
kernel + fused reduce / TF Adam, model_2.py:336-338, 369-383).  Two checks per path:

1. Every step, teacher-forced.  Before each engine step the test reads the engine's
   weights, Adam slots and beta powers; the oracle predicts that step from exactly that
   state (oracle.model_ref.loss_and_grads in float64 + AdamTF, the restated ApplyAdam).
   After the step:  |w - w_pred| <= 3e-4 lr + 2 ulp(w)   (a 3000th of one Adam step,
   plus the float32 rounding of the stored weight), and the pre-update losses rel 3e-5
   (CE falls from ~100 to ~3 while the logits stay ~1e3: the loss loses relative digits
   as training proceeds).  Achieved: <= 1.3e-4 lr and 8.9e-6 over all 50 steps.
2. Free-running.  The oracle runs its own 50-step float64 trajectory from the same
   initial weights (evaluated at float32-rounded weights); the engine's weights after 50
   steps:  |w - w_ref| <= 1e-3 |w_ref| + 1e-3 lr 50   (rtol 1e-3 of the weight, or of the
   largest displacement 50 Adam steps can make), per-step losses rel 1e-2.

   model_4 is held to "within 2 lr" and losses rel 3e-2 instead: its gradient is discontinuous (relu units
   and the hunk MLP hinge), and at step 7 of this trajectory one float32 rounding-level
   difference puts an element of phi_U_O1/o1_w1o on the other side of a kink; its Adam
   momentum then differs by O(lr) for the rest of the run (tools/diag_teacher.py: the
   step-8 gradient of element 125 is 6.2 on one trajectory and 2.6e-5 on the other).
   Each step is still exact to check 1; a float64 trajectory perturbed by 1e-7 relative
   does not cross it (tools/traj_floor.py, profiles/r03/traj_floor_m4.json).
Paths: model_2 fused (split), model_2 general, model_4 hybrid (fused step kernel +
general-path entity-edge stage).  Achieved errors go to the parity report
(tests/_errlog.py, HDG_PARITY_REPORT) and DESIGN.md 6.
"""
import os

import numpy as np
import pytest
import torch

from hdgnn import _lib, layout
from hdgnn.synth import synth_commits
from oracle import layout as olayout
from oracle import model_ref
from tests import _errlog

pytestmark = pytest.mark.gpu

STEPS = 50
B, NE, NC, SEED = 2, 200, 74, 21
LOSSES = ("ce", "loss_map", "loss_para", "total")


def _oracle(theta, cb, v, keys):
    params = model_ref.unflatten(np.asarray(theta, np.float64), v)
    out, grads = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                          cb.nlen, variant=v)
    return out, np.concatenate([grads[k].reshape(-1) for k in keys])


def _count(r):
    return int(round(r[4])) + (int(round(r[5])) << 16) + (int(round(r[6])) << 32)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("v,path", [(2, _lib.PATH_FUSED), (4, _lib.PATH_FUSED),
                                    (2, _lib.PATH_GENERAL)],
                         ids=["model2_fused", "model4_hybrid", "model2_general"])
def test_adam_trajectory_50_steps(v, path):
    from hdgnn import metrics
    from hdgnn.data import onehot_relations
    from hdgnn.engine import Engine
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    keys = [k for k, _, _ in olayout.keyed_specs(v)]
    cb = synth_commits(B, NE, NC, SEED)
    flat = layout.init_flat(SEED, v)
    eng = Engine(NE, NC, B, variant=v, path=path)
    assert eng.path == path
    eng.set_params(flat)
    db = eng.upload(cb)
    rel = onehot_relations(cb.y)
    lr = eng.lr

    theta_f = flat.astype(np.float64)            # free-running float64 trajectory
    opt_f = model_ref.AdamTF(len(flat))
    step_err, loss_tf, loss_free, cnt_bad = [], [], [], []
    for s in range(STEPS):
        w0 = eng.get_params().astype(np.float64)
        m0 = eng.m.cpu().numpy().astype(np.float64)
        v0 = eng.v.cpu().numpy().astype(np.float64)
        bp = eng.beta_pow.cpu().numpy()
        eng.train_step(db)
        torch.cuda.synchronize()
        w1 = eng.get_params().astype(np.float64)
        st = eng.stats.cpu().numpy().astype(np.float64)
        assert st[7] == 0                                 # no faulted step
        # 1. teacher-forced prediction of this step
        out, g = _oracle(w0, cb, v, keys)
        opt = model_ref.AdamTF(len(flat))
        opt.m, opt.v = m0, v0
        opt.b1p, opt.b2p = np.float32(bp[0]), np.float32(bp[1])
        wp = opt.step(w0, g)
        ulp = np.spacing(np.abs(wp).astype(np.float32)).astype(np.float64)
        step_err.append(float((np.abs(w1 - wp) / (3e-4 * lr + 2 * ulp)).max()))
        ref = np.array([float(out[k]) for k in LOSSES])
        loss_tf.append(np.abs(st[:4] - ref) / np.abs(ref))
        # the count may differ only on pairs whose logit difference is within the logit
        # tolerance of a tie (1e-5 of the commit's largest |logit|, tests/test_gpu_parity)
        p = out["probs"].transpose(0, 2, 1)
        z = out["logits"]
        scale = np.abs(z).reshape(B, -1).max(1)[:, None]
        nnear = int((np.abs(z[..., 1] - z[..., 0]) < 1e-5 * scale).sum())
        cnt_bad.append(abs(_count(st) - metrics.top_acc_count(rel, p)) > nnear)
        # 2. free-running float64 trajectory
        outf, gf = _oracle(theta_f.astype(np.float32), cb, v, keys)
        reff = np.array([float(outf[k]) for k in LOSSES])
        loss_free.append(np.abs(st[:4] - reff) / np.abs(reff))
        theta_f = opt_f.step(theta_f, gf)
    w_eng = eng.get_params().astype(np.float64)
    loss_tf, loss_free = np.asarray(loss_tf), np.asarray(loss_free)

    _errlog.record("teacher_step_update", max(step_err) * 3e-4, max(step_err),
                   note="err_over_scale in units of lr")
    ltol = 3e-2 if v == 4 else 1e-2
    _errlog.record("teacher_losses", loss_tf.max(), loss_tf.max() / 3e-5)
    _errlog.record("free_losses@1..50", loss_free.max(), loss_free.max() / ltol,
                   per_step=[float(x) for x in loss_free.max(1)])
    err = np.abs(w_eng - theta_f)
    tol = 1e-3 * np.abs(theta_f) + 1e-3 * lr * STEPS
    worst = []
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        e, r = err[o:o + n], theta_f[o:o + n]
        _errlog.record("free_weights@50:" + name, e.max() / max(np.abs(r).max(), 1e-12),
                       e.max() / (2 * lr) if v == 4 else (e / tol[o:o + n]).max(),
                       err_over_lr=float(e.max() / lr))
        if not np.all(e <= tol[o:o + n]):
            worst.append("%s: max err %.3g = %.3g lr (|w| %.3g)" % (
                name, e.max(), e.max() / lr, np.abs(r).max()))
    moved = np.abs(theta_f - flat.astype(np.float64)).max()
    _errlog.record("free_weights@50", err.max() / np.abs(theta_f).max(),
                   err.max() / (2 * lr) if v == 4 else (err / tol).max(),
                   err_over_lr=float(err.max() / lr), max_displacement=float(moved),
                   tolerance="2 lr" if v == 4 else "1e-3 |w| + 1e-3 lr steps")

    assert moved > 1e-3                                   # the weights did train
    assert max(step_err) <= 1.0, "teacher-forced step error %.3g x (3e-4 lr + 2 ulp)" % max(step_err)
    assert np.all(loss_tf <= 3e-5), "teacher-forced losses: max rel err %.3g" % loss_tf.max()
    assert not any(cnt_bad), "top_ACC counts differ on %d steps" % sum(cnt_bad)
    assert np.all(loss_free <= ltol), "free-run losses: max rel err %.3g" % loss_free.max()
    if v == 4:
        assert err.max() <= 2 * lr, "free-run weights: %.3g lr" % (err.max() / lr)
    else:
        assert not worst, "free-run weights after %d steps:\n  %s" % (STEPS, "\n  ".join(worst))
