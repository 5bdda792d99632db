"""Teacher-forced per-step update check at glide (GPU diagnostic, test infrastructure).

For each of N steps: read the engine's weights and Adam state, run one engine train step,
and predict the same step on the CPU from that exact state (oracle float64 gradient at the
engine's weights + AdamTF with the engine's m, v and beta powers).  Reports per variable
the max |w_engine - w_pred| / lr, i.e. the step's error as a fraction of one Adam step, and
the element-wise relative gradient error where it matters to Adam (|g| > 1e-3 sqrt(v))."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-gnn_amd")]
from hdgnn import _lib, layout  # noqa: E402
from hdgnn.engine import Engine  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402
from oracle import layout as olayout  # noqa: E402
from oracle import model_ref  # noqa: E402

FUSED_STEP = os.environ.get("DIAG_TRAIN_STEP", "1") == "1"


def run(v, path, steps):
    keys = [k for k, _, _ in olayout.keyed_specs(v)]
    cb = synth_commits(2, 200, 74, 21)
    flat = layout.init_flat(21, v)
    eng = Engine(200, 74, 2, variant=v, path=path)
    eng.set_params(flat)
    db = eng.upload(cb)
    rows = []
    theta_f = flat.astype(np.float64)             # the free-running float64 trajectory
    opt_f = model_ref.AdamTF(len(flat))
    for s in range(steps):
        w0 = eng.get_params().astype(np.float64)
        m0 = eng.m.cpu().numpy().astype(np.float64)
        v0 = eng.v.cpu().numpy().astype(np.float64)
        bp = eng.beta_pow.cpu().numpy()
        if FUSED_STEP:               # hdg_train_step: step kernel + fused reduce / Adam
            eng.train_step(db)
            torch.cuda.synchronize()
            g_eng = np.zeros(len(flat))
        else:                        # hdg_fwd_bwd, then hdg_adam_tf
            eng.fwd_bwd(db)
            torch.cuda.synchronize()
            g_eng = eng.grad.cpu().numpy().astype(np.float64)[:len(flat)]
            eng.adam()
            torch.cuda.synchronize()
        w1 = eng.get_params().astype(np.float64)
        params = model_ref.unflatten(w0, v)
        out, gr = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                           cb.nlen, variant=v)
        g_ref = np.concatenate([gr[k].reshape(-1) for k in keys])
        opt = model_ref.AdamTF(len(flat))
        opt.m, opt.v = m0.copy(), v0.copy()
        opt.b1p, opt.b2p = np.float32(bp[0]), np.float32(bp[1])
        wp = opt.step(w0, g_ref)
        # the engine's raw gradient excludes loss_para / loss_map (added in the Adam kernel)
        g_reg = 0.001 * w0
        n = len(w0)
        for off in (n - 4, n - 2):
            th = w0[off:off + 2]
            g_reg[off:off + 2] += 0.001 * th / np.linalg.norm(th)
        ge = g_eng + g_reg
        row = {"step": s + 1}
        for name, (o, shape) in layout.offsets(v).items():
            k = int(np.prod(shape))
            du = np.abs(w1[o:o + k] - wp[o:o + k]) / eng.lr
            gr_ = g_ref[o:o + k]
            gerr = np.abs(ge[o:o + k] - gr_)
            rel = gerr / np.maximum(np.abs(gr_), 1e-30)
            imp = np.abs(gr_) > 1e-3 * np.sqrt(opt.v[o:o + k])
            row[name] = [float(du.max()), float(rel[imp].max()) if imp.any() else 0.0,
                         float(np.abs(gr_).min())]
        pf = model_ref.unflatten(theta_f.astype(np.float32).astype(np.float64), v)
        outf, grf = model_ref.loss_and_grads(pf, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                             cb.nlen, variant=v)
        theta_f = opt_f.step(theta_f, np.concatenate([grf[k].reshape(-1) for k in keys]))
        dfree = np.abs(w1 - theta_f) / eng.lr
        i = int(np.argmax(dfree))
        name_i = [nm for nm, (o, sh) in layout.offsets(v).items() if o <= i < o + int(np.prod(sh))][0]
        row["free"] = [float(dfree.max()), name_i, i, float(g_ref[i]), float(opt.v[i]),
                       float(outf["ce"]), float(out["ce"])]
        print("   free-run max |w - w_f64|/lr %.3g at %s[%d] g %.3g v %.3g  ce_f64 %.9g ce@eng %.9g"
              % tuple([row["free"][0], name_i, i - layout.offsets(v)[name_i][0]] + row["free"][3:]),
              flush=True)
        rows.append(row)
        print("step %d  worst update err/lr: %s" % (s + 1, max(
            ((r[0], k) for k, r in row.items() if k != "step"))), flush=True)
    return rows


if __name__ == "__main__":
    res = {}
    for tag, v, path in (("m2_fused", 2, _lib.PATH_FUSED), ("m4_hybrid", 4, _lib.PATH_FUSED),
                         ("m4_general", 4, _lib.PATH_GENERAL)):
        print(tag, flush=True)
        res[tag] = run(v, path, int(sys.argv[1]) if len(sys.argv) > 1 else 6)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "teacher.json"), "w") as f:
        json.dump(res, f)
