"""How far an fp32 evaluation of the reference graph drifts from float64 over a TF-Adam
trajectory (CPU, test infrastructure): oracle.model_ref in float32 with float32 weights and
Adam slots (what TF1 does: fp32 variables, fp32 ApplyAdam) vs float64 from the same initial
weights, each with its own AdamTF.  The drift bounds what any fp32 implementation
(TF itself included) can promise for 50-step weights and losses; tests/test_trajectory_gpu
measures the engine against the same float64 trajectory.

    python tools/traj_floor.py [--variant 2] [--steps 50]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-gnn_amd")]

from hdgnn import layout  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402
from oracle import layout as olayout  # noqa: E402
from oracle import model_ref  # noqa: E402


def trajectory(flat, cb, v, steps, dtype, f32_state=False):
    """f32_state: keep the weights and Adam slots in float32 between steps, as TF's
    variables and ApplyAdam (and the engine) do; else float64 master copies."""
    keys = [k for k, _, _ in olayout.keyed_specs(v)]
    theta = flat.astype(np.float64)
    opt = model_ref.AdamTF(len(flat))
    losses = []
    for _ in range(steps):
        params = model_ref.unflatten(theta.astype(np.float32).astype(np.float64), v)
        out, g = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                          cb.nlen, variant=v, dtype=dtype)
        losses.append([float(out[k]) for k in ("ce", "loss_map", "loss_para", "total")])
        theta = opt.step(theta, np.concatenate([g[k].reshape(-1) for k in keys]).astype(np.float64))
        if f32_state:
            theta = theta.astype(np.float32).astype(np.float64)
            opt.m = opt.m.astype(np.float32).astype(np.float64)
            opt.v = opt.v.astype(np.float32).astype(np.float64)
    return theta, np.asarray(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=2)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--seed", type=int, default=21)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    v = a.variant
    cb = synth_commits(2, 200, 74, a.seed)
    flat = layout.init_flat(a.seed, v)
    w64, l64 = trajectory(flat, cb, v, a.steps, torch.float64)
    w32, l32 = trajectory(flat, cb, v, a.steps, torch.float32, f32_state=True)
    lrel = np.abs(l32 - l64) / np.abs(l64)
    err = np.abs(w32 - w64)
    atol = 1e-3 * 3e-4 * a.steps      # tests/test_trajectory_gpu.py: 1e-3 |w| + 1e-3 lr steps
    per = {}
    for name, (o, shape) in layout.offsets(v).items():
        n = int(np.prod(shape))
        e, r = err[o:o + n], w64[o:o + n]
        per[name] = {"max_err": float(e.max()), "max_abs_w": float(np.abs(r).max()),
                     "max_err_over_tol": float((e / (1e-3 * np.abs(r) + atol)).max())}
    res = {"variant": v, "steps": a.steps, "shape": "B=2 Ne=200 Nc=74 seed %d" % a.seed,
           "loss_rel_max_per_step": lrel.max(1).tolist(),
           "weights_max_err": float(err.max()),
           "weights_max_err_over_tol": float((err / (1e-3 * np.abs(w64) + atol)).max()),
           "tolerance": "1e-3 |w_ref| + 1e-3 lr steps (tests/test_trajectory_gpu.py)",
           "per_variable": per}
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(json.dumps({k: res[k] for k in ("weights_max_err", "weights_max_err_over_tol")}))
    print("loss rel per step:", " ".join("%.1e" % x for x in lrel.max(1)))


if __name__ == "__main__":
    main()
