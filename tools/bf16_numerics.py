"""What bf16 arithmetic does to the HD-GNN step at the BASELINE shapes (CPU, test
infrastructure; DESIGN.md 8, the bf16 decision for BASELINE configs 3 and 5).

The oracle graph (oracle.model_ref, the reference's op sequence) is evaluated in float64,
float32 and bfloat16 (torch CPU: bf16 storage and bf16-rounded results of every op) at
the untrained initial weights on synthetic commits of each shape, and the logits / CE
are compared with SURVEY 8(d)'s bf16 tolerances (logits atol 5e-2, CE rel 1e-2).
    python tools/bf16_numerics.py [--out profiles/r03/bf16_numerics.json]
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
from oracle import model_ref  # noqa: E402


def run(B, ne, nc, seed, dtype):
    cb = synth_commits(B, ne, nc, seed)
    P = model_ref.to_torch_params(model_ref.unflatten(layout.init_flat(seed).astype(np.float64)),
                                  dtype)
    with torch.no_grad():
        out = model_ref.forward(P, cb.x.astype(np.float64), cb.a, cb.y, cb.hid, cb.nlen, 2, dtype)
    return out["logits"].double().numpy(), float(out["ce"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = []
    for tag, (B, ne, nc) in (("glide (configs 1-2)", (2, 200, 74)),
                             ("step=3 (config 3)", (1, 250, 114))):
        l64, c64 = run(B, ne, nc, 3, torch.float64)
        row = {"shape": tag, "B": B, "ne": ne, "nc": nc, "max_abs_logit": float(np.abs(l64).max())}
        for name, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
            l, c = run(B, ne, nc, 3, dt)
            err = np.abs(l - l64)
            row[name] = {"logits_max_abs_err": float(err.max()),
                         "logits_frac_within_atol_5e-2": float((err <= 5e-2).mean()),
                         "ce_rel_err": abs(c - c64) / abs(c64)}
        res.append(row)
        print(json.dumps(row))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
