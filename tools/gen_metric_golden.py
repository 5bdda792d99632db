"""Generate tests/golden/metrics_tiny.{npz,json} by running the REFERENCE metrics.

Imports /root/reference/EvaluationFuncs.py (numpy / scipy / sklearn only, importable
here) and evaluates top_ACC, prec, recall, f1, AUC unmodified on seeded random inputs
shaped like model_2's outputs (B, 2, Ncr).  Graph 1 has a single label class so AUC's
skip path runs; the last graph has both (AUC divides by the count of the last graph).
Only the arrays and the resulting numbers are committed.

Run from the repo root:  python tools/gen_metric_golden.py
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"


def main():
    sys.path.insert(0, REF)
    import EvaluationFuncs as ef
    rng = np.random.default_rng(20250301)
    B, R = 5, 42
    lab = (rng.random((B, R)) < 0.3).astype(np.float32)
    lab[1] = 0.0
    label = np.stack([1 - lab, lab], 1)                          # one-hot over Dr=2
    p1 = rng.random((B, R)).astype(np.float32)
    p1[2, :5] = 0.5                                              # argmax ties
    probs = np.stack([1 - p1, p1], 1)
    out = {}
    for name in ("top_ACC", "prec", "recall", "f1", "AUC"):
        out[name] = float(getattr(ef, name)(label.copy(), probs.copy()))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gdir = os.path.join(root, "tests", "golden")
    np.savez(os.path.join(gdir, "metrics_tiny.npz"), label=label, probs=probs)
    with open(os.path.join(gdir, "metrics_tiny.json"), "w") as f:
        json.dump({"values": out, "generator": "tools/gen_metric_golden.py",
                   "reference": "EvaluationFuncs.py @ fanmengdan/HD-GNN 2025-03-01"}, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
