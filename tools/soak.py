"""GPU box: long-run check of the split-mode step (two co-resident blocks per commit trading
partial sums through tagged words): N training steps as HIP-graph replays at the bench
workload, twice from the same initial state in fresh engines.  Reports whether any launch
set the sticky status word (an exchange timeout), whether the final losses are finite,
and whether the two runs end bitwise equal (parameters and Adam state).

  python tools/soak.py [--variant 2] [--steps 20000] [--out gpurun_out/soak.json]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-gnn_amd")]


def run(variant, ne, nc, batch, steps, gsteps):
    import torch
    from hdgnn import layout
    from hdgnn.engine import Engine
    from hdgnn.synth import synth_commits
    eng = Engine(ne, nc, batch, variant=variant)
    eng.set_params(layout.init_flat(0, variant))
    db = eng.upload(synth_commits(batch, ne, nc, 1))
    eng.capture(db, steps=gsteps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // gsteps):
        eng.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.state.cpu().numpy()
    return {"split": bool(eng.split), "path": int(eng.path), "status": int(eng.status.item()),
            "loss": float(eng.stats[3].item()), "fault_slot": float(eng.stats[7].item()),
            "state_sha256": hashlib.sha256(st.tobytes()).hexdigest(),
            "finite": bool(torch.isfinite(eng.state).all().item()),
            "seconds": dt, "ms_per_step": 1e3 * dt / steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=2)
    ap.add_argument("--ne", type=int, default=200)
    ap.add_argument("--nc", type=int, default=74)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--graph-steps", type=int, default=50)
    ap.add_argument("--out", default="gpurun_out/soak.json")
    a = ap.parse_args()
    runs = [run(a.variant, a.ne, a.nc, a.batch, a.steps, a.graph_steps) for _ in range(2)]
    res = {"variant": a.variant, "ne": a.ne, "nc": a.nc, "batch": a.batch, "steps": a.steps,
           "runs": runs,
           "no_fault": all(r["status"] == 0 and r["fault_slot"] == 0.0 for r in runs),
           "bitwise_equal": runs[0]["state_sha256"] == runs[1]["state_sha256"]}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "a") as f:
        f.write(json.dumps(res) + "\n")
    print(json.dumps(res))
    if not (res["no_fault"] and res["bitwise_equal"] and all(r["finite"] for r in runs)):
        sys.exit(1)


if __name__ == "__main__":
    main()
