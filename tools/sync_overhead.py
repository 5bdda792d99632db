"""GPU box: the fixed cost of one timed region (graph launch + the final synchronize) at the
bench workload, with HIP's default scheduling and with hipDeviceScheduleSpin set before
the device is initialised.  Median over repeats of: sync; t0; one replay of S steps; sync.

  python tools/sync_overhead.py [--spin] [--steps 20]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-gnn_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    if a.spin:   # hipDeviceScheduleSpin = 1, before any HIP call initialises the device
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))
        print("hipSetDeviceFlags(spin) rc", rc)
    import torch
    from hdgnn import layout
    from hdgnn.engine import Engine
    from hdgnn.synth import synth_commits
    eng = Engine(200, 74, 100, variant=2)
    eng.set_params(layout.init_flat(0, 2))
    db = eng.upload(synth_commits(100, 200, 74, 1))
    eng.capture(db, steps=a.steps)
    eng.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        eng.replay()                      # warm-up replay, as bench.py
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.replay()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    first = [round(1e3 * x / a.steps, 5) for x in ts[:6]]
    ts.sort()
    t0 = time.perf_counter()
    for _ in range(40):
        eng.replay()
    torch.cuda.synchronize()
    per_step = (time.perf_counter() - t0) / (40 * a.steps)
    med = ts[len(ts) // 2]
    print(json.dumps({"spin": a.spin, "steps": a.steps, "region_ms_median": 1e3 * med,
                      "ms_per_step_region": 1e3 * med / a.steps,
                      "ms_per_step_streamed": 1e3 * per_step,
                      "fixed_us": 1e6 * (med - a.steps * per_step),
                      "first_regions_ms_per_step": first}))


if __name__ == "__main__":
    main()
