#!/usr/bin/env python
"""Training-step throughput of the HD-GNN/S engine on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step = the fused step kernel + the gradient reduction + TF Adam on 100 resident
synthetic glide-shaped commits per GPU (weak scaling); under torch.distributed.run the
reduction kernel also all-reduces the flat gradient over xGMI (hdg_train_step_dp; RCCL
when HDG_DP_ALLREDUCE=rccl or the ranks span hosts).  Rank 0 prints
one JSON line.  Per-kernel durations come from HIP events recorded on the launch stream;
the CPU baseline is oracle/literal.py (the TF graph's op sequence on torch-CPU).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "training-step commits/sec, glide Ne=200 Nc=74 batch=100; 1/2/4/8 GPU"
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak (spec)
HBM_PEAK_GBS = 8000.0


def _prof(name):
    """The newest round's copy of a committed profile file (profiles/rNN/<name>)."""
    pd = os.path.join(ROOT, "profiles")
    rounds = sorted(d for d in os.listdir(pd) if d.startswith("r") and d[1:].isdigit()) \
        if os.path.isdir(pd) else []
    for d in reversed(rounds):
        if os.path.exists(os.path.join(pd, d, name)):
            return os.path.join(pd, d, name)
    return os.path.join(pd, "r02", name)


def flops_per_commit(ne, nc, variant=2):
    """Algorithmic training FLOPs per commit, SURVEY 8(d) / BASELINE.md:
    3 * F_fwd(model_2), F_fwd = 1008 Pe + 880 Ne + 2200 Pc (the dense TF graph's pair
    MLPs, sums, node MLPs and classifier; padding / recompute not counted);
    F_fwd(model_4) = F_fwd(model_2) + 1960 Pe; model_1 / model_3 (TF evaluates only the
    fetched subgraph, so model_3's entity-edge stage is never run): 8 Pe + 2200 Pc.
    The engine executes far fewer operations (sorted-x entity sums),
    so this is work-equivalent throughput."""
    pe, pc = ne * (ne - 1), nc * (nc - 1)
    f = {1: 8 * pe + 2200 * pc, 3: 8 * pe + 2200 * pc,
         2: 1008 * pe + 880 * ne + 2200 * pc,
         4: 1008 * pe + 880 * ne + 2200 * pc + 1960 * pe}[variant]
    return 3 * f


def algorithmic_bytes_per_commit(ne, nc):
    """SURVEY 8(d) / BASELINE.md bytes per commit: 4 Ne^2 + 4 Nc^2 + 4 Pe + 8 Pc (the f32
    entity adjacency, the f32 label adjacency, int16 src + tgt hunk maps per entity pair,
    the f32 two-class output per hunk pair)."""
    pe, pc = ne * (ne - 1), nc * (nc - 1)
    return 4 * ne * ne + 4 * nc * nc + 4 * pe + 8 * pc


def compact_bytes_per_commit(ne, nc):
    """What the engine's compact form must move per commit and step: inputs (x, a bits and
    their transpose, y bits, the prepared x tables, the two u16 count matrices), the probs
    output (C_edge_output2, fetched by the training sess.run) and one partial-gradient row
    per block (two per commit in split mode)."""
    we, wc = (ne + 31) // 32, (nc + 31) // 32
    inp = 4 * ne + 2 * 4 * ne * we + 4 * nc * wc + 16 * ne
    kmat = 2 * (2 * nc * ne)
    return inp + kmat + 8 * nc * (nc - 1) + 2 * 4 * 2136


def cpu_baseline(cb, steps, threads):
    """oracle/literal.py (same dense op sequence and FLOPs as the TF1 CPU graph) on the
    GPU box's host cores: fwd + autograd bwd + TF-Adam on the same synthetic batch."""
    from oracle import layout as olayout
    from oracle import literal, model_ref
    torch.set_num_threads(threads)
    B, ne, nc = cb.B, cb.Ne, cb.Nc
    params = model_ref.init_params(0)
    P = model_ref.to_torch_params(params, dtype=torch.float32)
    D = literal.build_dense(cb.x, cb.a, cb.y, cb.hid, cb.nlen, dtype=torch.float32)
    keys = [k for k, _, _ in olayout.keyed_specs(2)]
    theta = np.concatenate([params[k].reshape(-1) for k in keys]).astype(np.float64)
    opt = model_ref.AdamTF(theta.size)

    def one():
        for p in P.values():
            p.grad = None
        out = literal.forward(P, D, B, ne, nc)
        out["total"].backward()
        g = np.concatenate([P[k].grad.numpy().reshape(-1) for k in keys]).astype(np.float64)
        th = opt.step(theta, g)
        with torch.no_grad():
            o = 0
            for k in keys:
                n = P[k].numel()
                P[k].copy_(torch.from_numpy(th[o:o + n].reshape(P[k].shape)))
                o += n

    one()                                     # warm-up (allocator, thread pool)
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    dt = time.perf_counter() - t0
    return {"value": round(B * steps / dt, 3), "unit": "commits/s", "cores": threads,
            "kind": "port",
            "sample": "%d train steps (fwd+bwd+TF-Adam) of oracle/literal.py, fp32 torch-CPU, "
                      "B=%d Ne=%d Nc=%d, %.1f s timed after 1 warm-up step" % (steps, B, ne, nc, dt)}


def e2e_train(B, ne, nc, v, epochs, dev):
    """The reference training loop as main.py --Type train runs it (model_2.py:335-424):
    graph2graph.train for `epochs` epochs, one Mini_batch = B step per epoch (2B synthetic
    commits split 50/50 as utils2 does), with its per-epoch result line, result file and
    checkpoint save, in a scratch directory.  Includes the upload + prepare of the batch."""
    import importlib
    import tempfile
    from hdgnn.synth import synth_commits
    mod = importlib.import_module("hdgnn.model" + ("" if v == 2 else "_%d" % v))
    cb = synth_commits(2 * B, ne, nc, 20250301 + 7)
    train, test = cb.slice(0, B), cb.slice(B, 2 * B)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            class Args:
                checkpoint_dir, Repo = os.path.join(d, "ck"), "glide"
            m = mod.graph2graph(None, Ds=1, Ne=ne, Nc=nc, Ner=ne * (ne - 1), Ncr=nc * (nc - 1),
                                Dr=2, De_e=20, De_er=20, Mini_batch=B, checkpoint_dir=Args.checkpoint_dir,
                                epoch=epochs, Ds_inter=1, Dr_inter=2, Step=2, Repo="glide",
                                device=dev, compact=(train, test, train))
            import contextlib
            import io
            with contextlib.redirect_stdout(io.StringIO()):
                m.train(Args)                      # warm: allocations, first checkpoint
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                m.train(Args)
                torch.cuda.synchronize(dev)
            wall = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
    return {"epochs": epochs, "commits_per_epoch": B, "wall_s": round(wall, 4),
            "commits_per_s": round(epochs * B / wall, 1),
            "ms_per_epoch": round(1e3 * wall / epochs, 3),
            "note": "graph2graph.train as main.py runs it: upload + hdg_prepare of the batch, "
                    "then per epoch one training step, one device->host read of the epoch's "
                    "losses / count, the result line + file and a TF-bundle checkpoint save"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=100, help="commits per GPU")
    ap.add_argument("--ne", type=int, default=200)
    ap.add_argument("--nc", type=int, default=74)
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch kernels eagerly")
    ap.add_argument("--graph-steps", type=int, default=50,
                    help="training steps captured per HIP graph (a divisor of --steps)")
    ap.add_argument("--variant", type=int, default=2, choices=(1, 2, 3, 4),
                    help="model_<variant>.py (the BASELINE metric is model_2)")
    ap.add_argument("--path", type=int, default=0, choices=(0, 1, 2),
                    help="engine path: 0 auto, 1 fused, 2 general (include/hdgnn.h)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"))
    ap.add_argument("--edensity", type=float, default=0.05,
                    help="synthetic entity-adjacency density (data-dependence runs)")
    ap.add_argument("--hdensity", type=float, default=0.10,
                    help="synthetic hunk-label density (data-dependence runs)")
    ap.add_argument("--xkind", default="int10", choices=("int10", "real"),
                    help="node attributes: integers 0..9, or Ne distinct signed reals")
    ap.add_argument("--e2e", type=int, default=50, metavar="EPOCHS",
                    help="also time graph2graph.train (the main.py --Type train loop) for "
                         "EPOCHS epochs of one --batch-commit step each (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run (any world size, so the RCCL step can be exercised on
    # one GPU) every step all-reduces the flat gradient inside the captured graph
    launched = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if launched:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from hdgnn.engine import Engine
    from hdgnn import layout
    from hdgnn.synth import seed_for, synth_commits
    from hdgnn import _lib

    B, ne, nc, v = args.batch, args.ne, args.nc, args.variant
    knobs = {"edensity": args.edensity, "hdensity": args.hdensity, "xkind": args.xkind}
    default_data = knobs == {"edensity": 0.05, "hdensity": 0.10, "xkind": "int10"}
    cb = synth_commits(B, ne, nc, seed_for(1, rank), **knobs)
    eng = Engine(ne, nc, B, variant=v, device=dev, batch_global=B * world, path=args.path,
                 process_group=torch.distributed.group.WORLD if launched else None)
    eng.set_params(layout.init_flat(0, v))
    eng.upload(cb)                               # warm the upload / prepare path once
    torch.cuda.synchronize(dev)
    t_up = time.perf_counter()
    db = eng.upload(cb)                          # host arrays -> HBM + hdg_prepare
    torch.cuda.synchronize(dev)
    upload_ms = 1e3 * (time.perf_counter() - t_up)

    def barrier():
        if launched:
            torch.distributed.barrier()

    # S training steps per HIP graph launch (S = the largest divisor of --steps up to
    # --graph-steps), so the timed region is exactly --steps steps
    gsteps = 1
    if not args.no_graph:
        gsteps = max(d for d in range(1, max(1, args.graph_steps) + 1) if args.steps % d == 0)
    if args.no_graph:
        step = lambda: eng.train_step(db)
    else:
        eng.capture(db, steps=gsteps)            # one HIP graph per gsteps training steps
        step = eng.replay
    for _ in range(max(1, args.warmup // gsteps)):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps // gsteps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    eng.check_status()             # a failed launch (exchange timeout) voids the run: raise
    if launched:
        t = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    value = world * B * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # per-kernel durations (HIP events on the launch stream), separate instrumented pass
    ev = _lib.HipEvents(3)
    # model_2 on the fused path: the step kernel and the reduction timed apart; model_4 on
    # the fused path (entity-edge stage on general-path kernels around the step kernel) and
    # the general path: the whole fwd+bwd
    fused = eng.path == _lib.PATH_FUSED and v == 2
    names = (["k_commit_step", "k_grad_reduce"] if fused else
             ["hybrid_fwd_bwd" if eng.path == _lib.PATH_FUSED else "general_fwd_bwd", "none"])
    acc = dict.fromkeys(names, 0.0)
    nev = max(10, min(args.steps, 50))
    import ctypes
    tails = []                  # data parallel: the all-reduce + Adam tail after fwd_bwd
    for _ in range(nev):
        bstruct = db.struct()
        _lib.check(eng.lib.hdg_fwd_bwd_events(ctypes.byref(eng.shape), ctypes.byref(bstruct),
                                              ctypes.c_void_p(eng.params.data_ptr()),
                                              ctypes.c_void_p(eng.grad_local.data_ptr()),
                                              ctypes.byref(eng._out),
                                              ctypes.c_void_p(eng.workspace.data_ptr()),
                                              eng._stream(), ev.ev))
        for i, n in enumerate(names):
            acc[n] += ev.elapsed_ms(i, i + 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if not eng.xgmi:         # xGMI: adam() exchanges + updates in one kernel
            eng.allreduce()
        eng.adam()
        e1.record()
        tails.append((e0, e1))
    torch.cuda.synchronize(dev)
    kern_ms = {n: acc[n] / nev for n in names}
    tail_ms = sum(a.elapsed_time(b) for a, b in tails) / nev

    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    dom = names[0]
    dense_launch = flops_per_commit(ne, nc, v) * B
    dense_tflops = dense_launch / (kern_ms[dom] * 1e-3) / 1e12
    # executed FP32 FLOPs of one launch (rocprofv3 PMC, calibrated: tools/flops_summary.py)
    exec_flops, flops_src = None, None
    fj = _prof("flops_pmc.json")
    if fused and os.path.exists(fj):
        with open(fj) as f:
            pj = json.load(f)
        if pj["config"] == {"ne": ne, "nc": nc, "batch": B} and v == 2:
            ks = [k for k in pj["kernels"] if k.startswith(dom)]
            if ks:
                exec_flops = pj["kernels"][ks[0]]["executed_flops_per_launch"]
                flops_src = (os.path.relpath(fj, ROOT) + ": 64 x SQ_INSTS_VALU_FLOPS_FP32 + 512 x "
                             "SQ_INSTS_VALU_MFMA_MOPS_F32 per launch, counters calibrated "
                             "on known instruction streams (tools/probe/flops_cal.hip)")
    achieved = exec_flops / (kern_ms[dom] * 1e-3) / 1e12 if exec_flops else None
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if (tj.get("kernel") == dom and tj.get("batch") == B and tj.get("ne") == ne
                and tj.get("nc") == nc and fused and default_data):
            traffic = tj.get("bytes_per_launch")
    executed = None              # executed-instruction view (SQ counters, tools/valu_issue.py)
    vj = _prof("valu_issue.json")
    if fused and (ne, nc, B) == (200, 74, 100) and default_data and os.path.exists(vj):
        with open(vj) as f:
            ev = json.load(f)
        executed = {"valu_wave_insts_per_launch": ev.get("sq_insts_valu_per_launch"),
                    "issue_frac_chip": round(ev.get("issue_frac_chip", 0.0), 4),
                    "issue_frac_busy_cus": round(ev.get("issue_frac_busy_cus", 0.0), 4),
                    "source": os.path.relpath(vj, ROOT) + " (rocprofv3 SQ_INSTS_VALU over the "
                              "kernel's rocprof duration; 4 cycles per wave64 VALU op per SIMD)"}
    # bound: VALU issue.  The kernel's work is FP32 on the vector ALUs (2/3 of its executed
    # FLOPs) and MFMA; what binds it is instruction issue and latency, not the FP32 FLOP
    # roof, so achieved/peak is the executed-FLOP fraction of the 157.3 TFLOP/s FP32 peak
    # and executed.issue_frac_* is the issue-slot fraction next to it
    roofline = {"bound": "valu-issue" if fused else "mfma",
                "achieved": round(achieved, 3) if achieved else None,
                "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4) if achieved else None,
                "traffic": traffic, "kernel": dom,
                "flops_per_launch": exec_flops, "flops_source": flops_src,
                "avg_launch_ms": round(kern_ms[dom], 5),
                "algorithmic_bytes_per_launch": algorithmic_bytes_per_commit(ne, nc) * B,
                "compact_bytes_per_launch": compact_bytes_per_commit(ne, nc) * B,
                "hbm_frac": (round(traffic / (kern_ms[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                             if traffic else None),
                "dense_equivalent": {
                    "flops_per_launch": dense_launch, "tflops": round(dense_tflops, 3),
                    "note": "SURVEY 8(d) per-commit figure (3 F_fwd: the TF graph's dense "
                            "incidence-matrix work) over the same launch time; the engine's "
                            "sorted-x / per-node algebra (DESIGN.md 3) needs ~13x fewer "
                            "operations, so this is work-equivalent throughput, not a "
                            "hardware roofline (no frac)"},
                "executed": executed}
    e2e = None
    if world == 1 and args.e2e > 0:
        try:                     # a side measurement: never costs the bench line
            e2e = e2e_train(B, ne, nc, v, args.e2e, dev)
        except Exception as ex:  # noqa: BLE001
            e2e = {"error": "%s: %s" % (type(ex).__name__, ex)}
    cpu = None
    if world == 1 and not args.no_cpu and v == 2:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(cb, args.cpu_steps, threads)
    line = {"metric": METRIC, "value": round(value, 2), "unit": "commits/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "allreduce": {"xgmi": "in-kernel xGMI exchange of the flat gradient per step "
                                  "(hdg_train_step_dp: tagged words into every peer's "
                                  "mailbox, rank-order sum, TF Adam in the same kernel)",
                          "rccl": "rccl all_reduce of the flat gradient per step"}.get(
                              eng.allreduce_kind) if launched else None,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic glide-shaped commits (SURVEY 8(d) generator, resident in HBM)" + (
                "" if default_data else "; data knobs %s" % json.dumps(knobs)),
            "config": {"workload": "model_%d (%s) train step: fwd+bwd+TF-Adam, %s" % (
                           v, {1: "HD-GNN/ES", 2: "HD-GNN/S", 3: "HD-GNN/E", 4: "HD-GNN"}[v],
                           "glide step=2" if (ne, nc) == (200, 74) else "Ne=%d Nc=%d" % (ne, nc)),
                       "engine_path": {_lib.PATH_FUSED: "fused", _lib.PATH_GENERAL: "general"}[
                           eng.path] + (" (entity-edge stage on general kernels)"
                                        if eng.path == _lib.PATH_FUSED and v == 4 else ""),
                       "launch": "eager" if args.no_graph else
                                 "hipGraph replay, %d training steps per graph" % gsteps,
                       "ne": ne, "nc": nc, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": "dp%d" % world,
                       **({} if default_data else {"data_knobs": knobs})},
            "roofline": roofline, "cpu_baseline": cpu,
            "dp": {"allreduce": eng.allreduce_kind, "selftest": eng.allreduce_selftest,
                   "tail_ms_per_step": round(tail_ms, 5),
                   "tail": "k_grad_reduce excluded; xgmi: hdg_adam_dp (exchange + Adam, the "
                           "k_dp_tail work); rccl: all_reduce + hdg_adam_tf"} if launched else None,
            "upload_prepare_ms": round(upload_ms, 3),
            "pcie_inclusive_commits_per_s": round(world * B / ((ms_per_step + upload_ms) * 1e-3), 1),
            "kernels_ms": {k: round(v, 5) for k, v in kern_ms.items()}}
    if e2e:
        line["e2e"] = e2e
    print(json.dumps(line), flush=True)
    if launched:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
