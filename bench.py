#!/usr/bin/env python
"""Training-step throughput of the HD-GNN/S engine on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` without a launcher starts the N ranks itself (a torch.distributed.run child);
under a launcher WORLD_SIZE must equal --gpus.  Rank r runs on device r mod device_count;
more ranks than devices (a rehearsal) share them over a gloo control plane.

A step = the fused step kernel + the gradient reduction + TF Adam on 100 resident
synthetic glide-shaped commits per GPU (weak scaling); under torch.distributed.run the
reduction kernel also all-reduces the flat gradient over xGMI (hdg_train_step_dp; RCCL
when HDG_DP_ALLREDUCE=rccl or the ranks span hosts).  Rank 0 prints
one JSON line.  Per-kernel durations come from HIP events recorded on the launch stream;
the CPU baseline is oracle/literal.py (the TF graph's op sequence on torch-CPU).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "training-step commits/sec, glide Ne=200 Nc=74 batch=100; 1/2/4/8 GPU"
WARM_S = 0.03      # seconds of back-to-back steps before the steady-state re-timing
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak (spec)
HBM_PEAK_GBS = 8000.0
CLOCK_HZ = 2.4e9              # gfx950 peak engine clock (MI355X_MICROARCH.md)


def find_profile(variant, path, ne, nc, batch, hunk="auto"):
    """The newest committed rocprofv3 profile of this exact workload:
    profiles/rNN/<config>/roofline.json (tools/roofline_profile.py) whose config matches
    (variant, engine path, Ne, Nc, batch per GPU, hunk pair-pass form) on the default
    synthetic data."""
    pd = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(pd) if d.startswith("r") and d[1:].isdigit()),
                    reverse=True) if os.path.isdir(pd) else []
    want = {"variant": variant, "path": path, "ne": ne, "nc": nc, "batch": batch}
    for d in rounds:
        for sub in sorted(os.listdir(os.path.join(pd, d))):
            f = os.path.join(pd, d, sub, "roofline.json")
            if os.path.isfile(f):
                with open(f) as fh:
                    pj = json.load(fh)
                if ({k: pj["config"].get(k) for k in want} == want
                        and pj["config"].get("hunk", "auto") == hunk):
                    return f, pj
    return None, None


def build_roofline(dom, kern_ms, variant, path, ne, nc, batch, default_data, hunk="auto"):
    """Roofline of the step's dominant kernel (the longest of the live per-kernel HIP-event
    times) from the committed profile of the same workload: executed FP32 FLOPs per launch
    (calibrated PMC counters) and HBM bytes per launch, over the LIVE average duration."""
    f, pj = find_profile(variant, path, ne, nc, batch, hunk) if default_data else (None, None)
    t = kern_ms[dom] * 1e-3
    dense = flops_per_commit(ne, nc, variant) * batch
    r = {"bound": None, "achieved": None, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
         "frac": None, "traffic": None, "kernel": dom, "avg_launch_ms": round(kern_ms[dom], 5),
         "algorithmic_bytes_per_launch": algorithmic_bytes_per_commit(ne, nc) * batch,
         "compact_bytes_per_launch": compact_bytes_per_commit(ne, nc) * batch,
         "dense_equivalent": {
             "flops_per_step": dense,
             "tflops": round(dense / (sum(kern_ms.values()) * 1e-3) / 1e12, 3),
             "note": "SURVEY 8(d) per-commit figure (3 F_fwd: the TF graph's dense "
                     "incidence-matrix work) over the whole fwd+bwd; the engine's sorted-x / "
                     "per-node algebra (DESIGN.md 3) executes ~13x fewer operations, so this "
                     "is work-equivalent throughput, not a hardware roofline (no frac)"},
         "profile": None}
    # SURVEY 8(d)'s algorithmic bytes over the live launch time: the contract's byte roofline
    alg = r["algorithmic_bytes_per_launch"]
    r["alg_hbm_gbs"] = round(alg / t / 1e9, 2)
    r["alg_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBS, 4)
    r["frac_basis"] = ("executed FP32 FLOPs per launch (calibrated rocprofv3 PMC counters of "
                       "the committed profile) / fp32 peak; alg_hbm_frac = SURVEY 8(d) "
                       "algorithmic bytes / live launch time / 8 TB/s")
    if pj is None:
        r["profile"] = "no committed profile of this workload (tools/profile_config.sh)"
        return r
    kp = pj["kernels"].get(dom)
    r["profile"] = os.path.relpath(f, ROOT)
    if kp is None:
        r["profile"] += ": kernel %s not in the profile" % dom
        return r
    fl = kp.get("executed_flops")
    if fl:
        r["achieved"] = round(fl / t / 1e12, 3)
        r["frac"] = round(fl / t / 1e12 / FP32_PEAK_TFLOPS, 4)
        r["flops_per_launch"] = fl
    r["traffic"] = kp.get("hbm_bytes")
    r["traffic_bounds"] = [kp.get("hbm_bytes_lower"), kp.get("hbm_bytes_upper")]
    r["traffic_note"] = pj.get("traffic_note")
    if r["traffic"]:
        r["hbm_frac"] = round(r["traffic"] / t / 1e9 / HBM_PEAK_GBS, 4)
    vi = kp.get("valu_wave_insts")
    if vi:           # a wave64 VALU instruction holds a SIMD for 4 cycles; 4 SIMDs per CU
        r["executed"] = {"valu_wave_insts_per_launch": vi,
                         "issue_frac_chip": round(vi / (t * CLOCK_HZ / 4 * 256 * 4), 4),
                         "wait_any_frac": kp.get("wait_any_frac")}
    issue = r.get("executed", {}).get("issue_frac_chip") or 0.0
    r["bound"] = "valu-issue" if issue >= (r.get("hbm_frac") or 0.0) else "hbm"
    # the whole step (every kernel of fwd+bwd) from the same profile
    ks = [k for k in kern_ms if k in pj["kernels"] and pj["kernels"][k].get("executed_flops")]
    if ks:
        tot_t = sum(kern_ms.values()) * 1e-3
        tot_f = sum(pj["kernels"][k]["executed_flops"] for k in ks)
        tot_b = sum(pj["kernels"][k].get("hbm_bytes") or 0 for k in kern_ms if k in pj["kernels"])
        r["step"] = {"kernels": len(kern_ms), "executed_flops": tot_f,
                     "tflops": round(tot_f / tot_t / 1e12, 3),
                     "frac": round(tot_f / tot_t / 1e12 / FP32_PEAK_TFLOPS, 4),
                     "hbm_bytes": tot_b, "hbm_frac": round(tot_b / tot_t / 1e9 / HBM_PEAK_GBS, 4)}
    return r


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
                    "then per epoch one training step, the epoch's stats and state read to "
                    "pinned host memory (epochs pipelined one deep), the result line + file "
                    "and a TF-bundle checkpoint written by libhdgnn on the saver thread"}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: run the N ranks as one
    torch.distributed.run child (one process per rank, rendezvous on 127.0.0.1) and return
    its exit code.  This process has not touched the GPU (nothing is exec'd: the child is a
    fresh process tree; rank 0's JSON line reaches stdout through the inherited pipe)."""
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd, env=env)


def rank_layout(world, local):
    """(device index, ranks share a device) for this rank: local rank modulo the node's
    device count.  torch.cuda.device_count() does not initialise the GPU on this image."""
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("bench.py needs a HIP device (torch.cuda.device_count() == 0)")
    return local % ndev, world > ndev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU; default: WORLD_SIZE under a launcher, "
                         "else 1).  Without a launcher, N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=100, help="commits per GPU")
    ap.add_argument("--ne", type=int, default=200)
    ap.add_argument("--nc", type=int, default=74)
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch kernels eagerly")
    ap.add_argument("--no-steady", action="store_true",
                    help="skip the steady-state re-timing after the clock-ramp warm-up")
    ap.add_argument("--graph-steps", type=int, default=50,
                    help="training steps captured per HIP graph (a divisor of --steps)")
    ap.add_argument("--variant", type=int, default=2, choices=(1, 2, 3, 4),
                    help="model_<variant>.py (the BASELINE metric is model_2)")
    ap.add_argument("--path", type=int, default=0, choices=(0, 1, 2),
                    help="engine path: 0 auto, 1 fused, 2 general (include/hdgnn.h)")
    ap.add_argument("--hunk", default="auto", choices=("auto", "dense", "sorted", "tiled"),
                    help="general path's hunk pair sums: the automatic form by Nc (include/hdgnn.h "
                         "HDG_HUNK_SORTED_MIN_NC / HDG_HUNK_TILED_MIN_NC), or forced dense / "
                         "sorted / tiled")
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

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        sys.exit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks; refusing "
                 "to report n_gpus=%d for a %d-rank run" % (args.gpus, world, args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run (any world size, so the RCCL step can be exercised on
    # one GPU) every step all-reduces the flat gradient inside the captured graph
    launched = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    didx, shared = rank_layout(world, local) if launched else (0, False)
    if launched:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(didx)
        if shared:
            # more ranks than devices (a rehearsal on a smaller box): RCCL refuses two ranks
            # on one GPU, so the control plane runs on gloo and the gradient exchange must
            # be the xGMI mailboxes (IPC-mapped between the processes)
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", didx))
    dev = torch.device("cuda", didx)

    from hdgnn.engine import Engine
    from hdgnn import layout
    from hdgnn.synth import seed_for, synth_commits
    from hdgnn import _lib

    B, ne, nc, v = args.batch, args.ne, args.nc, args.variant
    knobs = {"edensity": args.edensity, "hdensity": args.hdensity, "xkind": args.xkind}
    default_data = knobs == {"edensity": 0.05, "hdensity": 0.10, "xkind": "int10"}
    cb = synth_commits(B, ne, nc, seed_for(1, rank), **knobs)
    hflags = {"auto": 0, "dense": _lib.FLAG_HUNK_DENSE, "sorted": _lib.FLAG_HUNK_SORTED,
              "tiled": _lib.FLAG_HUNK_TILED}[args.hunk]
    eng = Engine(ne, nc, B, variant=v, device=dev, batch_global=B * world, path=args.path,
                 process_group=torch.distributed.group.WORLD if launched else None,
                 flags=hflags, allreduce="xgmi" if shared else None)
    if shared:
        # the fused split mode needs both blocks of a commit resident at once; ranks
        # sharing a device compete for its CUs, so one block per commit
        eng.set_split(False)
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
    # Warm-up: exactly the requested W training steps (eager launches of the same kernels;
    # the graph capture's own warm step restores the state it changed and is not counted),
    # then the timed region of exactly K steps: this is the headline `value`.
    for _ in range(args.warmup):
        eng.train_step(db)
    torch.cuda.synchronize(dev)

    def timed():
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps // gsteps):
            step()
        torch.cuda.synchronize(dev)
        barrier()
        el = time.perf_counter() - t0
        eng.check_status()         # a failed launch (exchange timeout) voids the run: raise
        if launched:
            t = torch.tensor([el], device="cpu" if shared else dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = t.item()
        return el

    elapsed = timed()
    value = world * B * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # Steady state, reported beside the headline: the device reaches its steady clocks only
    # after a few ms of back-to-back steps (20-step regions right after start-up: 0.0576,
    # 0.0565, 0.0560, 0.0554, then 0.0548 ms/step; tools/sync_overhead.py), so after WARM_S
    # more seconds of steps the same K steps are timed again.  The replay count is agreed
    # across ranks (every rank replays the same graphs: their exchanges must pair up).
    steady = None
    if not args.no_steady:
        t_w = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        extra = int(math.ceil(WARM_S / max(time.perf_counter() - t_w, 1e-6)))
        if launched:
            te = torch.tensor([float(extra)], device="cpu" if shared else dev)
            torch.distributed.all_reduce(te, op=torch.distributed.ReduceOp.MAX)
            extra = int(te.item())
        for _ in range(extra):
            step()
        torch.cuda.synchronize(dev)
        el2 = timed()
        steady = {"warmup": args.warmup + args.steps + (1 + extra) * gsteps,
                  "value": round(world * B * args.steps / el2, 2),
                  "ms_per_step": round(1e3 * el2 / args.steps, 5),
                  "note": "the same %d timed steps again after %g ms more of back-to-back "
                          "steps (the device's clock ramp); not the headline" % (
                              args.steps, 1e3 * WARM_S)}

    # per-kernel durations: HIP events on the launch stream after every kernel launch of
    # the step (hdg_fwd_bwd_kernel_events), eager launches, a separate instrumented pass
    # with the training step's outputs (probs, as the training sess.run fetches; no logits)
    import ctypes
    NEV = 40
    ev = _lib.HipEvents(NEV)
    kn = (ctypes.c_char_p * (NEV - 1))()
    nk = ctypes.c_int32()
    acc, order = {}, []
    nev = max(10, min(args.steps, 50))
    tails = []                  # data parallel: the all-reduce + Adam tail after fwd_bwd
    for _ in range(nev):
        bstruct = db.struct()
        _lib.check(eng.lib.hdg_fwd_bwd_kernel_events(
            ctypes.byref(eng.shape), ctypes.byref(bstruct), ctypes.c_void_p(eng.params.data_ptr()),
            ctypes.c_void_p(eng.grad_local.data_ptr()), ctypes.byref(eng._outputs(True, False)),
            ctypes.c_void_p(eng.workspace.data_ptr()), eng._stream(), ev.ev, NEV, kn,
            ctypes.byref(nk)))
        for i in range(nk.value):
            n = kn[i].decode()
            if n not in acc:
                acc[n] = 0.0
                order.append(n)
            acc[n] += ev.elapsed_ms(i, i + 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if not eng.xgmi:         # xGMI: adam() exchanges + updates in one kernel
            eng.allreduce()
        eng.adam()
        e1.record()
        tails.append((e0, e1))
    torch.cuda.synchronize(dev)
    kern_ms = {n: acc[n] / nev for n in order}
    tail_ms = sum(a.elapsed_time(b) for a, b in tails) / nev

    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    path_name = {_lib.PATH_FUSED: "fused", _lib.PATH_GENERAL: "general"}[eng.path]
    dom = max(kern_ms, key=kern_ms.get)          # the dominant kernel of the step
    roofline = build_roofline(dom, kern_ms, v, path_name, ne, nc, B, default_data, args.hunk)
    # the general path's hunk pair-sum form this run used (include/hdgnn.h's rule by Nc)
    hunk_form = args.hunk if args.hunk != "auto" else (
        "tiled" if nc >= _lib.HUNK_TILED_MIN_NC else
        "sorted" if nc >= _lib.HUNK_SORTED_MIN_NC else "dense") + " (auto)"
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
    ndev = min(world, torch.cuda.device_count()) if launched else 1
    line = {"metric": METRIC, "value": round(value, 2), "unit": "commits/s", "n_gpus": ndev,
            "n_ranks": world,
            "steps": args.steps, "warmup": args.warmup, "warmup_requested": args.warmup,
            "warmup_note": "exactly the requested W untimed training steps before the timed "
                           "region (plus the HIP-graph capture's state-neutral warm step)",
            "ms_per_step": round(ms_per_step, 5),
            "steady_state": steady,
            **({"rehearsal": "%d ranks share %d device(s): not a %d-GPU measurement" % (
                world, ndev, world)} if shared else {}),
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
                       "engine_path": path_name + (" (entity-edge stage on general kernels)"
                                        if eng.path == _lib.PATH_FUSED and v == 4 else ""),
                       "launch": "eager" if args.no_graph else
                                 "hipGraph replay, %d training steps per graph" % gsteps,
                       "ne": ne, "nc": nc, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": "dp%d" % world,
                       **({"ranks_share_device": "%d ranks on %d device(s): gloo control plane, "
                                                 "xGMI-mailbox gradient exchange, one block per "
                                                 "commit" % (world, torch.cuda.device_count())}
                          if shared else {}),
                       **({"hunk_sums": hunk_form} if eng.path == _lib.PATH_GENERAL else {}),
                       **({} if default_data else {"data_knobs": knobs})},
            "roofline": roofline, "cpu_baseline": cpu,
            "dp": {"allreduce": eng.allreduce_kind, "selftest": eng.allreduce_selftest,
                   "tail_ms_per_step": round(tail_ms, 5),
                   "tail": "k_grad_reduce excluded; xgmi: hdg_adam_dp (exchange + Adam, the "
                           "k_dp_tail work); rccl: all_reduce + hdg_adam_tf"} if launched else None,
            "upload_prepare_ms": round(upload_ms, 3),
            "pcie_inclusive_commits_per_s": round(world * B / ((ms_per_step + upload_ms) * 1e-3), 1),
            "kernels_ms": {k: round(t, 5) for k, t in kern_ms.items()},
            "fwd_bwd_ms": round(sum(kern_ms.values()), 5)}
    if e2e:
        line["e2e"] = e2e
    print(json.dumps(line), flush=True)
    if launched:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
