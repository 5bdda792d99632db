"""Data parallelism over xGMI mailboxes (include/hdgnn.h hdg_*_dp, hdgnn/xgmi.py) on the
GPU box.  The box has one GPU, so the ranks are processes sharing it: the mailboxes are
still separate allocations mapped into each other through HIP IPC, and every exchange
word still travels as a system-scope write-through store into another process's
memory -- the same protocol the 8-GPU node runs over xGMI links.  The handles go over a
gloo group (RCCL refuses two ranks on one GPU).

Checks: the DP step (fused and general path; eager, HIP-graph replay, and the split
fwd_bwd / adam calls; world 2 and 4; the one-rank-per-device tails and the shared-device
tails of HDG_DP_SHARED) equals the single-process step on the whole batch and keeps the
replicas bitwise equal; the plain all-reduce sums in rank order bit for bit (world 4);
a rank that stops exchanging makes its peer fail loudly (HDG_STATUS_DP_TIMEOUT, no
update) instead of hanging.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hdgnn import _lib, layout
from hdgnn.synth import synth_commits

pytestmark = pytest.mark.gpu
BL, NE, NC, SEED, STEPS = 4, 60, 21, 8, 3
VARIANTS = (2, 4)          # fused path / general path (model_4)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _train_main(rank, world, port, out_dir, shared=None):
    from hdgnn.engine import Engine
    _init(rank, world, port)
    cb = synth_commits(BL * world, NE, NC, SEED)
    shard = cb.slice(rank * BL, (rank + 1) * BL)
    res = {}
    for v in VARIANTS:
        flat = layout.init_flat(5, v)
        for mode in ("eager", "graph", "calls"):
            eng = Engine(NE, NC, BL, variant=v, batch_global=BL * world,
                         process_group=dist.group.WORLD, allreduce="xgmi", dp_shared=shared)
            assert eng.allreduce_kind == "xgmi"
            res["flags"] = np.array(eng.xgmi.dp.flags)
            eng.set_params(flat)
            db = eng.upload(shard)
            if mode == "graph":
                eng.capture(db, steps=STEPS)
                eng.replay()
            elif mode == "calls":             # bench.py's event pass: fwd_bwd, allreduce, adam
                for _ in range(STEPS):
                    eng.fwd_bwd(db)
                    eng.allreduce()
                    eng.adam()
            else:
                for _ in range(STEPS):
                    eng.train_step(db)
            torch.cuda.synchronize()
            eng.check_status()
            res["v%d_%s_params" % (v, mode)] = eng.get_params()
            res["v%d_%s_stats" % (v, mode)] = eng.stats.cpu().numpy()
            res["v%d_%s_count" % (v, mode)] = np.array(eng.correct_count())
            eng.xgmi.close()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,shared", [(2, False), (2, None), (4, None)],
                         ids=["w2-per-device-tails", "w2-auto", "w4-auto"])
def test_xgmi_step_equals_single_process(tmp_path, world, shared):
    """world 4 is the DP training step above world 2: on the one-GPU box the
    four ranks share the device, so `auto` detects it and runs the shared-device tails
    (HDG_DP_SHARED); (2, False) keeps the one-rank-per-device tails (k_dp_tail<PART> on the
    fused path) covered, whose small grids here still fit beside each other."""
    mp.spawn(_train_main, args=(world, _port(), str(tmp_path), shared), nprocs=world,
             join=True)
    from hdgnn.engine import Engine
    r = [np.load(os.path.join(tmp_path, "rank%d.npz" % k)) for k in range(world)]
    want_flags = (_lib.DP_SHARED if torch.cuda.device_count() < world else 0) \
        if shared is None else 0
    for k in range(world):
        assert int(r[k]["flags"]) == want_flags
    cb = synth_commits(BL * world, NE, NC, SEED)
    for v in VARIANTS:
        single = Engine(NE, NC, BL * world, variant=v)
        single.set_params(layout.init_flat(5, v))
        db = single.upload(cb)
        for _ in range(STEPS):
            single.train_step(db)
        torch.cuda.synchronize()
        want_p, want_s = single.get_params(), single.stats.cpu().numpy()
        want_c = single.correct_count()
        for mode in ("eager", "graph", "calls"):
            k = "v%d_%s_" % (v, mode)
            # replicas bitwise equal: every rank sums the world's words in rank order
            for q in range(1, world):
                np.testing.assert_array_equal(r[0][k + "params"], r[q][k + "params"])
                np.testing.assert_array_equal(r[0][k + "stats"], r[q][k + "stats"])
            np.testing.assert_allclose(r[0][k + "params"], want_p, rtol=0, atol=1e-6,
                                       err_msg=k)
            np.testing.assert_allclose(r[0][k + "stats"], want_s, rtol=1e-5, err_msg=k)
            assert int(r[0][k + "count"]) == want_c, k
        # the three ways of issuing the step agree bit for bit
        np.testing.assert_array_equal(r[0]["v%d_eager_params" % v], r[0]["v%d_graph_params" % v])


def _sum_main(rank, world, port, out_dir, shared=None):
    from hdgnn.xgmi import XgmiGroup
    _init(rank, world, port)
    lib = _lib.load()
    grp = XgmiGroup.create(lib, dist.group.WORLD, torch.device("cuda", 0), required=True,
                           shared=shared)
    dev = torch.device("cuda", 0)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    outs = []
    for n in (1, 17, 2131, _lib.DP_MAX_LEN):
        x = torch.from_numpy(np.random.default_rng(100 * n + rank).standard_normal(n)
                             .astype(np.float32)).to(dev)
        out = torch.empty_like(x)
        grp.allreduce(x, out, status)
        outs.append(out.cpu().numpy())
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "sum%d.npz" % rank), status=status.cpu().numpy(), *outs)
    # a rank that stops exchanging: rank 0 issues one more all-reduce than the others
    dist.barrier()
    status.zero_()
    grp.dp.wait_ticks = 30_000_000                          # 0.3 s
    if rank == 0:
        x = torch.ones(64, device=dev)
        out = torch.zeros(64, device=dev)
        grp.allreduce(x, out, status)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, "late.npy"), status.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("shared", [None, False], ids=["auto", "per-device-tails"])
def test_xgmi_allreduce_rank_order_and_timeout(tmp_path, shared):
    world = 4
    mp.spawn(_sum_main, args=(world, _port(), str(tmp_path), shared), nprocs=world, join=True)
    res = [np.load(os.path.join(tmp_path, "sum%d.npz" % k)) for k in range(world)]
    for i, n in enumerate((1, 17, 2131, _lib.DP_MAX_LEN)):
        xs = [np.random.default_rng(100 * n + k).standard_normal(n).astype(np.float32)
              for k in range(world)]
        want = xs[0].copy()
        for k in range(1, world):
            want = (want + xs[k]).astype(np.float32)       # rank order, fp32
        for k in range(world):
            np.testing.assert_array_equal(res[k]["arr_%d" % i], want)
            assert int(res[k]["status"][0]) == 0
    late = np.load(os.path.join(tmp_path, "late.npy"))
    assert int(late[0]) & _lib.STATUS_DP_TIMEOUT
