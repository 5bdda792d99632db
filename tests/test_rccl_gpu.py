"""RCCL data-parallel step on the GPU box (one GPU, so world size 1): the flat-gradient
all-reduce runs through torch.distributed's nccl (= RCCL) backend, both eagerly and
captured inside the per-step HIP graph, and matches the single-process step.  The
multi-rank decomposition itself is covered on CPU by tests/test_dp.py (gloo, world 2/4).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from hdgnn import layout
from hdgnn.synth import synth_commits

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture()
def world1():
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.mark.parametrize("v", [2, 4])
def test_rccl_step_matches_single_process(world1, v):
    from hdgnn.engine import Engine
    B, ne, nc = 4, 60, 21
    cb = synth_commits(B, ne, nc, 8)
    flat = layout.init_flat(5, v)
    single = Engine(ne, nc, B, variant=v)
    dp = Engine(ne, nc, B, variant=v, process_group=world1)
    dg = Engine(ne, nc, B, variant=v, process_group=world1)
    for e in (single, dp, dg):
        e.set_params(flat)
    db = single.upload(cb)
    dg.capture(db)                      # fwd_bwd + RCCL all_reduce + Adam in one HIP graph
    for _ in range(3):
        single.train_step(db)
        dp.train_step(db)               # eager: hdg_fwd_bwd -> all_reduce -> hdg_adam_tf
        dg.replay()
    torch.cuda.synchronize()
    for name, e in (("single", single), ("dp", dp), ("dg", dg)):
        assert bool(torch.isfinite(e.params).all()), name
    assert torch.equal(dp.params, dg.params) and torch.equal(dp.stats, dg.stats)
    np.testing.assert_allclose(dp.get_params(), single.get_params(), rtol=0, atol=1e-7)
    np.testing.assert_allclose(dp.stats.cpu().numpy(), single.stats.cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_gpus_n_starts_n_ranks(n):
    """`bench.py --gpus N` without a launcher starts the N ranks itself (the driver's
    scaling command shape).  On the one-GPU box the ranks share device 0: gloo control
    plane, the gradient over the xGMI mailboxes (IPC between the processes) with the
    shared-device tails (HDG_DP_SHARED: 8 light blocks per rank, so the waiting ranks can
    never hold every CU while the last rank's step kernel still needs one), one block per
    commit.  The line then counts the one device in n_gpus and the ranks in n_ranks."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "20",
           "--warmup", "5", "--no-cpu", "--e2e", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]          # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_ranks"] == n and d["n_gpus"] == min(n, torch.cuda.device_count())
    assert d["config"]["global_batch"] == n * d["config"]["batch_per_gpu"]
    assert d["config"]["parallelism"] == "dp%d" % n and d["value"] > 0
    assert d["warmup"] == d["warmup_requested"] == 5 and d["steps"] == 20
    dp = d["dp"]
    assert dp["allreduce"] == "xgmi" and dp["selftest"].startswith("passed")
    assert "over %d ranks" % n in dp["selftest"] and dp["tail_ms_per_step"] > 0
    if torch.cuda.device_count() < n:
        assert "ranks_share_device" in d["config"] and "rehearsal" in d
        assert "share a device" in dp["selftest"]


@pytest.mark.parametrize("mode", ["rccl", "auto"])
def test_bench_under_torchrun(mode):
    """bench.py under torch.distributed.run (world 1): HDG_DP_ALLREDUCE=rccl must run the
    RCCL all-reduce of the flat gradient (nccl backend = RCCL); auto picks the xGMI
    mailboxes when their self-test passes, else RCCL."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", HDG_DP_ALLREDUCE=mode)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5", "--warmup", "2",
           "--no-cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["allreduce"] and d["value"] > 0 and d["n_gpus"] == 1
    # the line explains the data-parallel path: which all-reduce, the xGMI self-test
    # verdict (world 1: the mailbox exchange with itself), the tail time per step
    dp = d["dp"]
    assert dp["allreduce"] in ("xgmi", "rccl") and dp["selftest"]
    if mode == "rccl":
        assert dp["allreduce"] == "rccl" and "not tried" in dp["selftest"]
    assert dp["allreduce"] != "xgmi" or dp["selftest"].startswith("passed")
    assert dp["tail_ms_per_step"] > 0
