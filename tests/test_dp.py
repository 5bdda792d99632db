"""Data-parallel path on CPU (gloo, world_size 2).

The engine's DP step is: each rank runs hdg_fwd_bwd on its contiguous shard of the
batch with the CE normalised by the GLOBAL batch (shape.batch_global), one SUM
all-reduce of the flat gradient (+ CE-sum trailer), then the same TF-Adam update on
every rank (reg terms added after the reduce).  These tests check that decomposition
with the oracle's gradients and a real gloo all-reduce, and the host shard plan that
graph2graph uses (hdgnn.model.shard_plan)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hdgnn.model import shard_plan
from hdgnn.synth import synth_commits
from oracle import layout as olayout
from oracle import model_ref

KEYS = [k for k, _, _ in olayout.keyed_specs(2)]
B, NE, NC, SEED = 4, 9, 6, 3


@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("n_commits,mb", [(100, 50), (103, 20), (8, 4)])
def test_shard_plan_partitions_every_batch(n_commits, mb, world):
    if mb % world:
        pytest.skip("not divisible")
    plans = [shard_plan(n_commits, mb, world, r) for r in range(world)]
    nb = n_commits // mb
    assert all(len(p) == nb for p in plans)
    for j in range(nb):
        commits = sorted(c for p in plans for c in range(*p[j][0]))
        pos = sorted(q for p in plans for q in range(*p[j][1]))
        assert commits == list(range(j * mb, (j + 1) * mb))
        assert pos == list(range(mb))        # maps of batch positions 0..mb-1 (B.2 quirk)


def test_shard_plan_rejects_indivisible():
    with pytest.raises(ValueError):
        shard_plan(100, 50, 3, 0)


def _flat(grads):
    return np.concatenate([grads[k].reshape(-1) for k in KEYS])


def _reg_grad(flat):
    g = 0.001 * flat.astype(np.float64)
    for off in (2123, 2125):
        th = flat[off:off + 2]
        g[off:off + 2] += 0.001 * th / np.linalg.norm(th)
    return g


def _rank_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cb = synth_commits(B, NE, NC, SEED)
    params = model_ref.init_params(SEED)
    theta = model_ref.flatten(params).astype(np.float64)
    (c0, c1), _ = shard_plan(B, B, world, rank)[0]
    sh = cb.slice(c0, c1)
    out, g = model_ref.loss_and_grads(params, sh.x.astype(np.float64), sh.a, sh.y, sh.hid,
                                      sh.nlen)
    w = (c1 - c0) / B                                   # CE mean over the global batch
    data = (_flat(g) - _reg_grad(theta)) * w
    buf = torch.from_numpy(np.concatenate([data, [float(out["ce"]) * w]]))
    dist.all_reduce(buf)                                # the one collective per step
    g_dp = buf.numpy()[:-1] + _reg_grad(theta)
    opt = model_ref.AdamTF(theta.size)
    new = opt.step(theta, g_dp)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), grad=g_dp, ce=buf.numpy()[-1],
             theta=new)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_two_rank_step_equals_single_process(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    cb = synth_commits(B, NE, NC, SEED)
    params = model_ref.init_params(SEED)
    theta = model_ref.flatten(params).astype(np.float64)
    out, g = model_ref.loss_and_grads(params, cb.x.astype(np.float64), cb.a, cb.y, cb.hid,
                                      cb.nlen)
    ref_new = model_ref.AdamTF(theta.size).step(theta, _flat(g))
    r = [np.load(os.path.join(tmp_path, "rank%d.npz" % k)) for k in range(world)]
    np.testing.assert_array_equal(r[0]["theta"], r[1]["theta"])     # replicas stay equal
    np.testing.assert_allclose(r[0]["grad"], _flat(g), rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(float(r[0]["ce"]), float(out["ce"]), rtol=1e-12)
    np.testing.assert_allclose(r[0]["theta"], ref_new, rtol=0, atol=1e-12)


def _trailer_main(rank, world, port, out_dir):
    """Each rank's gradient trailer as hdg_fwd_bwd leaves it (include/hdgnn.h): count as
    three 16-bit parts, rank 1 reports one timed-out block; one fp32 SUM all-reduce."""
    from hdgnn import _lib
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    count = [(1 << 24) + 12345, (1 << 26) + 777][rank]     # each beyond fp32's 2^24
    tr = np.zeros(_lib.TRAILER, np.float32)
    tr[_lib.TR_CE] = 0.5 + rank
    tr[_lib.TR_COUNT] = count & 0xFFFF
    tr[_lib.TR_COUNT + 1] = (count >> 16) & 0xFFFF
    tr[_lib.TR_FAULT] = float(rank == 1)
    buf = torch.from_numpy(np.concatenate([np.ones(5, np.float32), tr]))
    dist.all_reduce(buf)
    np.save(os.path.join(out_dir, "tr%d.npy" % rank), buf.numpy()[5:])
    dist.destroy_process_group()


def test_gloo_trailer_sums_exactly(tmp_path):
    """The correct-prediction count survives the float all-reduce exactly past 2^24 and a
    fault on any rank reaches every rank (so every replica skips that Adam update)."""
    from hdgnn import _lib
    world = 2
    mp.spawn(_trailer_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = (1 << 24) + 12345 + (1 << 26) + 777
    for k in range(world):
        tr = np.load(os.path.join(tmp_path, "tr%d.npy" % k))
        assert _lib.trailer_count(tr) == want
        assert tr[_lib.TR_FAULT] == 1.0
        assert tr[_lib.TR_CE] == 2.0
    assert float(np.float32(want)) != want                 # one fp32 slot would round it


def test_header_trailer_constants_match_binding():
    """include/hdgnn.h's trailer / status constants == the Python binding's."""
    import re
    from conftest import ROOT
    from hdgnn import _lib
    txt = open(os.path.join(ROOT, "include", "hdgnn.h")).read()
    val = {m.group(1): int(m.group(2)) for m in
           re.finditer(r"#define (HDG_\w+)\s+(\d+)u?\b", txt)}
    assert val["HDG_ABI_VERSION"] == _lib.ABI_VERSION
    assert val["HDG_TRAILER"] == _lib.TRAILER
    assert (val["HDG_TR_CE"], val["HDG_TR_COUNT"], val["HDG_TR_FAULT"]) == (
        _lib.TR_CE, _lib.TR_COUNT, _lib.TR_FAULT)
    assert val["HDG_STATUS_XCH_TIMEOUT"] == _lib.STATUS_XCH_TIMEOUT
    assert val["HDG_STATUS_DP_TIMEOUT"] == _lib.STATUS_DP_TIMEOUT
    assert (val["HDG_DP_MAX_WORLD"], val["HDG_DP_HANDLE_BYTES"], val["HDG_DP_MAX_LEN"]) == (
        _lib.DP_MAX_WORLD, _lib.DP_HANDLE_BYTES, _lib.DP_MAX_LEN)
    assert (val["HDG_DP_SHARED"], val["HDG_DP_SHARED_BLOCKS"]) == (
        _lib.DP_SHARED, _lib.DP_SHARED_BLOCKS)


def test_dp_struct_and_mailbox_size():
    """hdg_dp's ctypes mirror has the C layout (int32 rank, world; u64 wait; 16 pointers;
    int32 flags, reserved) and the mailbox holds two parities x 16 senders x DP_MAX_LEN
    tagged words."""
    import ctypes
    from hdgnn import _lib
    assert ctypes.sizeof(_lib.Dp) == 4 + 4 + 8 + 8 * _lib.DP_MAX_WORLD + 4 + 4
    assert _lib.Dp.mailbox.offset == 16
    assert _lib.Dp.flags.offset == 16 + 8 * _lib.DP_MAX_WORLD
    # the shared-device tails: the waiting ranks' spinning blocks never cover the CUs
    assert (_lib.DP_MAX_WORLD - 1) * _lib.DP_SHARED_BLOCKS < 256
    lib = _lib.load()
    assert lib.hdg_dp_mailbox_bytes() >= 2 * _lib.DP_MAX_WORLD * _lib.DP_MAX_LEN * 8
    assert _lib.DP_MAX_LEN >= lib.hdg_grad_len(4) and _lib.DP_MAX_LEN % 16 == 0
    # argument errors are reported without touching a device
    dp = _lib.Dp()
    dp.world, dp.rank = 2, 2
    rc = lib.hdg_dp_allreduce(ctypes.byref(dp), None, None, 4, None, None)
    assert rc == 1000 and b"out of range" in lib.hdg_last_error()
