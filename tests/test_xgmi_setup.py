"""xGMI mailbox set-up protocol on CPU (gloo, world 2) with a stand-in for the library's
mailbox calls: every outcome of XgmiGroup.create is agreed by all ranks (a failure on
any rank -- allocation, opening a peer handle, the self-test -- gives every rank the RCCL
fallback, or an error on every rank when xGMI is required), and whatever a failed set-up
allocated or mapped is released.  The exchange itself runs on the GPU box
(tests/test_xgmi_gpu.py)."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeLib:
    """hdg_dp_mailbox_* with scripted failures; records what was freed / closed."""

    def __init__(self, rank, fail):
        self.rank, self.fail, self.log = rank, fail, []

    def hdg_last_error(self):
        return b"scripted failure"

    def hdg_dp_mailbox_alloc(self, ref, handle):
        if ("alloc", self.rank) in self.fail:
            return 1
        ref._obj.value = 0x1000 * (self.rank + 1)
        for k in range(64):
            handle[k] = (self.rank * 7 + k) & 0xFF
        self.log.append("alloc")
        return 0

    def hdg_dp_mailbox_open(self, handle, ref):
        if ("open", self.rank) in self.fail:
            return 1
        peer = (handle[0] // 7) if handle[0] % 7 == 0 else -1
        ref._obj.value = 0x100000 + peer
        self.log.append("open")
        return 0

    def hdg_dp_mailbox_close(self, p):
        self.log.append("close")
        return 0

    def hdg_dp_mailbox_free(self, p):
        self.log.append("free")
        return 0


def _main(rank, world, port, out_dir, fail, required):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hdgnn import xgmi
    lib = FakeLib(rank, set(fail))
    orig = xgmi.XgmiGroup.selftest
    xgmi.XgmiGroup.selftest = (lambda self: "scripted" if ("selftest", self.rank) in lib.fail
                               else None)
    res = {"ok": 0, "raised": 0, "log": ",".join(lib.log)}
    try:
        grp = xgmi.XgmiGroup.create(lib, dist.group.WORLD, torch.device("cpu"),
                                    required=required)
        res["ok"] = int(grp is not None)
        if grp is not None:
            res["mailbox"] = [grp.dp.mailbox[r] for r in range(world)]
            res["wait"] = int(grp.dp.wait_ticks)
            grp._own = None                    # nothing real to release
    except RuntimeError:
        res["raised"] = 1
    res["log"] = ",".join(lib.log)
    xgmi.XgmiGroup.selftest = orig
    with open(os.path.join(out_dir, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, fail, required=False):
    world = 2
    mp.spawn(_main, args=(world, _port(), str(tmp_path), list(fail), required), nprocs=world,
             join=True)
    out = []
    for r in range(world):
        with open(os.path.join(tmp_path, "r%d.json" % r)) as f:
            out.append(json.load(f))
    return out


def test_setup_succeeds_on_every_rank(tmp_path):
    r = _run(tmp_path, [])
    assert [x["ok"] for x in r] == [1, 1]
    # rank r's own slot is its allocation, the peer's slot the mapping of the peer's handle
    assert r[0]["mailbox"] == [0x1000, 0x100001] and r[1]["mailbox"] == [0x100000, 0x2000]
    assert r[0]["wait"] == 10 * 100_000_000


@pytest.mark.parametrize("fail", [[("alloc", 1)], [("open", 0)], [("selftest", 1)]])
def test_any_failure_falls_back_on_every_rank(tmp_path, fail):
    r = _run(tmp_path, fail)
    assert [x["ok"] for x in r] == [0, 0] and [x["raised"] for x in r] == [0, 0]
    for x in r:                                   # nothing left allocated or mapped
        log = x["log"].split(",") if x["log"] else []
        assert log.count("alloc") == log.count("free")
        assert log.count("open") == log.count("close")


def test_required_xgmi_raises_on_every_rank(tmp_path):
    r = _run(tmp_path, [("selftest", 0)], required=True)
    assert [x["raised"] for x in r] == [1, 1]
