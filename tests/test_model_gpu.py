"""hdgnn.model[_N].graph2graph (the drop-ins for model_N.graph2graph) end to end on the GPU:
train(args) for 2 epochs on the reference loader's golden 12-tuple (Ne=7, Nc=5,
50 train / 50 test commits, Mini_batch=25 -> 2 steps per epoch) against the oracle
driven through the same batch plan; then test(args) and its output files."""
import json
import os
import types

import numpy as np
import pytest
import torch

from hdgnn import data, layout
from oracle import model_ref

pytestmark = pytest.mark.gpu

NAMES = ["E_node_train", "E_node_test", "E_edge_train", "E_edge_test", "C_edge_train",
         "C_edge_test", "Es_data", "Et_data", "Cs_label", "Ct_label", "Esc_data", "Etc_data"]


def _tuple(golden_dir):
    z = np.load(os.path.join(golden_dir, "loader_tiny.npz"))
    with open(os.path.join(golden_dir, "loader_tiny.json")) as f:
        meta = json.load(f)
    return tuple(z[n] for n in NAMES), meta


@pytest.mark.parametrize("v", [1, 2, 3, 4])
def test_graph2graph_train_and_test(v, golden_dir, tmp_path, monkeypatch):
    import importlib
    graph2graph = importlib.import_module("hdgnn.model" + ("" if v == 2 else "_%d" % v)).graph2graph
    assert graph2graph.variant == v
    tup, meta = _tuple(golden_dir)
    ne, nc, mb = meta["Ne"], meta["Nc"], 25
    monkeypatch.chdir(tmp_path)
    args = types.SimpleNamespace(Repo="tiny", checkpoint_dir=str(tmp_path / "ckpt"))
    m = graph2graph(None, Ds=1, Ne=ne, Nc=nc, Ner=ne * (ne - 1), Ncr=nc * (nc - 1), Dr=2,
                    De_e=20, De_er=20, Mini_batch=mb, checkpoint_dir=args.checkpoint_dir,
                    epoch=2, Ds_inter=1, Dr_inter=2, Step=2, Repo="tiny",
                    reader=lambda model, step: tup, seed=7)
    m.train(args)
    torch.cuda.synchronize()

    # oracle through the same plan: 2 epochs x 2 batches, maps of positions [:mb]
    train, test, maps = data.compact_from_read_data(tup, ne, nc, mb)
    theta = layout.init_flat(7, v).astype(np.float64)
    opt = model_ref.AdamTF(theta.size)
    epoch_theta = []
    for _ in range(2):
        for j in range(2):
            sh = train.slice(j * mb, (j + 1) * mb).with_maps(maps)
            P = model_ref.unflatten(theta.astype(np.float32).astype(np.float64), v)
            _, g = model_ref.loss_and_grads(P, sh.x.astype(np.float64), sh.a, sh.y, sh.hid,
                                            sh.nlen, variant=v)
            from oracle import layout as olayout
            keys = [k for k, _, _ in olayout.keyed_specs(v)]
            theta = opt.step(theta, np.concatenate([g[k].reshape(-1) for k in keys]))
            last = (P, sh)
        epoch_theta.append(theta.copy())
    np.testing.assert_allclose(m.engine.get_params(), theta, rtol=0, atol=5e-6)

    # C_edge_output2 = the last step's sess.run fetch (model_2.py:369-371): a host array of
    # the pre-update probabilities that later steps do not change
    fetched = m.C_edge_output2
    assert isinstance(fetched, np.ndarray) and fetched.shape == (mb, 2, nc * (nc - 1))
    P, sh = last
    o = model_ref.forward(model_ref.to_torch_params(P, requires_grad=False),
                          sh.x.astype(np.float64), sh.a, sh.y, sh.hid, sh.nlen, variant=v)
    np.testing.assert_allclose(fetched, o["probs"].detach().numpy().transpose(0, 2, 1), atol=1e-5)
    keep = fetched.copy()
    snap = m.engine.snapshot()
    db = m._device_batches(train, maps)[0]
    m.engine.train_step(db)                         # a later step overwrites engine.probs
    torch.cuda.synchronize()
    assert not torch.equal(m.engine.probs.cpu(), torch.from_numpy(keep))
    np.testing.assert_array_equal(m.C_edge_output2, keep)
    m.engine.restore(snap)                          # the checks below read the trained state

    res = tmp_path / "outputSelf" / "tiny" / ("model_%d" % v) / "2" / "result_2.npy"
    lines = res.read_text().splitlines()
    assert len(lines) == 2 and lines[0].startswith("Epoch 1 acc: ")
    ck = tmp_path / "ckpt" / "tiny" / ("model_%d" % v) / "2"
    assert (ck / "checkpoint").exists() and (ck / "g2g.model-3.index").exists()
    assert (ck / "g2g.model-3.data-00000-of-00001").exists()
    from hdgnn import tfckpt
    z = tfckpt.read(str(ck / "g2g.model-3"))
    first, shape = layout.specs(v)[0]
    np.testing.assert_array_equal(z[first.split(":")[0]].reshape(-1),
                                  m.engine.get_params()[:int(np.prod(shape))])
    # the epoch-1 bundle (written in the background while epoch 2 ran) holds epoch 1's state
    z1 = tfckpt.read(str(ck / "g2g.model-2"))
    np.testing.assert_allclose(z1[first.split(":")[0]].reshape(-1).astype(np.float64),
                               epoch_theta[0][:int(np.prod(shape))], rtol=0, atol=5e-6)
    assert not np.array_equal(z1[first.split(":")[0]], z[first.split(":")[0]])
    # resume: a fresh model restores weights, Adam slots and beta powers bit-exactly
    m2 = graph2graph(None, Ds=1, Ne=ne, Nc=nc, Ner=ne * (ne - 1), Ncr=nc * (nc - 1), Dr=2,
                     De_e=20, De_er=20, Mini_batch=mb, checkpoint_dir=args.checkpoint_dir,
                     epoch=2, Ds_inter=1, Dr_inter=2, Step=2, Repo="tiny",
                     reader=lambda model, step: tup, seed=99)
    m2._initialize()
    assert m2.load(args.checkpoint_dir)
    for a, b in ((m2.engine.params, m.engine.params), (m2.engine.m, m.engine.m),
                 (m2.engine.v, m.engine.v), (m2.engine.beta_pow, m.engine.beta_pow)):
        assert torch.equal(a, b)

    # test(): checkpoint looked up under checkpoint_dir/Repo/Repo/... (reference quirk)
    m.test(args)
    out = np.load(tmp_path / "outputSelf" / "tiny" / ("model_%d" % v) / "2" / "C_edge_t7.npy")
    assert out.shape == (50, 2, nc * (nc - 1))
    P0 = model_ref.unflatten(layout.init_flat(7, v).astype(np.float64), v)
    ref = []
    for j in range(2):
        sh = test.slice(j * mb, (j + 1) * mb).with_maps(maps)
        o = model_ref.forward(model_ref.to_torch_params(P0, requires_grad=False),
                              sh.x.astype(np.float64), sh.a, sh.y, sh.hid, sh.nlen, variant=v)
        ref.append(o["probs"].detach().numpy().transpose(0, 2, 1))
    np.testing.assert_allclose(out, np.concatenate(ref), atol=1e-5)


def test_graph2graph_fast_loader_equals_reference_loader(golden_dir, tmp_path, monkeypatch):
    """loader='fast' (hdgnn.loader on the dataset files) trains to the same weights and
    writes the same test outputs as the reference loader's 12-tuple."""
    from hdgnn.model import graph2graph
    from test_loader import _tree
    tup, meta = _tuple(golden_dir)
    z = np.load(os.path.join(golden_dir, "loader_tiny.npz"))
    ne, nc, mb = meta["Ne"], meta["Nc"], 25
    data_root = tmp_path / "data"
    data_root.mkdir()
    repo, step = _tree(str(data_root), z, meta)
    outs = {}
    for kind in ("utils2", "fast"):
        run = tmp_path / kind
        run.mkdir()
        monkeypatch.chdir(run)
        args = types.SimpleNamespace(Repo=repo, checkpoint_dir=str(run / "ckpt"))
        kw = dict(reader=lambda model, s: tup) if kind == "utils2" else dict(
            loader="fast", data_root=str(data_root))
        m = graph2graph(None, Ds=1, Ne=ne, Nc=nc, Ner=ne * (ne - 1), Ncr=nc * (nc - 1), Dr=2,
                        De_e=20, De_er=20, Mini_batch=mb, checkpoint_dir=args.checkpoint_dir,
                        epoch=2, Ds_inter=1, Dr_inter=2, Step=step, Repo=repo, seed=3, **kw)
        m.train(args)
        m.test(args)
        d = run / "outputSelf" / repo / "model_2" / str(step)
        outs[kind] = (m.engine.get_params(), np.load(d / ("C_edge_t%d.npy" % ne)),
                      np.load(d / ("C_edge_y%d.npy" % ne)))
    for a, b in zip(outs["utils2"], outs["fast"]):
        np.testing.assert_array_equal(a, b)
