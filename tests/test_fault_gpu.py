"""Failure path of the fused kernel's split mode (two blocks per commit exchanging partial
sums through tagged write-through words, csrc/hdgnn.hip pair_send / pair_recv_add).

A pair whose partner never arrives must fail loudly and leave the model untouched:
  * the sticky status word gets HDG_STATUS_XCH_TIMEOUT and Engine.check_status() raises;
  * forward-only launches poison the CE sum and the timed-out block's probs / logits rows;
  * training launches poison the CE, set the gradient trailer's fault slot and skip the
    Adam update (parameters, moments and beta powers bitwise unchanged), on the fused
    single-process path (k_reduce_adam; model_4: kw_reduce_adam) and on the
    data-parallel split (k_adam_tf);
  * the next clean launch is correct again (exchange tags are per launch epoch).
HDG_DEBUG_XCH_FAULT=1 makes block 1 of every pair send words its partner never accepts,
so block 0 (the even hunk rows) waits out every exchange (~20 ms each).  GPU only.
"""
import numpy as np
import pytest
import torch

from hdgnn import _lib, layout
from hdgnn.synth import synth_commits

pytestmark = pytest.mark.gpu

B, NE, NC = 3, 40, 17


@pytest.fixture(params=[2, 4], ids=["model_2", "model_4"])
def fused_split(monkeypatch, request):
    """model_4 runs its model_2-shaped part in the same step kernel (the entity-edge stage
    on general-path kernels around it, the reduction + Adam in kw_reduce_adam)."""
    monkeypatch.setenv("HDG_FUSED_SPLIT", "1")
    from hdgnn.engine import Engine
    v = request.param
    eng = Engine(NE, NC, B, variant=v, path=_lib.PATH_FUSED)
    eng.set_params(layout.init_flat(5, v))
    return eng, eng.upload(synth_commits(B, NE, NC, 7))


def _state(eng):
    return [t.clone() for t in (eng.params, eng.m, eng.v, eng.beta_pow)]


def _even_rows(a):
    """[B][2][Pc] -> the relations of hunk rows p = 0, 2, 4, ... (block 0's rows)."""
    r = a.reshape(a.shape[0], 2, NC, NC - 1)
    return r[:, :, 0::2], r[:, :, 1::2]


def test_forward_timeout_poisons_outputs(fused_split, monkeypatch):
    eng, db = fused_split
    probs, logits, ce = eng.forward(db)
    torch.cuda.synchronize()
    eng.check_status()
    good = probs.cpu().numpy().copy()
    monkeypatch.setenv("HDG_DEBUG_XCH_FAULT", "1")
    eng.probs.zero_()
    eng.logits.zero_()
    eng.forward(db)
    torch.cuda.synchronize()
    assert int(eng.status.item()) == _lib.STATUS_XCH_TIMEOUT
    with pytest.raises(RuntimeError, match="exchange"):
        eng.check_status()
    assert np.isnan(eng.ce_sum.item())
    ev, _ = _even_rows(eng.probs.cpu().numpy())    # block 1's rows are void too (built
    assert np.isnan(ev).all()                       # from its partner's bad partials)
    lev, _ = _even_rows(eng.logits.cpu().numpy())
    assert np.isnan(lev).all()
    # recovery: the next clean launch is exact again, status stays sticky until cleared
    monkeypatch.delenv("HDG_DEBUG_XCH_FAULT")
    eng.forward(db)
    torch.cuda.synchronize()
    assert int(eng.status.item()) == _lib.STATUS_XCH_TIMEOUT
    eng.clear_status()
    assert np.array_equal(eng.probs.cpu().numpy(), good)
    eng.check_status()


def test_train_timeout_skips_update(fused_split, monkeypatch):
    eng, db = fused_split
    before = _state(eng)
    monkeypatch.setenv("HDG_DEBUG_XCH_FAULT", "1")
    eng.train_step(db)                      # hdg_train_step: k_reduce_adam / kw_reduce_adam
    torch.cuda.synchronize()
    for a, b in zip(before, _state(eng)):
        assert torch.equal(a, b)
    tr = eng.grad[eng.np:].cpu().numpy()
    assert np.isnan(tr[_lib.TR_CE])
    # block 0 of every pair timed out; block 1 may too (block 0 sends each later exchange
    # ~20 ms late, after its own wait)
    assert B <= tr[_lib.TR_FAULT] <= 2 * B
    assert np.isnan(eng.stats[0].item())
    with pytest.raises(RuntimeError):
        eng.check_status()
    # the data-parallel decomposition (fwd_bwd -> all-reduce -> hdg_adam_tf) skips too
    eng.clear_status()
    eng.fwd_bwd(db)
    eng.adam()
    torch.cuda.synchronize()
    for a, b in zip(before, _state(eng)):
        assert torch.equal(a, b)
    assert int(eng.status.item()) == _lib.STATUS_XCH_TIMEOUT
    # clean again: the step equals a fresh engine's first step
    monkeypatch.delenv("HDG_DEBUG_XCH_FAULT")
    eng.clear_status()
    eng.train_step(db)
    torch.cuda.synchronize()
    eng.check_status()
    from hdgnn.engine import Engine
    ref = Engine(NE, NC, B, variant=eng.variant, path=_lib.PATH_FUSED)
    ref.set_params(layout.init_flat(5, eng.variant))
    ref.train_step(ref.upload(synth_commits(B, NE, NC, 7)))
    torch.cuda.synchronize()
    assert torch.equal(eng.params, ref.params)
    assert eng.grad[eng.np + _lib.TR_FAULT].item() == 0.0


def test_count_beyond_fp32_integer_range():
    """top_ACC numerator past 2^24 (B * Nc (Nc - 1) = 19.3 M relations; the classifier
    reduced to its output bias, so every relation predicts class 0 and the ~90 % with
    label 0 are correct): exact through the integer trailer parts (it used
    to be one fp32 slot)."""
    from hdgnn import metrics
    from hdgnn.data import onehot_relations
    from hdgnn.engine import Engine
    b, ne, nc = 16, 40, 1100
    cb = synth_commits(b, ne, nc, 11)
    eng = Engine(ne, nc, b, variant=2, path=_lib.PATH_GENERAL)
    flat = layout.init_flat(3)
    offs = layout.offsets(2)
    for name in ("phi_U_R1/C_edge_w1:0", "phi_U_R1/o1_w2r:0"):
        o, shp = offs[name]
        flat[o:o + int(np.prod(shp))] = 0.0
    off = offs["phi_U_R1/o1_b2r:0"][0]                   # classifier output bias
    flat[off], flat[off + 1] = 3.0, -3.0
    eng.set_params(flat)
    eng.fwd_bwd(eng.upload(cb))
    torch.cuda.synchronize()
    want = metrics.top_acc_count(onehot_relations(cb.y), eng.probs.cpu().numpy())
    assert want > 2 ** 24
    assert eng.correct_count() == want


def test_train_timeout_retried_in_one_block_mode(fused_split, monkeypatch):
    """Engine.train_step_checked: the faulted split step (update skipped) is re-run with one
    block per commit (HDG_FLAG_NO_SPLIT) and the run stays there; the result equals a
    clean one-block step.  HDG_DEBUG_XCH_FAULT only corrupts split-mode exchanges."""
    eng, db = fused_split
    monkeypatch.setenv("HDG_DEBUG_XCH_FAULT", "1")
    with pytest.warns(RuntimeWarning, match="one-block"):
        eng.train_step_checked(db)
    assert not eng.split and int(eng.status.item()) == 0
    eng.train_step_checked(db)                 # stays in one-block mode: no new fault
    torch.cuda.synchronize()
    monkeypatch.delenv("HDG_DEBUG_XCH_FAULT")
    from hdgnn.engine import Engine
    ref = Engine(NE, NC, B, variant=eng.variant, path=_lib.PATH_FUSED)
    ref.set_split(False)
    ref.set_params(layout.init_flat(5, eng.variant))
    rdb = ref.upload(synth_commits(B, NE, NC, 7))
    ref.train_step(rdb)
    ref.train_step(rdb)
    torch.cuda.synchronize()
    assert torch.equal(eng.params, ref.params)
    assert torch.equal(eng.m, ref.m) and torch.equal(eng.beta_pow, ref.beta_pow)


def test_model_train_epoch_retry(monkeypatch, tmp_path):
    """graph2graph.train re-runs a faulted epoch from its starting state in one-block mode
    (the losses it prints and the parameters equal a clean one-block run)."""
    from hdgnn.model import graph2graph
    monkeypatch.setenv("HDG_FUSED_SPLIT", "1")
    monkeypatch.chdir(tmp_path)
    cb = synth_commits(2 * B, NE, NC, 9)
    tr, te = cb.slice(0, B), cb.slice(B, 2 * B)

    class Args:
        checkpoint_dir, Repo = str(tmp_path / "ck"), "glide"

    def run(fault, split):
        if fault:
            monkeypatch.setenv("HDG_DEBUG_XCH_FAULT", "1")
        else:
            monkeypatch.delenv("HDG_DEBUG_XCH_FAULT", raising=False)
        m = graph2graph(None, 1, NE, NC, NE * (NE - 1), NC * (NC - 1), 2, 20, 20, B,
                        Args.checkpoint_dir, 2, 1, 2, 2, "glide", compact=(tr, te, tr))
        m.engine.set_split(split)
        m.train(Args)
        return m

    with pytest.warns(RuntimeWarning, match="one-block"):
        got = run(True, True)
    want = run(False, False)
    assert not got.engine.split
    assert torch.equal(got.engine.params, want.engine.params)
    assert got.loss_Hedge_mse == want.loss_Hedge_mse


def test_model_train_late_fault_polls_and_retries(monkeypatch, tmp_path, capsys):
    """The two paths of graph2graph.train's pipelined loop that a fault in epoch 0 never
    reaches: a split-mode fault that starts inside epoch 1 of a many-step epoch
    while epoch 2 is already queued.  The fault poll (every FAULT_POLL steps, lagged one
    poll) stops the faulted epoch early, the host retries epoch 1 from the state after
    epoch 0 in one-block mode and drops the stale epoch 2.  Parameters, Adam state, printed
    lines, result file and every checkpoint equal a clean run that leaves split mode at
    the same step boundary (epoch 0 split, epochs 1-2 one block per commit)."""
    import hdgnn.model as hm
    from hdgnn.engine import Engine
    monkeypatch.setenv("HDG_FUSED_SPLIT", "1")
    monkeypatch.setattr(hm, "FAULT_POLL", 4)
    nb, epochs, mb = 12, 3, B                 # polls at steps 4 and 8 of every epoch
    cb = synth_commits(nb * mb + mb, NE, NC, 13)
    tr, te = cb.slice(0, nb * mb), cb.slice(nb * mb, nb * mb + mb)
    orig = Engine.step_call

    def run(tag, fault_from=None, one_block_from=None):
        monkeypatch.delenv("HDG_DEBUG_XCH_FAULT", raising=False)
        count = {"n": 0}

        def step_call(self, *a, **k):       # enqueue-order hook: the host's step counter
            call = orig(self, *a, **k)

            def step():
                n = count["n"]
                if fault_from is not None and n == fault_from:
                    monkeypatch.setenv("HDG_DEBUG_XCH_FAULT", "1")
                if one_block_from is not None and n == one_block_from:
                    self.set_split(False)
                count["n"] += 1
                return call()
            return step

        monkeypatch.setattr(Engine, "step_call", step_call)
        d = tmp_path / tag
        d.mkdir()
        monkeypatch.chdir(d)

        class Args:
            checkpoint_dir, Repo = str(d / "ck"), "glide"

        m = hm.graph2graph(None, 1, NE, NC, NE * (NE - 1), NC * (NC - 1), 2, 20, 20, mb,
                           Args.checkpoint_dir, epochs, 1, 2, 2, "glide", compact=(tr, te, tr))
        m.train(Args)
        monkeypatch.setattr(Engine, "step_call", orig)
        out = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Epoch")]
        return m, d, out, count["n"]

    with pytest.warns(RuntimeWarning, match="one-block"):
        got, gd, gout, gsteps = run("fault", fault_from=nb + 2)
    want, wd, wout, wsteps = run("clean", one_block_from=nb)
    assert not got.engine.split and not want.engine.split
    # the faulted epoch 1 stopped at its second poll (step 8), epoch 2's stale launch too,
    # then epochs 1 and 2 ran again in full: fewer steps than 3 full epochs twice over
    assert gsteps == nb + 8 + 8 + 2 * nb, gsteps
    assert wsteps == epochs * nb
    assert torch.equal(got.engine.state, want.engine.state)       # params, m, v, beta powers
    assert gout == wout and len(gout) == epochs
    rel = "outputSelf/glide/model_2/2/result_2.npy"
    assert (gd / rel).read_bytes() == (wd / rel).read_bytes()
    ck = "ck/glide/model_2/2"
    names = sorted(p.name for p in (wd / ck).iterdir())
    assert names == sorted(p.name for p in (gd / ck).iterdir()) and len(names) > 3
    for n in names:
        if n != "checkpoint":
            assert (gd / ck / n).read_bytes() == (wd / ck / n).read_bytes(), n
