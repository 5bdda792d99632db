"""Pair-explicit torch-CPU restatement of graph2graph (TEST INFRASTRUCTURE ONLY).

Every stage evaluates the reference MLPs on every relation exactly as the TF
graph does (no algebraic hoisting), but replaces the one-hot incidence
matmuls (Es/Et/Cs/Ct/Esc/Etc) by the index gathers / index_add scatters they
are equivalent to.  ``literal.py`` keeps the incidence matmuls; the test-suite
checks the two against each other.  Gradients: torch.autograd.  Default dtype
float64 so the oracle's own rounding is far below the fp32 tolerances.

Input contract (compact form, see loader_ref.py):
    x    (B, Ne)      float  node attribute  = E_node[:, 0, :]       (utils2.py:29-36)
    a    (B, Ne, Ne)  int    entity edge class, off-diagonal         (utils2.py:46, 82)
    y    (B, Nc, Nc)  int    hunk edge class (label AND input)       (utils2.py:47, 105)
    hid  (B, Ne)      int    hunk row of index line i' (-1: 'null' / >= Nc / absent)
    nlen (B,)         int    n = len(readlines()[:Ne])               (utils2.py:121-137)
"""
import math

import numpy as np
import torch

from . import layout


# ----------------------------------------------------------------------------
# relation enumeration
# ----------------------------------------------------------------------------
def pair_index(n):
    """(I, J) of the r-th relation of an n-node complete digraph, row-major over
    i with j != i -- the order utils2 fills Es/Et (utils2.py:64-83), Cs/Ct
    (86-106) and Esc/Etc (123-137)."""
    if n < 2:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    r = np.arange(n * (n - 1), dtype=np.int64)
    i = r // (n - 1)
    jj = r % (n - 1)
    j = jj + (jj >= i)
    return i, j


def relation_maps(hid, nlen, ne, nc):
    """Per-relation source/target hunk rows s_r, t_r (B, Ne(Ne-1)), -1 = none.

    utils2.py:123-137: relation counter cnt2 walks the n-grid (n = nlen[b]),
    which is misaligned with the Ne-grid whenever n < Ne; relations with
    cnt2 >= n(n-1) have no hunk.
    """
    hid = np.asarray(hid)
    nlen = np.asarray(nlen)
    B = hid.shape[0]
    pe = ne * (ne - 1)
    s = np.full((B, pe), -1, np.int64)
    t = np.full((B, pe), -1, np.int64)
    for b in range(B):
        n = int(nlen[b])
        if n < 2:
            continue
        ii, jj = pair_index(n)
        m = n * (n - 1)
        s[b, :m] = hid[b, ii]
        t[b, :m] = hid[b, jj]
    s[s >= nc] = -1
    t[t >= nc] = -1
    return s, t


# ----------------------------------------------------------------------------
# parameters
# ----------------------------------------------------------------------------
def truncated_normal(rng, shape, stddev=0.1):
    """tf.truncated_normal: N(0, stddev) re-drawn outside 2 stddev."""
    out = rng.standard_normal(shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * stddev).astype(np.float32)


def init_params(seed=0, variant=2):
    """Reference initialisers (truncated_normal(0.1) weights & thetas, zero
    biases: model_2.py:167-173, 196-201, 257-264, 311-319, 329-330)."""
    rng = np.random.default_rng(seed)
    biases = {"r1_b1o", "r1_b5o", "o1_b1o", "o1_b2o", "r1_b1r", "r1_b2r", "o1_b1r",
              "o1_b2r", "b1", "b2", "C_edge_b1"}
    out = {}
    for key, name, shape in layout.keyed_specs(variant):
        if name.split("/")[-1] in biases:
            out[key] = np.zeros(shape, np.float32)
        else:
            out[key] = truncated_normal(rng, shape)
    return out


def flatten(params, variant=2):
    return np.concatenate([np.asarray(params[k], np.float32).reshape(-1)
                           for k, _, _ in layout.keyed_specs(variant)])


def unflatten(vec, variant=2):
    out, o = {}, 0
    for k, _, shape in layout.keyed_specs(variant):
        n = int(np.prod(shape))
        out[k] = np.asarray(vec[o:o + n]).reshape(shape)
        o += n
    assert o == len(vec)
    return out


# ----------------------------------------------------------------------------
# forward
# ----------------------------------------------------------------------------
def _mlp_pair_entity(P, B1):
    """mlp_entity_B1 (model_2.py:161-179): relu(B@w1+b1)@w5+b5, no output relu."""
    h1 = torch.relu(B1 @ P["E1.w1"] + P["E1.b1"])
    return h1 @ P["E1.w5"] + P["E1.b5"]


def _row_col_sum(vals, I, J, n):
    """(V Es^T) + (V Et^T) restated: per node, sum over relations whose source
    is the node plus relations whose target is the node (model_2.py:186)."""
    Bsz, _, D = vals.shape
    out = torch.zeros(Bsz, n, D, dtype=vals.dtype)
    out.index_add_(1, torch.as_tensor(I), vals)
    out.index_add_(1, torch.as_tensor(J), vals)
    return out


def _row_sum(vals, I, n):
    Bsz, _, D = vals.shape
    out = torch.zeros(Bsz, n, D, dtype=vals.dtype)
    out.index_add_(1, torch.as_tensor(I), vals)
    return out


def forward(P, x, a, y, hid, nlen, variant=2, dtype=torch.float64):
    """Returns dict(logits (B,Pc,2), probs, ce, loss_map, loss_para, total, theta).

    P: dict short_key -> torch tensor (leaf, requires_grad for gradients).
    """
    x = torch.as_tensor(np.asarray(x), dtype=dtype)
    a = np.asarray(a)
    y = np.asarray(y)
    Bsz, Ne = x.shape
    Nc = y.shape[1]
    I, J = pair_index(Ne)
    Ip, Jq = pair_index(Nc)
    tI, tJ = torch.as_tensor(I), torch.as_tensor(J)
    tIp, tJq = torch.as_tensor(Ip), torch.as_tensor(Jq)

    # E_edge one-hot per relation (utils2.py:82): class = a_ij
    acls = torch.as_tensor(a[:, I, J].astype(np.int64))
    E_edge = torch.stack([(acls == 0), (acls == 1)], -1).to(dtype)        # (B, Pe, 2)
    ycls = torch.as_tensor(y[:, Ip, Jq].astype(np.int64))
    C_edge = torch.stack([(ycls == 0), (ycls == 1)], -1).to(dtype)        # (B, Pc, 2)

    # marshalling_B1 (model_2.py:141-144): [O.Es, O.Et, E_edge]
    B1 = torch.cat([x[:, tI, None], x[:, tJ, None], E_edge], -1)          # (B, Pe, 4)

    if variant in (2, 4):
        # mlp_entity_B1 -> agg_entity_B1 -> mlp2_entity_B1 (model_2.py:89-91)
        e = _mlp_pair_entity(P, B1)                                        # (B, Pe, 20)
        Ebar = _row_col_sum(e, I, J, Ne)                                   # (B, Ne, 20)
        Cin = torch.cat([x[..., None], Ebar], -1)                          # concat [O, E_bar] (188)
        h = torch.relu(Cin @ P["E3.w1"] + P["E3.b1"])
        xp = torch.relu(h @ P["E3.w2"] + P["E3.b2"])[..., 0]              # relu on output (202)
    else:
        xp = None

    E_edge2 = E_edge
    if variant in (3, 4):
        # mlp_entityedge_B1 (model_4.py:206-243): shared w1 = [w1_1; w1_1; w1_2]
        w1 = torch.cat([P["EE.w11"], P["EE.w11"], P["EE.w12"]], 0)
        k1 = torch.relu(B1 @ w1 + P["EE.b1"])
        k2 = k1 @ P["EE.w2"] + P["EE.b2"]                                  # (B, Pe, 20)
        Srow = _row_sum(k2, I, Ne)                                         # h2 Es^T
        Tcol = _row_sum(k2, J, Ne)                                         # h2 Et^T
        eff = Srow[:, tI] + Tcol[:, tJ]                                    # (.)Es + (.)Et
        # agg_entityedge_B1 (282-284): concat [E_edge, effects]
        CR = torch.cat([E_edge, eff], -1)
        # mlp2_entityedge_B1 (286-304)
        zl = torch.relu(CR @ P["EC.w1"] + P["EC.b1"]) @ P["EC.w2"] + P["EC.b2"]
        probs_e = torch.softmax(zl, -1)
        if variant == 4:
            E_edge2 = probs_e                                              # model_4.py:97

    if variant == 1 or variant == 3:
        B2 = B1                                                            # model_1.py:76 / model_3.py:97
    else:
        B2 = torch.cat([xp[:, tI, None], xp[:, tJ, None], E_edge2], -1)   # model_2.py:94

    # marshalling_B2 (model_2.py:146-159): n_c = sum_r (Esc[c,r]+Etc[c,r]) B2_r
    s, t = relation_maps(hid, nlen, Ne, Nc)
    nbr = torch.zeros(Bsz * (Nc + 1), 4, dtype=dtype)
    B2f = B2.reshape(Bsz * len(I), 4)
    base = (np.arange(Bsz)[:, None] * (Nc + 1))
    sidx = torch.as_tensor((base + np.where(s < 0, Nc, s)).reshape(-1))
    tidx = torch.as_tensor((base + np.where(t < 0, Nc, t)).reshape(-1))
    nbr = nbr.index_add(0, sidx, B2f).index_add(0, tidx, B2f)
    nbr = nbr.reshape(Bsz, Nc + 1, 4)[:, :Nc]                              # (B, Nc, 4)
    B3 = torch.cat([nbr[:, tIp], nbr[:, tJq], C_edge], -1)                # (B, Pc, 10)

    # mlp_hunk_B2 (model_2.py:245-277)
    g = torch.relu(B3 @ P["H1.w1"] + P["H1.b1"]) @ P["H1.w2"] + P["H1.b2"]
    S = _row_sum(g, Ip, Nc)                                                # (g Cs^T)
    T = _row_sum(g, Jq, Nc)                                                # (g Ct^T)
    eff_h = S[:, tIp] + T[:, tJq]                                          # (.)Cs + (.)Ct (275)

    # agg_edge_B1 (279-281): labels first
    HR = torch.cat([C_edge, eff_h], -1)                                    # (B, Pc, 22)
    # mlp_hunkedge_B2 (304-324)
    logits = torch.relu(HR @ P["H2.w1"] + P["H2.b1"]) @ P["H2.w2"] + P["H2.b2"]
    probs = torch.softmax(logits, -1)

    # losses (model_2.py:115-130, 326-333)
    ce = (-(C_edge * torch.log_softmax(logits, -1)).sum(-1)).mean()
    th1 = P["th1"].reshape(2)
    th2 = P["th2"].reshape(2)
    loss_map = 0.01 * (torch.sqrt(2 * (0.5 * (th2 * th2).sum()))
                       + torch.sqrt((0.5 * (th1 * th1).sum()) * 2))
    loss_para = 0
    for k, _, _ in layout.keyed_specs(variant):
        loss_para = loss_para + 0.001 * (0.5 * (P[k] * P[k]).sum())
    total = 10 * ce + 0.1 * loss_map + loss_para                           # model_2.py:336
    # loss_E_HR = 0.001 * l2_loss(C_edge_output) (model_2.py:122): computed, never fetched
    loss_E_HR = 0.001 * 0.5 * (eff_h * eff_h).sum()
    return dict(logits=logits, probs=probs, ce=ce, loss_map=loss_map,
                loss_para=loss_para, total=total, theta=P["th2"], xp=xp, nbr=nbr,
                loss_E_HR=loss_E_HR)


def to_torch_params(params, dtype=torch.float64, requires_grad=True):
    return {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=requires_grad)
            for k, v in params.items()}


def loss_and_grads(params, x, a, y, hid, nlen, variant=2, dtype=torch.float64):
    """Forward + autograd backward of train_loss; returns (out, grads dict numpy)."""
    P = to_torch_params(params, dtype)
    out = forward(P, x, a, y, hid, nlen, variant, dtype)
    out["total"].backward()
    grads = {k: P[k].grad.detach().numpy().copy() for k in P}
    det = {k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in out.items()
           if v is not None}
    return det, grads


# ----------------------------------------------------------------------------
# TF1 Adam (tf.train.AdamOptimizer(0.0003), model_2.py:337)
# ----------------------------------------------------------------------------
class AdamTF:
    """Restates TF1 ApplyAdam:  lr_t = lr*sqrt(1-b2^t)/(1-b1^t);
    m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  var -= lr_t m / (sqrt(v) + eps).
    beta powers are float32 variables in TF (initialised to b1, b2 and
    multiplied after every apply); emulated in float32 here."""

    def __init__(self, n, lr=3e-4, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps
        self.m = np.zeros(n, np.float64)
        self.v = np.zeros(n, np.float64)
        self.b1p = np.float32(b1)
        self.b2p = np.float32(b2)

    def step(self, theta, g):
        lr_t = self.lr * math.sqrt(1 - float(self.b2p)) / (1 - float(self.b1p))
        self.m = self.b1 * self.m + (1 - self.b1) * g
        self.v = self.b2 * self.v + (1 - self.b2) * g * g
        theta = theta - lr_t * self.m / (np.sqrt(self.v) + self.eps)
        self.b1p = np.float32(self.b1p * np.float32(self.b1))
        self.b2p = np.float32(self.b2p * np.float32(self.b2))
        return theta
