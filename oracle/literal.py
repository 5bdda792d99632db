"""Literal incidence-matrix restatement of model_2 (TEST INFRASTRUCTURE ONLY).

Runs the reference graph op for op (model_2.py:86-130): one-hot incidence
tensors Es/Et (B,Ne,Ner), Cs/Ct (B,Nc,Ncr), Esc/Etc (B,Nc,Ner) and batched
matmuls / transposes / concats exactly as written, in torch on the CPU.  It
performs the same dense FLOPs as the TF1 CPU graph, so it is what bench.py
times as the CPU baseline ("kind": "port"), and the tests use it to check the
pair-explicit oracle (model_ref.py) at small sizes.
"""
import numpy as np
import torch

from .model_ref import pair_index, relation_maps


def build_dense(x, a, y, hid, nlen, dtype=torch.float32):
    """The 12-tuple tensors utils2.read_data feeds for one batch (utils2.py:50-137)."""
    x = np.asarray(x)
    Bsz, Ne = x.shape
    Nc = np.asarray(y).shape[1]
    I, J = pair_index(Ne)
    Ip, Jq = pair_index(Nc)
    ner, ncr = len(I), len(Ip)
    r = np.arange(ner)
    rc = np.arange(ncr)
    Es = torch.zeros(Bsz, Ne, ner, dtype=dtype)
    Et = torch.zeros(Bsz, Ne, ner, dtype=dtype)
    Es[:, I, r] = 1
    Et[:, J, r] = 1
    Cs = torch.zeros(Bsz, Nc, ncr, dtype=dtype)
    Ct = torch.zeros(Bsz, Nc, ncr, dtype=dtype)
    Cs[:, Ip, rc] = 1
    Ct[:, Jq, rc] = 1
    acls = np.asarray(a)[:, I, J].astype(np.int64)
    E_edge = torch.zeros(Bsz, 2, ner, dtype=dtype)
    E_edge.scatter_(1, torch.as_tensor(acls)[:, None, :], 1.0)
    ycls = np.asarray(y)[:, Ip, Jq].astype(np.int64)
    C_edge = torch.zeros(Bsz, 2, ncr, dtype=dtype)
    C_edge.scatter_(1, torch.as_tensor(ycls)[:, None, :], 1.0)
    s, t = relation_maps(hid, nlen, Ne, Nc)
    Esc = torch.zeros(Bsz, Nc, ner, dtype=dtype)
    Etc = torch.zeros(Bsz, Nc, ner, dtype=dtype)
    bb, rr = np.nonzero(s >= 0)
    Esc[bb, s[bb, rr], rr] = 1
    bb, rr = np.nonzero(t >= 0)
    Etc[bb, t[bb, rr], rr] = 1
    E_node = torch.as_tensor(x, dtype=dtype)[:, None, :]
    return dict(E_node=E_node, E_edge=E_edge, C_edge=C_edge, Es=Es, Et=Et, Cs=Cs,
                Ct=Ct, Esc=Esc, Etc=Etc)


def forward(P, D, Bsz, Ne, Nc):
    """model_2 build_model, literally.  P: short-key -> tensor, D: build_dense()."""
    Ner, Ncr = Ne * (Ne - 1), Nc * (Nc - 1)
    Es, Et, E_edge = D["Es"], D["Et"], D["E_edge"]
    O = D["E_node"]

    def marshalling_B1(O, E_edge):                                          # 141-144
        return torch.cat([O @ Es, O @ Et, E_edge], 1)

    B_1 = marshalling_B1(O, E_edge)                                          # (B,4,Ner)
    Bt = B_1.transpose(1, 2).reshape(Bsz * Ner, 4)                           # 164-165
    h1 = torch.relu(Bt @ P["E1.w1"] + P["E1.b1"])                            # 170
    h5 = (h1 @ P["E1.w5"] + P["E1.b5"]).reshape(Bsz, Ner, 20).transpose(1, 2)  # 175-178
    E_bar = h5 @ Es.transpose(1, 2) + h5 @ Et.transpose(1, 2)               # 186
    Cc = torch.cat([O, E_bar], 1).transpose(1, 2).reshape(Bsz * Ne, 21)      # 188, 193-194
    hh = torch.relu(Cc @ P["E3.w1"] + P["E3.b1"])                            # 199
    O2 = torch.relu(hh @ P["E3.w2"] + P["E3.b2"]).reshape(Bsz, Ne, 1).transpose(1, 2)  # 202-204
    B_2 = marshalling_B1(O2, E_edge)                                         # 94
    # marshalling_B2 (146-159)
    B_t = B_2.transpose(1, 2)
    neighbors = D["Esc"] @ B_t + D["Etc"] @ B_t                              # (B,Nc,4)
    Cs_t, Ct_t = D["Cs"].transpose(1, 2), D["Ct"].transpose(1, 2)
    B_3 = torch.cat([(Cs_t @ neighbors).transpose(1, 2),
                     (Ct_t @ neighbors).transpose(1, 2), D["C_edge"]], 1)   # (B,10,Ncr)
    # mlp_hunk_B2 (245-277)
    Bh = B_3.transpose(1, 2).reshape(Bsz * Ncr, 10)
    g1 = torch.relu(Bh @ P["H1.w1"] + P["H1.b1"])
    g2 = (g1 @ P["H1.w2"] + P["H1.b2"]).reshape(Bsz, Ncr, 20).transpose(1, 2)
    bar1 = g2 @ D["Cs"].transpose(1, 2)
    bar2 = g2 @ D["Ct"].transpose(1, 2)
    effects = bar1 @ D["Cs"] + bar2 @ D["Ct"]                                # (B,20,Ncr)
    HR = torch.cat([D["C_edge"], effects], 1)                                # 280
    He = HR.transpose(1, 2).reshape(Bsz * Ncr, 22)                           # 307-308
    k1 = torch.relu(He @ P["H2.w1"] + P["H2.b1"])
    logits = (k1 @ P["H2.w2"] + P["H2.b2"]).reshape(Bsz, Ncr, 2).transpose(1, 2)  # (B,2,Ncr)
    probs = torch.softmax(logits, 1)
    ce = (-(D["C_edge"] * torch.log_softmax(logits, 1)).sum(1)).mean()       # 115-118
    th1, th2 = P["th1"].reshape(2), P["th2"].reshape(2)
    loss_map = 0.01 * (torch.sqrt(2 * (0.5 * (th2 ** 2).sum()))
                       + torch.sqrt((0.5 * (th1 ** 2).sum()) * 2))
    loss_para = sum(0.001 * 0.5 * (v ** 2).sum() for v in P.values())
    total = 10 * ce + 0.1 * loss_map + loss_para
    return dict(logits=logits, probs=probs, ce=ce, loss_map=loss_map,
                loss_para=loss_para, total=total)
