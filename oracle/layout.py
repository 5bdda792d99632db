"""Variable layout of the reference graphs (TEST INFRASTRUCTURE ONLY).

Order = tf.global_variables() creation order inside build_model, weights are
(in, out) as TF's ``x @ W``.  Shapes follow the defaults Ds=1, Dr=2,
De_e=De_er=20, h_size=20, map_loss(k=2).

model_2.py:161-179 (phi_E_O1), 190-205 (phi_U_O1), 245-277 (mlp_hunk_B2),
304-324 (phi_U_R1), 326-333 (map_conv); model_4.py:206-243 / 286-304 add the
entity-edge blocks (phi_E_R1 / phi_U_R1).
"""

E1 = [("phi_E_O1/r1_w1o", (4, 20)), ("phi_E_O1/r1_b1o", (20,)),
      ("phi_E_O1/r1_w5o", (20, 20)), ("phi_E_O1/r1_b5o", (20,))]
E3 = [("phi_U_O1/o1_w1o", (21, 20)), ("phi_U_O1/o1_b1o", (20,)),
      ("phi_U_O1/o1_w2o", (20, 1)), ("phi_U_O1/o1_b2o", (1,))]
EE = [("phi_E_R1/r1_w1r1", (1, 20)), ("phi_E_R1/r1_w1r2", (2, 20)),
      ("phi_E_R1/r1_b1r", (20,)), ("phi_E_R1/r1_w2r", (20, 20)),
      ("phi_E_R1/r1_b2r", (20,))]
EC = [("phi_U_R1/o1_w1r", (22, 20)), ("phi_U_R1/o1_b1r", (20,)),
      ("phi_U_R1/o1_w2r", (20, 2)), ("phi_U_R1/o1_b2r", (2,))]
H1 = [("mlp_hunk_B2/w1", (10, 20)), ("mlp_hunk_B2/b1", (20,)),
      ("mlp_hunk_B2/r1_w2r", (20, 20)), ("mlp_hunk_B2/b2", (20,))]


def _h2(scope):
    return [(scope + "/C_edge_w1", (22, 20)), (scope + "/C_edge_b1", (20,)),
            (scope + "/o1_w2r", (20, 2)), (scope + "/o1_b2r", (2,))]


TH = [("map_conv/map_theta1", (1, 2, 1, 1)), ("map_conv/map_theta2", (1, 2, 1, 1))]

# TF uniquifies the re-entered "phi_U_R1" scope as phi_U_R1_1 when the
# entity-edge classifier already opened it (model_3 / model_4).
VARIANTS = {
    1: H1 + _h2("phi_U_R1") + TH,                       # HD-GNN/ES  (model_1.py)
    2: E1 + E3 + H1 + _h2("phi_U_R1") + TH,             # HD-GNN/S   (model_2.py)
    3: EE + EC + H1 + _h2("phi_U_R1_1") + TH,           # HD-GNN/E   (model_3.py)
    4: E1 + E3 + EE + EC + H1 + _h2("phi_U_R1_1") + TH,  # HD-GNN     (model_4.py)
}


def specs(variant=2):
    return list(VARIANTS[variant])


def short(name):
    """Scope-free key used by the restatements ('phi_E_O1/r1_w1o' -> 'E1.w1')."""
    return _SHORT[name]


_SHORT = {
    "phi_E_O1/r1_w1o": "E1.w1", "phi_E_O1/r1_b1o": "E1.b1",
    "phi_E_O1/r1_w5o": "E1.w5", "phi_E_O1/r1_b5o": "E1.b5",
    "phi_U_O1/o1_w1o": "E3.w1", "phi_U_O1/o1_b1o": "E3.b1",
    "phi_U_O1/o1_w2o": "E3.w2", "phi_U_O1/o1_b2o": "E3.b2",
    "phi_E_R1/r1_w1r1": "EE.w11", "phi_E_R1/r1_w1r2": "EE.w12",
    "phi_E_R1/r1_b1r": "EE.b1", "phi_E_R1/r1_w2r": "EE.w2", "phi_E_R1/r1_b2r": "EE.b2",
    "phi_U_R1/o1_w1r": "EC.w1", "phi_U_R1/o1_b1r": "EC.b1",
    "phi_U_R1/o1_w2r": "EC.w2", "phi_U_R1/o1_b2r": "EC.b2",
    "mlp_hunk_B2/w1": "H1.w1", "mlp_hunk_B2/b1": "H1.b1",
    "mlp_hunk_B2/r1_w2r": "H1.w2", "mlp_hunk_B2/b2": "H1.b2",
    "phi_U_R1/C_edge_w1": "H2.w1", "phi_U_R1/C_edge_b1": "H2.b1",
    "phi_U_R1/o1_w2r#H2": "H2.w2", "phi_U_R1/o1_b2r#H2": "H2.b2",
    "phi_U_R1_1/C_edge_w1": "H2.w1", "phi_U_R1_1/C_edge_b1": "H2.b1",
    "phi_U_R1_1/o1_w2r": "H2.w2", "phi_U_R1_1/o1_b2r": "H2.b2",
    "map_conv/map_theta1": "th1", "map_conv/map_theta2": "th2",
}


def keyed_specs(variant=2):
    """[(short_key, tf_name, shape)] in creation order.

    In model_2 the hunk classifier's o1_w2r/o1_b2r live in scope phi_U_R1 (no
    entity-edge classifier exists there), so the two names are disambiguated
    by position: the last phi_U_R1/o1_* pair always belongs to H2.
    """
    out = []
    sp = specs(variant)
    n_ec = sum(1 for n, _ in sp if n.startswith("phi_U_R1/o1_w2r"))
    seen = 0
    for name, shape in sp:
        key = name
        if name in ("phi_U_R1/o1_w2r", "phi_U_R1/o1_b2r"):
            if name.endswith("w2r"):
                seen += 1
            is_h2 = (variant in (1, 2)) or (n_ec == 2 and seen == 2)
            key = name + "#H2" if is_h2 else name
        out.append((_SHORT[key], name, shape))
    return out


def n_params(variant=2):
    tot = 0
    for _, shape in specs(variant):
        k = 1
        for s in shape:
            k *= s
        tot += k
    return tot
