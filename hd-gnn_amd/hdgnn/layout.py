"""Flat parameter layout of the engine (tf.global_variables order, (in,out) weights).

model_2.py:161-179 phi_E_O1, 190-205 phi_U_O1, 245-277 mlp_hunk_B2, 304-324 phi_U_R1,
326-333 map_conv; model_4.py:206-243 phi_E_R1, 286-304 phi_U_R1 (entity-edge blocks).
Offsets match hdg::param_offsets in csrc/hdgnn.hip (and m2:: for model_2).
"""
import numpy as np

_E1 = [("phi_E_O1/r1_w1o:0", (4, 20)), ("phi_E_O1/r1_b1o:0", (20,)),
       ("phi_E_O1/r1_w5o:0", (20, 20)), ("phi_E_O1/r1_b5o:0", (20,))]
_E3 = [("phi_U_O1/o1_w1o:0", (21, 20)), ("phi_U_O1/o1_b1o:0", (20,)),
       ("phi_U_O1/o1_w2o:0", (20, 1)), ("phi_U_O1/o1_b2o:0", (1,))]
_EE = [("phi_E_R1/r1_w1r1:0", (1, 20)), ("phi_E_R1/r1_w1r2:0", (2, 20)),     # model_4.py:218-221
       ("phi_E_R1/r1_b1r:0", (20,)), ("phi_E_R1/r1_w2r:0", (20, 20)), ("phi_E_R1/r1_b2r:0", (20,))]
_EC = [("phi_U_R1/o1_w1r:0", (22, 20)), ("phi_U_R1/o1_b1r:0", (20,)),      # model_4.py:293-299
       ("phi_U_R1/o1_w2r:0", (20, 2)), ("phi_U_R1/o1_b2r:0", (2,))]
_H1 = [("mlp_hunk_B2/w1:0", (10, 20)), ("mlp_hunk_B2/b1:0", (20,)),
       ("mlp_hunk_B2/r1_w2r:0", (20, 20)), ("mlp_hunk_B2/b2:0", (20,))]


def _h2(scope):   # TF uniquifies the re-entered phi_U_R1 scope when EC opened it first
    return [(scope + "/C_edge_w1:0", (22, 20)), (scope + "/C_edge_b1:0", (20,)),
            (scope + "/o1_w2r:0", (20, 2)), (scope + "/o1_b2r:0", (2,))]


_TH = [("map_conv/map_theta1:0", (1, 2, 1, 1)), ("map_conv/map_theta2:0", (1, 2, 1, 1))]

MODEL2 = _E1 + _E3 + _H1 + _h2("phi_U_R1") + _TH
VARIANTS = {
    1: _H1 + _h2("phi_U_R1") + _TH,                        # model_1.py  HD-GNN/ES
    2: MODEL2,                                              # model_2.py  HD-GNN/S
    3: _EE + _EC + _H1 + _h2("phi_U_R1_1") + _TH,           # model_3.py  HD-GNN/E
    4: _E1 + _E3 + _EE + _EC + _H1 + _h2("phi_U_R1_1") + _TH,   # model_4.py  HD-GNN
}
BIASES = {"r1_b1o", "r1_b5o", "o1_b1o", "o1_b2o", "b1", "b2", "C_edge_b1", "o1_b2r", "r1_b1r",
          "r1_b2r", "o1_b1r"}


def specs(variant=2):
    return VARIANTS[variant]


def n_params(variant=2):
    return int(sum(np.prod(s) for _, s in specs(variant)))


def offsets(variant=2):
    out, o = {}, 0
    for name, shape in specs(variant):
        n = int(np.prod(shape))
        out[name] = (o, shape)
        o += n
    return out


STATE_ALIGN = 16     # floats: each slice of the flat training state starts on 64 bytes


def state_offsets(variant=2):
    """Offsets of [params | adam_m | adam_v | beta_pow] in the engine's flat training state
    (Engine.state) and its length: each slice starts on a 64-byte boundary, so a vector
    access (float4) to any of them through hdg_state is aligned."""
    P = n_params(variant)
    S = -(-P // STATE_ALIGN) * STATE_ALIGN
    return {"params": 0, "m": S, "v": 2 * S, "beta_pow": 3 * S, "len": 3 * S + 2}


def split(flat, variant=2):
    return {name: np.asarray(flat[o:o + int(np.prod(s))]).reshape(s)
            for name, (o, s) in offsets(variant).items()}


def init_flat(seed=0, variant=2):
    """Reference initialisers: tf.truncated_normal(stddev=0.1) weights/thetas, zero biases."""
    rng = np.random.default_rng(seed)
    parts = []
    for name, shape in specs(variant):
        short = name.split("/")[-1].split(":")[0]
        if short in BIASES:
            parts.append(np.zeros(int(np.prod(shape)), np.float32))
        else:
            z = rng.standard_normal(int(np.prod(shape)))
            bad = np.abs(z) > 2
            while bad.any():
                z[bad] = rng.standard_normal(int(bad.sum()))
                bad = np.abs(z) > 2
            parts.append((0.1 * z).astype(np.float32))
    return np.concatenate(parts)
