"""Flat parameter layout of the engine (tf.global_variables order, (in,out) weights).

model_2.py:161-179 phi_E_O1, 190-205 phi_U_O1, 245-277 mlp_hunk_B2, 304-324 phi_U_R1,
326-333 map_conv.  Offsets here match the m2:: constants in csrc/hdgnn.hip.
"""
import numpy as np

MODEL2 = [
    ("phi_E_O1/r1_w1o:0", (4, 20)), ("phi_E_O1/r1_b1o:0", (20,)),
    ("phi_E_O1/r1_w5o:0", (20, 20)), ("phi_E_O1/r1_b5o:0", (20,)),
    ("phi_U_O1/o1_w1o:0", (21, 20)), ("phi_U_O1/o1_b1o:0", (20,)),
    ("phi_U_O1/o1_w2o:0", (20, 1)), ("phi_U_O1/o1_b2o:0", (1,)),
    ("mlp_hunk_B2/w1:0", (10, 20)), ("mlp_hunk_B2/b1:0", (20,)),
    ("mlp_hunk_B2/r1_w2r:0", (20, 20)), ("mlp_hunk_B2/b2:0", (20,)),
    ("phi_U_R1/C_edge_w1:0", (22, 20)), ("phi_U_R1/C_edge_b1:0", (20,)),
    ("phi_U_R1/o1_w2r:0", (20, 2)), ("phi_U_R1/o1_b2r:0", (2,)),
    ("map_conv/map_theta1:0", (1, 2, 1, 1)), ("map_conv/map_theta2:0", (1, 2, 1, 1)),
]
VARIANTS = {2: MODEL2}
BIASES = {"r1_b1o", "r1_b5o", "o1_b1o", "o1_b2o", "b1", "b2", "C_edge_b1", "o1_b2r"}


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
