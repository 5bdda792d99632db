"""Drop-in for the reference's model_4.graph2graph (HD-GNN; model_4.py:86-97: entity stage + entity-edge probabilities in B_2).
Same constructor, train / test / save / load as hdgnn.model.graph2graph."""
from .model import graph2graph as _g2g


class graph2graph(_g2g):
    variant = 4
