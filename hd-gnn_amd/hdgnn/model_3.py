"""Drop-in for the reference's model_3.graph2graph (HD-GNN/E; model_3.py:82-102: entity-edge stage built, hunk stage on B_1).
Same constructor, train / test / save / load as hdgnn.model.graph2graph."""
from .model import graph2graph as _g2g


class graph2graph(_g2g):
    variant = 3
