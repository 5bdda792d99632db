"""Drop-in for the reference's model_1.graph2graph (HD-GNN/ES; model_1.py:75-91: hunk stage on B_1, no entity stages).
Same constructor, train / test / save / load as hdgnn.model.graph2graph."""
from .model import graph2graph as _g2g


class graph2graph(_g2g):
    variant = 1
