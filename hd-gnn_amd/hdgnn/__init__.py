"""MI355X-native HD-GNN training-step engine (drop-in for fanmengdan/HD-GNN's graph2graph).

    from hdgnn.model import graph2graph       # reference constructor / train / test
    from hdgnn.engine import Engine           # raw device step runner (libhdgnn.so)
"""
__version__ = "0.1.0"
