"""Host-side cProfile of graph2graph.train (the main.py --Type train loop) at glide, one
B = 100 step per epoch, as bench.py --e2e runs it (GPU box):
    python tools/e2e_profile.py [epochs]
Prints the wall time per epoch and the functions with the most own time."""
import contextlib
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
from hdgnn.model import graph2graph  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402


def main(epochs):
    B, ne, nc = 100, 200, 74
    dev = torch.device("cuda:0")
    cb = synth_commits(2 * B, ne, nc, 20250301 + 7)
    train, test = cb.slice(0, B), cb.slice(B, 2 * B)
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)

        class Args:
            checkpoint_dir, Repo = os.path.join(d, "ck"), "glide"
        m = graph2graph(None, Ds=1, Ne=ne, Nc=nc, Ner=ne * (ne - 1), Ncr=nc * (nc - 1), Dr=2,
                        De_e=20, De_er=20, Mini_batch=B, checkpoint_dir=Args.checkpoint_dir,
                        epoch=epochs, Ds_inter=1, Dr_inter=2, Step=2, Repo="glide", device=dev,
                        compact=(train, test, train))
        with contextlib.redirect_stdout(io.StringIO()):
            m.train(Args)                                  # warm
            torch.cuda.synchronize(dev)
            pr = cProfile.Profile()
            t0 = time.perf_counter()
            pr.enable()
            m.train(Args)
            pr.disable()
            torch.cuda.synchronize(dev)
            wall = time.perf_counter() - t0
    print("epochs %d wall %.4f s: %.1f us per epoch, %.0f commits/s" % (
        epochs, wall, 1e6 * wall / epochs, epochs * B / wall))
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
