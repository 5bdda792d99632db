"""Upload + hdg_prepare of one glide batch (B=100) and one stress batch (B=32), 5 times
each: run under rocprofv3 --kernel-trace to time the prepare kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hd-gnn_amd"))
import torch  # noqa: E402
from hdgnn.synth import synth_commits  # noqa: E402

for B, ne, nc, path in ((100, 200, 74, 1), (32, 1024, 512, 2)):
    cb = synth_commits(B, ne, nc, 3)
    for _ in range(5):
        cb.to_device("cuda:0", 2, path)
    torch.cuda.synchronize()
print("ok")
