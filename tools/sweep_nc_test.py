import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "hd-gnn_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np
import test_general_gpu as T
from hdgnn.synth import synth_commits
from hdgnn import _lib
for split in ("1", "0"):
    os.environ["HDG_FUSED_SPLIT"] = split
    res = []
    for nc in (81, 90, 96, 97, 100, 114, 120, 127, 128, 129, 140, 150, 159, 160):
        try:
            T._run_and_check(synth_commits(2, 40, nc, 3), 2, 3, _lib.PATH_FUSED)
            res.append("%d:ok" % nc)
        except AssertionError as e:
            res.append("%d:FAIL" % nc)
    print("split", split, " ".join(res), flush=True)
