"""Generate tests/golden/loader_tiny.{npz,json} by running the REFERENCE loader.

Builds a tiny synthetic Adjset/dataset tree in a temp dir, imports
/root/reference/utils2.py (importable here: numpy/joblib/tqdm only) and runs
its read_data(self, step) unmodified.  The 12 returned arrays plus the raw
inputs are committed as fixtures; the reference itself never travels.

The tree is chosen to hit every bookkeeping edge case utils2.py has:
  * 100 commits (utils2.py:50-61 hard-codes 100 rows)
  * index files shorter than Ne (n < Ne: Esc/Etc stride n-1), equal, longer
  * 'null' lines, hunk ids >= Nc (dropped), a negative hunk id (numpy wrap)
  * a -1 off-diagonal adjacency value (class index wraps to 1)
  * non-integer diagonal node attributes

Run from the repo root:  python tools/gen_loader_golden.py
"""
import json
import os
import sys
import tempfile

import joblib
import numpy as np

REF = "/root/reference"
NE, NC, STEP, REPO = 7, 5, 2, "tiny"
NCOMMITS = 100


def build_tree(root, rng):
    adj = os.path.join(root, "Adjset", REPO, "Cutting_Adjs")
    os.makedirs(adj)
    os.makedirs(os.path.join(root, "dataset", REPO, "IndexPathList"))
    os.makedirs(os.path.join(root, "dataset", REPO, "HunkIDdict"))
    os.makedirs(os.path.join(root, "Intermediate_products", REPO))   # utils2 never mkdirs it
    idx_dir = os.path.join(root, "index")
    os.makedirs(idx_dir)

    x = (rng.random((NCOMMITS, NE, NE)) < 0.3).astype(np.float64)
    diag = np.round(rng.random((NCOMMITS, NE)) * 9.0, 1)           # non-integer attributes
    for k in range(NCOMMITS):
        np.fill_diagonal(x[k], diag[k])
    x[3, 0, 1] = -1.0                                                 # class-index wrap
    y = (rng.random((NCOMMITS, NC, NC)) < 0.35).astype(np.float64)
    y = np.maximum(y, y.transpose(0, 2, 1))
    np.save(os.path.join(adj, "CAdjs_%d.npy" % STEP), x)
    np.save(os.path.join(adj, "CHunkAdjs_%d.npy" % STEP), y)

    paths, maps, lines_all = [], [], []
    for k in range(NCOMMITS):
        n = [3, NE, NE + 3, 5, 1][k % 5]                               # shorter / equal / longer
        keys = {}
        lines = []
        for i in range(n):
            if rng.random() < 0.2:
                lines.append("null")
                continue
            key = "h%d_%d" % (k, rng.integers(0, 9))
            if key not in keys:
                hid = int(rng.integers(0, int(1.25 * NC) + 1))
                keys[key] = hid
            lines.append(key)
        if k == 7 and lines:
            lines[0] = "neg"
            keys["neg"] = -1                                           # numpy negative index
        p = os.path.join(idx_dir, "idx_%03d.txt" % k)
        with open(p, "w") as f:
            f.write("\n".join("  %s " % ln for ln in lines) + ("\n" if lines else ""))
        paths.append(p)
        maps.append(keys)
        lines_all.append(lines)
    with open(os.path.join(root, "dataset", REPO, "IndexPathList",
                           "IndexPathList_%d.pkl" % STEP), "wb") as f:
        joblib.dump(paths, f)
    with open(os.path.join(root, "dataset", REPO, "HunkIDdict",
                           "HunkIDmap_%d.pkl" % STEP), "wb") as f:
        joblib.dump(maps, f)
    return x, y, lines_all, maps


class _Self:
    Repo, Ne, Nc, Dr = REPO, NE, NC, 2
    Ner, Ncr = NE * (NE - 1), NC * (NC - 1)


def main():
    sys.path.insert(0, REF)
    import utils2  # noqa: reference loader, run unmodified

    rng = np.random.default_rng(20250301)
    here = os.getcwd()
    with tempfile.TemporaryDirectory() as root:
        x, y, lines, maps = build_tree(root, rng)
        os.chdir(root)
        try:
            out = utils2.read_data(_Self(), STEP)
        finally:
            os.chdir(here)
    names = ["E_node_train", "E_node_test", "E_edge_train", "E_edge_test",
             "C_edge_train", "C_edge_test", "Es_data", "Et_data", "Cs_label",
             "Ct_label", "Esc_data", "Etc_data"]
    arrays = {n: np.asarray(v) for n, v in zip(names, out)}
    arrays["CAdjs"] = x
    arrays["CHunkAdjs"] = y
    os.makedirs("tests/golden", exist_ok=True)
    np.savez_compressed("tests/golden/loader_tiny.npz", **arrays)
    with open("tests/golden/loader_tiny.json", "w") as f:
        json.dump({"Ne": NE, "Nc": NC, "step": STEP, "index_lines": lines,
                   "hunkmaps": maps, "generator": "tools/gen_loader_golden.py",
                   "reference": "utils2.read_data @ fanmengdan/HD-GNN 2025-03-01"}, f)
    print({k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
