"""Fast compact loader: the dataset files utils2.read_data reads, straight
to CommitBatches, bit-exact with utils2.read_data + data.compact_from_read_data.

utils2.read_data (utils2.py:11-253) builds twelve dense arrays (~9 GB at glide step 2,
minutes of Python loops and progress-bar sleeps) from four inputs per step:
    Adjset/<repo>/Cutting_Adjs/CAdjs_<step>.npy        entity adjacency, diagonal = x
    Adjset/<repo>/Cutting_Adjs/CHunkAdjs_<step>.npy    hunk adjacency (the labels)
    dataset/<repo>/IndexPathList/IndexPathList_<step>.pkl   per commit: index file path
    dataset/<repo>/HunkIDdict/HunkIDmap_<step>.pkl          per commit: {line key: hunk id}
This module reads the same four and produces the compact form directly, reproducing the
reference's bookkeeping on purpose:
    x     = diagonal of CAdjs (f64, fed to TF as f32)                    utils2.py:29-36
    class = int(value) used as an index into Dr=2: truncation toward 0,
            -1 -> class 1, -2 -> class 0, anything else outside {0,1} raises    82, 105
    index = the first n = len(readlines()[:Ne]) lines; 'null' -> no hunk; a hunk id
            >= Nc is dropped; a negative id wraps like a numpy index (row Nc + id)  111-137
    split = first int(N/2) commits train, the rest test                  140-149
The pickles are read with an unpickler that refuses every global: they hold plain
lists / dicts / strings (what joblib.dump writes for them), nothing executable.
"""
import os
import pickle

import numpy as np

from .data import CommitBatch


class _PlainUnpickler(pickle.Unpickler):
    """Builds only built-in containers / strings / numbers; any class reference raises."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(
            "refusing to load %s.%s: the index-path and hunk-map pickles hold plain lists "
            "and dicts" % (module, name))


def load_plain_pickle(path):
    with open(path, "rb") as f:
        head = f.read(4)
        if head[:1] != b"\x80" and head[:1] not in (b"(", b"]", b"}"):
            raise pickle.UnpicklingError("%s is not an uncompressed pickle (joblib compression "
                                         "is not supported)" % path)
        f.seek(0)
        return _PlainUnpickler(f).load()


def edge_classes(m, dr=2):
    """int(value) as an index into Dr classes (utils2.py:82, 105), vectorised."""
    m = np.asarray(m, dtype=np.float64)
    if not np.all(np.isfinite(m)):
        raise ValueError("adjacency holds non-finite values")
    c = np.trunc(m).astype(np.int64)
    bad = (c < -dr) | (c >= dr)
    if bad.any():
        v = m[bad].flat[0]
        raise IndexError("edge value %r is not a valid class index for Dr=%d" % (v, dr))
    return (c % dr).astype(np.uint8)


def hunk_rows(lines, hunkmap, ne, nc):
    """(hid[ne], n) of one commit's index file (utils2.py:121-137)."""
    lines = list(lines)[:ne]
    hid = np.full(ne, -1, np.int32)
    for i, ln in enumerate(lines):
        key = ln.strip()
        if key == "null":
            continue
        num = int(hunkmap[key])                  # KeyError like the reference
        if num >= nc:
            continue
        if num < -nc:
            raise IndexError("hunk id %d out of range for Nc=%d" % (num, nc))
        hid[i] = num % nc
    return hid, len(lines)


def compact_from_arrays(cadjs, chunkadjs, index_lines, hunkmaps, ne, nc):
    """Raw per-step inputs -> CommitBatch over all N commits (x f32, a/y u8 classes with a
    zero diagonal, hid/nlen of each commit's own index file)."""
    cadjs = np.asarray(cadjs)
    chunkadjs = np.asarray(chunkadjs)
    N = cadjs.shape[0]
    if cadjs.shape != (N, ne, ne) or chunkadjs.shape != (N, nc, nc):
        raise ValueError("CAdjs %s / CHunkAdjs %s do not match Ne=%d, Nc=%d"
                         % (cadjs.shape, chunkadjs.shape, ne, nc))
    if len(index_lines) < N or len(hunkmaps) < N:
        raise ValueError("index paths / hunk maps cover %d / %d of %d commits"
                         % (len(index_lines), len(hunkmaps), N))
    x = np.diagonal(cadjs, axis1=1, axis2=2).astype(np.float64).astype(np.float32)
    off_e = ~np.eye(ne, dtype=bool)
    off_c = ~np.eye(nc, dtype=bool)
    a = edge_classes(np.where(off_e, cadjs, 0.0)) * off_e
    y = edge_classes(np.where(off_c, chunkadjs, 0.0)) * off_c
    hid = np.full((N, ne), -1, np.int32)
    nlen = np.zeros(N, np.int32)
    for k in range(N):
        hid[k], nlen[k] = hunk_rows(index_lines[k], hunkmaps[k], ne, nc)
    return CommitBatch(x, a.astype(np.uint8), y.astype(np.uint8), hid, nlen)


def read_step_files(repo, step, root="."):
    """The four inputs of one step (paths exactly as utils2.py:22-27 builds them)."""
    adj = os.path.join(root, "Adjset", repo, "Cutting_Adjs")
    cadjs = np.load(os.path.join(adj, "CAdjs_%d.npy" % step), allow_pickle=False)
    chunk = np.load(os.path.join(adj, "CHunkAdjs_%d.npy" % step), allow_pickle=False)
    paths = load_plain_pickle(os.path.join(root, "dataset", repo, "IndexPathList",
                                           "IndexPathList_%d.pkl" % step))
    maps = load_plain_pickle(os.path.join(root, "dataset", repo, "HunkIDdict",
                                          "HunkIDmap_%d.pkl" % step))
    lines = []
    for p in paths[:cadjs.shape[0]]:
        p = p if os.path.isabs(p) else os.path.join(root, p)   # utils2 opens it from its cwd
        with open(p) as f:
            lines.append(f.readlines())
    return cadjs, chunk, lines, maps


def read_compact(repo, step, ne, nc, mini_batch=None, root="."):
    """-> (train, test, maps) CommitBatches, the same triple data.compact_from_read_data
    returns for utils2.read_data's 12-tuple: train / test = first int(N/2) commits / the
    rest; maps = the hunk maps of the first Mini_batch commits, which the reference feeds
    for every batch (model_2.py:376-381, 495-500)."""
    cb = compact_from_arrays(*read_step_files(repo, step, root), ne, nc)
    half = int(cb.B / 2)
    train, test = cb.slice(0, half), cb.slice(half, cb.B)
    mb = mini_batch or half
    return train, test, cb.slice(0, mb)
