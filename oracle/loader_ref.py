"""Compact restatement of utils2.read_data's bookkeeping (TEST INFRASTRUCTURE ONLY).

Pinned bit-exact against tests/golden/loader_tiny.npz, which holds the
12-tuple the reference utils2.read_data itself produced on a synthetic tree
(tools/gen_loader_golden.py).  Reproduces, on purpose:
  * node attribute = diagonal of CAdjs, float64               (utils2.py:29-36)
  * edge class = int(value) used as an index into Dr=2, so -1 -> class 1,
    -2 -> class 0, anything else outside {0,1} raises              (82, 105)
  * Esc/Etc walk the first n = len(readlines()[:Ne]) index lines with their own
    relation counter (stride n-1, misaligned with Es when n < Ne); 'null' lines
    still advance it; hunk ids >= Nc are dropped; negative ids wrap like a numpy
    index (row Nc+id)                                              (111-137)
"""
import numpy as np


def edge_class(v, dr=2):
    c = int(v)                      # python int(): truncation toward zero
    if c < -dr or c >= dr:
        raise IndexError("edge value %r is not a valid class index for Dr=%d" % (v, dr))
    return c % dr


def hunk_row(num, nc):
    """HunkIDmap value -> Esc row, or -1 when dropped (utils2.py:130-136)."""
    num = int(num)
    if num >= nc:
        return -1
    if num < -nc:
        raise IndexError("hunk id %d out of range for Nc=%d" % (num, nc))
    return num % nc


def compact_from_raw(cadjs, chunkadjs, index_lines, hunkmaps, ne, nc):
    """(x f64 (N,Ne), a i8 (N,Ne,Ne), y i8 (N,Nc,Nc), hid i32 (N,Ne), nlen i32 (N,))."""
    cadjs = np.asarray(cadjs)
    chunkadjs = np.asarray(chunkadjs)
    N = cadjs.shape[0]
    x = np.zeros((N, ne), np.float64)
    a = np.zeros((N, ne, ne), np.int8)
    y = np.zeros((N, nc, nc), np.int8)
    for k in range(N):
        x[k] = np.diagonal(cadjs[k]).astype(np.float64)
        for i in range(ne):
            for j in range(ne):
                if i != j:
                    a[k, i, j] = edge_class(cadjs[k, i, j] * 1.0)
        for i in range(nc):
            for j in range(nc):
                if i != j:
                    y[k, i, j] = edge_class(chunkadjs[k, i, j] * 1.0)
    hid = np.full((N, ne), -1, np.int32)
    nlen = np.zeros(N, np.int32)
    for k in range(N):
        lines = list(index_lines[k])[:ne]
        nlen[k] = len(lines)
        for i, ln in enumerate(lines):
            key = ln.strip()
            if key != "null":
                hid[k, i] = hunk_row(hunkmaps[k][key], nc)
    return x, a, y, hid, nlen
