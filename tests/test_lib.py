"""The C-ABI library loads on CPU and exports every symbol include/hdgnn.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

from conftest import ROOT


def _declared():
    with open(os.path.join(ROOT, "include", "hdgnn.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(hdg_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    names = _declared()
    for want in ("hdg_fwd_bwd", "hdg_adam_tf", "hdg_train_step", "hdg_forward",
                 "hdg_workspace_bytes", "hdg_last_error", "hdg_version"):
        assert want in names


def test_library_exports_every_declared_symbol():
    from hdgnn import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (hdg_\w+)", out))
    assert set(_declared()) <= exported


def test_host_only_entry_points():
    from hdgnn import _lib
    lib = _lib.load()
    assert lib.hdg_version() == _lib.ABI_VERSION == 9
    for v, n in ((1, 1146), (2, 2127), (3, 2148), (4, 3129)):
        assert lib.hdg_param_count(v) == n
        assert lib.hdg_grad_len(v) == n + _lib.TRAILER
    assert lib.hdg_param_count(5) == -1
    ok = _lib.Shape(100, 200, 74, 2, 100, 0)
    assert lib.hdg_resolve_path(ctypes.byref(ok)) == _lib.PATH_FUSED
    assert lib.hdg_workspace_bytes(ctypes.byref(ok)) > 0
    assert lib.hdg_prep_bytes(ctypes.byref(ok)) > 0
    for ne, nc in ((250, 114), (250, 150), (256, 160), (2, 2)):   # s3, s5, fused limits
        sh = _lib.Shape(100, ne, nc, 2, 100, 0)
        assert lib.hdg_resolve_path(ctypes.byref(sh)) == _lib.PATH_FUSED
        assert lib.hdg_workspace_bytes(ctypes.byref(sh)) > 0, lib.hdg_last_error()
    # beyond the fused kernel (stress shape, other variants): the general path
    for v, ne, nc in ((2, 1024, 512), (2, 300, 74), (1, 200, 74), (3, 200, 74), (4, 300, 74),
                      (4, 1024, 512)):
        sh = _lib.Shape(32, ne, nc, v, 256, 0)
        assert lib.hdg_resolve_path(ctypes.byref(sh)) == _lib.PATH_GENERAL
        assert lib.hdg_workspace_bytes(ctypes.byref(sh)) > 0, lib.hdg_last_error()
        assert lib.hdg_prep_bytes(ctypes.byref(sh)) > 0
    # model_4 within the fused engine's limits: the fused path with the entity-edge stage on
    # the general kernels; its prep / workspace hold both paths' parts
    m4 = _lib.Shape(100, 200, 74, 4, 100, 0)
    assert lib.hdg_resolve_path(ctypes.byref(m4)) == _lib.PATH_FUSED
    m4g = _lib.Shape(100, 200, 74, 4, 100, _lib.PATH_GENERAL)
    m2 = _lib.Shape(100, 200, 74, 2, 100, 0)
    # (the general path's own batches also carry the hunk label lists of its sorted passes,
    # which the hybrid's entity-edge half does not need)
    assert (lib.hdg_prep_bytes(ctypes.byref(m2)) < lib.hdg_prep_bytes(ctypes.byref(m4))
            <= lib.hdg_prep_bytes(ctypes.byref(m2)) + lib.hdg_prep_bytes(ctypes.byref(m4g)))
    assert lib.hdg_workspace_bytes(ctypes.byref(m4)) > lib.hdg_workspace_bytes(ctypes.byref(m4g))
    forced = _lib.Shape(4, 200, 74, 2, 4, _lib.PATH_GENERAL)
    assert lib.hdg_resolve_path(ctypes.byref(forced)) == _lib.PATH_GENERAL
    bad = _lib.Shape(100, 300, 74, 2, 100, _lib.PATH_FUSED)
    assert lib.hdg_workspace_bytes(ctypes.byref(bad)) == 0
    assert b"fused path" in lib.hdg_last_error()
    bad = _lib.Shape(100, 5000, 74, 2, 100, 0)
    assert lib.hdg_workspace_bytes(ctypes.byref(bad)) == 0
    assert b"ne must be" in lib.hdg_last_error()
    bad_v = _lib.Shape(4, 20, 10, 5, 4, 0)
    assert lib.hdg_workspace_bytes(ctypes.byref(bad_v)) == 0
    assert b"variant" in lib.hdg_last_error()


def test_prep_counts_layout_host():
    """hdg_prep_counts_layout: the count tables sit inside each commit's prep block."""
    from hdgnn import _lib
    lib = _lib.load()
    for v, ne, nc, path in ((2, 200, 74, 0), (2, 250, 150, 0), (4, 200, 74, 0),
                            (2, 1024, 512, 0), (2, 200, 74, _lib.PATH_GENERAL)):
        sh = _lib.Shape(8, ne, nc, v, 8, path)
        st, ks, kt, ncst = (ctypes.c_int64() for _ in range(4))
        assert lib.hdg_prep_counts_layout(ctypes.byref(sh), ctypes.byref(st), ctypes.byref(ks),
                                          ctypes.byref(kt), ctypes.byref(ncst)) == 0
        kw = (nc * ne + 1) // 2                       # u16 [Nc][Ne] in words
        assert 0 <= ks.value and ks.value + kw <= kt.value or kt.value + kw <= ks.value
        assert max(ks.value, kt.value) + kw <= st.value and ncst.value + 2 * nc <= st.value
        assert 8 * st.value * 4 <= lib.hdg_prep_bytes(ctypes.byref(sh))
    bad = _lib.Shape(4, 5000, 74, 2, 4, 0)
    z = ctypes.c_int64()
    assert lib.hdg_prep_counts_layout(ctypes.byref(bad), *(ctypes.byref(z) for _ in range(4))) != 0


def test_python_mirror_matches_header_constants():
    """hdgnn._lib's flag values and the general path's automatic hunk-form thresholds are
    the ones include/hdgnn.h defines (bench.py reports the form from the Python mirror)."""
    from hdgnn import _lib
    with open(os.path.join(ROOT, "include", "hdgnn.h")) as f:
        defs = dict(re.findall(r"#define\s+(HDG_[A-Z_0-9]+)\s+(0x[0-9a-fA-F]+|\d+)", f.read()))
    val = {k: int(v, 0) for k, v in defs.items()}
    assert val["HDG_FLAG_NO_SPLIT"] == _lib.FLAG_NO_SPLIT
    assert val["HDG_FLAG_HUNK_DENSE"] == _lib.FLAG_HUNK_DENSE
    assert val["HDG_FLAG_HUNK_SORTED"] == _lib.FLAG_HUNK_SORTED
    assert val["HDG_FLAG_HUNK_TILED"] == _lib.FLAG_HUNK_TILED
    assert val["HDG_HUNK_SORTED_MIN_NC"] == _lib.HUNK_SORTED_MIN_NC
    assert val["HDG_HUNK_TILED_MIN_NC"] == _lib.HUNK_TILED_MIN_NC
    assert val["HDG_PATH_FUSED"] == _lib.PATH_FUSED and val["HDG_PATH_GENERAL"] == _lib.PATH_GENERAL
