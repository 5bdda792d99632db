"""The device code's hand-written cross-lane instructions keep their wait states.

row16_sums / swap16 / swap32 (hdgnn.hip, wide.hip) are inline asm, which the compiler's
hazard recognizer does not see into; a DPP or permlane-swap read issued < 2 wait states
after the VALU write of its operand returns stale lanes -- wrong sums whose presence
depends on the schedule.  Compiles both sources to gfx950 assembly (CPU only) and scans
every cross-lane read with tools/dpp_hazards.py.
"""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not shutil.which(HIPCC), reason="hipcc not available")
def test_no_cross_lane_read_hazards(tmp_path):
    import dpp_hazards
    csrc = os.path.join(ROOT, "hd-gnn_amd", "csrc")
    procs, outs = [], []
    for f in ("hdgnn.hip", "wide.hip"):
        out = str(tmp_path / (f + ".s"))
        outs.append(out)
        procs.append(subprocess.Popen(
            [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
             "-I" + os.path.join(ROOT, "include"), "-o", out, os.path.join(csrc, f)],
            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=str(tmp_path)))
    for p in procs:
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err.decode(errors="replace")[-2000:]
    bad = [(o, b) for o in outs for b in dpp_hazards.scan(o)]
    assert not bad, bad[:5]
    # the scan sees the hand-written reductions (guards against a vacuous pass)
    text = open(outs[0]).read()
    assert text.count("v_add_f32_dpp") > 100 and "v_permlane16_swap_b32" in text


def test_scanner_flags_a_close_write(tmp_path):
    import dpp_hazards
    s = tmp_path / "k.s"
    s.write_text("f:\n\tv_add_f32_e32 v29, v31, v99\n"
                 "\tv_add_f32_dpp v29, v29, v29 row_mirror row_mask:0xf bank_mask:0xf\n"
                 "\tv_pk_fma_f32 v[4:5], v[0:1], v[2:3], v[6:7]\n\ts_nop 0\n"
                 "\tv_permlane16_swap_b32 v5, v8\n"
                 "\tv_mov_b32_e32 v9, v1\n\ts_nop 1\n"
                 "\tv_add_f32_dpp v9, v9, v9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n")
    bad = dpp_hazards.scan(str(s))
    assert [b[2].split()[0] for b in bad] == ["v_add_f32_dpp", "v_permlane16_swap_b32"]


def test_scanner_follows_control_flow(tmp_path):
    """A write at the end of a predecessor block (fall-through into a label, a loop back
    edge, a conditional branch's target) reaches a cross-lane read at the top of the next
    block; an s_nop at the block start covers every path."""
    import dpp_hazards
    s = tmp_path / "k.s"
    s.write_text("g:\n\tv_add_f32_e32 v5, v1, v2\n.LBB0_1:\n"
                 "\tv_add_f32_dpp v5, v5, v5 row_mirror row_mask:0xf bank_mask:0xf\n"
                 "\ts_cbranch_scc1 .LBB0_3\n\tv_add_f32_e32 v9, v1, v2\n.LBB0_3:\n"
                 "\tv_permlane16_swap_b32 v7, v9\n\ts_endpgm\n"
                 "h:\n.LBB1_1:\n\ts_nop 1\n"
                 "\tv_add_f32_dpp v3, v3, v3 row_mirror row_mask:0xf bank_mask:0xf\n"
                 "\tv_add_f32_e32 v3, v4, v4\n\ts_cbranch_scc1 .LBB1_1\n\ts_endpgm\n"
                 "k:\n.LBB2_1:\n"
                 "\tv_add_f32_dpp v6, v6, v6 row_mirror row_mask:0xf bank_mask:0xf\n"
                 "\tv_add_f32_e32 v6, v4, v4\n\ts_cbranch_scc1 .LBB2_1\n\ts_endpgm\n")
    bad = dpp_hazards.scan(str(s))
    got = sorted((b[0], b[1].split()[1].rstrip(",")) for b in bad)
    assert got == [("g", "v5"), ("g", "v9"), ("k", "v6")], bad
