"""The gather's inline v_dot4_i32_i8 blocks keep gfx950's dot-result wait states (no GPU needed):
the sources are compiled to gfx950 assembly with the library's flags and every inline dot's
destination must stay unread for three wait states (tools/dot_hazard_scan.py).  A read that comes
earlier sees the register's old value on the hardware — measured as dropped photons in a gather
variant whose schedule did that (profiles/r05h_gather_two_hitpoints_ab.txt)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dot_hazard_scan as dhs  # noqa: E402


def test_scanner_flags_an_early_read_and_accepts_padding():
    early = """
    v_dot4_i32_i8 v6, v2, v1, 0
    v_cmp_gt_i32_e32 vcc, s4, v6
    """
    padded = """
    v_dot4_i32_i8 v6, v2, v1, 0
    v_dot4_i32_i8 v7, v3, v1, 0
    s_nop 2
    v_cmp_gt_i32_e32 vcc, s4, v6
    v_cmp_gt_i32_e32 vcc, s4, v7
    """
    ranged = """
    v_dot4_i32_i8 v6, v2, v1, 0
    v_mov_b32 v9, 0
    v_pk_add_f32 v[4:5], v[6:7], v[2:3]
    """
    branch = """
    v_dot4_i32_i8 v6, v2, v1, 0
    s_cbranch_vccz .LBB0_2
    """
    assert dhs.scan_text(early)[1] and dhs.scan_text(ranged)[1] and dhs.scan_text(branch)[1]
    assert dhs.scan_text(padded) == (2, [])


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_shipped_inline_dots_keep_their_wait_states():
    results = dhs.build_and_scan()
    assert "orx_kernels.hip" in results
    ndots, bad = results["orx_kernels.hip"]
    assert ndots >= 16  # the union (two instances) and per-lane gathers' four-dot blocks
    assert not bad, bad[:5]
