"""CPU: static audit of the shipped gfx950 code for the MFMA operand write-after-read hazard (tools/audit_mfma_war.py).

Round 5 root-caused wrong 16-column groups in the register-dequant GEMM to a VALU that overwrote an A / B source register
of the MFMA issued just before it, at two waves per SIMD.  These tests read the .s that the build keeps
(-save-temps) and fail when any kernel that can run two waves per SIMD has a VALU write to an in-flight MFMA's A / B /
scale register within 8 issue slots on some control-flow path.  Kernels whose registers allow one wave per SIMD only
(hipcc's `; Occupancy: 1`) are reported, not failed: round 5's attention kernel (attn2, now the ACE_MI_ATTN_KH=0 /
non-f8c path) is one of them, and that it stays so is asserted below.  Round 6's f8c kernel (attn_kh_kernel) runs two
waves per SIMD by design: it must be clean of VALU AND LDS-read overwrites (--loads)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "ace-step-1.5-ggml_amd", "build")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import audit_mfma_war as aw  # noqa: E402

FILES = ["gemm", "gemm_q", "gemm_a8", "attention", "vae"]


def _s(name):
    p = os.path.join(BUILD, f"{name}-hip-amdgcn-amd-amdhsa-gfx950.s")
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: build the library first (make -C ace-step-1.5-ggml_amd/csrc, or __graft_entry__.build())")
    return p


@pytest.mark.parametrize("name", FILES)
def test_no_exposed_mfma_operand_overwrite(name):
    res = aw.audit(_s(name), window=8)
    exposed = {k: v for k, v in res.items() if (v[0] or 1) >= 2}
    msg = "\n".join(f"{k[:120]}: occupancy {occ}, {len(h)} pairs, first d={h[0][0]} {h[0][2]} {h[0][3]} (line {h[0][5]})"
                    for k, (occ, h) in list(exposed.items())[:10])
    assert not exposed, f"unguarded MFMA operand overwrites in two-wave kernels:\n{msg}"


def test_attn2_instances_are_single_wave():
    """attn2 (f32 for the condition / text encoders and the q8 mode; f8c with ACE_MI_ATTN_KH=0) must keep one wave per
    SIMD: its hand-laid stream reuses P-pack and address registers right after the MFMAs that read them"""
    funcs = aw.parse(_s("attention"))
    attn2 = {k: f for k, f in funcs.items() if "attn2_kernel" in k}
    assert attn2, "no attn2_kernel instance in attention.s"
    for k, f in attn2.items():
        assert f.occupancy == 1, f"{k}: occupancy {f.occupancy}"


def test_two_wave_attention_kernel_is_clean_of_operand_overwrites():
    """attn_kh_kernel (the f8c default, 8 waves = two per SIMD): no VALU and no LDS / memory load may write an A / B /
    scale register within 8 issue slots of the MFMA that reads it (fragment liveness + phase-end wait states)"""
    s = _s("attention")
    funcs = aw.parse(s)
    kh = {k: f for k, f in funcs.items() if "attn_kh_kernel" in k}
    assert len(kh) == 4, sorted(kh)  # bf16 / fp16 output x key bias
    for k, f in kh.items():
        assert f.occupancy == 2, f"{k}: occupancy {f.occupancy}"
    res = aw.audit(s, window=8, ksub="attn_kh_kernel", valu_only=False)
    assert res == {}, {k[:80]: (occ, h[:3]) for k, (occ, h) in res.items()}


def _fake(tmp_path, body, occupancy):
    p = tmp_path / "fake.s"
    p.write_text("k:\n" + body + f"\n; Occupancy: {occupancy}\n")
    return str(p)


def test_audit_flags_a_close_overwrite(tmp_path):
    body = "\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]\n\tv_add_u32_e32 v5, v1, v2\n\ts_endpgm"
    res = aw.audit(_fake(tmp_path, body, 2))
    assert "k" in res and res["k"][1][0][0] == 1


def test_audit_counts_nops_and_follows_branches(tmp_path):
    # 16 wait states between the MFMA and the write: clean
    body = ("\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]\n\ts_nop 7\n\ts_nop 7\n"
            "\tv_add_u32_e32 v5, v1, v2\n\ts_endpgm")
    assert aw.audit(_fake(tmp_path, body, 2)) == {}
    # the write sits on the other side of an unconditional branch (another wave role's code): clean
    body = ("\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]\n\ts_branch .LBB0_2\n"
            ".LBB0_1:\n\tv_add_u32_e32 v5, v1, v2\n\ts_endpgm\n.LBB0_2:\n\ts_endpgm")
    assert aw.audit(_fake(tmp_path, body, 2)) == {}
    # ... but on the taken side of a conditional branch it is a hit
    body = ("\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]\n\ts_cbranch_scc1 .LBB0_1\n\ts_endpgm\n"
            ".LBB0_1:\n\tv_add_u32_e32 v9, v1, v2\n\ts_endpgm")
    res = aw.audit(_fake(tmp_path, body, 2))
    assert res["k"][1][0][0] == 2
    # block-scaled MFMA: its scale VGPRs count as sources
    body = ("\tv_mfma_scale_f32_32x32x64_f8f6f4 a[0:15], v[2:9], v[10:17], a[0:15], v24, v23 op_sel_hi:[0,0,0]\n"
            "\tv_mov_b32_e32 v23, 0\n\ts_endpgm")
    assert aw.audit(_fake(tmp_path, body, 1))["k"][1][0][3] == "v23"
