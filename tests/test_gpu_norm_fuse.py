"""GPU: the row RMSNorm + AdaLN modulation fused into the residual GEMMs' epilogue (launch_gemm_resid_norm,
kernels/gemm_common.h norm_fuse) against the standalone kernel (ops.hip rmsnorm_mod_canon_kernel), which sums x^2
in the same order (kernels/norm_math.h): whole forwards with the fusion on, on without waiting (every column tile
but the last of its row block hands its normalisation over to that last one, which reads the x it stored back
from memory) and off (mode 3: the standalone kernel in that order) give the same bits.  Every tile family the
fusion runs on (forced), batched items whose token counts are not multiples of the row tile (a tile spans two
items: per-item modulation), at the tiny and the full width (2 layers; T = 3000 is the 240 s shape).  The fusion
is an opt-in mode (ACE_MI_NORM_FUSE=1): measured slower than the standalone launch on MI355X."""
import numpy as np
import pytest

from test_gpu_forward import _batched

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [-1, 6, 7, 8, 9, 12, 13, 14])
@pytest.mark.parametrize("width", ["tiny", "full"])
def test_fused_norm_is_bit_exact(tiny_ckpt, monkeypatch, width, variant):
    from acestep_mi355x import capi
    from acestep_mi355x.capi import GGMLCAPIBridge
    if width == "tiny":
        d, H, cases = tiny_ckpt, 256, [(1, 37, 5), (2, 301, 9), (3, 1001, 17)]
    else:
        from acestep_mi355x.synthetic import cached_checkpoint, make_config
        d, H = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch"), 2048
        cases = [(2, 601, 64)] if variant >= 0 else [(2, 601, 64), (1, 3000, 512)]
        monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    br = GGMLCAPIBridge()
    br.load_dit(d)
    outs = {}
    try:
        capi.gemm_variant(variant)
        for mode in (1, 2, 3):
            capi.norm_fuse(mode)
            for B, T, L in cases:
                r = np.random.default_rng(B * 7 + T)
                h = r.standard_normal((B, T, 64)).astype(np.float32)
                c = r.standard_normal((B, T, 128)).astype(np.float32)
                e = r.standard_normal((B, L, H)).astype(np.float32)
                outs[(mode, B, T)] = _batched(br, h, c, e, 0.7)
    finally:
        capi.gemm_variant(-1)
        capi.norm_fuse(-1)
        br.close()
    for B, T, L in cases:
        ref = outs[(3, B, T)]
        assert np.isfinite(ref).all()
        np.testing.assert_array_equal(outs[(1, B, T)], ref, err_msg=f"fused B={B} T={T}")
        np.testing.assert_array_equal(outs[(2, B, T)], ref, err_msg=f"hand-over B={B} T={T}")


def test_fused_norm_repeated_launches_stay_exact(tiny_ckpt):
    """The per-row-block counters and claims are left at zero by every launch (the row block's last tile resets
    them): many forwards in a row, alternating the hand-over and the waiting path, keep giving the same bits."""
    from acestep_mi355x import capi
    from acestep_mi355x.capi import GGMLCAPIBridge
    rng = np.random.default_rng(3)
    B, T, L = 2, 301, 9
    h = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    br = GGMLCAPIBridge()
    br.load_dit(tiny_ckpt)
    try:
        capi.norm_fuse(3)
        ref = _batched(br, h, c, e, 0.5)
        for i in range(12):
            capi.norm_fuse(1 + i % 2)
            np.testing.assert_array_equal(_batched(br, h, c, e, 0.5), ref, err_msg=f"forward {i}")
    finally:
        capi.norm_fuse(-1)
        br.close()
