"""GPU parity of the quantized-weight paths: the dequant-fused GEMM kernel (Q8_0 / Q4_K / Q6_K planes)
against an fp64 product of bf16 activations with bf16(dequant(W)), and whole DiT forwards with
online-quantized (ACE_GGML_DIT_WEIGHT_QTYPE) and GGUF weights against the oracle."""
import os
import tempfile

import numpy as np
import pytest

from oracle.ggml_numerics import bf16_bits_to_f32, f32_to_bf16_bits
from test_gpu_forward import check, check_product_vs_ggml, rel_errors

pytestmark = pytest.mark.gpu


def _capi():
    from acestep_mi355x import capi
    return capi


def _q_ref(a_bits, w_blocks, qtype):
    """fp64 product of the bf16 activations with bf16(dequant(W)) — the values the kernel's MFMAs see."""
    from oracle import ggml_numerics as g
    deq = {"q8_0": lambda r: g.dequantize_q8_0(*g.unpack_q8_0(r)), "q4_k": g.dequantize_q4_k,
           "q6_k": g.dequantize_q6_k}[qtype](w_blocks)
    wv = g.round_bf16(deq).astype(np.float64)
    av = bf16_bits_to_f32(a_bits).astype(np.float64)
    return av @ wv.T, np.abs(av) @ np.abs(wv).T


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("N,K", [(1, 256), (7, 512), (256, 2048), (96, 6144)])
def test_staged_dequant_kernel_is_exact(qtype, N, K):
    """launch_dequant_bf16 (the staged dequant's kernel) equals bf16(ggml dequant(W)), bit for bit except the
    sign of zero: q = 0 with a negative Q6_K scale is -0 in ggml's d*sc*q and +0 in the kernel's
    fma(q + 128, s, -128 s) (the dequant-fused GEMM computes the same +0; a product term of either sign is 0)."""
    from oracle import ggml_numerics as g
    rng = np.random.default_rng(N + K)
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = _capi().quantize(w, qtype)
    deq = {"q8_0": lambda r: g.dequantize_q8_0(*g.unpack_q8_0(r)), "q4_k": g.dequantize_q4_k,
           "q6_k": g.dequantize_q6_k}[qtype](blocks)
    want = f32_to_bf16_bits(np.asarray(deq, dtype=np.float32).reshape(N, K))
    got = _capi().kernel_dequant(blocks, qtype)
    bad = np.argwhere((got != want) & ~(((got | want) & 0x7FFF) == 0))
    assert len(bad) == 0, (len(bad), bad[:8].tolist())


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("variant", [-1, 1, 2, 3, 4, 5, 7, 20, 21, 22, 23, 24, 25, 222, 223, 423])
@pytest.mark.parametrize("M,N,K", [(1, 256, 256), (300, 512, 512), (1000, 256, 2048), (129, 768, 6144)])
def test_gemm_q_matches_dequantized_product(qtype, variant, M, N, K):
    """Both dequant-fused kernels (round 1's LDS-dequant tiles 1-7; the register-dequant tiles 20-24, + 100 S for
    split-K over S blocks) against an fp64 product of the same bf16 operands."""
    capi = _capi()
    if variant in (2, 5, 21) and N % 256:
        pytest.skip("256-wide tiles need N % 256 == 0")
    if variant >= 100 and K // 64 < 2 * (variant // 100):
        pytest.skip("split-K needs two k-tiles per part")
    rng = np.random.default_rng(M + K + variant)
    a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = capi.quantize(w, qtype)
    bias = rng.standard_normal(N).astype(np.float32)
    got = capi.kernel_gemm_q(a, blocks, qtype, epi=0, variant=variant, bias=bias)
    ref, scale = _q_ref(a, blocks, qtype)
    ref = ref + bias
    assert np.all(np.abs(got - ref) <= 2e-6 * scale + 1e-6), np.max(np.abs(got - ref) / (scale + 1e-6))


@pytest.mark.parametrize("variant", [-1, 1, 3, 4, 20, 22, 23, 24, 25])
@pytest.mark.parametrize("M,K", [(1100, 128), (1100, 64), (300, 128)])
def test_gemm_q_short_k_q8_0(variant, M, K):
    """Q8_0 rows of K = 128 / 64 (four / two blocks): the warp-specialised tile (25, what pick_variant_q takes at
    M > 1024 with N <= 2048 whatever K is) with only two / one k-tile in its 3-slot ring -- its prologue's counted wait
    (round 6 fix) -- and the other fused tiles' short pipelines."""
    capi = _capi()
    N = 256
    rng = np.random.default_rng(M + K + variant)
    a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = capi.quantize(w, "q8_0")
    bias = rng.standard_normal(N).astype(np.float32)
    got = capi.kernel_gemm_q(a, blocks, "q8_0", epi=0, variant=variant, bias=bias)
    ref, scale = _q_ref(a, blocks, "q8_0")
    ref = ref + bias
    assert np.all(np.abs(got - ref) <= 2e-6 * scale + 1e-6), np.max(np.abs(got - ref) / (scale + 1e-6))


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("variant", [-1, 20, 21, 22, 23, 24, 25, 222, 423])
@pytest.mark.parametrize("epi", [2, 3])
def test_gemm_q_residual_epilogues(qtype, variant, epi):
    """x += A.bf16(dequant(W))^T (* gate[n]) in place (the o / cross-o / down projections) through the
    register-dequant tiles, M edges included."""
    capi = _capi()
    M, N, K = 300, 512, 512
    if variant in (21,) and N % 256:
        pytest.skip("256-wide tiles need N % 256 == 0")
    rng = np.random.default_rng(7 * epi + variant + 100)
    a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = capi.quantize(w, qtype)
    x = rng.standard_normal((M, N)).astype(np.float32)
    gate = rng.standard_normal(N).astype(np.float32) if epi == 2 else None
    got = capi.kernel_gemm_q(a, blocks, qtype, epi=epi, variant=variant, bias=gate, x=x)
    acc, scale = _q_ref(a, blocks, qtype)
    g = gate.astype(np.float64) if epi == 2 else np.ones(N)
    ref = x.astype(np.float64) + acc * g
    assert np.all(np.abs(got - ref) <= (2e-6 * scale + 1e-6) * np.abs(g) + 2e-7 * np.abs(ref)), \
        np.max(np.abs(got - ref))


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k"])
def test_gemm_q_swiglu_epilogue(qtype):
    M, I, K = 200, 256, 512
    rng = np.random.default_rng(21)
    a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
    w = (rng.standard_normal((2 * I, K)) * 0.05).astype(np.float32)
    blocks = _capi().quantize(w, qtype)
    got = bf16_bits_to_f32(_capi().kernel_gemm_q(a, blocks, qtype, epi=4))
    ref, _ = _q_ref(a, blocks, qtype)
    gcols = np.concatenate([np.arange(grp * 32, grp * 32 + 16) for grp in range(I // 16)])
    ucols = gcols + 16
    gv, uv = ref[:, gcols], ref[:, ucols]
    sw = gv / (1.0 + np.exp(-gv)) * uv
    np.testing.assert_allclose(got, sw, rtol=2 ** -7, atol=1e-3 * np.abs(sw).max())


# ---------------------------------------------------------------- online-quantized weights (a14)
def engine_view(W):
    """The oracle weights as the MI355X engine computes with them in a quantized mode: every
    quantized matrix as bf16(dequant(q)) with bf16 activations (the dequant-fused GEMM), instead of
    ggml's Q8_0 / Q8_K activation quantization.  Test-side helper, not part of the oracle."""
    import copy
    from oracle import ggml_numerics as g

    def fix(x):
        if isinstance(x, g.GgmlWeight) and x.wtype in ("q8_0", "q4_k", "q6_k"):
            return g.GgmlWeight(g.round_bf16(x.values), "bf16")
        if isinstance(x, dict):
            return {k: fix(v) for k, v in x.items()}
        if isinstance(x, list):
            return [fix(v) for v in x]
        return x

    W2 = copy.deepcopy(W)
    for k, v in list(vars(W2).items()):
        setattr(W2, k, fix(v))
    return W2


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
def test_quantized_tiny_matches_dequant_semantics(tiny_ckpt, monkeypatch, qtype):
    """ACE_GGML_DIT_WEIGHT_QTYPE=<q>: the loader quantizes every eligible 2-D weight with the ggml
    encoders and the DiT runs on the dequant-fused GEMM; checked against the oracle on the same
    quantized bytes with bf16(dequant) weights and bf16 activations (the engine's arithmetic)."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from oracle.dit_oracle import DitWeights, forward_with_floor
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    br = GGMLCAPIBridge()
    br.load_dit(tiny_ckpt)
    rng = np.random.default_rng(31)
    T, L = 301, 20
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, 256)).astype(np.float32)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.7, 0.7)
    br.close()
    W = DitWeights(tiny_ckpt, qtype=qtype)
    ref, floor = forward_with_floor(engine_view(W), h, c, e, None, None, T, L, 0.7, 0.7)
    check(got, ref, floor, f"tiny {qtype} (dequant semantics)")
    # distance to ggml's own Q8 activation path, reported (see the full-width test for the bound)
    ggml_ref = forward_with_floor(W, h, c, e, None, None, T, L, 0.7, 0.7)
    l2, _ = rel_errors(got, ggml_ref[0])
    print(f"tiny {qtype}: vs ggml Q8-activation semantics rel_l2={l2:.3e} (ggml floor {ggml_ref[1]:.3e})")


@pytest.mark.slow
@pytest.mark.parametrize("qtype", ["q8_0", "q4_k"])
def test_quantized_full_width_vs_ggml_semantics(monkeypatch, qtype):
    """Full width, 2 layers, T = 400, against the oracle WITH ggml's activation quantization (Q8_0 blocks for Q8_0
    weights, Q8_K for K-quants): the ggml-faithful mode (ACE_MI_QUANT_ACT=q8, kernels/gemm_a8.hip) within 1.5x the
    oracle's own floor, element-wise too.  The product path (bf16 activations) is checked against its own arithmetic
    and held to GGML_PRODUCT_K (1.75) x the ggml path's floor against ggml's semantics: 8-bit activation rounding
    amplifies any f32 difference much harder than bf16 does (measured 1.3-1.6x, DESIGN.md "Parity")."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor, forward_with_floor_stats
    cfg = make_config(num_hidden_layers=2)
    d = cached_checkpoint(cfg, seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    rng = np.random.default_rng(77)
    T, L = 400, 64
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    got = {}
    for mode in ("bf16", "q8"):
        monkeypatch.setenv("ACE_MI_QUANT_ACT", mode)
        br = GGMLCAPIBridge()
        br.load_dit(d)
        got[mode] = br.dit_forward_tfirst(h, c, e, None, None, 0.8, 0.8)
        br.close()
    W = DitWeights(d, qtype=qtype)
    ref, floor, fmax = forward_with_floor_stats(W, h, c, e, None, None, T, L, 0.8, 0.8, max_layers=2)
    check_product_vs_ggml(got["bf16"], ref, floor, fmax, f"full-width {qtype}")
    check(got["q8"], ref, floor, f"full-width {qtype} ACE_MI_QUANT_ACT=q8 (ggml semantics)", fmax)
    eng = forward_with_floor(engine_view(W), h, c, e, None, None, T, L, 0.8, 0.8, max_layers=2)
    check(got["bf16"], eng[0], eng[1], f"full-width {qtype} product path (dequant semantics)")


# ---------------------------------------------------------------- GGUF weights (a14 / SURVEY §8f)
@pytest.mark.parametrize("quant", ["Q8", "Q4", "F16"])
def test_gguf_tiny_matches_oracle(tiny_ckpt, monkeypatch, quant):
    """model.gguf next to config.json (resolve_gguf_path, acestep_dit_model.cpp:47-70): types kept as
    stored, proj_in/proj_out converted to F32 (the engine's fp16 hi/lo triple GEMM), no online
    quantization even if ACE_GGML_DIT_WEIGHT_QTYPE is set."""
    import shutil
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import write_gguf
    from oracle.dit_oracle import DitWeights, forward_with_floor
    d = tempfile.mkdtemp(prefix="acemi_gguf_")
    shutil.copy(os.path.join(tiny_ckpt, "config.json"), d)
    path = write_gguf(os.path.join(tiny_ckpt, "model.safetensors"), os.path.join(d, "model.gguf"), quant=quant)
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", "q6_k")   # ignored on the GGUF path
    br = GGMLCAPIBridge()
    br.load_dit(d)
    rng = np.random.default_rng(41)
    T, L = 150, 12
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, 256)).astype(np.float32)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6)
    br.close()
    W = DitWeights(d, gguf=path)
    ref, floor = forward_with_floor(engine_view(W), h, c, e, None, None, T, L, 0.6, 0.6)
    check(got, ref, floor, f"tiny GGUF {quant}")




@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("width", ["tiny", "full", "240s"])
def test_staged_dequant_equals_fused(tiny_ckpt, monkeypatch, qtype, width):
    """The staged dequant (ACE_MI_QUANT_STAGED, default: each layer's bf16 weight image expanded right before the
    layer, dense GEMMs) and the dequant-fused GEMMs (ACE_MI_QUANT_STAGED=0) give the same bits: both multiply
    bf16 activations by bf16(dequant(W)) with the same per-element summation order."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    if width == "tiny":
        d, H, T, L = tiny_ckpt, 256, 301, 20
    elif width == "240s":  # M = 3000: the register-dequant 192-row tiles (incl. their attention-prep epilogue)
        from acestep_mi355x.synthetic import cached_checkpoint, make_config
        d, H, T, L = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch"), 2048, 6000, 512
        monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    else:
        from acestep_mi355x.synthetic import cached_checkpoint, make_config
        d, H, T, L = cached_checkpoint(make_config(num_hidden_layers=3), seed=0, backend="torch"), 2048, 400, 64
        monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "3")
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    rng = np.random.default_rng(5)
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, H)).astype(np.float32)
    # short sequences: the same 96 x 128 tiles on both paths (the automatic dense pick there splits the K = 6144
    # down projection over two blocks, a different summation order from the unsplit fused tile); at 240 s both
    # paths run their automatic tiles (staged: dense 192 / 96-row; fused: the register-dequant 192-row tiles)
    from acestep_mi355x import capi
    outs = []
    for staged in ("1", "0"):
        monkeypatch.setenv("ACE_MI_QUANT_STAGED", staged)
        br = GGMLCAPIBridge()
        br.load_dit(d)
        capi.gemm_variant(-1 if width == "240s" else 7)
        try:
            outs.append(br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6))
            outs.append(br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6))  # slot reused by a second forward
        finally:
            capi.gemm_variant(-1)
        br.close()
    assert np.isfinite(outs[0]).all()
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k"])
def test_sampling_call_scope_staging_equals_per_layer(tiny_ckpt, monkeypatch, qtype):
    """ace_mi_dit_sample_ex with quantized weights: the bf16 images kept for the model (ACE_MI_QUANT_STAGE_SCOPE=
    model, default) or expanded once per sampling call (=call; steps 1.. reuse them) give the same bits as expanding them
    before every layer of every step (=layer) and as the dequant-fused GEMMs (ACE_MI_QUANT_STAGED=0).
    A first call on fewer layers (ACE_GGML_DIT_MAX_LAYERS) must not leave images a later call reuses."""
    import torch
    from acestep_mi355x.capi import GGMLCAPIBridge
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    rng = np.random.default_rng(9)
    B, T, L = 2, 301, 20
    x0 = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    sched = [1.0, 0.75, 0.5, 0.25]
    dc, de = (torch.from_numpy(a).cuda() for a in (c, e))
    outs = []
    for scope, staged in (("model", "1"), ("call", "1"), ("layer", "1"), ("call", "0")):
        monkeypatch.setenv("ACE_MI_QUANT_STAGE_SCOPE", scope)
        monkeypatch.setenv("ACE_MI_QUANT_STAGED", staged)
        br = GGMLCAPIBridge()
        br.load_dit(tiny_ckpt)
        monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "1")
        xt = torch.from_numpy(x0).cuda()
        torch.cuda.synchronize()
        br.dit_sample_ex_device(B, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, sched)
        br.synchronize()
        monkeypatch.delenv("ACE_GGML_DIT_MAX_LAYERS")
        for _ in range(2):  # the second call expands the images again and must give the same bits
            xt = torch.from_numpy(x0).cuda()
            torch.cuda.synchronize()
            br.dit_sample_ex_device(B, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, sched)
            br.synchronize()
            outs.append(xt.cpu().numpy())
        br.close()
    assert np.isfinite(outs[0]).all()
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])
