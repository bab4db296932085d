"""CPU tests of the oracle (test infrastructure) against golden vectors and closed forms."""
import json
import math
import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ggml_numerics as gn
from oracle.dit_oracle import (DitWeights, apply_rope_neox, build_key_bias, forward_dit, rms_norm, rope_tables,
                               timestep_freq)


def test_bf16_rounding_matches_torch_rne():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(100000).astype(np.float32) * 10,
                        np.array([0.0, -0.0, 1.0, 1.00390625, 1.01171875, 3.4e38, -3.4e38, 1e-40, np.inf, -np.inf],
                                 dtype=np.float32)])
    ref = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    got = gn.round_bf16(x)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.isnan(gn.round_bf16(np.array([np.nan], np.float32)))[0]


def test_q8_0_weight_roundtrip_matches_metal_formula():
    # ggml-metal-embed.metal:3110-3128 quantize (d = amax/127, q = round(x/d)) and :3328-3339 dequant (q*d)
    rng = np.random.default_rng(1)
    w = rng.standard_normal((8, 64)).astype(np.float32)
    d, q = gn.quantize_q8_0_weights(w)
    assert d.dtype == np.float16 and q.dtype == np.int8 and q.shape == (8, 2, 32)
    blk = w.reshape(8, 2, 32)
    amax = np.abs(blk).max(axis=2)
    np.testing.assert_array_equal(d, (amax / 127).astype(np.float16))
    assert np.abs(q).max() <= 127
    deq = gn.dequantize_q8_0(d, q)
    err = np.abs(deq - w).reshape(8, 2, 32).max(axis=2)
    assert np.all(err <= d.astype(np.float32) * 0.5 + amax * 2e-3)
    raw = gn.pack_q8_0(d, q)
    assert raw.shape == (8, 2, 34)
    d2, q2 = gn.unpack_q8_0(raw)
    np.testing.assert_array_equal(d2, d)
    np.testing.assert_array_equal(q2, q)


def test_q8_0_zero_block_and_half_rounding():
    w = np.zeros((1, 32), np.float32)
    d, q = gn.quantize_q8_0_weights(w)
    assert float(d[0, 0]) == 0 and not q.any()
    # roundf rounds halves away from zero for weights; activations use round-half-even (AVX)
    x = np.zeros((1, 32), np.float32)
    x[0, 0] = 127.0
    x[0, 1] = 0.5
    x[0, 2] = -2.5
    _, qw = gn.quantize_q8_0_weights(x)
    _, qa = gn.quantize_q8_0_activations(x)
    assert qw[0, 0, 1] == 1 and qw[0, 0, 2] == -3
    assert qa[0, 0, 1] == 0 and qa[0, 0, 2] == -2


def test_q4_k_layout_and_dequant():
    rng = np.random.default_rng(2)
    w = rng.standard_normal((4, 512)).astype(np.float32) * 0.05
    raw = gn.quantize_q4_k_weights(w)
    assert raw.shape == (4, 2, 144)
    deq = gn.dequantize_q4_k(raw)
    rel = np.linalg.norm(deq - w) / np.linalg.norm(w)
    assert rel < 0.12, rel
    # 6-bit scale/min packing is exactly invertible (get_scale_min_k4, metal :3429-3432)
    ls = rng.integers(0, 64, size=(5, 8)).astype(np.uint8)
    lm = rng.integers(0, 64, size=(5, 8)).astype(np.uint8)
    sc = np.zeros((5, 12), np.uint8)
    sc[:, 0:4] = ls[:, 0:4]
    sc[:, 4:8] = lm[:, 0:4]
    sc[:, 8:12] = (ls[:, 4:8] & 0xF) | ((lm[:, 4:8] & 0xF) << 4)
    sc[:, 0:4] |= (ls[:, 4:8] >> 4) << 6
    sc[:, 4:8] |= (lm[:, 4:8] >> 4) << 6
    s2, m2 = gn._q4k_scale_min(sc)
    np.testing.assert_array_equal(s2, ls)
    np.testing.assert_array_equal(m2, lm)


def test_q8_k_activation_roundtrip():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((3, 512)).astype(np.float32)
    y = gn.q8_k_activation_roundtrip(x)
    blk = np.abs(x.reshape(3, 2, 256)).max(axis=2)
    assert np.all(np.abs(y - x).reshape(3, 2, 256).max(axis=2) <= blk / 127 * 0.5 + 1e-6)


def test_mul_mat_rounds_activation_to_weight_type():
    rng = np.random.default_rng(4)
    w = gn.round_bf16(rng.standard_normal((16, 64)).astype(np.float32))
    x = rng.standard_normal((3, 64)).astype(np.float32)
    W = gn.GgmlWeight(w, "bf16")
    np.testing.assert_allclose(gn.mul_mat(W, x), gn.round_bf16(x) @ w.T, rtol=1e-6, atol=1e-6)


def test_rope_table_close_to_closed_form():
    cos, sin = rope_tables(300, 128, 1000000.0)
    pos = np.arange(300)[:, None].astype(np.float64)
    inv = 1000000.0 ** (-np.arange(64) * 2 / 128)
    ang = pos * inv[None, :]
    # the running f32 product of ggml's rope cache drifts by a few ulp of the angle
    assert np.abs(cos - np.cos(ang)).max() < 2e-4
    assert np.abs(sin - np.sin(ang)).max() < 2e-4
    x = np.random.default_rng(5).standard_normal((300, 2, 128)).astype(np.float32)
    y = apply_rope_neox(x, cos, sin)
    np.testing.assert_allclose(np.linalg.norm(y, axis=-1), np.linalg.norm(x, axis=-1), rtol=1e-5)


def test_attention_mask_semantics():
    # build_attention_mask (acestep_dit_model.cpp:1132-1173), causal = false
    b = build_key_bias(6, 6, np.array([1, 1, 1, 1, 0, 1]), True, 2)
    allow = np.isfinite(b)
    for q in range(6):
        for k in range(6):
            assert allow[q, k] == (abs(q - k) <= 2 and k != 4)
    assert build_key_bias(4, 4, None, False, 0) is None


def test_rms_norm_and_timestep_freq():
    x = np.array([[3.0, 4.0]], np.float32)
    np.testing.assert_allclose(rms_norm(x, None, 0.0), x / math.sqrt(12.5), rtol=1e-6)
    f = timestep_freq(0.5)
    assert f.shape == (1, 256)
    np.testing.assert_allclose(f[0, 0], math.cos(500.0), rtol=1e-5)
    np.testing.assert_allclose(f[0, 128], math.sin(500.0), rtol=1e-4, atol=1e-5)


def test_oracle_forward_matches_golden():
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    z = np.load(os.path.join(GOLDEN, "dit_tiny.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    with tempfile.TemporaryDirectory() as d:
        write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
        W = DitWeights(d)
        for n in names:
            T, L, t, r = z[f"{n}/meta"]
            T, L = int(T), int(L)
            m = z[f"{n}/mask"]
            em = z[f"{n}/enc_mask"]
            out = forward_dit(W, z[f"{n}/hidden"], z[f"{n}/context"], z[f"{n}/enc"] if L > 0 else None,
                              m if m.size else None, em if em.size else None, T, L, float(t), float(r))
            np.testing.assert_allclose(out, z[f"{n}/out"], rtol=2e-5, atol=2e-5)


def test_oracle_padding_and_masks_behave():
    """Odd T is zero padded to the patch (:1343-1348) and cropped back; a frame mask that
    zeroes whole patches changes the result; an all-valid mask equals no mask."""
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    rng = np.random.default_rng(7)
    with tempfile.TemporaryDirectory() as d:
        write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
        W = DitWeights(d)
        T, L = 21, 6
        h = rng.standard_normal((T, 64)).astype(np.float32)
        c = rng.standard_normal((T, 128)).astype(np.float32)
        e = rng.standard_normal((L, 256)).astype(np.float32)
        a = forward_dit(W, h, c, e, None, None, T, L, 0.6, 0.6)
        b = forward_dit(W, h, c, e, np.ones(T, np.int32), np.ones(L, np.int32), T, L, 0.6, 0.6)
        np.testing.assert_array_equal(a, b)
        mk = np.ones(T, np.int32)
        mk[:4] = 0
        cm = forward_dit(W, h, c, e, mk, None, T, L, 0.6, 0.6)
        assert a.shape == (T, 64) and np.abs(cm - a).max() > 1e-4
