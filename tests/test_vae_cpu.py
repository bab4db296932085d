"""VAE decoder oracle (oracle/vae_oracle.py) checked against independent implementations of the
same operators (torch CPU float64 conv1d / conv_transpose1d / weight_norm), the MLX Snake text, and
the reference tiled-decode window plan (scripts/run_non_ggml_real_case.py:597-649)."""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import vae_oracle as V
from oracle.ggml_numerics import round_f16


def test_conv1d_matches_torch_on_f16_operands():
    rng = np.random.default_rng(0)
    for (T, cin, cout, k, d) in [(50, 64, 128, 7, 1), (33, 128, 128, 7, 9), (20, 128, 128, 1, 1)]:
        x = rng.standard_normal((T, cin)).astype(np.float32)
        w = round_f16(rng.standard_normal((cout, cin, k)).astype(np.float32) * 0.05)
        b = rng.standard_normal(cout).astype(np.float32)
        pad = (k - 1) * d // 2
        got = V.conv1d(x, w, b, d, pad)
        ref = torch.nn.functional.conv1d(torch.from_numpy(round_f16(x).T[None].astype(np.float64)),
                                         torch.from_numpy(w.astype(np.float64)), torch.from_numpy(b.astype(np.float64)),
                                         padding=pad, dilation=d)[0].T.numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("stride", [2, 3, 4, 6, 10])
def test_conv_transpose_with_center_crop_matches_torch_padding(stride):
    """ggml conv_transpose_1d(p0=0) + center crop == PyTorch ConvTranspose1d(padding=ceil(s/2))."""
    rng = np.random.default_rng(stride)
    T, cin, cout = 17, 64, 32
    x = rng.standard_normal((T, cin)).astype(np.float32)
    w = round_f16(rng.standard_normal((cin, cout, 2 * stride)).astype(np.float32) * 0.05)
    b = rng.standard_normal(cout).astype(np.float32)
    pad = (stride + 1) // 2
    got = V.conv_transpose1d(x, w, b, stride, pad)
    ref = torch.nn.functional.conv_transpose1d(torch.from_numpy(round_f16(x).T[None].astype(np.float64)),
                                               torch.from_numpy(w.astype(np.float64)),
                                               torch.from_numpy(b.astype(np.float64)), stride=stride,
                                               padding=pad)[0].T.numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


def test_weight_norm_fold_matches_torch():
    rng = np.random.default_rng(3)
    v = rng.standard_normal((16, 8, 7)).astype(np.float32)
    g = rng.random((16, 1, 1)).astype(np.float32) + 0.5
    got = V.fold_weight_norm(g, v)
    ref = torch._weight_norm(torch.from_numpy(v.astype(np.float64)), torch.from_numpy(g.astype(np.float64)), 0).numpy()
    np.testing.assert_allclose(got, ref, rtol=2 ** -10, atol=1e-6)


def test_snake_is_mlx_form_without_epsilon():
    """acestep/mlx_vae/model.py:55: x + 1/(e^b + 1e-9) * sin(e^a x)^2 — ggml has no 1e-9."""
    rng = np.random.default_rng(4)
    x = rng.standard_normal((40, 8)).astype(np.float32)
    a = rng.standard_normal(8).astype(np.float32) * 0.3
    b = rng.standard_normal(8).astype(np.float32) * 0.3
    got = V.snake(x, a, b)
    ref = x.astype(np.float64) + np.sin(np.exp(a) * x.astype(np.float64)) ** 2 / np.exp(b.astype(np.float64))
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


def _ref_tile_plan(T, chunk_size, overlap):
    # run_non_ggml_real_case.py:597-611 restated
    max_overlap = max(0, (chunk_size // 2) - 1)
    if overlap > max_overlap:
        overlap = max_overlap
    stride = chunk_size - 2 * overlap
    if stride <= 0:
        overlap = max(0, chunk_size // 4)
        stride = chunk_size - 2 * overlap
        if stride <= 0:
            stride = max(1, chunk_size)
            overlap = 0
    import math
    out = []
    for i in range(int(math.ceil(T / float(stride)))):
        cs = i * stride
        ce = min(cs + stride, T)
        out.append((cs, ce, max(0, cs - overlap), min(T, ce + overlap)))
    return out


@pytest.mark.parametrize("T,chunk,overlap", [(100, 32, 8), (33, 32, 8), (250, 16, 20), (7, 2, 1), (64, 3, 0)])
def test_tile_plan_matches_reference(T, chunk, overlap):
    from acestep_mi355x.hook import _tile_plan
    assert _tile_plan(T, chunk, overlap) == _ref_tile_plan(T, chunk, overlap)


def test_synthetic_vae_checkpoint_decodes_in_oracle():
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    d = tempfile.mkdtemp()
    write_vae_checkpoint(d, VAE_TINY_CONFIG)
    W = V.VaeWeights(d)
    assert W.cfg.hop_length == 6 and W.cfg.upsampling_ratios == [3, 2]
    lat = np.random.default_rng(0).standard_normal((20, 64)).astype(np.float32)
    y = V.decode(W, lat)
    # odd stride 3: PyTorch ConvTranspose1d length (20+1)*3 - 2*2 = 59, then (59+1)*2 - 2 = 118
    assert y.shape == (118, 2) and np.all(np.isfinite(y))


def test_implicit_gemm_formulation_reproduces_the_oracle():
    """The layouts and index maps used by kernels/vae.hip + runtime/vae.cpp, restated in numpy:
    weights re-laid out as the loader does, A rows gathered as conv_gemm_kernel's stage() does
    (row m, tap -> input row m + tap*dil - pad, zero outside), output columns mapped as its epilogue
    does (conv_t: n = r*Cout + co -> u = s*m + r - crop).  Must reproduce the oracle's decoder."""
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    d = tempfile.mkdtemp()
    write_vae_checkpoint(d, VAE_TINY_CONFIG)
    W = V.VaeWeights(d)

    def gemm_conv(S, Wm, taps, dil, pad, M, T_in, Cin):
        A = np.zeros((M, taps * Cin), np.float64)
        for m in range(M):
            for tap in range(taps):
                t = m + tap * dil - pad
                if 0 <= t < T_in:
                    A[m, tap * Cin:(tap + 1) * Cin] = S[t]
        return A @ Wm.T

    def conv_layout(w):            # [Cout][Cin][K] -> [Cout][K*Cin]
        return np.transpose(w, (0, 2, 1)).reshape(w.shape[0], -1).astype(np.float64)

    def convt_layout(w, s):        # [Cin][Cout][2s] -> [s*Cout][2*Cin]
        cin, cout, _ = w.shape
        out = np.zeros((s * cout, 2 * cin))
        for r in range(s):
            for tap in range(2):
                out[r * cout:(r + 1) * cout, tap * cin:(tap + 1) * cin] = w[:, :, r + tap * s].T
        return out

    def snake(v, sn):
        return V.snake(v.astype(np.float32), sn["alpha"], sn["beta"])

    lat = np.random.default_rng(1).standard_normal((13, 64)).astype(np.float32)
    S = round_f16(lat).astype(np.float64)
    X = gemm_conv(S, conv_layout(W.conv1["w"]), 7, 1, 3, 13, 13, 64) + W.conv1["b"]
    L = 13
    for blk in W.blocks:
        s = blk["stride"]
        p = (s + 1) // 2
        Sa = round_f16(snake(X, blk["snake1"])).astype(np.float64)
        full = (L + 1) * s
        Lo = full - 2 * p
        cout = blk["conv_t1"]["w"].shape[1]
        G = gemm_conv(Sa, convt_layout(blk["conv_t1"]["w"], s), 2, -1, 0, L + 1, L, Sa.shape[1])
        Xn = np.zeros((Lo, cout))
        for m in range(L + 1):
            for n in range(s * cout):
                r, co = divmod(n, cout)
                u = m * s + r - p
                if 0 <= u < Lo:
                    Xn[u, co] = G[m, n] + blk["conv_t1"]["b"][co]
        X, L = Xn, Lo
        for ru in blk["res"]:
            Sb = round_f16(snake(X, ru["snake1"])).astype(np.float64)
            Y = gemm_conv(Sb, conv_layout(ru["conv1"]["w"]), 7, ru["dil"], 3 * ru["dil"], L, L, Sb.shape[1])
            Sc = round_f16(snake(Y + ru["conv1"]["b"], ru["snake2"])).astype(np.float64)
            X = X + (gemm_conv(Sc, conv_layout(ru["conv2"]["w"]), 1, 1, 0, L, L, Sc.shape[1]) + ru["conv2"]["b"])
    Sf = round_f16(snake(X, W.snake1)).astype(np.float64)
    out = gemm_conv(Sf, conv_layout(W.conv2["w"]), 7, 1, 3, L, L, Sf.shape[1])
    ref = V.decode(W, lat)
    assert out.shape == ref.shape
    rel = np.linalg.norm(out - ref) / np.linalg.norm(ref)
    assert rel < 2e-3, rel


@pytest.mark.parametrize("stride", [2, 4, 6])
def test_strided_conv_matches_torch(stride):
    """encoder downsampling conv: ggml_conv_1d(s0=s, p0=ceil(s/2)), kernel 2s."""
    rng = np.random.default_rng(stride + 10)
    T, cin, cout = 61, 64, 32
    x = rng.standard_normal((T, cin)).astype(np.float32)
    w = round_f16(rng.standard_normal((cout, cin, 2 * stride)).astype(np.float32) * 0.05)
    b = rng.standard_normal(cout).astype(np.float32)
    pad = (stride + 1) // 2
    got = V.conv1d(x, w, b, 1, pad, stride=stride)
    ref = torch.nn.functional.conv1d(torch.from_numpy(round_f16(x).T[None].astype(np.float64)),
                                     torch.from_numpy(w.astype(np.float64)), torch.from_numpy(b.astype(np.float64)),
                                     stride=stride, padding=pad)[0].T.numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


def test_encoder_round_trip_shapes():
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    d = tempfile.mkdtemp()
    write_vae_checkpoint(d, VAE_TINY_CONFIG)
    W = V.VaeWeights(d)
    audio = np.random.default_rng(2).standard_normal((120, 2)).astype(np.float32)
    z = V.encode(W, audio)
    assert z.shape == (20, 64) and np.all(np.isfinite(z))
