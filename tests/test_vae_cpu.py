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
