"""The oracle's reading of the DiT graph (oracle/dit_oracle.py, from acestep_dit_model.cpp:1316-1560) against an
independent float64 restatement of the reference's second implementation of the same model, the MLX decoder
(tests/mlx_restatement.py, from acestep/mlx_dit/model.py:413-629).  F32 weights, so ggml rounds no activation
and the two differ only by f32-vs-f64 arithmetic and ggml's RoPE running product; all-valid inputs (the MLX
decoder applies no key-padding or encoder mask).  CPU only."""
import os
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT, os.path.dirname(os.path.abspath(__file__))]

from mlx_restatement import mlx_forward  # noqa: E402


def _run(cfg, T, L, seed, t, r):
    from acestep_mi355x.synthetic import _read_safetensors_f32, write_checkpoint
    from oracle.dit_oracle import DitWeights, forward_dit
    with tempfile.TemporaryDirectory() as d:
        write_checkpoint(d, cfg, seed=seed, dtype="F32")
        W = DitWeights(d)
        st = {k: v.astype(np.float64) for k, v in _read_safetensors_f32(os.path.join(d, "model.safetensors")).items()}
    rng = np.random.default_rng(seed + 1)
    H = cfg["hidden_size"]
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, cfg["in_channels"] - 64)).astype(np.float32)
    e = rng.standard_normal((L, H)).astype(np.float32)
    got = forward_dit(W, h, c, e, None, None, T, L, t, r).astype(np.float64)
    ref = mlx_forward(st, cfg, h.astype(np.float64), c.astype(np.float64), e.astype(np.float64), float(np.float32(t)),
                      float(np.float32(r)))
    rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    sel = np.abs(ref) > 1e-2 * np.sqrt(np.mean(ref * ref))
    rel_max = float(np.max(np.abs(got - ref)[sel] / np.abs(ref[sel])))
    return rel, rel_max


@pytest.mark.parametrize("T,t,r", [(61, 0.8, 0.8), (96, 0.6, 0.25)])
def test_oracle_matches_mlx_reading_tiny(T, t, r):
    """Tiny config (2 layers: one sliding with window 16, one full), odd T (patch padding), r != t."""
    from acestep_mi355x.synthetic import TINY_CONFIG
    rel, rel_max = _run(TINY_CONFIG, T, 7, 3, t, r)
    print(f"tiny T={T}: oracle vs MLX restatement rel_l2={rel:.2e} rel_max={rel_max:.2e}")
    assert rel < 2e-6 and rel_max < 1e-3


def test_oracle_matches_mlx_reading_full_width():
    """Full width (hidden 2048, 16/8 heads, MLP 6144), 2 layers (sliding w = 128 then full), N = 150 tokens so
    the window mask bites."""
    from acestep_mi355x.synthetic import make_config
    rel, rel_max = _run(make_config(num_hidden_layers=2), 300, 16, 5, 0.7, 0.7)
    print(f"full width 2 layers T=300: oracle vs MLX restatement rel_l2={rel:.2e} rel_max={rel_max:.2e}")
    assert rel < 5e-6 and rel_max < 1e-3
