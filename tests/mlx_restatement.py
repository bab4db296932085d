"""Independent float64 restatement of the reference's SECOND reading of the DiT: the MLX decoder
(`acestep/mlx_dit/model.py`, read as text; `mlx` is Darwin-only and is not imported here), used to check
that oracle/dit_oracle.py (the restatement of the ggml graph, acestep_dit_model.cpp:1316-1560) reads the
model the same way.  TEST INFRASTRUCTURE ONLY.

It deliberately follows the MLX module structure rather than the ggml graph, so that a misreading shared
by the oracle and the HIP kernels (pack order, RoPE pairing, GQA head map, which norm is modulated, the
t - r embedding, the output head's pre-SiLU temb, the de-patchify order) shows up as a disagreement:

* weights in their PyTorch layouts as stored in the checkpoint: Conv1d [out][in][k] for `proj_in`
  (model.py:464-471), ConvTranspose1d [in][out][k] for `proj_out` (:491-497), Linear [out][in];
* RoPE from `inv_freq = base^(-arange(0, D, 2)/D)` and `rotate_half` (:16-34, :62-88) — not ggml's running
  product;
* sliding layers as an additive -1e9 mask on |i - j| > window (:37-55); no key-padding and no
  encoder mask (the MLX decoder passes `encoder_attention_mask=None`, :598-606), so callers compare
  on all-valid inputs;
* GQA by `repeat_kv` (:183-191): query head h reads kv head h // n_rep;
* every op in float64, no activation rounding.
"""
import math

import numpy as np


def _rms(x, w, eps):
    return x / np.sqrt(np.mean(x * x, axis=-1, keepdims=True) + eps) * w


def _silu(x):
    return x / (1.0 + np.exp(-x))


def _linear(x, W, b=None):
    y = x @ W.T
    return y if b is None else y + b


def _timestep_embedding(st, tag, t):
    """MLXTimestepEmbedding (:355-411) for one scalar t: (temb [D], proj [6][D])."""
    half = 128
    freqs = np.exp(-math.log(10000.0) * np.arange(half, dtype=np.float64) / half)
    args = (t * 1000.0) * freqs
    f = np.concatenate([np.cos(args), np.sin(args)])
    p = f"decoder.{tag}."
    temb = _linear(_silu(_linear(f, st[p + "linear_1.weight"], st[p + "linear_1.bias"])),
                   st[p + "linear_2.weight"], st[p + "linear_2.bias"])
    proj = _linear(_silu(temb), st[p + "time_proj.weight"], st[p + "time_proj.bias"])
    return temb, proj.reshape(6, -1)


def _rope(n, D, base):
    inv = 1.0 / (base ** (np.arange(0, D, 2, dtype=np.float64) / D))
    fr = np.arange(n, dtype=np.float64)[:, None] * inv[None, :]
    fr = np.concatenate([fr, fr], axis=-1)
    return np.cos(fr), np.sin(fr)


def _rotate_half(x):
    h = x.shape[-1] // 2
    return np.concatenate([-x[..., h:], x[..., :h]], axis=-1)


def _attn(st, pre, cfg, x, enc, cos_sin, mask):
    """MLXAttention (:138-239) for one item: x [L][H], enc [Le][H] or None (self-attention)."""
    hq, hkv, D = cfg["num_attention_heads"], cfg["num_key_value_heads"], cfg["head_dim"]
    eps = cfg["rms_norm_eps"]
    L = x.shape[0]
    src = x if enc is None else enc
    Lk = src.shape[0]
    q = _rms(_linear(x, st[pre + "q_proj.weight"]).reshape(L, hq, D), st[pre + "q_norm.weight"], eps)
    k = _rms(_linear(src, st[pre + "k_proj.weight"]).reshape(Lk, hkv, D), st[pre + "k_norm.weight"], eps)
    v = _linear(src, st[pre + "v_proj.weight"]).reshape(Lk, hkv, D)
    if enc is None and cos_sin is not None:
        cos, sin = cos_sin
        q = q * cos[:, None, :] + _rotate_half(q) * sin[:, None, :]
        k = k * cos[:, None, :] + _rotate_half(k) * sin[:, None, :]
    rep = hq // hkv
    k = np.repeat(k, rep, axis=1)  # [Lk][hq][D], head h <- kv head h // rep
    v = np.repeat(v, rep, axis=1)
    s = np.einsum("qhd,khd->hqk", q, k) * (D ** -0.5)
    if mask is not None:
        s = s + mask[None]
    s = s - s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(axis=-1, keepdims=True)
    o = np.einsum("hqk,khd->qhd", p, v).reshape(L, hq * D)
    return _linear(o, st[pre + "o_proj.weight"])


def mlx_forward(st, cfg, hidden, context, enc, t, r):
    """MLXDiTDecoder.__call__ (:517-608) for one item (batch of 1).  st: name -> float64 array in the
    checkpoint's layout; hidden [T][64], context [T][C_ctx], enc [Le][H]; returns [T][64]."""
    eps = cfg["rms_norm_eps"]
    P = cfg["patch_size"]
    H = cfg["hidden_size"]
    temb_t, proj_t = _timestep_embedding(st, "time_embed", t)
    temb_r, proj_r = _timestep_embedding(st, "time_embed_r", t - r)
    temb = temb_t + temb_r
    tproj = proj_t + proj_r
    x = np.concatenate([context, hidden], axis=-1)  # context first (:546)
    T = x.shape[0]
    if T % P:
        x = np.concatenate([x, np.zeros((P - T % P, x.shape[1]))], axis=0)
    # Conv1d(kernel = stride = P): y[n][o] = sum_{c,k} W[o][c][k] x[nP + k][c] + b[o]
    Wi = st["decoder.proj_in.1.weight"]
    xp = x.reshape(-1, P, x.shape[1])
    h = np.einsum("nkc,ock->no", xp, Wi) + st["decoder.proj_in.1.bias"]
    e = _linear(enc, st["decoder.condition_embedder.weight"], st["decoder.condition_embedder.bias"])
    n = h.shape[0]
    cos_sin = _rope(n, cfg["head_dim"], cfg["rope_theta"])
    idx = np.arange(n)
    smask = np.where(np.abs(idx[:, None] - idx[None, :]) <= cfg["sliding_window"], 0.0, -1e9)
    for i, lt in enumerate(cfg["layer_types"][:cfg["num_hidden_layers"]]):
        p = f"decoder.layers.{i}."
        mod = st[p + "scale_shift_table"].reshape(6, H) + tproj
        shift, scale, gate, c_shift, c_scale, c_gate = mod
        nrm = _rms(h, st[p + "self_attn_norm.weight"], eps) * (1.0 + scale) + shift
        h = h + _attn(st, p + "self_attn.", cfg, nrm, None, cos_sin,
                      smask if lt == "sliding_attention" else None) * gate
        nrm = _rms(h, st[p + "cross_attn_norm.weight"], eps)
        h = h + _attn(st, p + "cross_attn.", cfg, nrm, e, None, None)
        nrm = _rms(h, st[p + "mlp_norm.weight"], eps) * (1.0 + c_scale) + c_shift
        ff = _linear(_silu(_linear(nrm, st[p + "mlp.gate_proj.weight"])) * _linear(nrm, st[p + "mlp.up_proj.weight"]),
                     st[p + "mlp.down_proj.weight"])
        h = h + ff * c_gate
    oss = st["decoder.scale_shift_table"].reshape(2, H) + temb[None, :]
    h = _rms(h, st["decoder.norm_out.weight"], eps) * (1.0 + oss[1]) + oss[0]
    # ConvTranspose1d(kernel = stride = P): y[nP + k][o] = sum_c W[c][o][k] h[n][c] + b[o]
    Wo = st["decoder.proj_out.1.weight"]
    y = np.einsum("nc,cok->nko", h, Wo).reshape(n * P, -1) + st["decoder.proj_out.1.bias"]
    return y[:T]
