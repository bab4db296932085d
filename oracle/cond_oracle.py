"""numpy restatement of the condition encoders — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, with the ggml-cpu numerics of oracle/ggml_numerics.py:
  forward_lyric_encoder   acestep_dit_model.cpp:1562-1651
  forward_timbre_encoder  acestep_dit_model.cpp:1653-1737
  ace_project_tokens_linear            acestep_ggml.cpp:1624-1678
  ace_pack_sequences_single_batch      acestep_ggml.cpp:1729-1801
  the encoder_hidden_states assembly of ace_generate_audio_style_lyric_timbre_impl
                                       acestep_ggml.cpp:2414-2556
Weights come from oracle.dit_oracle.DitWeights (text_proj / lyric / timbre).
"""
from __future__ import annotations

import numpy as np

from . import ggml_numerics
from .dit_oracle import DitWeights, attention, mul_mat, rms_norm, rope_tables, silu


class EncoderFailed(Exception):
    """forward_*_encoder returned nullptr (missing weights / shape mismatch)."""


def _lyric_in_dim(c):
    return c.text_hidden_dim if c.text_hidden_dim > 0 else 1024


def _timbre_in_dim(c):
    return c.timbre_hidden_dim if c.timbre_hidden_dim > 0 else (
        c.audio_acoustic_hidden_dim if c.audio_acoustic_hidden_dim > 0 else 64)


def encoder_blocks(W: DitWeights, enc: dict, x: np.ndarray, max_layers: int | None = None) -> np.ndarray:
    """The EncoderLayer loop + final norm shared by both encoders (:1614-1645 / :1705-1730):
    x += attn(rms_norm(x)); x += mlp(rms_norm(x)); x = rms_norm(x, norm).  Token mask all ones, RoPE
    positions 0..n-1, sliding layers |q - k| <= window."""
    c = W.cfg
    n = x.shape[0]
    rope = rope_tables(n, c.head_dim, c.rope_theta)
    layers = enc["layers"] if max_layers is None else enc["layers"][:max_layers]
    for L in layers:
        xn = rms_norm(x, L["input_norm"], c.rms_norm_eps)
        a = attention(c, L["self_attn"], xn, xn, np.ones(n, np.int32), L["sliding"], c.sliding_window, rope)
        h = (x + a).astype(np.float32)
        hn = rms_norm(h, L["post_norm"], c.rms_norm_eps)
        g = mul_mat(L["mlp"]["gate"], hn)
        u = mul_mat(L["mlp"]["up"], hn)
        act = (silu(g) * u).astype(np.float32)
        x = (h + mul_mat(L["mlp"]["down"], act)).astype(np.float32)
    if enc["norm"] is not None:
        x = rms_norm(x, enc["norm"], c.rms_norm_eps)
    return x


def _project(w, b, x):
    y = mul_mat(w, np.asarray(x, np.float32))
    return (y + b).astype(np.float32) if b is not None else y


def forward_lyric_encoder(W: DitWeights, lyric_hidden_states, max_layers: int | None = None) -> np.ndarray:
    """[n][in_dim] -> [n][H]; the projection is embed_tokens (+ bias), else the text projector."""
    c = W.cfg
    proj_w = W.lyric["embed"] if W.lyric["embed"] is not None else W.text_proj
    proj_b = W.lyric["embed_b"] if W.lyric["embed"] is not None else None
    if proj_w is None or proj_w.values.shape != (c.hidden_size, _lyric_in_dim(c)):
        raise EncoderFailed("forward_lyric_encoder failed")
    x = _project(proj_w, proj_b, lyric_hidden_states)
    return encoder_blocks(W, W.lyric, x, max_layers)


def forward_timbre_encoder(W: DitWeights, refer_audio_hidden_states, max_layers: int | None = None) -> np.ndarray:
    """One reference [refer_len][in_dim] -> its first output token [H] ("use first time step as timbre
    embedding", :1732-1736)."""
    c = W.cfg
    w = W.timbre["embed"]
    if w is None or w.values.shape != (c.hidden_size, _timbre_in_dim(c)):
        raise EncoderFailed("forward_timbre_encoder failed")
    x = _project(w, W.timbre["embed_b"], refer_audio_hidden_states)
    return encoder_blocks(W, W.timbre, x, max_layers)[0]


def project_tokens_linear(W: DitWeights, states) -> np.ndarray:
    """ace_project_tokens_linear(text_projector_w, bias = nullptr)."""
    return _project(W.text_proj, None, states)


def pack_sequences_single_batch(h1, m1, h2, m2):
    """Valid rows (mask != 0) first in stable order, then the rest; mask = 1 for the first n_valid."""
    len1 = 0 if h1 is None else len(h1)
    len2 = 0 if h2 is None else len(h2)
    if len1 <= 0 and len2 <= 0:
        return np.zeros((0, 0), np.float32), np.zeros(0, np.int32)
    if len2 <= 0:
        return np.asarray(h1, np.float32), np.asarray(m1, np.int32)
    if len1 <= 0:
        return np.asarray(h2, np.float32), np.asarray(m2, np.int32)
    h = np.concatenate([h1, h2]).astype(np.float32)
    valid = np.concatenate([np.asarray(m1) != 0, np.asarray(m2) != 0])
    order = np.concatenate([np.nonzero(valid)[0], np.nonzero(~valid)[0]])
    mask = np.zeros(len(h), np.int32)
    mask[: int(valid.sum())] = 1
    return h[order], mask


def build_condition(W: DitWeights, style_states=None, lyric_embeds=None, refer=None, text_hidden=None,
                    allow_text_mismatch: bool = False):
    """(encoder_hidden_states [len][H], mask [len]) as ace_generate_audio_style_lyric_timbre_impl builds
    them from text-encoder style states, lyric token embeddings and timbre references
    [n_refer][refer_len][timbre_in]."""
    c = W.cfg
    H = c.hidden_size
    has_style = style_states is not None and len(style_states) > 0
    has_lyric = lyric_embeds is not None and len(lyric_embeds) > 0
    has_timbre = refer is not None and len(refer) > 0
    if not (has_style or has_lyric or has_timbre):
        raise ValueError("empty style/lyric/timbre inputs")
    style_enc = lyric_enc = None
    if has_style and W.text_proj is not None:
        if W.text_proj.values.shape[1] != text_hidden:
            raise EncoderFailed("linear projection weight shape mismatch")
        style_enc = project_tokens_linear(W, style_states)
    if has_lyric and (W.lyric["embed"] is not None or W.text_proj is not None):
        try:
            if text_hidden != _lyric_in_dim(c):
                raise EncoderFailed("lyric input width")
            lyric_enc = forward_lyric_encoder(W, lyric_embeds)
        except EncoderFailed:
            lyric_enc = None  # fallback: copy the embeddings (:2447-2451)
    timbre = None
    if has_timbre:
        timbre = np.stack([forward_timbre_encoder(W, r) for r in refer]).astype(np.float32)
    if ((has_style and style_enc is None) or (has_lyric and lyric_enc is None)) and text_hidden != H \
            and not allow_text_mismatch:
        raise EncoderFailed("text encoder hidden size mismatch with dit")
    cpy = min(text_hidden or H, H)

    def widen(x):
        out = np.zeros((len(x), H), np.float32)
        out[:, :cpy] = np.asarray(x, np.float32)[:, :cpy]
        return out

    enc, mask = None, None
    if has_lyric:
        enc = lyric_enc if lyric_enc is not None else widen(lyric_embeds)
        mask = np.ones(len(enc), np.int32)
    if has_timbre:
        enc, mask = pack_sequences_single_batch(enc, mask, timbre, np.ones(len(timbre), np.int32))
    if has_style:
        sh = style_enc if style_enc is not None else widen(style_states)
        enc, mask = pack_sequences_single_batch(enc, mask, sh, np.ones(len(sh), np.int32))
    return np.ascontiguousarray(enc, np.float32), mask


def encode_with_floor(fn, *args, perturb: float = 1e-7, **kw):
    """(out, floor) for an encoder forward: the relative L2 change when every mul_mat result is
    perturbed by `perturb` (see dit_oracle.forward_with_floor)."""
    out = fn(*args, **kw)
    old = ggml_numerics.MULMAT_PERTURB
    ggml_numerics.MULMAT_PERTURB = perturb
    try:
        pert = fn(*args, **kw)
    finally:
        ggml_numerics.MULMAT_PERTURB = old
    floor = float(np.linalg.norm(np.asarray(pert, np.float64) - out) / np.linalg.norm(np.asarray(out, np.float64)))
    return out, floor
