"""numpy restatement of the reference's end-to-end generation — TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py).

  ace_generate_audio_from_encoder             acestep_ggml.cpp:1901-2238
  ace_ggml_generate_audio_simple              acestep_ggml.cpp:2240-2322
  ace_generate_audio_style_lyric_timbre_impl  acestep_ggml.cpp:2324-2556
  ace_get_shift_schedule                      acestep_ggml.cpp:1484-1500
and the x_T generator, std::mt19937(seed) + std::normal_distribution<float> (:2043-2048), restated from
the C++ standard library the reference is built with (libstdc++: MT19937 of [rand.eng.mers];
normal_distribution = Marsaglia's polar method over generate_canonical<float, 24>, bits/random.tcc).
logf is taken from the C library through ctypes so that x_T matches bit for bit.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

from . import cond_oracle, vae_oracle
from .dit_oracle import forward_dit

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]


class MT19937:
    """std::mt19937 (32-bit Mersenne twister, seed via init_genrand)."""

    def __init__(self, seed: int):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.idx = 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def __call__(self) -> int:
        if self.idx >= 624:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def reference_noise(seed: int, n: int) -> np.ndarray:
    """n draws of std::normal_distribution<float>(0, 1) on std::mt19937(seed)."""
    g = MT19937(np.uint32(np.int64(seed) & 0xFFFFFFFF).item())
    f32 = np.float32

    def canonical():  # generate_canonical<float, 24>: one 32-bit draw / 2^32, clamped below 1
        r = f32(g()) / f32(4294967296.0)
        return r if r < f32(1.0) else np.nextafter(f32(1.0), f32(0.0))

    out = np.empty(n, np.float32)
    saved = None
    for i in range(n):
        if saved is not None:
            out[i], saved = saved, None
            continue
        while True:
            x = f32(np.float64(f32(2.0) * canonical()) - 1.0)
            y = f32(np.float64(f32(2.0) * canonical()) - 1.0)
            r2 = f32(x * x + y * y)
            if not (r2 > 1.0 or r2 == 0.0):
                break
        mult = np.sqrt(f32(f32(-2.0) * f32(_libm.logf(float(r2)))) / r2, dtype=np.float32)
        saved = f32(x * mult)
        out[i] = f32(y * mult)
    return out


def shift_schedule(shift: float):
    s1 = [1.0, 0.875, 0.75, 0.625, 0.5, 0.375, 0.25, 0.125]
    s2 = [1.0, 0.9333333333, 0.8571428571, 0.7692307692, 0.6666666667, 0.5454545455, 0.4, 0.2222222222]
    s3 = [1.0, 0.9545454545, 0.9, 0.8333333333, 0.75, 0.6428571429, 0.5, 0.3]
    sh = np.float32(shift)
    d1, d2, d3 = (abs(sh - np.float32(v)) for v in (1.0, 2.0, 3.0))
    s = s1 if (d1 <= d2 and d1 <= d3) else (s2 if (d2 <= d1 and d2 <= d3) else s3)
    return [np.float32(v) for v in s]


def silence_context(VW, seq_len: int, audio_dim: int, ctx_dim: int, hop: int, audio_channels: int,
                    chunk_frames: int | None = None):
    """context_latents of :1948-2041 with silence latents from the VAE encoder (chunked as the reference
    chunks them: 64 frames when seq_len > 128, else the whole sequence) and an all-ones chunk mask."""
    src_dim = min(audio_dim, ctx_dim)
    chunk = chunk_frames or (64 if seq_len > 128 else seq_len)
    src = np.zeros((seq_len, src_dim), np.float32)
    for f0 in range(0, seq_len, chunk):
        cur = min(chunk, seq_len - f0)
        lat = vae_oracle.encode(VW, np.zeros((cur * hop, audio_channels), np.float32))
        src[f0:f0 + cur] = lat[:cur, :src_dim]
    ctx = np.ones((seq_len, ctx_dim), np.float32)
    ctx[:, :src_dim] = src
    return ctx


def decode_windowed(VW, xt, hop: int, audio_channels: int):
    """The VAE decode of :2114-2223 (128-frame windows with 32 frames of overlap when seq_len > 128)."""
    seq_len = len(xt)
    chunk = 128 if seq_len > 128 else 0
    if not (0 < chunk < seq_len):
        return vae_oracle.decode(VW, xt)
    overlap = min(64, max(1, chunk // 4))
    if overlap * 2 >= chunk:
        overlap = max(0, chunk // 2 - 1)
    stride = chunk - 2 * overlap
    parts = []
    for core0 in range(0, seq_len, stride):
        core1 = min(core0 + stride, seq_len)
        w0, w1 = max(0, core0 - overlap), min(seq_len, core1 + overlap)
        # the reference decodes into a zeroed buffer of win_frames * hop samples and trims by that size
        dec = vae_oracle.decode(VW, xt[w0:w1])
        audio = np.zeros(((w1 - w0) * hop, audio_channels), np.float32)
        audio[:min(len(dec), len(audio))] = dec[:len(audio)]
        up = len(audio) / (w1 - w0)
        ts = int(np.floor((core0 - w0) * up + 0.5))   # std::llround (halves away from zero)
        te = int(np.floor((w1 - core1) * up + 0.5))
        parts.append(audio[ts:len(audio) - te])
    return np.concatenate(parts)


def generate_from_encoder(DW, VW, enc, enc_mask, seq_len: int, shift: float, seed: int, hop: int, audio_channels: int):
    c = DW.cfg
    audio_dim = c.audio_acoustic_hidden_dim
    ctx = silence_context(VW, seq_len, audio_dim, c.in_channels - audio_dim, hop, audio_channels)
    xt = reference_noise(seed, seq_len * audio_dim).reshape(seq_len, audio_dim)
    sched = shift_schedule(shift)
    for i, t in enumerate(sched):
        v = forward_dit(DW, xt, ctx, enc, None, enc_mask, seq_len, len(enc), t, t)
        dt = t if i + 1 == len(sched) else np.float32(t - sched[i + 1])
        xt = (xt - v * dt).astype(np.float32)
    return decode_windowed(VW, xt, hop, audio_channels), xt


def generate_style_lyric_timbre(DW, VW, TW, style_ids, lyric_ids, refer, seq_len, shift, seed, hop, audio_channels):
    from .text_oracle import forward_text_encoder_embeddings, forward_text_encoder_layers
    style = forward_text_encoder_layers(TW, style_ids) if style_ids is not None and len(style_ids) else None
    lyric = forward_text_encoder_embeddings(TW, lyric_ids) if lyric_ids is not None and len(lyric_ids) else None
    enc, mask = cond_oracle.build_condition(DW, style, lyric, refer, text_hidden=TW.cfg.hidden_size)
    return generate_from_encoder(DW, VW, enc, mask, seq_len, shift, seed, hop, audio_channels)


def forward_text_encoder_layers_for_simple(TW, token_ids):
    """encoder_hidden_states of ace_ggml_generate_audio_simple: the text states as they are (:2289-2297)."""
    from .text_oracle import forward_text_encoder_layers
    return forward_text_encoder_layers(TW, token_ids)
