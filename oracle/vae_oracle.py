"""numpy restatement of the Oobleck VAE decoder (`ace_vae::forward_decode`) — TEST INFRASTRUCTURE
ONLY (see oracle/__init__.py).

Follows `acestep_ggml/cpp/acestep_vae_model.cpp`:
  * config (`load_config` :55-125): upsampling_ratios = reversed(downsampling_ratios),
    hop_length = prod(downsampling_ratios);
  * weight-norm fold at load (`load_conv_weight_norm` :520-588): per slice i of dim 0,
    ss = sum(v^2) in double, scale = g_i / sqrtf((float)ss + 1e-12f), w = v * scale, stored F16
    (conv_t too, unless ACE_GGML_VAE_TRANSPOSE_CONV_F32);
  * snake (`snake_forward` :682-692): x + sin(exp(alpha) * x)^2 / exp(beta), all f32 (no 1e-9);
  * conv (`conv_forward` :694-712): ggml_conv_1d = im2col to F16 + F16 mul_mat with f32
    accumulation; ggml_conv_transpose_1d with p0 = 0 (input rounded to F16, f32 accumulation),
    then a center crop to the PyTorch output length; bias added after;
  * residual unit (:724-733), decoder block (:735-742), decode (:957-1002): latents
    [T][64] -> audio [T*hop][audio_channels] (`ace_ggml_vae_decode` returns it time-major,
    acestep_ggml.cpp:936-940).
Parity: ggml cannot be built here -> parity unpinned against real ggml; the Snake
form is cross-checked against `acestep/mlx_vae/model.py:24-56` (which adds 1e-9 to beta; the
ggml path does not).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

from .dit_oracle import read_safetensors
from .ggml_numerics import round_f16


# Test-only knob (as ggml_numerics.MULMAT_PERTURB): relative perturbation of every conv result, used to measure the
# decoder's own sensitivity to f32 summation order (fp16 re-rounding of every conv input amplifies it) -- the floor
# two correct implementations agree to.  Independent per-element noise y * (1 + p * N(0, 1)) (PERTURB_RNG, re-seeded by
# the floor helpers), like the DiT oracle's: a different summation order changes each dot product by ~1e-7 with no
# correlation between elements.  (Rounds 1-4 scaled every conv output coherently by (1 + p), which the next Snake and
# fp16 rounding see as a smooth change: a looser floor for the L2 statistic and none for the element-wise one.)
CONV_PERTURB = 0.0
PERTURB_RNG = np.random.default_rng(0)
# the restatement of the VAE's test-only ACE_MI_TEST_VAE_FAULT hook (runtime/vae.cpp): (block, row, col, amp) adds amp
# to rows [row, row + 16) x channels [col, col + 128) of the residual stream after the block's first residual unit
FAULT = None


def _perturb(y):
    if CONV_PERTURB:
        noise = PERTURB_RNG.standard_normal(y.shape)
        return (y.astype(np.float64) * (1.0 + CONV_PERTURB * noise)).astype(np.float32)
    return y


@dataclass
class VaeConfig:
    audio_channels: int
    decoder_channels: int
    decoder_input_channels: int
    downsampling_ratios: list
    channel_multiples: list
    upsampling_ratios: list = field(default_factory=list)
    hop_length: int = 1

    @staticmethod
    def load(path: str) -> "VaeConfig":
        o = json.load(open(path))
        c = VaeConfig(audio_channels=int(o["audio_channels"]), decoder_channels=int(o["decoder_channels"]),
                      decoder_input_channels=int(o["decoder_input_channels"]),
                      downsampling_ratios=[int(v) for v in o["downsampling_ratios"]],
                      channel_multiples=[int(v) for v in o["channel_multiples"]])
        c.upsampling_ratios = list(reversed(c.downsampling_ratios))  # :119-120
        c.hop_length = int(np.prod(c.downsampling_ratios))           # :121-124
        return c


def fold_weight_norm(g: np.ndarray, v: np.ndarray) -> np.ndarray:
    """`load_conv_weight_norm` (:541-555) -> the f32 values of the F16 weight."""
    v = np.asarray(v, np.float32)
    d0 = v.shape[0]
    flat = v.reshape(d0, -1)
    ss = np.sum(flat.astype(np.float64) ** 2, axis=1)
    scale = (np.asarray(g, np.float32).reshape(d0) / np.sqrt((ss.astype(np.float32) + np.float32(1e-12))
                                                            .astype(np.float32))).astype(np.float32)
    w = (flat * scale[:, None]).astype(np.float32)
    return round_f16(w).reshape(v.shape)


def snake(x, alpha, beta):
    """snake_forward (:682-692): per channel (last axis of x [T][C])."""
    a = np.exp(np.asarray(alpha, np.float32).reshape(-1)).astype(np.float32)
    b = np.exp(np.asarray(beta, np.float32).reshape(-1)).astype(np.float32)
    s = (a[None, :] * x).astype(np.float32)
    s = np.sin(s).astype(np.float32)
    s = (s * s).astype(np.float32)
    s = (s / b[None, :]).astype(np.float32)
    return (x + s).astype(np.float32)


def conv1d(x, w, bias, dilation=1, padding=0, stride=1):
    """ggml_conv_1d(w [Cout][Cin][K], x [T][Cin], s0=stride, p0=padding, d0=dilation): F16 operands,
    f32 accumulation; + bias.  Output length (T + 2p - d(K-1) - 1) / s + 1."""
    xh = round_f16(x).astype(np.float32)
    T, cin = xh.shape
    cout, cin2, K = w.shape
    assert cin == cin2
    T_out = (T + 2 * padding - dilation * (K - 1) - 1) // stride + 1
    xp = np.zeros((T + 2 * padding + stride, cin), np.float32)
    xp[padding:padding + T] = xh
    out = np.zeros((T_out, cout), np.float32)
    for k in range(K):
        out += xp[k * dilation:k * dilation + (T_out - 1) * stride + 1:stride] @ w[:, :, k].T.astype(np.float32)
    out = _perturb(out)
    if bias is not None:
        out += np.asarray(bias, np.float32)[None, :]
    return out


def conv_transpose1d(x, w, bias, stride, padding):
    """ggml_conv_transpose_1d(w [Cin][Cout][K], x, s0=stride, p0=0) + center crop (:697-708) + bias."""
    xh = round_f16(x).astype(np.float32)
    T, cin = xh.shape
    cin2, cout, K = w.shape
    assert cin == cin2
    full_len = (T - 1) * stride + K
    full = np.zeros((full_len, cout), np.float32)
    for k in range(K):
        full[k:k + (T - 1) * stride + 1:stride] += xh @ w[:, :, k].astype(np.float32)
    full = _perturb(full)
    target = (T - 1) * stride - 2 * padding + (K - 1) + 1
    if padding > 0 and 0 < target < full_len:
        start = (full_len - target) // 2
        full = full[start:start + target]
    if bias is not None:
        full = full + np.asarray(bias, np.float32)[None, :]
    return full.astype(np.float32)


class VaeWeights:
    """Decoder weights as ggml holds them (F16 folded conv weights, f32 snake params/biases)."""

    def __init__(self, model_dir: str):
        self.cfg = VaeConfig.load(os.path.join(model_dir, "config.json"))
        st = read_safetensors(os.path.join(model_dir, "diffusion_pytorch_model.safetensors"))

        def arr(name):
            dt, shape, v = st[name]
            return v.astype(np.float32).reshape(shape)

        def conv(prefix, bias=True):
            w = fold_weight_norm(arr(prefix + ".weight_g"), arr(prefix + ".weight_v"))
            return dict(w=w, b=arr(prefix + ".bias").reshape(-1) if bias else None)

        def snk(prefix):
            return dict(alpha=arr(prefix + ".alpha").reshape(-1), beta=arr(prefix + ".beta").reshape(-1))

        self.conv1 = conv("decoder.conv1")
        self.blocks = []
        for i, s in enumerate(self.cfg.upsampling_ratios):
            p = f"decoder.block.{i}"
            blk = dict(stride=s, snake1=snk(p + ".snake1"), conv_t1=conv(p + ".conv_t1"), res=[])
            for j, dil in enumerate((1, 3, 9)):
                q = f"{p}.res_unit{j + 1}"
                blk["res"].append(dict(dil=dil, snake1=snk(q + ".snake1"), conv1=conv(q + ".conv1"),
                                       snake2=snk(q + ".snake2"), conv2=conv(q + ".conv2")))
            self.blocks.append(blk)
        self.snake1 = snk("decoder.snake1")
        self.conv2 = conv("decoder.conv2", bias=False)
        # encoder (load_model_from_dir :925-937): optional here, required by encode()
        self.enc = None
        if "encoder.conv1.weight_v" in st:
            enc = dict(conv1=conv("encoder.conv1"), blocks=[], snake1=snk("encoder.snake1"), conv2=conv("encoder.conv2"))
            for i, s_ in enumerate(self.cfg.downsampling_ratios):
                p = f"encoder.block.{i}"
                blk = dict(stride=s_, res=[], snake1=snk(p + ".snake1"), conv1=conv(p + ".conv1"))
                for j, dil in enumerate((1, 3, 9)):
                    q = f"{p}.res_unit{j + 1}"
                    blk["res"].append(dict(dil=dil, snake1=snk(q + ".snake1"), conv1=conv(q + ".conv1"),
                                           snake2=snk(q + ".snake2"), conv2=conv(q + ".conv2")))
                enc["blocks"].append(blk)
            self.enc = enc


def residual_unit(ru, x, skip=None):
    """residual_forward (:724-733): skip + conv2(snake2(conv1(snake1(x)))), skip = x (the test-only FAULT restatement
    passes a different skip: the faulted residual stream beside the clean unit input)."""
    y = conv1d(snake(x, **ru["snake1"]), ru["conv1"]["w"], ru["conv1"]["b"], ru["dil"], 3 * ru["dil"])
    y = conv1d(snake(y, **ru["snake2"]), ru["conv2"]["w"], ru["conv2"]["b"], 1, 0)
    skip = x if skip is None else skip
    n = min(len(skip), len(y))
    cx, cy = (len(skip) - n) // 2, (len(y) - n) // 2
    return (skip[cx:cx + n] + y[cy:cy + n]).astype(np.float32)


def decode(W: VaeWeights, latents: np.ndarray) -> np.ndarray:
    """forward_decode (:957-1002): latents [T][C_lat] -> audio [T*hop][audio_channels]."""
    x = conv1d(np.asarray(latents, np.float32), W.conv1["w"], W.conv1["b"], 1, 3)
    for bi, blk in enumerate(W.blocks):
        s = blk["stride"]
        x = snake(x, **blk["snake1"])
        x = conv_transpose1d(x, blk["conv_t1"]["w"], blk["conv_t1"]["b"], s, (s + 1) // 2)
        skip = None
        for ri, ru in enumerate(blk["res"]):
            x = residual_unit(ru, x, skip)
            skip = None
            if FAULT is not None and FAULT[0] == bi and ri == 0:  # ACE_MI_TEST_VAE_FAULT, restated: the engine adds
                _, r0, c0, amp = FAULT                             # the tile to the f32 residual stream after the unit;
                skip = x.copy()                                    # the next unit's input Snake was already formed
                skip[r0:r0 + 16, c0:c0 + 128] = (skip[r0:r0 + 16, c0:c0 + 128] + np.float32(amp)).astype(np.float32)
    x = snake(x, **W.snake1)
    return conv1d(x, W.conv2["w"], None, 1, 3)


def encode(W: VaeWeights, audio: np.ndarray) -> np.ndarray:
    """forward_encode (:1004-1044): audio [n_samples][audio_channels] -> latent mean
    [n_frames][decoder_input_channels] (the first half of encoder.conv2's [mean, scale] channels)."""
    E = W.enc
    x = conv1d(np.asarray(audio, np.float32), E["conv1"]["w"], E["conv1"]["b"], 1, 3)
    for blk in E["blocks"]:
        for ru in blk["res"]:
            x = residual_unit(ru, x)
        s = blk["stride"]
        x = snake(x, **blk["snake1"])
        x = conv1d(x, blk["conv1"]["w"], blk["conv1"]["b"], 1, (s + 1) // 2, stride=s)
    x = snake(x, **E["snake1"])
    x = conv1d(x, E["conv2"]["w"], E["conv2"]["b"], 1, 1)
    return x[:, :W.cfg.decoder_input_channels].copy()


def decode_with_floor(W: VaeWeights, latents, perturb: float = 1e-7):
    """(audio, floor): decode() and its relative L2 change under an independent `perturb` relative
    perturbation of every conv result element (see CONV_PERTURB)."""
    out, floor, _ = decode_with_floor_stats(W, latents, perturb=perturb)
    return out, floor


def floor_stats(fn, perturb: float = 1e-7):
    """(out, floor_l2, floor_maxabs) of a decode-like callable: its output, and the relative L2 and the element-wise
    max|pert - out| / rms(out) of its change when every conv result element is perturbed (the DiT oracle's
    forward_with_floor_stats, restated for the decoder)."""
    global CONV_PERTURB, PERTURB_RNG
    out = fn()
    old = CONV_PERTURB
    CONV_PERTURB = perturb
    PERTURB_RNG = np.random.default_rng(12345)
    try:
        pert = fn()
    finally:
        CONV_PERTURB = old
    o64, p64 = out.astype(np.float64), pert.astype(np.float64)
    floor = float(np.linalg.norm(p64 - o64) / np.linalg.norm(o64))
    maxabs = float(np.max(np.abs(p64 - o64)) / np.sqrt(np.mean(o64 * o64)))
    return out, floor, maxabs


def decode_with_floor_stats(W: VaeWeights, latents, perturb: float = 1e-7):
    return floor_stats(lambda: decode(W, latents), perturb=perturb)
