"""numpy restatement of `ace_dit::forward_dit` — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Every function cites the reference lines it restates.  Numerics follow ggml-cpu
(oracle/ggml_numerics.py): activations are converted to the weight's
vec_dot_type before each `ggml_mul_mat`, attention runs in f32
(`acestep_dit_model.cpp:1238-1251`), norms/modulation/residuals in f32.
"""
from __future__ import annotations

import json
import math
import os
import struct
from dataclasses import dataclass, field

import numpy as np

from . import ggml_numerics
from .ggml_numerics import GgmlWeight, make_weight, mul_mat, bf16_bits_to_f32

# --------------------------------------------------------------------------
# config.json  (acestep_dit_config.cpp:19-93)
# --------------------------------------------------------------------------
@dataclass
class DitConfig:
    hidden_size: int
    intermediate_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    head_dim: int
    max_position_embeddings: int
    rms_norm_eps: float
    patch_size: int
    in_channels: int
    audio_acoustic_hidden_dim: int
    rope_theta: float = 1000000.0
    sliding_window: int = 0
    use_sliding_window: bool = False
    layer_types: list = field(default_factory=list)
    text_hidden_dim: int = 0
    num_lyric_encoder_hidden_layers: int = 0
    timbre_hidden_dim: int = 0
    num_timbre_encoder_hidden_layers: int = 0

    @staticmethod
    def load(path: str) -> "DitConfig":
        with open(path, "r", encoding="utf-8") as f:
            o = json.load(f)
        return DitConfig(
            hidden_size=int(o["hidden_size"]),
            intermediate_size=int(o["intermediate_size"]),
            num_hidden_layers=int(o["num_hidden_layers"]),
            num_attention_heads=int(o["num_attention_heads"]),
            num_key_value_heads=int(o["num_key_value_heads"]),
            head_dim=int(o["head_dim"]),
            max_position_embeddings=int(o["max_position_embeddings"]),
            rms_norm_eps=float(o["rms_norm_eps"]),
            patch_size=int(o["patch_size"]),
            in_channels=int(o["in_channels"]),
            audio_acoustic_hidden_dim=int(o["audio_acoustic_hidden_dim"]),
            rope_theta=float(o.get("rope_theta", 1000000.0)),
            sliding_window=int(o.get("sliding_window", 0) or 0),
            use_sliding_window=bool(o.get("use_sliding_window", False)),
            layer_types=list(o["layer_types"]),
            text_hidden_dim=int(o.get("text_hidden_dim", 0) or 0),
            num_lyric_encoder_hidden_layers=int(o.get("num_lyric_encoder_hidden_layers", 0) or 0),
            timbre_hidden_dim=int(o.get("timbre_hidden_dim", 0) or 0),
            num_timbre_encoder_hidden_layers=int(o.get("num_timbre_encoder_hidden_layers", 0) or 0),
        )


# --------------------------------------------------------------------------
# safetensors reader (independent of the product's C++ reader)
# --------------------------------------------------------------------------
def read_safetensors(path: str) -> dict:
    """Returns name -> (dtype, shape, f32 ndarray)."""
    out = {}
    with open(path, "rb") as f:
        (hlen,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(hlen))
        base = 8 + hlen
        mm = np.memmap(path, dtype=np.uint8, mode="r")
        for name, info in header.items():
            if name == "__metadata__":
                continue
            s, e = info["data_offsets"]
            raw = np.asarray(mm[base + s: base + e])
            dt = info["dtype"]
            shape = tuple(info["shape"])
            if dt == "BF16":
                arr = bf16_bits_to_f32(raw.view("<u2"))
            elif dt == "F16":
                arr = raw.view("<f2").astype(np.float32)
            elif dt == "F32":
                arr = raw.view("<f4").astype(np.float32)
            else:
                raise ValueError(f"unsupported dtype {dt} for {name}")
            out[name] = (dt, shape, arr.reshape(shape))
    return out


# --------------------------------------------------------------------------
# weight loading  (acestep_dit_model.cpp:753-1088)
# --------------------------------------------------------------------------
def read_gguf(path: str) -> dict:
    """Independent numpy GGUF v2/v3 reader (format of llama.cpp's GGUFWriter, used by
    acestep_ggml/tools/export_safetensors_to_gguf.py): name -> (ggml type, ne list, raw bytes)."""
    import struct as _st
    data = open(path, "rb").read()
    pos = 0

    def rd(fmt):
        nonlocal pos
        v = _st.unpack_from("<" + fmt, data, pos)
        pos += _st.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def rstr():
        nonlocal pos
        n = rd("Q")
        out = data[pos:pos + n].decode("utf-8")
        pos += n
        return out

    sizes = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4, 5: 4, 6: 4, 7: 1, 10: 8, 11: 8, 12: 8}

    def skip_value(t):
        nonlocal pos
        if t == 8:
            rstr()
        elif t == 9:
            et, n = rd("I"), rd("Q")
            for _ in range(n):
                skip_value(et)
        else:
            pos += sizes[t]

    assert data[:4] == b"GGUF"
    pos = 4
    version, n_t, n_kv = rd("I"), rd("Q"), rd("Q")
    assert version in (2, 3)
    align = 32
    for _ in range(n_kv):
        key, t = rstr(), rd("I")
        if key == "general.alignment" and t in (4, 5, 10, 11):
            align = int(_st.unpack_from("<" + {4: "I", 5: "i", 10: "Q", 11: "q"}[t], data, pos)[0])
        skip_value(t)
    infos = []
    for _ in range(n_t):
        name = rstr()
        nd = rd("I")
        ne = [rd("Q") for _ in range(nd)]
        gt, off = rd("I"), rd("Q")
        infos.append((name, ne, gt, off))
    base = (pos + align - 1) // align * align
    row_bytes = {0: lambda n: 4 * n, 1: lambda n: 2 * n, 30: lambda n: 2 * n, 8: lambda n: n // 32 * 34,
                 12: lambda n: n // 256 * 144, 14: lambda n: n // 256 * 210}
    out = {}
    for name, ne, gt, off in infos:
        rows = int(np.prod(ne[1:])) if len(ne) > 1 else 1
        nb = row_bytes[gt](ne[0]) * rows
        out[name] = (gt, ne, data[base + off: base + off + nb])
    return out


_GGUF_QT = {8: "q8_0", 12: "q4_k", 14: "q6_k"}


def _gguf_values(gt, ne, raw):
    """f32 values of a GGUF tensor in numpy (row-major, reversed ne) shape."""
    from .ggml_numerics import dequantize_q4_k, dequantize_q6_k, dequantize_q8_0, unpack_q8_0
    shape = list(reversed(ne))
    rows = int(np.prod(ne[1:])) if len(ne) > 1 else 1
    if gt == 0:
        v = np.frombuffer(raw, "<f4").astype(np.float32)
    elif gt == 1:
        v = np.frombuffer(raw, "<f2").astype(np.float32)
    elif gt == 30:
        v = (np.frombuffer(raw, "<u2").astype(np.uint32) << 16).view(np.float32)
    elif gt == 8:
        v = dequantize_q8_0(*unpack_q8_0(np.frombuffer(raw, np.uint8).reshape(rows, ne[0] // 32, 34)))
    elif gt == 12:
        v = dequantize_q4_k(np.frombuffer(raw, np.uint8).reshape(rows, ne[0] // 256, 144))
    elif gt == 14:
        v = dequantize_q6_k(np.frombuffer(raw, np.uint8).reshape(rows, ne[0] // 256, 210))
    else:
        raise ValueError(f"unsupported gguf type {gt}")
    return np.asarray(v, np.float32).reshape(shape)


class DitWeights:
    def __init__(self, model_dir: str, qtype: str | None = None, gguf: str | None = None):
        """Weights of load_model_from_dir (acestep_dit_model.cpp:753-1088).  `gguf`: load the tensors
        from a GGUF file instead (the `use_gguf` branch: types kept as stored, conv weights converted
        to F32, no online quantization, :526-718)."""
        self.cfg = DitConfig.load(os.path.join(model_dir, "config.json"))
        st = read_gguf(gguf) if gguf else read_safetensors(os.path.join(model_dir, "model.safetensors"))
        self.qtype = None if gguf else qtype
        qtype = self.qtype
        c = self.cfg

        if gguf:
            def w2(name):  # load_tensor_2d_from_gguf: type kept
                gt, ne, raw = st[name]
                v = _gguf_values(gt, ne, raw).reshape(ne[1], ne[0])
                wt = _GGUF_QT.get(gt) or {0: "f32", 1: "f16", 30: "bf16"}[gt]
                return GgmlWeight(v, wt)

            def w3as2(name):  # load_tensor_3d_as_2d_from_gguf + cast_f32
                gt, ne, raw = st[name]
                return GgmlWeight(_gguf_values(gt, ne, raw).reshape(ne[1], ne[0]), "f32")

            def v1(name):
                gt, ne, raw = st[name]
                return _gguf_values(gt, ne, raw).reshape(-1)

            def conv_w(name):  # read_gguf_tensor_as_f32 -> values, stored as an F32 matrix
                gt, ne, raw = st[name]
                return "F32", tuple(reversed(ne)), _gguf_values(gt, ne, raw)
        else:
            def w2(name):  # load_tensor_2d_transposed :228-277
                dt, shape, v = st[name]
                return make_weight(v.reshape(shape[0], shape[1]), dt, qtype)

            def w3as2(name):  # load_tensor_3d_as_2d :279-332 ([1, r, c] -> r rows of c)
                dt, shape, v = st[name]
                return make_weight(v.reshape(shape[1], shape[2]), dt, qtype)

            def v1(name):  # load_tensor_1d + cast_f32
                return st[name][2].astype(np.float32).reshape(-1)

            def conv_w(name):
                dt, shape, v = st[name]
                return dt, tuple(shape), np.asarray(v).reshape(shape)

        # proj_in: conv1d [out, in, k] -> linear [out][in + k*in]  (:334-411; GGUF :602-637 -> F32)
        dt, (co, ci, kk), wv = conv_w("decoder.proj_in.1.weight")
        mat = np.transpose(wv, (0, 2, 1)).reshape(co, kk * ci)  # index k*ci + c
        self.proj_in_w = GgmlWeight(mat, "f32") if gguf else make_weight(mat, dt, qtype)
        self.proj_in_b = v1("decoder.proj_in.1.bias")
        # proj_out: convtranspose1d [in, out, k] -> linear [(out + k*out_ch)][in]  (:413-490; GGUF :639-677)
        dt, (ci2, co2, k2), wv = conv_w("decoder.proj_out.1.weight")
        mat = np.transpose(wv, (2, 1, 0)).reshape(k2 * co2, ci2)  # row o + k*co2
        self.proj_out_w = GgmlWeight(mat, "f32") if gguf else make_weight(mat, dt, qtype)
        self.proj_out_b = v1("decoder.proj_out.1.bias")
        self.condition_w = w2("decoder.condition_embedder.weight")
        self.condition_b = v1("decoder.condition_embedder.bias")
        self.norm_out = v1("decoder.norm_out.weight")
        self.out_table = w3as2("decoder.scale_shift_table").values  # cast_f32 (dequantized if quantized)
        self.time_embed = {}
        for tag in ("time_embed", "time_embed_r"):
            p = f"decoder.{tag}."
            self.time_embed[tag] = dict(
                w1=w2(p + "linear_1.weight"), b1=v1(p + "linear_1.bias"),
                w2=w2(p + "linear_2.weight"), b2=v1(p + "linear_2.bias"),
                wp=w2(p + "time_proj.weight"), bp=v1(p + "time_proj.bias"))
        self.layers = []
        for i in range(c.num_hidden_layers):
            p = f"decoder.layers.{i}."
            L = {}
            L["self_attn_norm"] = v1(p + "self_attn_norm.weight")
            L["cross_attn_norm"] = v1(p + "cross_attn_norm.weight")
            L["mlp_norm"] = v1(p + "mlp_norm.weight")
            for a in ("self_attn", "cross_attn"):
                L[a] = dict(q=w2(p + f"{a}.q_proj.weight"), k=w2(p + f"{a}.k_proj.weight"),
                            v=w2(p + f"{a}.v_proj.weight"), o=w2(p + f"{a}.o_proj.weight"),
                            q_norm=v1(p + f"{a}.q_norm.weight"), k_norm=v1(p + f"{a}.k_norm.weight"))
            L["mlp"] = dict(gate=w2(p + "mlp.gate_proj.weight"), up=w2(p + "mlp.up_proj.weight"),
                            down=w2(p + "mlp.down_proj.weight"))
            L["table"] = w3as2(p + "scale_shift_table").values  # [6][H]
            L["sliding"] = i < len(c.layer_types) and c.layer_types[i] == "sliding_attention"  # :1078-1080
            L["cross"] = True  # Layer::use_cross_attention default (acestep_dit_model.h:47)
            self.layers.append(L)

        # condition encoders, all optional (:885-996); consumed by oracle/cond_oracle.py
        self.text_proj = w2("encoder.text_projector.weight") if "encoder.text_projector.weight" in st else None
        self.lyric = self._encoder(st, "encoder.lyric_encoder.", c.num_lyric_encoder_hidden_layers, w2, v1)
        self.timbre = self._encoder(st, "encoder.timbre_encoder.", c.num_timbre_encoder_hidden_layers, w2, v1)

    def _encoder(self, st, pre, n_layers, w2, v1):
        """EncoderLayer stack of one condition encoder (:889-937 lyric, :941-994 timbre)."""
        c = self.cfg
        e = dict(embed=w2(pre + "embed_tokens.weight") if pre + "embed_tokens.weight" in st else None,
                 embed_b=v1(pre + "embed_tokens.bias") if pre + "embed_tokens.bias" in st else None,
                 norm=v1(pre + "norm.weight") if pre + "norm.weight" in st else None, layers=[])
        for i in range(n_layers):
            p = f"{pre}layers.{i}."
            e["layers"].append(dict(
                input_norm=v1(p + "input_layernorm.weight"),
                post_norm=v1(p + "post_attention_layernorm.weight"),
                self_attn=dict(q=w2(p + "self_attn.q_proj.weight"), k=w2(p + "self_attn.k_proj.weight"),
                               v=w2(p + "self_attn.v_proj.weight"), o=w2(p + "self_attn.o_proj.weight"),
                               q_norm=v1(p + "self_attn.q_norm.weight"), k_norm=v1(p + "self_attn.k_norm.weight")),
                mlp=dict(gate=w2(p + "mlp.gate_proj.weight"), up=w2(p + "mlp.up_proj.weight"),
                         down=w2(p + "mlp.down_proj.weight")),
                sliding=i < len(c.layer_types) and c.layer_types[i] == "sliding_attention"))
        return e


# --------------------------------------------------------------------------
# graph pieces
# --------------------------------------------------------------------------
def rms_norm(x: np.ndarray, w: np.ndarray | None, eps: float) -> np.ndarray:
    """ggml_rms_norm (sum of squares in ggml_float=double, scale = 1/sqrtf(mean+eps)) then
    ggml_mul by the f32 weight (acestep_dit_model.cpp:1097-1106)."""
    x = np.asarray(x, dtype=np.float32)
    ss = np.sum((x * x).astype(np.float64), axis=-1, keepdims=True)
    mean = (ss / x.shape[-1]).astype(np.float32)
    scale = (np.float32(1.0) / np.sqrt(mean + np.float32(eps))).astype(np.float32)
    y = (x * scale).astype(np.float32)
    if w is not None:
        y = (y * w).astype(np.float32)
    return y


def silu(x):
    x = np.asarray(x, dtype=np.float32)
    return (x / (np.float32(1.0) + np.exp(-x))).astype(np.float32)


def timestep_freq(t: float, dim: int = 256, scale: float = 1000.0) -> np.ndarray:
    """build_timestep_freq (:1261-1284), f32 arithmetic with correctly rounded exp / cos / sin (evaluated in
    float64, rounded once: what an accurate libm returns; ggml-cpu's vectorised expf is within an ulp or two of
    it).  The sinusoid is ill-conditioned -- arg reaches ~1000, so one ulp of the frequency moves the feature
    by ~6e-5 -- so under the floor knob (ggml_numerics.MULMAT_PERTURB) the frequencies get the same relative
    noise as the products: the spread of legitimate f32 evaluations of this node belongs in the floor."""
    half = dim // 2
    t_scaled = np.float32(t) * np.float32(scale)
    i = np.arange(half, dtype=np.float32)
    log_max = np.float32(math.log(10000.0))
    exponent = ((-log_max) * i / np.float32(half)).astype(np.float32)
    f = ggml_numerics.perturb(np.exp(exponent.astype(np.float64)).astype(np.float32))
    arg = (t_scaled * f).astype(np.float32)
    out = np.zeros((1, dim), dtype=np.float32)
    out[0, :half] = np.cos(arg.astype(np.float64)).astype(np.float32)
    out[0, half:2 * half] = np.sin(arg.astype(np.float64)).astype(np.float32)
    return out


def timestep_forward(tw: dict, t: float):
    """timestep_forward (:1286-1308): temb = W2 silu(W1 f + b1) + b2; proj = Wp silu(temb) + bp."""
    f = timestep_freq(t)
    h = silu(mul_mat(tw["w1"], f) + tw["b1"])
    temb = (mul_mat(tw["w2"], h) + tw["b2"]).astype(np.float32)
    proj = (mul_mat(tw["wp"], silu(temb)) + tw["bp"]).astype(np.float32)
    return temb.reshape(-1), proj.reshape(6, -1)


def rope_tables(n: int, head_dim: int, theta_base: float):
    """ggml_rope_ext NEOX (:1205-1210): theta_i = p * theta_scale^i with the f32 running
    product of ggml's rope cache (theta *= theta_scale), theta_scale = base^(-2/n_dims)."""
    theta_scale = np.float32(math.pow(theta_base, -2.0 / head_dim))
    half = head_dim // 2
    theta = np.empty((n, half), dtype=np.float32)
    cur = np.arange(n, dtype=np.float32)
    for i in range(half):
        theta[:, i] = cur
        cur = (cur * theta_scale).astype(np.float32)
    # correctly rounded cos / sin of the f32 angles (ggml_rope_cache_init calls libm cosf / sinf)
    return np.cos(theta.astype(np.float64)).astype(np.float32), np.sin(theta.astype(np.float64)).astype(np.float32)


def apply_rope_neox(x: np.ndarray, cos: np.ndarray, sin: np.ndarray) -> np.ndarray:
    """x [n, heads, D]; rotate-half pairs (i, i + D/2)."""
    half = x.shape[-1] // 2
    x0 = x[..., :half]
    x1 = x[..., half:]
    c = cos[:, None, :]
    s = sin[:, None, :]
    return np.concatenate([x0 * c - x1 * s, x0 * s + x1 * c], axis=-1).astype(np.float32)


def build_key_bias(q_len, k_len, key_mask, sliding, window, causal=False):
    """build_attention_mask (:1132-1173) as an additive f32 [q][k] mask, or None when nothing is
    masked.  causal (the text encoder's mask, qwen_model.cpp:618-637): key k > query q masked."""
    if key_mask is None and not sliding and not causal:
        return None
    allow = np.ones((q_len, k_len), dtype=bool)
    if causal:
        allow &= np.arange(k_len)[None, :] <= np.arange(q_len)[:, None]
    if sliding:
        qi = np.arange(q_len)[:, None]
        ki = np.arange(k_len)[None, :]
        allow &= np.abs(qi - ki) <= window
    if key_mask is not None:
        allow &= (np.asarray(key_mask)[None, :k_len] != 0)
    return np.where(allow, np.float32(0.0), np.float32(-np.inf)).astype(np.float32)


def attention(cfg: DitConfig, w: dict, xq, xkv, key_mask, sliding, window, rope, causal=False):
    """attention() (:1175-1259): projections (weight vec_dot rules), per-head QK-RMSNorm,
    NEOX RoPE, f32 softmax(QK^T/sqrt(D) + mask) V with GQA head h -> kv h // n_rep."""
    nh, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    q_len, k_len = xq.shape[0], xkv.shape[0]
    q = mul_mat(w["q"], xq).reshape(q_len, nh, D)
    k = mul_mat(w["k"], xkv).reshape(k_len, nkv, D)
    v = mul_mat(w["v"], xkv).reshape(k_len, nkv, D)
    q = rms_norm(q, w["q_norm"], cfg.rms_norm_eps)
    k = rms_norm(k, w["k_norm"], cfg.rms_norm_eps)
    if rope is not None:
        cos, sin = rope
        q = apply_rope_neox(q, cos[:q_len], sin[:q_len])
        k = apply_rope_neox(k, cos[:k_len], sin[:k_len])
    scale = np.float32(1.0 / math.sqrt(D))
    bias = build_key_bias(q_len, k_len, key_mask, sliding, window, causal)
    rep = nh // nkv
    out = np.empty((q_len, nh, D), dtype=np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        for h in range(nh):
            kh = k[:, h // rep, :]
            vh = v[:, h // rep, :]
            s = ggml_numerics.perturb((q[:, h, :] @ kh.T).astype(np.float32)) * scale
            if bias is not None:
                s = s + bias
            m = np.max(s, axis=1, keepdims=True)
            p = np.exp(s - m).astype(np.float32)
            ssum = np.sum(p.astype(np.float64), axis=1, keepdims=True)
            p = (p * (1.0 / ssum)).astype(np.float32)
            out[:, h, :] = ggml_numerics.perturb((p @ vh).astype(np.float32))
    return mul_mat(w["o"], out.reshape(q_len, nh * D))


# (layer, row, col, amp): add amp to x[row:row+16, col:col+128] after that layer's self-attention residual --
# the restatement of the engine's test-only ACE_MI_TEST_FAULT hook (negative-control tests); None = off
FAULT = None


def forward_dit(W: DitWeights, hidden_states, context_latents, encoder_hidden_states,
                attention_mask, encoder_attention_mask, seq_len: int, enc_len: int,
                timestep: float, timestep_r: float, max_layers: int | None = None) -> np.ndarray:
    """forward_dit (:1316-1560) for one sample.  Inputs are host f32 row-major
    [seq_len][64], [seq_len][ctx], [enc_len][H]; masks int32 or None.  Returns [seq_len][64]."""
    c = W.cfg
    audio = c.audio_acoustic_hidden_dim
    ctx_dim = c.in_channels - audio
    P = c.patch_size
    H = c.hidden_size
    pad = (P - seq_len % P) % P
    Tp = seq_len + pad
    Np = Tp // P
    # input pack, context first (:1350-1377)
    x0 = np.zeros((Tp, c.in_channels), dtype=np.float32)
    if context_latents is not None:
        x0[:seq_len, :ctx_dim] = np.asarray(context_latents, dtype=np.float32).reshape(seq_len, ctx_dim)
    if hidden_states is not None:
        x0[:seq_len, ctx_dim:] = np.asarray(hidden_states, dtype=np.float32).reshape(seq_len, audio)
    x = mul_mat(W.proj_in_w, x0.reshape(Np, P * c.in_channels)) + W.proj_in_b  # :1379-1382
    enc = None
    if enc_len > 0:  # :1384-1414
        e = np.zeros((enc_len, H), dtype=np.float32) if encoder_hidden_states is None else \
            np.asarray(encoder_hidden_states, dtype=np.float32).reshape(enc_len, H)
        enc = (mul_mat(W.condition_w, e) + W.condition_b).astype(np.float32)
    temb_t, proj_t = timestep_forward(W.time_embed["time_embed"], timestep)  # :1420-1424
    temb_r, proj_r = timestep_forward(W.time_embed["time_embed_r"], np.float32(timestep) - np.float32(timestep_r))
    temb = (temb_t + temb_r).astype(np.float32)
    proj = (proj_t + proj_r).astype(np.float32)
    patch_mask = None
    if attention_mask is not None:  # :1433-1449
        am = np.asarray(attention_mask, dtype=np.int32)
        pm = np.zeros(Np, dtype=np.int32)
        for p in range(Np):
            for k in range(P):
                idx = p * P + k
                if idx < seq_len and am[idx] != 0:
                    pm[p] = 1
                    break
        patch_mask = pm
    rope = rope_tables(Np, c.head_dim, c.rope_theta)
    n_layers = len(W.layers) if max_layers is None else min(len(W.layers), max_layers)
    for i in range(n_layers):  # :1466-1535
        L = W.layers[i]
        mod = (L["table"] + proj).astype(np.float32)  # [6][H]
        shift_msa, scale_msa, gate_msa, c_shift, c_scale, c_gate = mod
        norm = rms_norm(x, L["self_attn_norm"], c.rms_norm_eps)
        norm_msa = (norm * (scale_msa + np.float32(1.0)) + shift_msa).astype(np.float32)
        a = attention(c, L["self_attn"], norm_msa, norm_msa, patch_mask, L["sliding"], c.sliding_window,
                      rope)
        x = (x + a * gate_msa).astype(np.float32)
        if FAULT is not None and FAULT[0] == i:  # the engine's ACE_MI_TEST_FAULT hook, restated
            _, r0, c0, amp = FAULT
            x[r0:r0 + 16, c0:c0 + 128] = (x[r0:r0 + 16, c0:c0 + 128] + np.float32(amp)).astype(np.float32)
        if L["cross"] and enc is not None:
            cn = rms_norm(x, L["cross_attn_norm"], c.rms_norm_eps)
            co = attention(c, L["cross_attn"], cn, enc, encoder_attention_mask, False, 0, None)
            x = (x + co).astype(np.float32)
        mn = rms_norm(x, L["mlp_norm"], c.rms_norm_eps)
        mlp_in = (mn * (c_scale + np.float32(1.0)) + c_shift).astype(np.float32)
        g = mul_mat(L["mlp"]["gate"], mlp_in)
        u = mul_mat(L["mlp"]["up"], mlp_in)
        act = (silu(g) * u).astype(np.float32)
        down = mul_mat(L["mlp"]["down"], act)
        x = (x + down * c_gate).astype(np.float32)
    # output head (:1537-1559)
    oss = (W.out_table + temb[None, :]).astype(np.float32)
    out_shift, out_scale = oss[0], oss[1]
    no = rms_norm(x, W.norm_out, c.rms_norm_eps)
    y = (no * (out_scale + np.float32(1.0)) + out_shift).astype(np.float32)
    y_lin = mul_mat(W.proj_out_w, y)  # [Np][P*audio], column o + k*audio
    y2 = y_lin.reshape(Np * P, audio) + W.proj_out_b
    return np.ascontiguousarray(y2[:seq_len].astype(np.float32))


def maxabs_rms(a, ref) -> float:
    """max|a - ref| / rms(ref): the element-wise parity statistic (a localised error of a few rows shows up
    here at full size, where the relative L2 over the whole output dilutes it)."""
    a64, r64 = np.asarray(a, np.float64), np.asarray(ref, np.float64)
    return float(np.max(np.abs(a64 - r64)) / np.sqrt(np.mean(r64 * r64)))


def forward_with_floor_stats(W: DitWeights, *args, perturb: float = 1e-7, **kw):
    """(out, floor_l2, floor_maxabs): forward_with_floor's output and floor, plus the floor of the
    element-wise statistic max|pert - out| / rms(out) under the same perturbation (maxabs_rms)."""
    out = forward_dit(W, *args, **kw)
    old = ggml_numerics.MULMAT_PERTURB
    ggml_numerics.MULMAT_PERTURB = perturb
    ggml_numerics.PERTURB_RNG = np.random.default_rng(12345)
    try:
        pert = forward_dit(W, *args, **kw)
    finally:
        ggml_numerics.MULMAT_PERTURB = old
    o64, p64 = out.astype(np.float64), pert.astype(np.float64)
    floor = float(np.linalg.norm(p64 - o64) / np.linalg.norm(o64))
    return out, floor, maxabs_rms(p64, o64)


def forward_with_floor(W: DitWeights, *args, perturb: float = 1e-7, **kw):
    """(out, floor): the oracle output and its relative L2 change when every mul_mat result is
    perturbed by `perturb` (a stand-in for another f32 summation order).  bf16 activation
    rounding turns such a change of e into ~sqrt(e * 2^-8) per rounding site, so this floor,
    not 0, is what two correct implementations of the same graph can agree to."""
    out = forward_dit(W, *args, **kw)
    old = ggml_numerics.MULMAT_PERTURB
    ggml_numerics.MULMAT_PERTURB = perturb
    ggml_numerics.PERTURB_RNG = np.random.default_rng(12345)
    try:
        pert = forward_dit(W, *args, **kw)
    finally:
        ggml_numerics.MULMAT_PERTURB = old
    floor = float(np.linalg.norm(pert.astype(np.float64) - out) / np.linalg.norm(out.astype(np.float64)))
    return out, floor
