"""Synthetic DiT checkpoints with the real ACE-Step 1.5 tensor names and shapes.

No checkpoints are available offline, so tests and benchmarks use random
weights written in the reference's on-disk format: `config.json` with the keys
read by acestep_dit_config.cpp:58-87 and `model.safetensors` with the
`decoder.*` names loaded by acestep_dit_model.cpp:870-1082.  2-D weights and
biases ~ N(0, 0.02); norm weights ~ 1 + N(0, 0.02); AdaLN tables ~ N(0, 0.02).
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import tempfile
from typing import Dict, Iterator, Tuple

import numpy as np

FULL_CONFIG = dict(
    hidden_size=2048, intermediate_size=6144, num_hidden_layers=24, num_attention_heads=16,
    num_key_value_heads=8, head_dim=128, max_position_embeddings=32768, rms_norm_eps=1e-6,
    rope_theta=1000000.0, patch_size=2, in_channels=192, audio_acoustic_hidden_dim=64,
    use_sliding_window=True, sliding_window=128, attention_bias=False,
)


def make_config(**overrides) -> dict:
    cfg = dict(FULL_CONFIG)
    cfg.update(overrides)
    n = cfg["num_hidden_layers"]
    # acestep/mlx_dit/model.py:447-451 default: even layers sliding, odd layers full
    cfg.setdefault("layer_types", ["sliding_attention" if (i + 1) % 2 else "full_attention" for i in range(n)])
    if len(cfg["layer_types"]) != n:
        cfg["layer_types"] = ["sliding_attention" if (i + 1) % 2 else "full_attention" for i in range(n)]
    return cfg


TINY_CONFIG = make_config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                          num_key_value_heads=2, head_dim=128, sliding_window=16)

# Condition-encoder keys (acestep_dit_config.cpp:69-73).  The released config values are not in the
# reference tree; these are the Qwen3-Embedding-0.6B text width and a guess at the layer counts, used
# only to size synthetic checkpoints.
COND_KEYS = dict(text_hidden_dim=1024, num_lyric_encoder_hidden_layers=8, timbre_hidden_dim=64,
                 num_timbre_encoder_hidden_layers=4, timbre_fix_frame=750)
TINY_COND_CONFIG = make_config(**{k: v for k, v in TINY_CONFIG.items() if k != "layer_types"},
                               text_hidden_dim=256, num_lyric_encoder_hidden_layers=2, timbre_hidden_dim=64,
                               num_timbre_encoder_hidden_layers=2, timbre_fix_frame=8)


def tensor_specs(cfg: dict) -> Iterator[Tuple[str, Tuple[int, ...], str]]:
    """(name, shape, kind) for every DiT decoder tensor; kind in {w, b, norm, table}."""
    H, I, D = cfg["hidden_size"], cfg["intermediate_size"], cfg["head_dim"]
    hq, hkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    cin, audio, P = cfg["in_channels"], cfg["audio_acoustic_hidden_dim"], cfg["patch_size"]
    yield "decoder.proj_in.1.weight", (H, cin, P), "w"
    yield "decoder.proj_in.1.bias", (H,), "b"
    yield "decoder.proj_out.1.weight", (H, audio, P), "w"
    yield "decoder.proj_out.1.bias", (audio,), "b"
    yield "decoder.condition_embedder.weight", (H, H), "w"
    yield "decoder.condition_embedder.bias", (H,), "b"
    yield "decoder.norm_out.weight", (H,), "norm"
    yield "decoder.scale_shift_table", (1, 2, H), "table"
    for tag in ("time_embed", "time_embed_r"):
        p = f"decoder.{tag}."
        yield p + "linear_1.weight", (H, 256), "w"
        yield p + "linear_1.bias", (H,), "b"
        yield p + "linear_2.weight", (H, H), "w"
        yield p + "linear_2.bias", (H,), "b"
        yield p + "time_proj.weight", (6 * H, H), "w"
        yield p + "time_proj.bias", (6 * H,), "b"
    for i in range(cfg["num_hidden_layers"]):
        p = f"decoder.layers.{i}."
        yield p + "self_attn_norm.weight", (H,), "norm"
        for a in ("self_attn", "cross_attn"):
            yield p + f"{a}.q_proj.weight", (hq * D, H), "w"
            yield p + f"{a}.k_proj.weight", (hkv * D, H), "w"
            yield p + f"{a}.v_proj.weight", (hkv * D, H), "w"
            yield p + f"{a}.o_proj.weight", (H, hq * D), "w"
            yield p + f"{a}.q_norm.weight", (D,), "norm"
            yield p + f"{a}.k_norm.weight", (D,), "norm"
        yield p + "cross_attn_norm.weight", (H,), "norm"
        yield p + "mlp_norm.weight", (H,), "norm"
        yield p + "mlp.gate_proj.weight", (I, H), "w"
        yield p + "mlp.up_proj.weight", (I, H), "w"
        yield p + "mlp.down_proj.weight", (H, I), "w"
        yield p + "scale_shift_table", (1, 6, H), "table"
    # condition encoders (acestep_dit_model.cpp:885-996), after the decoder so that adding them leaves
    # the decoder's random draws unchanged
    th = cfg.get("text_hidden_dim", 0)
    if th:
        yield "encoder.text_projector.weight", (H, th), "w"
    for tag, n_key, in_dim in (("lyric", "num_lyric_encoder_hidden_layers", th or 1024),
                               ("timbre", "num_timbre_encoder_hidden_layers",
                                cfg.get("timbre_hidden_dim", 0) or cfg["audio_acoustic_hidden_dim"])):
        n = cfg.get(n_key, 0)
        if not n:
            continue
        p = f"encoder.{tag}_encoder."
        yield p + "embed_tokens.weight", (H, in_dim), "w"
        yield p + "embed_tokens.bias", (H,), "b"
        yield p + "norm.weight", (H,), "norm"
        if tag == "timbre":
            yield p + "special_token", (1, 1, H), "table"
        for i in range(n):
            q = f"{p}layers.{i}."
            yield q + "input_layernorm.weight", (H,), "norm"
            yield q + "self_attn.q_proj.weight", (hq * D, H), "w"
            yield q + "self_attn.k_proj.weight", (hkv * D, H), "w"
            yield q + "self_attn.v_proj.weight", (hkv * D, H), "w"
            yield q + "self_attn.o_proj.weight", (H, hq * D), "w"
            yield q + "self_attn.q_norm.weight", (D,), "norm"
            yield q + "self_attn.k_norm.weight", (D,), "norm"
            yield q + "post_attention_layernorm.weight", (H,), "norm"
            yield q + "mlp.gate_proj.weight", (I, H), "w"
            yield q + "mlp.up_proj.weight", (I, H), "w"
            yield q + "mlp.down_proj.weight", (H, I), "w"


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    return ((u + (np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1)))) >> np.uint32(16)).astype("<u2")


def _encode(values: np.ndarray, dtype: str) -> bytes:
    if dtype == "BF16":
        return _bf16_bits(values).tobytes()
    if dtype == "F16":
        return values.astype("<f2").tobytes()
    if dtype == "F32":
        return values.astype("<f4").tobytes()
    raise ValueError(dtype)


# Qwen3-Embedding-0.6B, the ACE-Step text encoder (config keys of qwen_config.cpp:52-61; tensor names of
# qwen_model.cpp:425-467, no "model." prefix)
TEXT_FULL_CONFIG = dict(vocab_size=151669, hidden_size=1024, num_hidden_layers=28, num_attention_heads=16,
                        num_key_value_heads=8, intermediate_size=3072, head_dim=128, max_position_embeddings=32768,
                        rms_norm_eps=1e-6, rope_theta=1000000.0)
TEXT_TINY_CONFIG = dict(TEXT_FULL_CONFIG, vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                        num_attention_heads=4, num_key_value_heads=2, intermediate_size=512)


def text_tensor_specs(cfg: dict) -> Iterator[Tuple[str, Tuple[int, ...], str]]:
    H, I, D = cfg["hidden_size"], cfg["intermediate_size"], cfg["head_dim"]
    hq, hkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    yield "embed_tokens.weight", (cfg["vocab_size"], H), "w"
    yield "norm.weight", (H,), "norm"
    for i in range(cfg["num_hidden_layers"]):
        p = f"layers.{i}."
        yield p + "input_layernorm.weight", (H,), "norm"
        yield p + "post_attention_layernorm.weight", (H,), "norm"
        yield p + "self_attn.q_proj.weight", (hq * D, H), "w"
        yield p + "self_attn.k_proj.weight", (hkv * D, H), "w"
        yield p + "self_attn.v_proj.weight", (hkv * D, H), "w"
        yield p + "self_attn.o_proj.weight", (H, hq * D), "w"
        yield p + "self_attn.q_norm.weight", (D,), "norm"
        yield p + "self_attn.k_norm.weight", (D,), "norm"
        yield p + "mlp.gate_proj.weight", (I, H), "w"
        yield p + "mlp.up_proj.weight", (I, H), "w"
        yield p + "mlp.down_proj.weight", (H, I), "w"


def write_checkpoint(out_dir: str, cfg: dict, seed: int = 0, dtype: str = "BF16", std: float = 0.02,
                     backend: str = "numpy", specs=None, qk_norm_scale: float = 1.0,
                     qk_norm_tags=("self_attn", "cross_attn")) -> str:
    """Write config.json + model.safetensors into out_dir; returns out_dir.
    backend "numpy" (default, used by the golden fixtures) or "torch" (multi-threaded, ~10x
    faster for the 1.5 B-parameter benchmark checkpoint; different random values).
    specs: tensor list (default: the DiT's, tensor_specs(cfg); text_tensor_specs for Qwen3).
    qk_norm_scale: multiplies the DiT's q_norm / k_norm weights (self and cross attention), so the
    post-norm logits q.k/sqrt(D) have a standard deviation of ~scale^2 instead of ~1: the peaked-softmax
    regime of trained checkpoints (|logit| of tens) for the attention-precision tests; qk_norm_tags picks the
    attention blocks it applies to."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w", encoding="utf-8") as f:
        json.dump(cfg, f, indent=1)
    specs = list(tensor_specs(cfg) if specs is None else specs)
    esz = {"BF16": 2, "F16": 2, "F32": 4}[dtype]
    header: Dict[str, dict] = {}
    off = 0
    for name, shape, _ in specs:
        n = int(np.prod(shape)) * esz
        header[name] = {"dtype": dtype, "shape": list(shape), "data_offsets": [off, off + n]}
        off += n
    hjson = json.dumps(header, separators=(",", ":")).encode("utf-8")
    hjson += b" " * ((8 - len(hjson) % 8) % 8)
    rng = np.random.default_rng(seed)
    gen = None
    if backend == "torch":
        import torch
        gen = torch.Generator().manual_seed(seed)
    tmp = os.path.join(out_dir, "model.safetensors.tmp")
    with open(tmp, "wb") as f:
        f.write(struct.pack("<Q", len(hjson)))
        f.write(hjson)
        for name, shape, kind in specs:
            if gen is not None:
                import torch
                t = torch.randn(shape, generator=gen, dtype=torch.float32) * std
                if kind == "norm":
                    t = t + 1.0
                    if _is_qk_norm(name, qk_norm_tags):
                        t = t * qk_norm_scale
                tt = {"BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32}[dtype]
                f.write(t.to(tt).view(torch.int16 if dtype != "F32" else torch.int32).numpy().tobytes())
                continue
            v = rng.standard_normal(size=shape, dtype=np.float32) * np.float32(std)
            if kind == "norm":
                v = v + np.float32(1.0)
                if _is_qk_norm(name, qk_norm_tags):
                    v = v * np.float32(qk_norm_scale)
            f.write(_encode(v, dtype))
    os.replace(tmp, os.path.join(out_dir, "model.safetensors"))
    return out_dir


def _is_qk_norm(name: str, tags=("self_attn", "cross_attn")) -> bool:
    return (name.startswith("decoder.layers.") and name.endswith(("q_norm.weight", "k_norm.weight")) and
            any(f".{t}." in name for t in tags))


def cached_checkpoint(cfg: dict, seed: int = 0, dtype: str = "BF16", root: str | None = None,
                      backend: str = "numpy", kind: str = "dit", qk_norm_scale: float = 1.0,
                      qk_norm_tags=("self_attn", "cross_attn")) -> str:
    """Write the checkpoint once per (cfg, seed, dtype, backend, kind, qk_norm_scale) under a cache dir and
    reuse it.  kind "dit" (tensor_specs) or "text" (the Qwen3 text encoder, text_tensor_specs)."""
    key_parts = [cfg, seed, dtype, backend] + ([kind] if kind != "dit" else []) + \
        ([float(qk_norm_scale)] if qk_norm_scale != 1.0 else []) + \
        ([list(qk_norm_tags)] if tuple(qk_norm_tags) != ("self_attn", "cross_attn") else [])
    key = hashlib.sha1(json.dumps(key_parts, sort_keys=True).encode()).hexdigest()[:16]
    root = root or os.environ.get("ACE_MI_SYNTH_DIR") or os.path.join(tempfile.gettempdir(), "acestep_mi355x_synth")
    d = os.path.join(root, key)
    if not os.path.exists(os.path.join(d, "model.safetensors")):
        specs = text_tensor_specs(cfg) if kind == "text" else None
        write_checkpoint(d, cfg, seed=seed, dtype=dtype, backend=backend, specs=specs, qk_norm_scale=qk_norm_scale,
                         qk_norm_tags=qk_norm_tags)
    return d


# ----------------------------------------------------------------------------- VAE (Oobleck)
# diffusers AutoencoderOobleck layout read by acestep_vae_model.cpp:760-955 (decoder.* only: the
# MI355X engine implements decode; encode is out of scope this round).
VAE_FULL_CONFIG = dict(audio_channels=2, encoder_hidden_size=128, decoder_channels=128, decoder_input_channels=64,
                       sampling_rate=48000, downsampling_ratios=[2, 4, 4, 6, 10], channel_multiples=[1, 2, 4, 8, 16])
VAE_TINY_CONFIG = dict(VAE_FULL_CONFIG, downsampling_ratios=[2, 3], channel_multiples=[1, 2])


def vae_tensor_specs(cfg: dict) -> Iterator[Tuple[str, Tuple[int, ...], str]]:
    """(name, shape, kind) of every decoder tensor; kind in {g, v, b, snake}."""
    ch, lat, aud = cfg["decoder_channels"], cfg["decoder_input_channels"], cfg["audio_channels"]
    strides = list(reversed(cfg["downsampling_ratios"]))
    cm = [1] + list(cfg["channel_multiples"])
    n = len(strides)

    def conv(prefix, cout, cin, k, bias=True, transposed=False):
        d0 = cin if transposed else cout
        yield prefix + ".weight_g", (d0, 1, 1), "g"
        yield prefix + ".weight_v", ((cin, cout, k) if transposed else (cout, cin, k)), "v"
        if bias:
            yield prefix + ".bias", (cout,), "b"

    def snk(prefix, c):
        yield prefix + ".alpha", (1, c, 1), "snake"
        yield prefix + ".beta", (1, c, 1), "snake"

    yield from conv("decoder.conv1", ch * cm[-1], lat, 7)
    for i, s in enumerate(strides):
        cin, cout = ch * cm[n - i], ch * cm[n - i - 1]
        p = f"decoder.block.{i}"
        yield from snk(p + ".snake1", cin)
        yield from conv(p + ".conv_t1", cout, cin, 2 * s, transposed=True)
        for j in range(3):
            q = f"{p}.res_unit{j + 1}"
            yield from snk(q + ".snake1", cout)
            yield from conv(q + ".conv1", cout, cout, 7)
            yield from snk(q + ".snake2", cout)
            yield from conv(q + ".conv2", cout, cout, 1)
    yield from snk("decoder.snake1", ch)
    yield from conv("decoder.conv2", aud, ch, 7, bias=False)
    # encoder (diffusers OobleckEncoder; acestep_vae_model.cpp:925-937)
    eh = cfg["encoder_hidden_size"]
    dn = list(cfg["downsampling_ratios"])
    yield from conv("encoder.conv1", eh, aud, 7)
    for i, s in enumerate(dn):
        cin, cout = eh * cm[i], eh * cm[i + 1]
        p = f"encoder.block.{i}"
        for j in range(3):
            q = f"{p}.res_unit{j + 1}"
            yield from snk(q + ".snake1", cin)
            yield from conv(q + ".conv1", cin, cin, 7)
            yield from snk(q + ".snake2", cin)
            yield from conv(q + ".conv2", cin, cin, 1)
        yield from snk(p + ".snake1", cin)
        yield from conv(p + ".conv1", cout, cin, 2 * s)
    yield from snk("encoder.snake1", eh * cm[-1])
    yield from conv("encoder.conv2", eh, eh * cm[-1], 3)


def write_vae_checkpoint(out_dir: str, cfg: dict, seed: int = 0, dtype: str = "F32") -> str:
    """config.json + diffusion_pytorch_model.safetensors with weight-normed convs: weight_v ~ N(0,1),
    weight_g ~ 0.6 + U(0, 0.4) (keeps activations O(1) through the residual stack), biases ~ N(0, 0.02),
    snake alpha/beta ~ N(0, 0.1)."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w", encoding="utf-8") as f:
        json.dump(cfg, f, indent=1)
    specs = list(vae_tensor_specs(cfg))
    esz = {"BF16": 2, "F16": 2, "F32": 4}[dtype]
    header: Dict[str, dict] = {}
    off = 0
    for name, shape, _ in specs:
        nb = int(np.prod(shape)) * esz
        header[name] = {"dtype": dtype, "shape": list(shape), "data_offsets": [off, off + nb]}
        off += nb
    hjson = json.dumps(header, separators=(",", ":")).encode("utf-8")
    hjson += b" " * ((8 - len(hjson) % 8) % 8)
    rng = np.random.default_rng(seed)
    tmp = os.path.join(out_dir, "diffusion_pytorch_model.safetensors.tmp")
    with open(tmp, "wb") as f:
        f.write(struct.pack("<Q", len(hjson)))
        f.write(hjson)
        for name, shape, kind in specs:
            if kind == "v":
                v = rng.standard_normal(size=shape, dtype=np.float32)
            elif kind == "g":
                v = (np.float32(0.6) + np.float32(0.4) * rng.random(size=shape, dtype=np.float32))
            elif kind == "b":
                v = rng.standard_normal(size=shape, dtype=np.float32) * np.float32(0.02)
            else:
                v = rng.standard_normal(size=shape, dtype=np.float32) * np.float32(0.1)
            f.write(_encode(v, dtype))
    os.replace(tmp, os.path.join(out_dir, "diffusion_pytorch_model.safetensors"))
    return out_dir


# ----------------------------------------------------------------------------- GGUF export
GGML_TYPES = {"F32": 0, "F16": 1, "Q8_0": 8, "Q4_K": 12, "Q6_K": 14, "BF16": 30}
_QUANT_ARG = {"F16": None, "Q8": "Q8_0", "Q8_0": "Q8_0", "Q6": "Q6_K", "Q6_K": "Q6_K", "Q4": "Q4_K", "Q4_K": "Q4_K"}
_QBLOCK = {"Q8_0": 32, "Q4_K": 256, "Q6_K": 256}


def _read_safetensors_f32(path: str) -> Dict[str, np.ndarray]:
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        header = json.loads(f.read(n))
        base = 8 + n
        out = {}
        for name, info in header.items():
            if name == "__metadata__":
                continue
            b0, b1 = info["data_offsets"]
            f.seek(base + b0)
            raw = f.read(b1 - b0)
            dt = info["dtype"]
            if dt == "F32":
                v = np.frombuffer(raw, "<f4").astype(np.float32)
            elif dt == "F16":
                v = np.frombuffer(raw, "<f2").astype(np.float32)
            elif dt == "BF16":
                v = (np.frombuffer(raw, "<u2").astype(np.uint32) << 16).view(np.float32)
            else:
                raise ValueError(dt)
            out[name] = v.reshape(info["shape"])
    return out


def write_gguf(safetensors_path: str, out_path: str, quant: str = "Q8", arch: str = "acestep") -> str:
    """GGUF export with the rules of acestep_ggml/tools/export_safetensors_to_gguf.py:192-281: every
    float tensor with >= 2 dims whose last dim is a multiple of the block size is quantized (Q8/Q6/Q4),
    everything else is stored F16.  Block bytes come from this library's ggml encoders
    (ace_mi_quantize; the reference script uses gguf-py / ggml's C quantizer).  GGUF v3, alignment 32,
    numpy shape reversed into ggml ne order."""
    from . import capi
    qname = _QUANT_ARG[quant.upper()]
    tensors = _read_safetensors_f32(safetensors_path)
    entries = []
    for name, v in tensors.items():
        if qname and v.ndim >= 2 and v.shape[-1] % _QBLOCK[qname] == 0:
            rows = int(np.prod(v.shape[:-1]))
            data = capi.quantize(v.reshape(rows, v.shape[-1]), qname.lower()).tobytes()
            entries.append((name, v.shape, GGML_TYPES[qname], data))
        else:
            entries.append((name, v.shape, GGML_TYPES["F16"], v.astype("<f2").tobytes()))

    def s(x: str) -> bytes:
        b = x.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    kv = [("general.architecture", 8, s(arch)), ("general.type", 8, s("model")),
          ("general.quantization_version", 4, struct.pack("<I", 2))]
    head = b"GGUF" + struct.pack("<IQQ", 3, len(entries), len(kv))
    for k, t, val in kv:
        head += s(k) + struct.pack("<I", t) + val
    off = 0
    infos = b""
    for name, shape, gt, data in entries:
        ne = list(reversed(shape))
        infos += s(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", d) for d in ne)
        infos += struct.pack("<IQ", gt, off)
        off += (len(data) + 31) // 32 * 32
    blob = head + infos
    blob += b"\0" * ((32 - len(blob) % 32) % 32)
    tmp = out_path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(blob)
        for _, _, _, data in entries:
            f.write(data)
            f.write(b"\0" * ((32 - len(data) % 32) % 32))
    os.replace(tmp, out_path)
    return out_path
