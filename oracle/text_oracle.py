"""numpy restatement of the Qwen3 text encoder — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  load_config                    qwen_config.cpp:19-64
  load_model_from_dir            qwen_model.cpp:340-478 (online quantization :185-240)
  forward_text_encoder_layers    qwen_model.cpp:528-677 (causal mask :618-637)
  forward_text_encoder_embeddings qwen_model.cpp:690-703
with the ggml-cpu numerics of oracle/ggml_numerics.py and the DiT oracle's attention / rms_norm.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import numpy as np

from . import ggml_numerics
from .dit_oracle import attention, mul_mat, read_gguf, read_safetensors, rms_norm, rope_tables, silu, _gguf_values
from .ggml_numerics import GgmlWeight, make_weight


@dataclass
class TextConfig:
    vocab_size: int
    hidden_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    intermediate_size: int
    head_dim: int
    max_position_embeddings: int
    rms_norm_eps: float
    rope_theta: float = 1000000.0

    @staticmethod
    def load(path: str) -> "TextConfig":
        with open(path, "r", encoding="utf-8") as f:
            o = json.load(f)
        return TextConfig(*(int(o[k]) for k in ("vocab_size", "hidden_size", "num_hidden_layers",
                                                 "num_attention_heads", "num_key_value_heads", "intermediate_size",
                                                 "head_dim", "max_position_embeddings")),
                          rms_norm_eps=float(o["rms_norm_eps"]), rope_theta=float(o.get("rope_theta", 1000000.0)))


_GGUF_QT = {8: "q8_0", 12: "q4_k", 14: "q6_k"}


class TextWeights:
    def __init__(self, model_dir: str, qtype: str | None = None, gguf: str | None = None):
        self.cfg = c = TextConfig.load(os.path.join(model_dir, "config.json"))
        st = read_gguf(gguf) if gguf else read_safetensors(os.path.join(model_dir, "model.safetensors"))
        qtype = None if gguf else qtype

        if gguf:
            def w2(name):
                gt, ne, raw = st[name]
                return GgmlWeight(_gguf_values(gt, ne, raw).reshape(ne[1], ne[0]),
                                  _GGUF_QT.get(gt) or {0: "f32", 1: "f16", 30: "bf16"}[gt])

            def v1(name):
                gt, ne, raw = st[name]
                return _gguf_values(gt, ne, raw).reshape(-1)
        else:
            def w2(name):
                dt, shape, v = st[name]
                return make_weight(v.reshape(shape[0], shape[1]), dt, qtype)

            def v1(name):
                return st[name][2].astype(np.float32).reshape(-1)

        # get_rows + cast_f32 reads the stored (dequantized) values
        self.embed = w2("embed_tokens.weight").values.astype(np.float32)
        self.norm = v1("norm.weight")
        self.layers = []
        for i in range(c.num_hidden_layers):
            p = f"layers.{i}."
            self.layers.append(dict(
                input_norm=v1(p + "input_layernorm.weight"), post_norm=v1(p + "post_attention_layernorm.weight"),
                self_attn=dict(q=w2(p + "self_attn.q_proj.weight"), k=w2(p + "self_attn.k_proj.weight"),
                               v=w2(p + "self_attn.v_proj.weight"), o=w2(p + "self_attn.o_proj.weight"),
                               q_norm=v1(p + "self_attn.q_norm.weight"), k_norm=v1(p + "self_attn.k_norm.weight")),
                mlp=dict(gate=w2(p + "mlp.gate_proj.weight"), up=w2(p + "mlp.up_proj.weight"),
                         down=w2(p + "mlp.down_proj.weight"))))


def forward_text_encoder_embeddings(W: TextWeights, token_ids) -> np.ndarray:
    return W.embed[np.asarray(token_ids, np.int64)].astype(np.float32)


def forward_text_encoder_layers(W: TextWeights, token_ids, attention_mask=None, n_layers: int = -1,
                                apply_final_norm: bool = True, causal: bool = True) -> np.ndarray:
    c = W.cfg
    n = len(token_ids)
    run = c.num_hidden_layers if n_layers < 0 else min(n_layers, c.num_hidden_layers)
    x = forward_text_encoder_embeddings(W, token_ids)
    rope = rope_tables(n, c.head_dim, c.rope_theta)
    for L in W.layers[:run]:
        xn = rms_norm(x, L["input_norm"], c.rms_norm_eps)
        a = attention(c, L["self_attn"], xn, xn, attention_mask, False, 0, rope, causal=causal)
        h = (x + a).astype(np.float32)
        hn = rms_norm(h, L["post_norm"], c.rms_norm_eps)
        act = (silu(mul_mat(L["mlp"]["gate"], hn)) * mul_mat(L["mlp"]["up"], hn)).astype(np.float32)
        x = (h + mul_mat(L["mlp"]["down"], act)).astype(np.float32)
    if apply_final_norm and run == c.num_hidden_layers:
        x = rms_norm(x, W.norm, c.rms_norm_eps)
    return x


def forward_with_floor(W: TextWeights, *args, perturb: float = 1e-7, **kw):
    """(out, floor) as dit_oracle.forward_with_floor."""
    out = forward_text_encoder_layers(W, *args, **kw)
    old = ggml_numerics.MULMAT_PERTURB
    ggml_numerics.MULMAT_PERTURB = perturb
    try:
        pert = forward_text_encoder_layers(W, *args, **kw)
    finally:
        ggml_numerics.MULMAT_PERTURB = old
    floor = float(np.linalg.norm(pert.astype(np.float64) - out) / np.linalg.norm(out.astype(np.float64)))
    return out, floor
