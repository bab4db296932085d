"""Generates tests/golden/text_encoder_qwen3.npz: the text encoder's reference-side pin.

The reference checks its ggml Qwen3 text encoder against `transformers.AutoModel` (acestep_ggml/tools/
compare_text_encoder.py:133-183: embed_tokens -> layers with create_causal_mask and rotary_emb -> norm).  This script runs
that model -- transformers' Qwen3Model, here in float64 with eager attention -- on the synthetic tiny text checkpoint the
tests use (acestep_mi355x.synthetic TEXT_TINY_CONFIG, seed 6, BF16 weights: exactly representable, so ggml-style bf16
arithmetic and the float64 model see the same weights) and stores token ids, masks and hidden states.  The fixture holds
no weights: it records the sha256 of the checkpoint's safetensors bytes, which the tests re-create with the same writer
and check before comparing.

Cases: full forward (final norm) at n = 37 and 200, the same with the last 5 keys padding-masked (attention_mask), and
the first layer's output without the final norm (the harness's --layers 1 path).

Run from the repo root: python tests/golden/make_text_encoder_fixture.py"""
import hashlib
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))

from acestep_mi355x.synthetic import TEXT_TINY_CONFIG, text_tensor_specs, write_checkpoint  # noqa: E402
from oracle.dit_oracle import read_safetensors  # noqa: E402

SEED = 6
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "text_encoder_qwen3.npz")


def checkpoint(d):
    write_checkpoint(d, TEXT_TINY_CONFIG, seed=SEED, dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    path = os.path.join(d, "model.safetensors")
    with open(path, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    return path, sha


def hf_model(st_path):
    from transformers import Qwen3Config, Qwen3Model
    c = TEXT_TINY_CONFIG
    cfg = Qwen3Config(vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
                      num_hidden_layers=c["num_hidden_layers"], num_attention_heads=c["num_attention_heads"],
                      num_key_value_heads=c["num_key_value_heads"], head_dim=c["head_dim"],
                      max_position_embeddings=c["max_position_embeddings"], rms_norm_eps=c["rms_norm_eps"],
                      rope_theta=c["rope_theta"], attention_bias=False, tie_word_embeddings=False)
    cfg._attn_implementation = "eager"
    model = Qwen3Model(cfg).double().eval()
    sd = {k: torch.from_numpy(v[2].astype(np.float64)) for k, v in read_safetensors(st_path).items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all("rotary" in m for m in missing), (missing, unexpected)
    return model


def first_layer(model, ids):
    """compare_text_encoder.py:138-176 with layers = 1: embeddings, one decoder layer, no final norm"""
    from transformers.masking_utils import create_causal_mask
    x = model.embed_tokens(ids)
    position_ids = torch.arange(0, x.shape[1]).unsqueeze(0)
    # (transformers 5.x: create_causal_mask(config, inputs_embeds, ...); the explicit mask, never the is_causal skip, since
    # the eager attention path applies exactly the mask it is given)
    mask = create_causal_mask(config=model.config, inputs_embeds=x, attention_mask=None, past_key_values=None,
                              position_ids=position_ids, allow_is_causal_skip=False)
    pe = model.rotary_emb(x, position_ids)
    out = model.layers[0](x, attention_mask=mask, position_ids=position_ids, past_key_values=None, use_cache=False,
                          position_embeddings=pe)
    return out[0] if isinstance(out, tuple) else out


def main():
    d = tempfile.mkdtemp(prefix="acemi_te_fix_")
    st_path, sha = checkpoint(d)
    model = hf_model(st_path)
    rng = np.random.default_rng(2026)
    res = {"sha256": np.array(sha), "seed": np.array(SEED)}
    with torch.no_grad():
        for n in (37, 200):
            ids = rng.integers(0, TEXT_TINY_CONFIG["vocab_size"], n).astype(np.int32)
            t = torch.from_numpy(ids.astype(np.int64))[None]
            res[f"full{n}/ids"] = ids
            res[f"full{n}/out"] = model(input_ids=t).last_hidden_state[0].numpy().astype(np.float32)
            mask = np.ones(n, np.int32)
            mask[n - 5:] = 0
            res[f"masked{n}/ids"] = ids
            res[f"masked{n}/mask"] = mask
            res[f"masked{n}/out"] = model(input_ids=t, attention_mask=torch.from_numpy(mask.astype(np.int64))[None]) \
                .last_hidden_state[0].numpy().astype(np.float32)
            res[f"layer1_{n}/ids"] = ids
            res[f"layer1_{n}/out"] = first_layer(model, t)[0].numpy().astype(np.float32)
    np.savez_compressed(OUT, **res)
    print(OUT, sha, sorted(res))


if __name__ == "__main__":
    main()
