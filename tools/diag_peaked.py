"""Where does the GPU's extra error in the peaked-softmax regime come from?  (round-3 diagnostic, GPU box)
One full-width layer at 240 s (T = 6000) vs the oracle, with q/k-norm weights x3 on both attentions / only the
self-attention / only the cross-attention, with and without the encoder (L = 512 / 0), in fp16 and f32
attention; GPU fp16 vs GPU f32; error energy in the worst 1 % of tokens."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
sys.path.insert(0, ROOT)
from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config  # noqa: E402
from oracle.dit_oracle import DitWeights, forward_with_floor_stats, maxabs_rms  # noqa: E402

T = 6000
rng = np.random.default_rng(1234)
h = rng.standard_normal((T, 64)).astype(np.float32)
c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
e = rng.standard_normal((512, 2048)).astype(np.float32)
os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "1"


def gpu(d, L, prec):
    os.environ["ACE_MI_ATTN_PRECISION"] = prec
    br = GGMLCAPIBridge()
    br.load_dit(d)
    out = br.dit_forward_tfirst(h, c, e[:L] if L else np.zeros((0, 2048), np.float32), None, None, 0.9, 0.9)
    br.close()
    return out


def rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / np.linalg.norm(b.astype(np.float64)))


for tags in [("self_attn", "cross_attn"), ("self_attn",), ("cross_attn",)]:
    d = cached_checkpoint(make_config(num_hidden_layers=2, layer_types=["full_attention", "sliding_attention"]),
                          seed=0, backend="torch", qk_norm_scale=3.0, qk_norm_tags=tags)
    for L in (512, 0):
        ref, fl, fm = forward_with_floor_stats(DitWeights(d), h, c, e[:L] if L else None, None, None, T, L, 0.9,
                                               0.9, max_layers=1)
        g16, g32 = gpu(d, L, "fp16"), gpu(d, L, "f32")
        tok = np.sum((g16.astype(np.float64) - ref) ** 2, axis=1)
        top = np.sort(tok)[::-1]
        print(f"tags={tags} L={L}: floor {fl:.3e} | fp16 {rel(g16, ref):.3e} (maxabs {maxabs_rms(g16, ref):.3e}) "
              f"f32 {rel(g32, ref):.3e} | fp16 vs f32 {rel(g16, g32):.3e} | worst 1% tokens hold "
              f"{top[:T // 100].sum() / top.sum():.2f} of the fp16 error energy", flush=True)
