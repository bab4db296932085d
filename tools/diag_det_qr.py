"""Round-4 check of the round-3 anomaly "register-dequant tiles 22 / 23 (split-K or not) are not run-to-run identical
inside whole forwards" (GPU box): 3-layer full-width forwards with fused quantized weights, the tile forced, each
forward repeated 3 times; then the same against the staged (bf16 image) forward of the same weights."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402
from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config  # noqa: E402


def fwd(d, T, L, H):
    rng = np.random.default_rng(5)
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, H)).astype(np.float32)
    br = GGMLCAPIBridge()
    br.load_dit(d)
    o = [br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6) for _ in range(3)]
    br.close()
    return o


os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "3"
full = cached_checkpoint(make_config(num_hidden_layers=3), seed=0, backend="torch")
lib = capi.load_library()
for qt in os.environ.get("QTYPES", "q4_k,q8_0").split(","):
    os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qt
    os.environ["ACE_MI_QUANT_STAGED"] = "1"
    ref = fwd(full, 400, 64, 2048)[0]
    os.environ["ACE_MI_QUANT_STAGED"] = "0"
    for v in [int(x) for x in os.environ.get("VARIANTS", "22,23,222,223,423,20,21").split(",")]:
        capi.gemm_variant(v)
        try:
            o = fwd(full, 400, 64, 2048)
        finally:
            capi.gemm_variant(-1)
        print(f"{qt} v{v}: repeat max|d| {np.max(np.abs(o[0] - o[1])):.3e} {np.max(np.abs(o[0] - o[2])):.3e}  "
              f"vs staged {np.max(np.abs(o[0] - ref)):.3e}", flush=True)
