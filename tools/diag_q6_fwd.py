"""Diagnostic (GPU box): 2-layer 240 s forwards with Q6_K weights -- staged vs dequant-fused with the tile forced
(25 / 20 / 21 / automatic), each repeated: which path differs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402
from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config  # noqa: E402

os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "2"
d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
qt = os.environ.get("QT", "q6_k")
os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qt
rng = np.random.default_rng(5)
T, L, H = 6000, 512, 2048
h = rng.standard_normal((T, 64)).astype(np.float32)
c = rng.standard_normal((T, 128)).astype(np.float32)
e = rng.standard_normal((L, H)).astype(np.float32)
res = {}
for staged, v in [tuple(x.split(":")) for x in os.environ.get("RUNS", "1:-1,0:-1,0:25,0:20,0:21").split(",")]:
    v = int(v)
    os.environ["ACE_MI_QUANT_STAGED"] = staged
    br = GGMLCAPIBridge()
    br.load_dit(d)
    capi.gemm_variant(v)
    try:
        o = [br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6) for _ in range(int(os.environ.get("REPS", "2")))]
    finally:
        capi.gemm_variant(-1)
    br.close()
    res[(staged, v)] = o
    print(qt, "staged" if staged == "1" else f"fused v{v}", "repeats", [float(np.max(np.abs(o[0] - x))) for x in o[1:]],
          "vs staged", float(np.max(np.abs(o[0] - res[("1", -1)][0]))) if ("1", -1) in res else None, flush=True)
