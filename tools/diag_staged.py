"""GPU diagnostic: staged-dequant ring vs dequant-fused DiT forwards, per layer count and profiling mode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]
import numpy as np

from acestep_mi355x.capi import GGMLCAPIBridge
from acestep_mi355x.synthetic import cached_checkpoint, make_config

qt = sys.argv[1] if len(sys.argv) > 1 else "q4_k"
d = cached_checkpoint(make_config(num_hidden_layers=3), seed=0, backend="torch")
os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qt
rng = np.random.default_rng(5)
T, L, H = 400, 64, 2048
h = rng.standard_normal((T, 64)).astype(np.float32)
c = rng.standard_normal((T, 128)).astype(np.float32)
e = rng.standard_normal((L, H)).astype(np.float32)
for nl in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "3"]):
    os.environ["ACE_GGML_DIT_MAX_LAYERS"] = nl
    res = {}
    for mode in ("fused", "staged", "staged_prof", "dbg1", "dbg2"):
        os.environ["ACE_MI_QUANT_STAGED"] = "0" if mode == "fused" else "1"
        os.environ["ACE_MI_STAGE_DBG"] = mode[3:] if mode.startswith("dbg") else "0"
        br = GGMLCAPIBridge()
        br.load_dit(d)
        if mode == "staged_prof":
            br.profile_enable(True)
        res[mode] = [br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6) for _ in range(2)]
        br.close()
    f = res["fused"][0]
    for mode, outs in res.items():
        for i, o in enumerate(outs):
            dif = float(np.abs(o - f).max())
            print(f"{qt} layers={nl} {mode}[{i}] max|diff vs fused|={dif:.3e}", flush=True)
