"""Per-kernel HIP-event times of one 240 s DiT forward (full width, LAYERS layers) in the ggml-faithful mode
(ACE_MI_QUANT_ACT=q8) against the product path, Q8_0 weights: JSON lines {mode, kernel: avg us}.  GPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
import numpy as np  # noqa: E402

from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config  # noqa: E402

layers = int(os.environ.get("LAYERS", "2"))
qtype = os.environ.get("QTYPE", "q8_0")
d = cached_checkpoint(make_config(num_hidden_layers=layers), seed=0, backend="torch")
os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qtype
T, L = 6000, 512
rng = np.random.default_rng(0)
h = rng.standard_normal((T, 64)).astype(np.float32)
c = rng.standard_normal((T, 128)).astype(np.float32)
e = rng.standard_normal((L, 2048)).astype(np.float32)
for mode in ("bf16", "q8"):
    os.environ["ACE_MI_QUANT_ACT"] = mode
    br = GGMLCAPIBridge()
    br.load_dit(d)
    br.dit_forward_tfirst(h, c, e, None, None, 0.75, 0.75)  # warm-up (staged images, workspace)
    br.profile_enable(True)
    br.profile_reset()
    for _ in range(3):
        br.dit_forward_tfirst(h, c, e, None, None, 0.75, 0.75)
    prof = br.profile_get()
    br.profile_enable(False)
    br.close()
    print(json.dumps({"mode": mode, "qtype": qtype, "layers": layers,
                      "avg_us": {n: round(1000.0 * ms / max(k, 1), 2) for n, ms, k in prof}}), flush=True)
