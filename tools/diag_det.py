"""Forward determinism and staged == fused (round-3 diagnostic, GPU box): the same forward twice per mode, staged
vs fused quantized forwards, with the persistent rmsnorm on and off."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config, write_checkpoint  # noqa: E402


def fwd(d, T, L, H, env):
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    rng = np.random.default_rng(5)
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, H)).astype(np.float32)
    br = GGMLCAPIBridge()
    br.load_dit(d)
    o = [br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6) for _ in range(3)]
    br.close()
    return o


def md(a, b):
    return float(np.max(np.abs(a - b)))


os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "3"
full = cached_checkpoint(make_config(num_hidden_layers=3), seed=0, backend="torch")
for rms in ("2", "0"):
    os.environ["ACE_MI_RMSNORM_PERSIST"] = rms
    for qt in (None, "q8_0", "q4_k"):
        res = {}
        for staged in (("1", "0") if qt else ("1",)):
            o = fwd(full, 400, 64, 2048, {"ACE_GGML_DIT_WEIGHT_QTYPE": qt, "ACE_MI_QUANT_STAGED": staged})
            res[staged] = o
            print(f"rmsnorm_persist={rms} {qt or 'bf16'} staged={staged}: repeat max|d| {md(o[0], o[1]):.3e} "
                  f"{md(o[0], o[2]):.3e}", flush=True)
        if qt:
            print(f"rmsnorm_persist={rms} {qt}: staged vs fused max|d| {md(res['1'][0], res['0'][0]):.3e}", flush=True)
