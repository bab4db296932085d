"""GPU box: error pattern of the f8c attention kernel on one small case (run once per ACE_MI_ATTN_KH setting): output
vs the fp64 reference of the same (rounded) operands, by d-tile, by d within a 32-row tile (the O^T accumulator rows),
by query row within a wave's 32 and by head.  One JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ace-step-1.5-ggml_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acestep_mi355x import capi  # noqa: E402
from tests.test_gpu_kernels import MODES, _attn_ref  # noqa: E402

rng = np.random.default_rng(64)
B, hq, hkv, nq, nk = 1, 2, 1, 64, int(os.environ.get("NK", "64"))
q = rng.standard_normal((B, nq, hq * 128)).astype(np.float32) * 2.0
kv = rng.standard_normal((B, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
scale = 1.0 / np.sqrt(128.0)
got = capi.kernel_attention(q, kv, hq, hkv, window=0, kmask=None, scale=scale, **MODES[os.environ.get("MODE", "f8c")])
ref = _attn_ref(q, kv, hq, hkv, 0, None, scale, rnd=lambda x: np.asarray(x, np.float32))
err = np.abs(got - ref).reshape(B, nq, hq, 128)
out = {"kh": os.environ.get("ACE_MI_ATTN_KH", "1"), "nk": nk, "max": float(err.max()), "mean": float(err.mean()),
       "rel_l2": float(np.linalg.norm(got - ref) / np.linalg.norm(ref)),
       "by_dtile": [float(err[..., 32 * t:32 * t + 32].mean()) for t in range(4)],
       "by_d_mod32": [round(float(err[..., [d for d in range(128) if d % 32 == j]].mean()), 6) for j in range(32)],
       "by_q_mod32": [round(float(err[:, [i for i in range(nq) if i % 32 == j]].mean()), 6) for j in range(32)],
       "by_head": [float(err[:, :, h].mean()) for h in range(hq)]}
print(json.dumps(out))
