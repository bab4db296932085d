"""Does a DiT forward depend on the previous call's state?  (round-3 diagnostic, GPU box; bf16, 2 layers, 240 s)
The device 2-step loop and per-step forwards + torch Euler differ at the bf16 level although each piece matches
on its own (diag_loop.py); this isolates whether the second forward's result depends on what ran before it."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x.capi import GGMLCAPIBridge  # noqa: E402
from acestep_mi355x.synthetic import cached_checkpoint, make_config  # noqa: E402

os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "2"
T, L = 6000, 512
rng = np.random.default_rng(27)
h = rng.standard_normal((1, T, 64)).astype(np.float32)
c = np.concatenate([rng.standard_normal((1, T, 64)), np.ones((1, T, 64))], axis=-1).astype(np.float32)
e = rng.standard_normal((1, L, 2048)).astype(np.float32)
dev = torch.device("cuda:0")
x0, dc, de = (torch.from_numpy(a).to(dev) for a in (h, c, e))
d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
br = GGMLCAPIBridge()
br.load_dit(d)


def fwd(x, t):
    tt = torch.full((1,), float(t), dtype=torch.float32, device=dev)
    v = torch.empty_like(x)
    torch.cuda.synchronize()
    br.dit_forward_batched_device(1, T, L, x.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, tt.data_ptr(),
                                  tt.data_ptr(), v.data_ptr(), 0)
    br.synchronize()
    return v


def loop(x, sched):
    xt = x.clone()
    torch.cuda.synchronize()
    br.dit_sample_ex_device(1, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, list(sched), cache_cross=False)
    br.synchronize()
    return xt


def cmp(tag, a, b):
    print(f"{tag}: equal={bool(torch.equal(a, b))} max|d|={float((a - b).abs().max()):.3e}", flush=True)


v1 = fwd(x0, 1.0)
x = x0 - v1 * float(np.float32(1.0) - np.float32(0.9))
q_after_x0 = fwd(x, np.float32(0.9))
q_after_x = fwd(x, np.float32(0.9))
cmp("fwd(x1) after fwd(x0)  vs  after fwd(x1)", q_after_x0, q_after_x)
fwd(x0, np.float32(0.9))
cmp("fwd(x1) after fwd(x0, t=0.9)  vs  after fwd(x1)", fwd(x, np.float32(0.9)), q_after_x)
fwd(x, np.float32(1.0))
cmp("fwd(x1) after fwd(x1, t=1.0)  vs  after fwd(x1)", fwd(x, np.float32(0.9)), q_after_x)
ref = x - q_after_x * float(np.float32(0.9))
cmp("1-step loop from x1 at 0.9  vs  x1 - fwd(x1)*0.9", loop(x, [0.9]), ref)
a3 = loop(x0, [1.0, 0.9])
cmp("2-step loop  vs  per-step", a3, ref)
# the loop's own x1: recover from a 2-step SDE-free loop is impossible; run [1.0, 0.9, 0.9] dt=0 step instead
a_dt0 = loop(x0, [1.0, 0.9, 0.9])  # step 2 Euler with dt = 0 leaves x1; final step x1 - v*0.9 again
cmp("3-step loop with a dt=0 middle step  vs  2-step loop", a_dt0, a3)
br.close()
