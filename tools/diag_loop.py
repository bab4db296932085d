"""Device sampling loop vs per-step forwards (round-3 diagnostic, GPU box): determinism of repeated forwards and
loops, and the step at which ace_mi_dit_sample_ex and ace_mi_dit_forward_batched + torch Euler part ways."""
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
for qt, staged in (("", "1"), ("q8_0", "1"), ("q8_0", "0")):
    os.environ["ACE_MI_QUANT_STAGED"] = staged
    if qt:
        os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qt
    else:
        os.environ.pop("ACE_GGML_DIT_WEIGHT_QTYPE", None)
    qt = qt + ("" if staged == "1" else "-fused")
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

    def loop(sched):
        xt = x0.clone()
        torch.cuda.synchronize()
        br.dit_sample_ex_device(1, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, list(sched),
                                cache_cross=False)
        br.synchronize()
        return xt

    v1, v2 = fwd(x0, 1.0), fwd(x0, 1.0)
    print(qt or "bf16", "forward twice identical:", bool(torch.equal(v1, v2)), flush=True)
    a1, a2 = loop([1.0]), loop([1.0])
    print(qt or "bf16", "1-step loop twice identical:", bool(torch.equal(a1, a2)), flush=True)
    ref1 = x0 - v1 * 1.0
    print(qt or "bf16", "1-step loop == forward + euler:", bool(torch.equal(a1, ref1)),
          "max|d|", float((a1 - ref1).abs().max()), flush=True)
    a3 = loop([1.0, 0.9])
    print(qt or "bf16", "2-step loop twice identical:", bool(torch.equal(a3, loop([1.0, 0.9]))), flush=True)
    x = x0 - v1 * float(np.float32(1.0) - np.float32(0.9))
    # the torch Euler update against IEEE f32 mul-then-sub on the host
    xh = (x0.cpu().numpy() - (v1.cpu().numpy() * np.float32(np.float32(1.0) - np.float32(0.9))).astype(np.float32))
    print(qt or "bf16", "torch euler == host f32 euler:", bool(np.array_equal(xh, x.cpu().numpy())), flush=True)
    va = fwd(x, np.float32(0.9))
    print(qt or "bf16", "forward of the step-1 input twice identical:", bool(torch.equal(va, fwd(x, np.float32(0.9)))),
          flush=True)
    ref3 = x - va * float(np.float32(0.9))
    print(qt or "bf16", "2-step loop == per-step:", bool(torch.equal(a3, ref3)), "max|d|", float((a3 - ref3).abs().max()),
          flush=True)
    br.close()
