"""GPU test of the device generation loop ace_mi_dit_sample_ex (ODE with the cross-attention cache,
SDE re-noise with caller noise) against per-step forwards through the reference ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_generation_loop_ex_on_gpu(tiny_bridge):
    """ace_mi_dit_sample_ex (ODE + cross-attention cache, SDE with caller noise) vs per-step forwards."""
    import torch
    rng = np.random.default_rng(23)
    B, T, L = 2, 36, 6
    x0 = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    sched = [1.0, 0.8, 0.5, 0.25]
    noise = rng.standard_normal((3, B, T, 64)).astype(np.float32)
    dc, de, dn = (torch.from_numpy(a).cuda() for a in (c, e, noise))
    for sde in (False, True):
        xt = torch.from_numpy(x0).cuda()
        torch.cuda.synchronize()
        tiny_bridge.dit_sample_ex_device(B, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, sched,
                                         sde=sde, d_noise=dn.data_ptr(), cache_cross=True)
        tiny_bridge.synchronize()
        ref = x0.copy()
        for i, t in enumerate(sched):
            v = np.stack([tiny_bridge.dit_forward_tfirst(ref[b], c[b], e[b], None, None, t, t) for b in range(B)])
            if i + 1 == len(sched):
                ref = ref - v * np.float32(t)
            elif sde:
                tn = np.float32(sched[i + 1])
                ref = tn * noise[i] + (np.float32(1) - tn) * (ref - v * np.float32(t))
            else:  # dt in f32, as the reference C loop computes it (acestep_ggml.cpp:2056-2086)
                ref = ref - v * (np.float32(t) - np.float32(sched[i + 1]))
        # same per-step forwards; only the f32 order of the Euler / re-noise arithmetic may differ, and
        # bf16 activation rounding amplifies such 1-ulp differences over the steps (test_gpu_forward.py)
        got = xt.cpu().numpy()
        l2 = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        assert l2 < 1e-5, (sde, l2, float(np.abs(got - ref).max()))
