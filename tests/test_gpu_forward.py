"""GPU parity of the full DiT forward (ace_ggml_dit_forward and the MI355X extensions)
against the oracle restatement of ace_dit::forward_dit.

Tolerance (BASELINE.json north_star "within 1e-3 relative"):
  rel_l2 = ||gpu - ref||_2 / ||ref||_2 <= max(1e-3, FLOOR_K * floor)
where `floor` is the oracle's own rel_l2 change when every mul_mat result is perturbed by
1e-7 (oracle.dit_oracle.forward_with_floor).  Every bf16 activation rounding turns a
relative difference e into ~sqrt(e * 2^-8), so two correct implementations that differ
only in f32 summation order agree to this floor and no better: measured 1.3e-3 after 2
full-width layers and 3.4e-3 after 24 layers ("Parity").  Where the floor is
below 1e-3 (tiny configs, shallow depth) the plain 1e-3 bound applies.  The
element-wise statistic max|gpu - ref| / rms(ref) is asserted against 2.5x the oracle's own spread of
that statistic wherever the test computes it (the full-width cases here, tests/test_gpu_configs.py and
tests/test_gpu_parity_strict.py, whose fault-injection negative control shows that it catches one wrong
16 x 128 tile that the L2 bound lets through).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

REL_L2 = 1e-3
FLOOR_K = 1.5
MAXABS_K = 2.5
COS_MIN = 0.99999


def check(got, ref, floor, tag, floor_max=None):
    """rel-L2 floor-relative (module docstring).  With `floor_max` (the oracle's own perturbation spread of
    the element-wise statistic max|d| / rms(ref), dit_oracle.forward_with_floor_stats) the element-wise
    error is asserted against it with no absolute slack: max|got - ref| / rms(ref) <= MAXABS_K x floor_max,
    so a wrong tile on a few rows fails even when the L2 over the whole output absorbs it
    (test_gpu_parity_strict.py, fault-injection negative control).  SURVEY §8(d)'s max relative error over
    |ref| > 1e-2 rms(ref) is printed for reference.  Returns rel-L2."""
    l2, mx = rel_errors(got, ref)
    ma = maxabs_rms(got, ref)
    cos = float(np.dot(got.ravel().astype(np.float64), ref.ravel()) /
                (np.linalg.norm(got.astype(np.float64)) * np.linalg.norm(ref.astype(np.float64))))
    bound = max(REL_L2, FLOOR_K * floor)
    extra = ""
    if floor_max is not None:
        extra = (f" maxabs/rms={ma:.3e} floor_maxabs={floor_max:.3e} maxabs_ratio={ma / max(floor_max, 1e-12):.2f}"
                 f" maxabs_bound={MAXABS_K * floor_max:.3e}")
    print(f"{tag}: rel_l2={l2:.3e} floor={floor:.3e} ratio={l2 / max(floor, 1e-12):.2f} cos={cos:.7f} "
          f"rel_max={mx:.3e} bound={bound:.3e}{extra}")
    # cosine: 1 - cos ~ rel_l2^2 / 2, so it is held to the same bound (with 2x slack), never looser than 1e-5
    assert np.isfinite(l2) and l2 <= bound and 1.0 - cos <= max(1.0 - COS_MIN, bound * bound), (tag, l2, floor, cos)
    if floor_max is not None:
        assert ma <= MAXABS_K * floor_max, (tag, ma, floor_max)
    return l2


# The shipped quantized path (bf16 activations x bf16(dequant(W))) against ggml's OWN quantized arithmetic (Q8_0 / Q8_K
# activation blocks): its arithmetic differs from ggml's by the activation rounding, so it is held to a looser, asserted
# multiple of the ggml-semantics floor (measured 1.28-1.64x in round 5): rel-L2 <= GGML_PRODUCT_K x floor and
# max|d| / rms <= GGML_PRODUCT_K x MAXABS_K x that statistic's floor.  A regression that moves the product path away
# from ggml fails here even while it still matches its own arithmetic (check() against engine_view).
GGML_PRODUCT_K = 1.75


def check_product_vs_ggml(got, ref, floor, floor_max, tag):
    l2, _ = rel_errors(got, ref)
    ma = maxabs_rms(got, ref)
    print(f"{tag}: product path vs ggml semantics rel_l2={l2:.3e} floor={floor:.3e} ratio={l2 / floor:.2f} "
          f"maxabs/rms={ma:.3e} floor_maxabs={floor_max:.3e} maxabs_ratio={ma / floor_max:.2f} "
          f"(bounds {GGML_PRODUCT_K} / {GGML_PRODUCT_K * MAXABS_K})")
    assert np.isfinite(l2) and l2 <= GGML_PRODUCT_K * floor, (tag, l2, floor)
    assert ma <= GGML_PRODUCT_K * MAXABS_K * floor_max, (tag, ma, floor_max)
    return l2


def maxabs_rms(got, ref):
    from oracle.dit_oracle import maxabs_rms as f
    return f(got, ref)


def rel_errors(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    l2 = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    rms = np.sqrt(np.mean(ref * ref))
    sel = np.abs(ref) > 1e-2 * rms
    mx = float(np.max(np.abs(got - ref)[sel] / np.abs(ref[sel]))) if sel.any() else 0.0
    return float(l2), mx


def test_golden_tiny_cases(tiny_bridge):
    z = np.load(os.path.join(GOLDEN, "dit_tiny.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    for n in names:
        T, L, t, r = z[f"{n}/meta"]
        T, L = int(T), int(L)
        m = z[f"{n}/mask"]
        em = z[f"{n}/enc_mask"]
        enc = z[f"{n}/enc"] if L > 0 else np.zeros((0, 256), np.float32)
        got = tiny_bridge.dit_forward_tfirst(z[f"{n}/hidden"], z[f"{n}/context"], enc, m if m.size else None,
                                             em if em.size else None, float(t), float(r))
        l2, mx = rel_errors(got, z[f"{n}/out"])
        print(f"golden {n}: rel_l2={l2:.3e} rel_max={mx:.3e}")
        assert l2 <= REL_L2, (n, l2, mx)


def test_tiny_vs_live_oracle_long_sequence(tiny_ckpt, tiny_bridge):
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    W = DitWeights(tiny_ckpt)
    rng = np.random.default_rng(99)
    T, L = 1001, 130
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, 256)).astype(np.float32)
    # (a frame mask that empties a whole sliding window makes ggml's soft_max NaN; keep windows non-empty)
    mask = np.ones(T, np.int32)
    mask[990:] = 0
    mask[301:305] = 0
    emask = np.ones(L, np.int32)
    emask[100:] = 0
    ref, floor, fmax = forward_with_floor_stats(W, h, c, e, mask, emask, T, L, 0.8, 0.8)
    got = tiny_bridge.dit_forward_tfirst(h, c, e, mask, emask, 0.8, 0.8)
    check(got, ref, floor, "tiny T=1001", fmax)


def test_null_inputs_are_zeros(tiny_bridge):
    """hidden/context NULL are treated as zeros (acestep_dit_model.cpp:1358-1377)."""
    import ctypes
    rng = np.random.default_rng(5)
    T, L = 30, 4
    e = rng.standard_normal((L, 256)).astype(np.float32)
    zeros_h = np.zeros((T, 64), np.float32)
    zeros_c = np.zeros((T, 128), np.float32)
    a = tiny_bridge.dit_forward_tfirst(zeros_h, zeros_c, e, None, None, 0.5, 0.5)
    out = np.empty((T, 64), np.float32)
    fp = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    st = tiny_bridge.lib.ace_ggml_dit_forward(tiny_bridge.ctx, None, None, fp(e), None, None, T, L, 0.5, 0.5,
                                              fp(out), out.nbytes)
    assert st == 0
    np.testing.assert_array_equal(a, out)
    small = np.empty((T - 1, 64), np.float32)
    st = tiny_bridge.lib.ace_ggml_dit_forward(tiny_bridge.ctx, None, None, fp(e), None, None, T, L, 0.5, 0.5,
                                              fp(small), small.nbytes)
    assert st == 2 and tiny_bridge._last_error() == "output buffer too small"
    st = tiny_bridge.lib.ace_ggml_dit_forward(tiny_bridge.ctx, None, None, None, None, None, T, L, 0.5, 0.5,
                                              fp(out), out.nbytes)
    assert st == 1


def test_batched_device_entry_equals_serial_calls(tiny_bridge):
    import torch
    rng = np.random.default_rng(17)
    B, T, L = 3, 50, 7
    h = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    ts = np.array([1.0, 0.6, 0.3], np.float32)
    rs = np.array([1.0, 0.2, 0.3], np.float32)
    mask = np.ones((B, T), np.int32)
    mask[1, 40:] = 0
    serial = np.stack([tiny_bridge.dit_forward_tfirst(h[b], c[b], e[b], mask[b], None, ts[b], rs[b])
                       for b in range(B)])
    dev = torch.device("cuda:0")
    th = torch.from_numpy(h).to(dev)
    tc = torch.from_numpy(c).to(dev)
    te = torch.from_numpy(e).to(dev)
    tm = torch.from_numpy(mask).to(dev)
    tt = torch.from_numpy(ts).to(dev)
    tr = torch.from_numpy(rs).to(dev)
    out = torch.empty((B, T, 64), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    tiny_bridge.dit_forward_batched_device(B, T, L, th.data_ptr(), tc.data_ptr(), te.data_ptr(), tm.data_ptr(), 0,
                                           tt.data_ptr(), tr.data_ptr(), out.data_ptr(), 0)
    tiny_bridge.synchronize()
    got = out.cpu().numpy()
    for b in range(B):
        l2, mx = rel_errors(got[b], serial[b])
        assert l2 < 1e-6, (b, l2, mx)


def test_device_sampler_equals_host_euler_loop(tiny_bridge):
    import torch
    from acestep_mi355x.schedule import get_timestep_schedule
    rng = np.random.default_rng(23)
    B, T, L = 2, 40, 6
    x0 = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    sched = get_timestep_schedule(3.0)
    # host loop through the reference-ABI entry (acestep_ggml.cpp:2056-2086 order)
    ref = x0.copy()
    for b in range(B):
        xt = ref[b]
        for i, t in enumerate(sched):
            vt = tiny_bridge.dit_forward_tfirst(xt, c[b], e[b], None, None, t, t)
            dt = np.float32(t) if i + 1 == len(sched) else np.float32(np.float32(t) - np.float32(sched[i + 1]))
            xt = (xt - vt * dt).astype(np.float32)
        ref[b] = xt
    dev = torch.device("cuda:0")
    xt_d = torch.from_numpy(x0).to(dev)
    tc = torch.from_numpy(c).to(dev)
    te = torch.from_numpy(e).to(dev)
    torch.cuda.synchronize()
    tiny_bridge.dit_sample_device(B, T, L, xt_d.data_ptr(), tc.data_ptr(), te.data_ptr(), 0, 0, sched)
    tiny_bridge.synchronize()
    got = xt_d.cpu().numpy()
    l2, _ = rel_errors(got, ref)
    # same library, same arithmetic; the host loop's numpy Euler update and the batched (B = 2) GEMM
    # tiles differ from the device loop in the last f32 bit, which the bf16 activation roundings of
    # 8 forwards amplify (the DiT's floor, DESIGN.md "Parity")
    assert l2 < 1e-4, l2


@pytest.mark.slow
def test_full_width_two_layers_240s(monkeypatch):
    """Full DiT width (2048/6144, 16/8 heads) at the 240 s workload (T = 6000 frames at 25 Hz,
    N = 3000 tokens, L = 512), first 2 layers (ACE_GGML_DIT_MAX_LAYERS, :1457-1464): one
    sliding + one full layer, vs the oracle."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    cfg = make_config(num_hidden_layers=2)
    d = cached_checkpoint(cfg, seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    br = GGMLCAPIBridge()
    br.load_dit(d)
    rng = np.random.default_rng(1234)
    T, L = 6000, 512
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.9, 0.9)
    br.close()
    W = DitWeights(d)
    ref, floor, fmax = forward_with_floor_stats(W, h, c, e, None, None, T, L, 0.9, 0.9, max_layers=2)
    check(got, ref, floor, "full-width 2-layer 240s", fmax)


def test_context_destroy_then_new_context_60s(monkeypatch):
    """a context whose stream ran split-K GEMMs (the 60 s down projection, variant 213) is destroyed;
    a forward in a new context on the same device must still run (no sync of the dead stream, no stale error
    word) and give the same bits as the first context's forward."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    rng = np.random.default_rng(60)
    T, L = 1500, 512
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    outs = []
    for _ in range(2):
        br = GGMLCAPIBridge()
        br.load_dit(d)
        outs.append(br.dit_forward_tfirst(h, c, e, None, None, 0.7, 0.7))
        br.synchronize()
        br.close()
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.slow
def test_full_width_two_layers_600s(monkeypatch):
    """The largest BASELINE config's sequence (C5: 600 s, T = 15000 frames, N = 7500 tokens, L = 512)
    at full width, first 2 layers (one sliding, one full), vs the oracle: 118 key tiles per
    block, so the full layer runs the two-way key split with the merge kernel."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    cfg = make_config(num_hidden_layers=2)
    d = cached_checkpoint(cfg, seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    br = GGMLCAPIBridge()
    br.load_dit(d)
    rng = np.random.default_rng(600)
    T, L = 15000, 512
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.5, 0.5)
    br.close()
    ref, floor, fmax = forward_with_floor_stats(DitWeights(d), h, c, e, None, None, T, L, 0.5, 0.5, max_layers=2)
    check(got, ref, floor, "full-width 2-layer 600s", fmax)


@pytest.mark.slow
def test_full_model_24_layers_20s():
    """The complete 24-layer DiT (synthetic weights, real shapes) at 20 s of audio
    (T = 500 frames, N = 250 tokens, L = 256) vs the oracle: the error budget over full depth."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import FULL_CONFIG, cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    d = cached_checkpoint(make_config(), seed=0, backend="torch")
    br = GGMLCAPIBridge()
    br.load_dit(d)
    rng = np.random.default_rng(4321)
    T, L = 500, 256
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.6428571429, 0.6428571429)
    br.close()
    ref, floor, fmax = forward_with_floor_stats(DitWeights(d), h, c, e, None, None, T, L, 0.6428571429,
                                                0.6428571429)
    check(got, ref, floor, "full 24-layer 20s", fmax)


def test_decoder_forward_hook_device_path(tiny_bridge):
    """install_dit_backend on cuda tensors (device pointers, one batched call) == the reference
    host-pointer ABI per item; bf16 in/out like the PyTorch pipeline."""
    import types

    import torch
    from acestep_mi355x.hook import install_dit_backend
    dec = types.SimpleNamespace(forward=None)
    handler = types.SimpleNamespace(model=types.SimpleNamespace(decoder=dec))
    install_dit_backend(handler, tiny_bridge)
    rng = np.random.default_rng(41)
    B, T, L = 2, 44, 9
    h = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    em = np.ones((B, L), np.int64)
    em[0, 6:] = 0
    dev = torch.device("cuda:0")
    t = torch.tensor([0.9, 0.4], device=dev)
    pred, _ = handler.model.decoder.forward(
        hidden_states=torch.from_numpy(h).to(dev), timestep=t, timestep_r=t, attention_mask=None,
        encoder_hidden_states=torch.from_numpy(e).to(dev), encoder_attention_mask=torch.from_numpy(em).to(dev),
        context_latents=torch.from_numpy(c).to(dev))
    torch.cuda.synchronize()
    got = pred.cpu().numpy()
    for b in range(B):
        ref = tiny_bridge.dit_forward_tfirst(h[b], c[b], e[b], None, em[b].astype(np.int32), float(t[b]), float(t[b]))
        l2, _ = rel_errors(got[b], ref)
        assert l2 < 1e-6, (b, l2)


def _batched(br, h, c, e, t):
    import torch
    dev = torch.device("cuda:0")
    B, T = h.shape[:2]
    L = e.shape[1]
    th, tc, te = (torch.from_numpy(x).to(dev) for x in (h, c, e))
    tt = torch.full((B,), t, dtype=torch.float32, device=dev)
    out = torch.empty((B, T, 64), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    br.dit_forward_batched_device(B, T, L, th.data_ptr(), tc.data_ptr(), te.data_ptr(), 0, 0, tt.data_ptr(),
                                  tt.data_ptr(), out.data_ptr(), 0)
    br.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("variant", [-1, 10, 11, 16, 18])
@pytest.mark.parametrize("width", ["tiny", "full"])
def test_fused_qkv_prep_is_bit_exact(tiny_ckpt, monkeypatch, width, variant):
    """The QKV / cross-q GEMMs with QK-norm, RoPE and the attention re-layout fused into their epilogue
    (EPI_QKV_PREP) give the same bits as the f32 store + attn_prep pair (ACE_MI_UNFUSED_PREP=1): batched
    items whose token counts are not multiples of 16 or of the GEMM's row tile, so V^T key groups are cut
    by chunk and item edges; the automatic tile choice, the forced 8-wave 256-column tiles and the 8-wave
    (4 x 2) 192x128 tiles."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    if width == "tiny":
        d, H, cases = tiny_ckpt, 256, [(1, 37, 5), (2, 301, 9), (3, 1001, 17)]
    else:
        from acestep_mi355x.synthetic import cached_checkpoint, make_config
        d, H, cases = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch"), 2048, [(2, 601, 64)]
        monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    from acestep_mi355x import capi
    outs = {}
    for fused in (True, False):
        if fused:
            monkeypatch.delenv("ACE_MI_UNFUSED_PREP", raising=False)
        else:
            monkeypatch.setenv("ACE_MI_UNFUSED_PREP", "1")
        br = GGMLCAPIBridge()
        br.load_dit(d)
        for B, T, L in cases:
            r = np.random.default_rng(B * 7 + T)
            h = r.standard_normal((B, T, 64)).astype(np.float32)
            c = r.standard_normal((B, T, 128)).astype(np.float32)
            e = r.standard_normal((B, L, H)).astype(np.float32)
            # the same tiles on both sides (the 8-wave tiles' two-heads-per-tile prep: 10, 11), so only the prep
            # path differs (a split-K pick on one side would change the other GEMMs' summation order)
            capi.gemm_variant(variant)
            try:
                outs[(fused, B, T)] = _batched(br, h, c, e, 0.7)
            finally:
                capi.gemm_variant(-1)
        br.close()
    for B, T, L in cases:
        a, b = outs[(True, B, T)], outs[(False, B, T)]
        assert np.isfinite(a).all()
        np.testing.assert_array_equal(a, b, err_msg=f"B={B} T={T}")
