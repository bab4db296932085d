"""GPU parity at the BASELINE.json workloads, each against the oracle (not only against the library's own
serial path):

  configs[0]  F16-safetensors weights, 10 s (T = 250, N = 125), L = 512, all 24 layers
  configs[1]  bf16 weights, 60 s (T = 1500, N = 750), L = 512, 2 layers (the short-sequence GEMM tiles)
  configs[2]  Q8_0 weights, 240 s (T = 6000, N = 3000), L = 512, 2 layers: engine arithmetic and ggml's;
              and the bench's exact path, 3 steps of the device sampling loop (ace_mi_dit_sample_ex)
  configs[3]  bs = 8 at 240 s, 2 layers, every item of one batched call
  configs[4]  Q4_K weights at 600 s (T = 15000, N = 7500), 2 layers; the full-width VAE decode over 192
              latent frames through the windowed plan (128-frame windows, 32 frames of overlap)

Every comparison asserts both SURVEY §8(d) metrics floor-relatively: rel-L2 <= max(1e-3, 1.5 x the
oracle's own 1e-7-perturbation spread) and the max element-wise relative error over |ref| > 1e-2 rms(ref)
<= max(1e-3, MAX_K x the same spread of that metric) (test_gpu_forward.check).  Layer counts are capped
with ACE_GGML_DIT_MAX_LAYERS (acestep_dit_model.cpp:1457-1464) where the numpy oracle would otherwise
take minutes; the sequence lengths, widths and weight formats are the configs' own.
"""
import numpy as np
import pytest

from test_gpu_forward import check, check_product_vs_ggml
from test_gpu_quant import engine_view

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _inputs(T, L, seed, H=2048, B=None):
    rng = np.random.default_rng(seed)
    shp = (T,) if B is None else (B, T)
    h = rng.standard_normal(shp + (64,)).astype(np.float32)
    c = np.concatenate([rng.standard_normal(shp + (64,)), np.ones(shp + (64,))], axis=-1).astype(np.float32)
    e = rng.standard_normal(((L,) if B is None else (B, L)) + (H,)).astype(np.float32)
    return h, c, e


def test_config0_f16_weights_10s_full_model():
    """configs[0]: the reference's CPU plumbing case -- F16 weights, whose activations ggml rounds to fp16
    (3 more mantissa bits than bf16, so the floor is ~3x lower than with bf16 weights)."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    d = cached_checkpoint(make_config(), seed=0, dtype="F16", backend="torch")
    T, L = 250, 512
    h, c, e = _inputs(T, L, 1234)
    br = GGMLCAPIBridge()
    br.load_dit(d)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.6428571429, 0.6428571429)
    br.close()
    ref, floor, fmax = forward_with_floor_stats(DitWeights(d), h, c, e, None, None, T, L, 0.6428571429,
                                                0.6428571429)
    l2 = check(got, ref, floor, "configs[0] F16 10 s, 24 layers", fmax)
    print(f"configs[0]: rel_l2 {'<=' if l2 <= 1e-3 else '>'} 1e-3 (north-star literal bound)")


def test_config1_bf16_60s_two_layers(monkeypatch):
    """configs[1]'s shape: bf16 weights, 60 s (T = 1500 frames, N = 750 tokens), L = 512, first 2 layers
    (one sliding, one full): the M = 750 tile choice of the GEMMs and the 60 s attention grid vs the oracle."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    T, L = 1500, 512
    h, c, e = _inputs(T, L, 60)
    br = GGMLCAPIBridge()
    br.load_dit(d)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.85, 0.85)
    br.close()
    ref, floor, fmax = forward_with_floor_stats(DitWeights(d), h, c, e, None, None, T, L, 0.85, 0.85, max_layers=2)
    check(got, ref, floor, "configs[1] bf16 60 s, 2 layers", fmax)


def test_config2_q8_0_sampling_loop_240s(monkeypatch):
    """configs[2] through the bench's exact path: 3 steps of ace_mi_dit_sample_ex with Q8_0 weights at 240 s
    (full width, 2 layers, cross K/V recomputed every step as in the bench) equal, bit for bit, 3 per-step
    batched forwards (ace_mi_dit_forward_batched) with the same Euler updates; the first step's velocity is
    checked against the oracle on the same quantized bytes (engine arithmetic)."""
    import torch
    from acestep_mi355x import capi
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle import ggml_numerics
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", "q8_0")
    T, L = 6000, 512
    h, c, e = _inputs(T, L, 27)
    sched = np.array([1.0, 0.9, 0.75], np.float32)
    dev = torch.device("cuda:0")
    x0, dc, de = (torch.from_numpy(a[None]).to(dev) for a in (h, c, e))
    br = GGMLCAPIBridge()
    br.load_dit(d)
    xt = x0.clone()
    torch.cuda.synchronize()
    br.dit_sample_ex_device(1, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, list(sched),
                            cache_cross=False)
    br.synchronize()
    loop = xt.cpu().numpy()[0]
    # per-step forwards + the same f32 Euler arithmetic (x -= v * dt; the last step x0 = x - v * t)
    x = x0.clone()
    v = torch.empty_like(x)
    v0 = None
    for i, t in enumerate(sched):
        tt = torch.full((1,), float(t), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        br.dit_forward_batched_device(1, T, L, x.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, tt.data_ptr(),
                                      tt.data_ptr(), v.data_ptr(), 0)
        br.synchronize()
        if v0 is None:
            v0 = v.cpu().numpy()[0]
        dt = np.float32(t) if i + 1 == len(sched) else np.float32(np.float32(t) - np.float32(sched[i + 1]))
        x = x - v * float(dt)
    torch.cuda.synchronize()
    br.close()
    np.testing.assert_array_equal(loop, x.cpu().numpy()[0])
    monkeypatch.setattr(ggml_numerics, "QUANTIZER", capi.quantize)
    W = DitWeights(d, qtype="q8_0")
    ref, floor, fmax = forward_with_floor_stats(engine_view(W), h, c, e, None, None, T, L, float(sched[0]),
                                                float(sched[0]), max_layers=2)
    check(v0, ref, floor, "configs[2] Q8_0 sampling loop, step 0 velocity", fmax)


@pytest.mark.parametrize("qtype,T,seed", [("q8_0", 6000, 2), ("q4_k", 15000, 4)])
def test_quantized_configs_full_width(monkeypatch, qtype, T, seed):
    """configs[2] (Q8_0, 240 s) and configs[4] (Q4_K, 600 s) at full width, 2 layers:
      * the product path (bf16 activations x bf16(dequant W)) vs the oracle on the same quantized bytes with that
        arithmetic, floor-relative, element-wise too;
      * the ggml-faithful mode (ACE_MI_QUANT_ACT=q8: Q8_0 / Q8_K activation blocks, integer block dots, f32
        activations between the linears) vs the oracle with ggml's own activation quantization, within 1.5x that
        path's floor, element-wise too;
      * the product path against ggml's semantics too, within GGML_PRODUCT_K (1.75) x that floor, element-wise too."""
    from acestep_mi355x import capi
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle import ggml_numerics
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "2")
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    L = 512
    h, c, e = _inputs(T, L, seed)
    got = {}
    for mode in ("bf16", "q8"):
        monkeypatch.setenv("ACE_MI_QUANT_ACT", mode)
        br = GGMLCAPIBridge()
        br.load_dit(d)
        got[mode] = br.dit_forward_tfirst(h, c, e, None, None, 0.75, 0.75)
        br.close()
    monkeypatch.setattr(ggml_numerics, "QUANTIZER", capi.quantize)  # byte-identical C++ encoder (K-quants)
    W = DitWeights(d, qtype=qtype)
    ref, floor, fmax = forward_with_floor_stats(engine_view(W), h, c, e, None, None, T, L, 0.75, 0.75, max_layers=2)
    check(got["bf16"], ref, floor, f"{qtype} T={T} product path (dequant semantics)", fmax)
    gref, gfloor, gfmax = forward_with_floor_stats(W, h, c, e, None, None, T, L, 0.75, 0.75, max_layers=2)
    check_product_vs_ggml(got["bf16"], gref, gfloor, gfmax, f"{qtype} T={T}")
    check(got["q8"], gref, gfloor, f"{qtype} T={T} ACE_MI_QUANT_ACT=q8 (ggml semantics)", gfmax)


def test_config3_batch8_240s_every_item():
    """configs[3]'s per-GPU work at bs = 8: one batched call over 8 items of 240 s (M = 24000 rows: the
    256x256 GEMM tiles and the bs-8 attention grid), every item vs the oracle with its own timestep."""
    import torch
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle.dit_oracle import DitWeights, forward_dit, forward_with_floor_stats
    import os
    d = cached_checkpoint(make_config(num_hidden_layers=2), seed=0, backend="torch")
    os.environ["ACE_GGML_DIT_MAX_LAYERS"] = "2"
    try:
        B, T, L = 8, 6000, 512
        h, c, e = _inputs(T, L, 88, B=B)
        ts = np.linspace(1.0, 0.3, B).astype(np.float32)
        dev = torch.device("cuda:0")
        th, tc, te, tt = (torch.from_numpy(x).to(dev) for x in (h, c, e, ts))
        out = torch.empty((B, T, 64), dtype=torch.float32, device=dev)
        br = GGMLCAPIBridge()
        br.load_dit(d)
        torch.cuda.synchronize()
        br.dit_forward_batched_device(B, T, L, th.data_ptr(), tc.data_ptr(), te.data_ptr(), 0, 0, tt.data_ptr(),
                                      tt.data_ptr(), out.data_ptr(), 0)
        br.synchronize()
        got = out.cpu().numpy()
        br.close()
    finally:
        os.environ.pop("ACE_GGML_DIT_MAX_LAYERS", None)
    W = DitWeights(d)
    _, floor, fmax = forward_with_floor_stats(W, h[0], c[0], e[0], None, None, T, L, float(ts[0]), float(ts[0]),
                                              max_layers=2)
    for b in range(B):
        ref = forward_dit(W, h[b], c[b], e[b], None, None, T, L, float(ts[b]), float(ts[b]), max_layers=2)
        check(got[b], ref, floor, f"configs[3] bs=8 item {b}", fmax)


def _python_plan(T, chunk, overlap):
    """The reference tiled-decode window plan (scripts/run_non_ggml_real_case.py:597-611), restated."""
    overlap = min(overlap, max(0, chunk // 2 - 1))
    stride = chunk - 2 * overlap
    return [(cs, min(cs + stride, T), max(0, cs - overlap), min(T, cs + stride + overlap))
            for cs in range(0, T, stride)]


def test_config4_vae_decode_192_frames_windowed():
    """The full-size decoder (128 x [1,2,4,8,16] channels, hop 1920) over 192 latent frames through the
    decode hook with 128-frame windows and 32 frames of overlap (three windows of 96 / 128 / 96 frames,
    368,640 samples), vs the oracle decoding the same windows and trimming them the same way."""
    import torch
    import types
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.hook import install_vae_backend
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG
    from oracle import vae_oracle as V
    from test_gpu_vae import _ckpt
    d = _ckpt(VAE_FULL_CONFIG)
    br = GGMLCAPIBridge()
    br.load_vae(d)
    handler = types.SimpleNamespace()
    install_vae_backend(handler, br, chunk_size_default=128, overlap_default=32)
    T = 192
    lat = np.random.default_rng(19).standard_normal((1, 64, T)).astype(np.float32)
    got = handler.tiled_decode(torch.from_numpy(lat).cuda(), offload_wav_to_cpu=True).numpy()[0].T
    br.close()
    W = V.VaeWeights(d)

    def windowed():
        parts = []
        for cs, ce, ws, we in _python_plan(T, 128, 32):
            wav = V.decode(W, lat[0, :, ws:we].T)
            up = wav.shape[0] / max(1, we - ws)
            ts, te = int(round((cs - ws) * up)), int(round((we - ce) * up))
            parts.append(wav[ts:wav.shape[0] - te if te > 0 else wav.shape[0]])
        return np.concatenate(parts, axis=0)

    ref, floor, fmax = V.floor_stats(windowed)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    check(got, ref, floor, "full VAE, 192 frames windowed", fmax)


def test_config4_vae_decode_full_600s_windowed():
    """configs[4]'s whole decode: the 600 s latent (T = 15000 frames) through the installed tiled_decode hook with
    the reference C path's default plan (ACE_GGML_VAE_CHUNK_FRAMES 128, overlap 32: acestep_ggml.cpp:2114-2151)
    -- 235 windows.  Exact length (the hook's plan length and T x hop), finite everywhere, and three interior
    windows (first, middle, last) equal the oracle decoding the same window frames, trimmed the same way."""
    import torch
    import types
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.hook import install_vae_backend, tiled_out_len
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG
    from oracle import vae_oracle as V
    from test_gpu_vae import _ckpt
    d = _ckpt(VAE_FULL_CONFIG)
    br = GGMLCAPIBridge()
    br.load_vae(d)
    handler = types.SimpleNamespace()
    install_vae_backend(handler, br, chunk_size_default=128, overlap_default=32)
    T = 15000
    lat = np.random.default_rng(600).standard_normal((1, 64, T)).astype(np.float32)
    got = handler.tiled_decode(torch.from_numpy(lat).cuda(), offload_wav_to_cpu=True).numpy()[0].T  # [samples, ch]
    n_expect = tiled_out_len(br, T, 128, 32)
    hop = br.vae_out_len(1)
    br.close()
    assert got.shape == (n_expect, 2), (got.shape, n_expect)
    assert n_expect == T * hop, (n_expect, T, hop)
    assert np.isfinite(got).all()
    W = V.VaeWeights(d)
    plan = _python_plan(T, 128, 32)
    offs = np.cumsum([0] + [(ce - cs) * hop for cs, ce, _, _ in plan])

    def window(idx):
        cs, ce, ws, we = plan[idx]
        wav = V.decode(W, lat[0, :, ws:we].T)
        up = wav.shape[0] / max(1, we - ws)
        ts, te = int(round((cs - ws) * up)), int(round((we - ce) * up))
        return wav[ts:wav.shape[0] - te if te > 0 else wav.shape[0]]

    for idx in (0, len(plan) // 2, len(plan) - 1):
        ref, floor, fmax = V.floor_stats(lambda: window(idx))
        seg = got[offs[idx]:offs[idx + 1]]
        assert seg.shape == ref.shape, (idx, seg.shape, ref.shape)
        check(seg, ref, floor, f"600 s VAE decode, window {idx} of {len(plan)}", fmax)
