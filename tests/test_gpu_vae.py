"""GPU parity of the Oobleck VAE decoder (ace_ggml_vae_decode and the device entry) against the
oracle restatement of ace_vae::forward_decode (oracle/vae_oracle.py).

Tolerance: every conv re-rounds its input to fp16 (ggml im2col), so any f32 difference (summation
order, a 1-ulp sinf) can flip an fp16 rounding and propagate; the bound is
max(1e-3, FLOOR_K * floor), floor = the oracle's own rel-L2 change when every conv result element is
perturbed by independent 1e-7 relative noise (vae_oracle.floor_stats, as the DiT oracle's floor); the
full-size decodes also assert the element-wise max|gpu - ref| / rms(ref) <= MAXABS_K x the oracle's own
spread of that statistic (test_gpu_forward.check), which a wrong conv output tile fails even where the L2
absorbs it (test_vae_fault_injection_is_caught)."""
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_L2 = 1e-3
FLOOR_K = 1.5


def _ckpt(cfg):
    from acestep_mi355x.synthetic import write_vae_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_vae_")
    write_vae_checkpoint(d, cfg, seed=0)
    return d


@pytest.fixture(scope="module")
def tiny_vae():
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG
    d = _ckpt(VAE_TINY_CONFIG)
    br = GGMLCAPIBridge()
    br.load_vae(d)
    yield d, br
    br.close()


def _check(got, ref, floor, tag, floor_max=None):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    if floor_max is not None:  # rel-L2 and the element-wise bound (test_gpu_forward.check)
        from test_gpu_forward import check
        return check(got, ref, floor, tag, floor_max)
    l2 = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    bound = max(REL_L2, FLOOR_K * floor)
    print(f"{tag}: rel_l2={l2:.3e} floor={floor:.3e} bound={bound:.3e} max_abs={np.abs(got - ref).max():.3e}")
    assert np.isfinite(l2) and l2 <= bound, (tag, l2, floor)
    return l2


@pytest.mark.parametrize("T", [1, 20, 37])
def test_tiny_vae_decode_odd_stride(tiny_vae, T):
    from oracle.vae_oracle import VaeWeights, decode_with_floor
    d, br = tiny_vae
    assert (br.latent_channels, br.audio_channels, br.hop_length) == (64, 2, 6)
    lat = np.random.default_rng(T).standard_normal((T, 64)).astype(np.float32)
    ref, floor = decode_with_floor(VaeWeights(d), lat)
    n = br.vae_out_len(T)
    assert n == ref.shape[0]
    got = br.vae_decode_tfirst(lat)           # [T*hop, 2]; odd strides fill only the first n samples
    _check(got[:n], ref, floor, f"tiny VAE T={T}")


def test_vae_error_paths(tiny_vae):
    import ctypes
    from acestep_mi355x.capi import GGMLCAPIBridge
    d, br = tiny_vae
    lat = np.zeros((10, 64), np.float32)
    out = np.zeros((10 * 6 - 1, 2), np.float32)
    fp = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert br.lib.ace_ggml_vae_decode(br.ctx, fp(lat), 10, fp(out), out.nbytes) == 2
    assert br._last_error() == "output buffer too small"
    assert br.lib.ace_ggml_vae_decode(br.ctx, None, 10, fp(out), out.nbytes) == 2
    assert br.lib.ace_ggml_vae_decode(br.ctx, fp(lat), 0, fp(out), out.nbytes) == 2
    fresh = GGMLCAPIBridge()
    assert fresh.lib.ace_ggml_vae_decode(fresh.ctx, fp(lat), 10, fp(out), out.nbytes) == 1
    assert fresh._last_error() == "vae not loaded"
    assert fresh.lib.ace_ggml_vae_get_info(fresh.ctx, None, None, None) == 1
    assert fresh.lib.ace_ggml_load_vae(fresh.ctx, b"/nonexistent/vae") == 3
    fresh.close()


def test_device_entry_equals_host_entry(tiny_vae):
    import torch
    d, br = tiny_vae
    lat = np.random.default_rng(9).standard_normal((33, 64)).astype(np.float32)
    host = br.vae_decode_tfirst(lat)
    n = br.vae_out_len(33)
    dl = torch.from_numpy(lat).cuda()
    out = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    br.vae_decode_device(dl.data_ptr(), 33, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), host[:n])


def test_tiled_decode_hook_matches_windowed_oracle(tiny_vae):
    """install_vae_backend: dit_handler.tiled_decode on ROCm tensors, reference window plan."""
    import types
    import torch
    from acestep_mi355x.hook import _tile_plan, install_vae_backend
    from oracle.vae_oracle import VaeWeights, decode
    d, br = tiny_vae
    handler = types.SimpleNamespace()
    install_vae_backend(handler, br, chunk_size_default=16, overlap_default=4)
    B, T = 2, 40
    lat = np.random.default_rng(5).standard_normal((B, 64, T)).astype(np.float32)
    got = handler.tiled_decode(torch.from_numpy(lat).cuda(), offload_wav_to_cpu=True).numpy()
    W = VaeWeights(d)
    for b in range(B):
        parts = []
        for cs, ce, ws, we in _tile_plan(T, 16, 4):
            wav = decode(W, lat[b, :, ws:we].T)
            up = wav.shape[0] / max(1, we - ws)
            ts, te = int(round((cs - ws) * up)), int(round((we - ce) * up))
            parts.append(wav[ts:wav.shape[0] - te if te > 0 else wav.shape[0]])
        ref = np.concatenate(parts, axis=0).T
        assert got[b].shape == ref.shape
        l2 = np.linalg.norm(got[b] - ref) / np.linalg.norm(ref)
        print(f"tiled hook b={b}: rel_l2={l2:.3e}")
        assert l2 < 5e-3


@pytest.mark.parametrize("T", [37, 61])
def test_halo_staged_residual_convs_equal_generic(tiny_vae, T, monkeypatch):
    """The 128-channel residual units' k7 convs with the halo-staged A operand (default) give the same bits as
    the generic per-k-tile staging (ACE_MI_VAE_HALO=0): same products, same k order.  Odd T: ragged tiles at
    every stage.  Decode and encode (the encoder's 128-channel units run the unfused k7 conv)."""
    d, br = tiny_vae
    lat = np.random.default_rng(100 + T).standard_normal((T, 64)).astype(np.float32)
    audio = np.random.default_rng(200 + T).standard_normal((T * 6, 2)).astype(np.float32)
    n = br.vae_out_len(T)  # (the samples past n of the [T*hop] host buffer are not written)
    halo = br.vae_decode_tfirst(lat)[:n], br.vae_encode_tfirst(audio)
    monkeypatch.setenv("ACE_MI_VAE_HALO", "0")
    generic = br.vae_decode_tfirst(lat)[:n], br.vae_encode_tfirst(audio)
    for i, what in enumerate(("decode", "encode")):
        d = np.abs(halo[i].astype(np.float64) - generic[i])
        print(f"halo vs generic {what} T={T}: {int((d > 0).sum())} of {d.size} differ, max {d.max():.3e}")
        np.testing.assert_array_equal(halo[i], generic[i])


@pytest.mark.slow
@pytest.mark.parametrize("T", [6, 5])
def test_full_size_vae_decode(T):
    """The real ACE-Step 1.5 decoder shape (128 x [1,2,4,8,16] channels, strides 10,6,4,4,2,
    hop 1920) on 6 / 5 latent frames (11520 / 9600 samples; 5: ragged 128-row tiles in the 128-channel blocks),
    rel-L2 and element-wise against the oracle's noise floor."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG
    from oracle.vae_oracle import VaeWeights, decode_with_floor_stats
    d = _ckpt(VAE_FULL_CONFIG)
    br = GGMLCAPIBridge()
    br.load_vae(d)
    lat = np.random.default_rng(11).standard_normal((T, 64)).astype(np.float32)
    got = br.vae_decode_tfirst(lat)
    br.close()
    ref, floor, fmax = decode_with_floor_stats(VaeWeights(d), lat)
    _check(got, ref, floor, f"full VAE T={T}", fmax)


# one corrupted tile: 16 samples x 128 channels of the residual stream after block 3's first residual unit
# (the 128 x 2-channel block, 4800 rows at T = 5 frames), restated in the oracle as vae_oracle.FAULT
VAE_FAULT = (3, 2000, 0, 0.02)


def test_vae_fault_injection_is_caught(monkeypatch):
    """Negative control: a wrong conv output tile inside the decoder passes the rel-L2 bound but fails the element-wise
    bound; the faulted GPU output equals the oracle with the same fault restated (so the failure is the fault's)."""
    from acestep_mi355x.capi import GGMLCAPIBridge, selftest_library_path
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG
    from oracle import vae_oracle as V
    from test_gpu_forward import FLOOR_K as FK, MAXABS_K, check, maxabs_rms, rel_errors
    d = _ckpt(VAE_FULL_CONFIG)
    lat = np.random.default_rng(11).standard_normal((5, 64)).astype(np.float32)
    W = V.VaeWeights(d)
    ref, floor, fmax = V.decode_with_floor_stats(W, lat)
    monkeypatch.setenv("ACE_MI_TEST_VAE_FAULT", ",".join(str(v) for v in VAE_FAULT))
    br = GGMLCAPIBridge(lib_path=selftest_library_path())  # the fault hook is read by the self-test library only
    try:
        br.load_vae(d)
        bad = br.vae_decode_tfirst(lat)
    finally:
        br.close()
    l2, _ = rel_errors(bad, ref)
    ma = maxabs_rms(bad, ref)
    print(f"VAE faulted: rel_l2={l2:.3e} (bound {max(REL_L2, FK * floor):.3e}) maxabs/rms={ma:.3e} "
          f"(bound {MAXABS_K * fmax:.3e}, ratio {ma / fmax:.2f})")
    assert l2 <= max(REL_L2, FK * floor), "the L2 bound alone would have caught it: raise the control's subtlety"
    with pytest.raises(AssertionError):
        check(bad, ref, floor, "VAE negative control: faulted run", fmax)
    V.FAULT = VAE_FAULT
    try:
        fref = V.decode(W, lat)
    finally:
        V.FAULT = None
    check(bad, fref, floor, "VAE faulted GPU vs faulted oracle", fmax)


@pytest.mark.parametrize("n", [120, 126, 600])
def test_tiny_vae_encode(tiny_vae, n):
    """ace_ggml_vae_encode: encoder convs incl. the strided downsampling convs (the first conv's
    2 audio channels zero-padded to 64 for the GEMM) vs the oracle."""
    from oracle.vae_oracle import VaeWeights, encode
    import oracle.vae_oracle as V
    d, br = tiny_vae
    audio = np.random.default_rng(n).standard_normal((n, 2)).astype(np.float32)
    W = VaeWeights(d)
    ref = encode(W, audio)
    _, floor, _ = V.floor_stats(lambda: encode(W, audio))
    assert br.vae_enc_out_len(n) == ref.shape[0]
    got = br.vae_encode_tfirst(audio)
    _check(got[:ref.shape[0]], ref, floor, f"tiny VAE encode n={n}")
