"""The product's host code (runtime/*.cpp: ABI, loaders, engine orchestration) linked against a host
emulation of the kernels (tests/host/kernel_emul.cpp, each launch_* restated as plain loops on
host memory) and driven through the same ctypes bridge as the GPU tests.  This checks on the CPU
that every buffer, offset and launch argument of the DiT forward, the quantized and GGUF weight
paths, the batched/sampler entries and the VAE decode/encode is wired as the oracle's graph says;
the kernels themselves are checked by the -m gpu tests."""
import os
import shutil
import tempfile

import numpy as np
import pytest

from hostlib import CLANG, build_host_lib


@pytest.fixture(scope="module")
def host_lib():
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    return build_host_lib()


@pytest.fixture(scope="module")
def tiny_ckpt():
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_he_")
    write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
    return d


def bridge(lib):
    from acestep_mi355x.capi import GGMLCAPIBridge
    return GGMLCAPIBridge(lib_path=lib)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def engine_view(W):
    from test_gpu_quant import engine_view as ev
    return ev(W)


def inputs(seed, T, L, H=256):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((T, 64)).astype(np.float32), rng.standard_normal((T, 128)).astype(np.float32),
            rng.standard_normal((L, H)).astype(np.float32))


def test_dit_forward_bf16_with_masks(host_lib, tiny_ckpt):
    from oracle.dit_oracle import DitWeights, forward_with_floor
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    h, c, e = inputs(3, 77, 13)
    mask = np.ones(77, np.int32)
    mask[70:] = 0
    emask = np.ones(13, np.int32)
    emask[10:] = 0
    got = br.dit_forward_tfirst(h, c, e, mask, emask, 0.8, 0.3)
    ref, floor = forward_with_floor(DitWeights(tiny_ckpt), h, c, e, mask, emask, 77, 13, 0.8, 0.3)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    br.close()


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
def test_dit_forward_online_quantized(host_lib, tiny_ckpt, monkeypatch, qtype):
    from oracle.dit_oracle import DitWeights, forward_with_floor
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    h, c, e = inputs(5, 64, 9)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.6, 0.6)
    ref, floor = forward_with_floor(engine_view(DitWeights(tiny_ckpt, qtype=qtype)), h, c, e, None, None, 64, 9,
                                    0.6, 0.6)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    br.close()


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
def test_dit_forward_quant_act_ggml_semantics(host_lib, tiny_ckpt, monkeypatch, qtype):
    """ACE_MI_QUANT_ACT=q8 (DitEngine::forward_qact): f32 activations quantized to Q8_0 / Q8_K blocks before every
    quantized linear, against the oracle's ggml semantics (no engine_view) -- the orchestration of the mode, with
    the host restatement of its kernels; the sampler entry's precomputed timestep rows take the same path."""
    from oracle.dit_oracle import DitWeights, forward_with_floor
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    monkeypatch.setenv("ACE_MI_QUANT_ACT", "q8")
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    h, c, e = inputs(9, 70, 11)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.7, 0.4)
    ref, floor = forward_with_floor(DitWeights(tiny_ckpt, qtype=qtype), h, c, e, None, None, 70, 11, 0.7, 0.4)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    dq, dq_floor = forward_with_floor(engine_view(DitWeights(tiny_ckpt, qtype=qtype)), h, c, e, None, None, 70, 11,
                                      0.7, 0.4)
    assert rel(got, dq) > rel(got, ref), "the mode should sit closer to ggml's arithmetic than to bf16 activations"
    br.close()


@pytest.mark.parametrize("quant", ["Q8", "Q4", "F16"])
def test_dit_forward_gguf(host_lib, tiny_ckpt, quant):
    from acestep_mi355x.synthetic import write_gguf
    from oracle.dit_oracle import DitWeights, forward_with_floor
    d = tempfile.mkdtemp(prefix="acemi_heg_")
    shutil.copy(os.path.join(tiny_ckpt, "config.json"), d)
    path = write_gguf(os.path.join(tiny_ckpt, "model.safetensors"), os.path.join(d, "model.gguf"), quant=quant)
    br = bridge(host_lib)
    br.load_dit(d)
    h, c, e = inputs(7, 50, 6)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.5, 0.5)
    ref, floor = forward_with_floor(engine_view(DitWeights(d, gguf=path)), h, c, e, None, None, 50, 6, 0.5, 0.5)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    br.close()


def test_batched_entry_and_sampler_wiring(host_lib, tiny_ckpt):
    """ace_mi_dit_forward_batched / ace_mi_dit_sample on "device" pointers (host memory here)."""
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    B, T, L = 3, 40, 7
    rng = np.random.default_rng(11)
    h = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    t = np.array([0.9, 0.5, 0.2], np.float32)
    out = np.empty((B, T, 64), np.float32)
    p = lambda a: a.ctypes.data
    br.dit_forward_batched_device(B, T, L, p(h), p(c), p(e), 0, 0, p(t), p(t), p(out), 0)
    for b in range(B):
        ser = br.dit_forward_tfirst(h[b], c[b], e[b], None, None, float(t[b]), float(t[b]))
        np.testing.assert_array_equal(out[b], ser)
    # device sampler == host Euler loop
    sched = [1.0, 0.75, 0.5, 0.25]
    xt = h.copy()
    br.dit_sample_device(B, T, L, p(xt), p(c), p(e), 0, 0, sched, 0)
    ref = h.copy()
    for i, ti in enumerate(sched):
        for b in range(B):
            v = br.dit_forward_tfirst(ref[b], c[b], e[b], None, None, ti, ti)
            dt = ti if i + 1 == len(sched) else ti - sched[i + 1]
            ref[b] = ref[b] - v * np.float32(dt)
    np.testing.assert_allclose(xt, ref, rtol=1e-5, atol=1e-5)
    br.close()


def test_vae_decode_encode(host_lib):
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    from oracle.vae_oracle import VaeWeights, decode, decode_with_floor, encode
    d = tempfile.mkdtemp(prefix="acemi_hev_")
    write_vae_checkpoint(d, VAE_TINY_CONFIG, seed=1)
    br = bridge(host_lib)
    br.load_vae(d)
    W = VaeWeights(d)
    lat = np.random.default_rng(2).standard_normal((21, 64)).astype(np.float32)
    ref, floor = decode_with_floor(W, lat)
    n = br.vae_out_len(21)
    got = br.vae_decode_tfirst(lat)[:n]
    assert got.shape == ref.shape and rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    audio = np.random.default_rng(3).standard_normal((126, 2)).astype(np.float32)
    z = br.vae_encode_tfirst(audio)
    zr = encode(W, audio)
    assert z.shape == zr.shape and rel(z, zr) < 2e-3, rel(z, zr)
    br.close()


def test_abi_error_paths(host_lib, tiny_ckpt):
    import ctypes
    br = bridge(host_lib)
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    out = np.zeros((10, 64), np.float32)
    assert br.lib.ace_ggml_dit_forward(br.ctx, None, None, None, None, None, 10, 0, 0.5, 0.5, fp(out), out.nbytes) == 1
    assert br._last_error() == "dit not loaded"
    assert br.lib.ace_ggml_load_dit(br.ctx, b"/nonexistent") == 3
    br.load_dit(tiny_ckpt)
    assert br.lib.ace_ggml_dit_forward(br.ctx, None, None, None, None, None, 10, 0, 0.5, 0.5, fp(out),
                                       out.nbytes - 4) == 2
    assert br._last_error() == "output buffer too small"
    assert br.lib.ace_ggml_dit_forward(br.ctx, None, None, None, None, None, 0, 0, 0.5, 0.5, fp(out), out.nbytes) == 2
    # enc_len > 0 without encoder states
    assert br.lib.ace_ggml_dit_forward(br.ctx, None, None, None, None, None, 10, 4, 0.5, 0.5, fp(out), out.nbytes) == 1
    br.close()


def test_generation_loop_ex_ode_sde_cover_and_cross_cache(host_lib, tiny_ckpt):
    """ace_mi_dit_sample_ex == the reference loop of acestep/mlx_dit/generate.py:143-199 restated with
    per-step forwards: ODE with the cross-attention cache, SDE with caller noise, and the cover switch."""
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    B, T, L = 2, 30, 5
    rng = np.random.default_rng(21)
    x0 = rng.standard_normal((B, T, 64)).astype(np.float32)
    c = rng.standard_normal((B, T, 128)).astype(np.float32)
    e = rng.standard_normal((B, L, 256)).astype(np.float32)
    c_nc = rng.standard_normal((B, T, 128)).astype(np.float32)
    e_nc = rng.standard_normal((B, L, 256)).astype(np.float32)
    sched = [1.0, 0.9, 0.75, 0.5, 0.3]
    noise = rng.standard_normal((len(sched) - 1, B, T, 64)).astype(np.float32)
    p = lambda a: a.ctypes.data

    def ref_loop(sde, cover):
        xt = x0.copy()
        for i, t in enumerate(sched):
            cc, ee = (c_nc, e_nc) if (cover is not None and i >= cover) else (c, e)
            v = np.stack([br.dit_forward_tfirst(xt[b], cc[b], ee[b], None, None, t, t) for b in range(B)])
            if i + 1 == len(sched):
                xt = xt - v * np.float32(t)
            elif sde:
                xc = xt - v * np.float32(t)
                tn = np.float32(sched[i + 1])
                xt = tn * noise[i] + (np.float32(1.0) - tn) * xc
            else:
                xt = xt - v * (np.float32(t) - np.float32(sched[i + 1]))  # the library's f32 dt
        return xt

    for sde, cover, cache in ((False, None, True), (True, None, True), (False, 2, True), (True, 3, False)):
        xt = x0.copy()
        br.dit_sample_ex_device(B, T, L, p(xt), p(c), p(e), 0, 0, sched, sde=sde, d_noise=p(noise),
                                cover_steps=-1 if cover is None else cover,
                                d_context_nc=p(c_nc) if cover is not None else 0,
                                d_enc_nc=p(e_nc) if cover is not None else 0, cache_cross=cache)
        np.testing.assert_allclose(xt, ref_loop(sde, cover), rtol=1e-5, atol=1e-5, err_msg=str((sde, cover, cache)))
    br.close()


# ---------------------------------------------------------------- condition encoders
@pytest.fixture(scope="module")
def cond_ckpt():
    from acestep_mi355x.synthetic import TINY_COND_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_hec_")
    write_checkpoint(d, TINY_COND_CONFIG, seed=4, dtype="BF16")
    return d


def test_condition_encoders(host_lib, cond_ckpt):
    """Lyric encoder, batched timbre encoder, text projector and the packed encoder_hidden_states of
    ace_mi_build_condition against oracle/cond_oracle.py."""
    from oracle import cond_oracle as co
    from oracle.dit_oracle import DitWeights
    W = DitWeights(cond_ckpt)
    br = bridge(host_lib)
    br.load_dit(cond_ckpt)
    info = br.cond_info()
    assert (info.hidden_size, info.lyric_in_dim, info.timbre_in_dim, info.text_projector_in) == (256, 256, 64, 256)
    assert (info.lyric_layers, info.timbre_layers, info.has_lyric_encoder, info.has_timbre_encoder) == (2, 2, 1, 1)
    rng = np.random.default_rng(8)
    lyr = rng.standard_normal((45, 256)).astype(np.float32)
    ref, floor = co.encode_with_floor(co.forward_lyric_encoder, W, lyr)
    got = br.lyric_encode(lyr)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    refer = rng.standard_normal((3, 20, 64)).astype(np.float32)
    tim = br.timbre_encode(refer)
    for i in range(3):
        r, f = co.encode_with_floor(co.forward_timbre_encoder, W, refer[i])
        assert rel(tim[i], r) <= max(1e-3, 1.5 * f), (i, rel(tim[i], r), f)
    sty = rng.standard_normal((17, 256)).astype(np.float32)
    np.testing.assert_allclose(br.text_project(sty), co.project_tokens_linear(W, sty), rtol=1e-5, atol=1e-6)
    enc, mask = br.build_condition(sty, lyr, refer)
    eref, mref = co.build_condition(W, sty, lyr, refer, text_hidden=256)
    assert enc.shape == (45 + 3 + 17, 256) and np.array_equal(mask, mref)
    assert rel(enc, eref) <= max(1e-3, 1.5 * floor), rel(enc, eref)
    br.close()


def test_condition_encoder_layer_cap_and_fallbacks(host_lib, cond_ckpt, tiny_ckpt, monkeypatch):
    from oracle import cond_oracle as co
    from oracle.dit_oracle import DitWeights
    W = DitWeights(cond_ckpt)
    rng = np.random.default_rng(9)
    lyr = rng.standard_normal((30, 256)).astype(np.float32)
    monkeypatch.setenv("ACE_GGML_LYRIC_MAX_LAYERS", "1")
    br = bridge(host_lib)
    br.load_dit(cond_ckpt)
    ref, floor = co.encode_with_floor(co.forward_lyric_encoder, W, lyr, max_layers=1)
    got = br.lyric_encode(lyr)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor)
    # order mask: multi-batch references are not supported (acestep_ggml.cpp:1832-1834)
    import ctypes
    refer = rng.standard_normal((2, 9, 64)).astype(np.float32)
    with pytest.raises(RuntimeError, match="multi-batch refer_audio_order_mask is not supported"):
        br.timbre_encode(refer, order_mask=np.array([0, 1], np.int32))
    # lyric width != lyric encoder input: the copy fallback, widened to H (zero padded)
    lyr2 = rng.standard_normal((6, 96)).astype(np.float32)
    monkeypatch.setenv("ACE_GGML_ALLOW_TEXT_DIM_MISMATCH", "1")
    enc, mask = br.build_condition(lyric_embeds=lyr2)
    eref, _ = co.build_condition(W, lyric_embeds=lyr2, text_hidden=96, allow_text_mismatch=True)
    np.testing.assert_array_equal(enc, eref)
    monkeypatch.delenv("ACE_GGML_ALLOW_TEXT_DIM_MISMATCH")
    with pytest.raises(RuntimeError, match="text encoder hidden size mismatch with dit"):
        br.build_condition(lyric_embeds=lyr2)
    br.close()
    # a DiT checkpoint without encoder tensors
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    assert br.cond_info().has_timbre_encoder == 0
    with pytest.raises(RuntimeError, match="forward_lyric_encoder failed"):
        br.lyric_encode(lyr)
    with pytest.raises(RuntimeError, match="timbre encoder weights are not loaded"):
        br.timbre_encode(refer)
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    out = np.zeros((30, 256), np.float32)
    assert br.lib.ace_mi_text_project(br.ctx, fp(lyr), 30, 256, fp(out), out.nbytes) == 2
    br.close()


# ---------------------------------------------------------------- Qwen3 text encoder
@pytest.fixture(scope="module")
def text_ckpt():
    from acestep_mi355x.synthetic import TEXT_TINY_CONFIG, text_tensor_specs, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_het_")
    write_checkpoint(d, TEXT_TINY_CONFIG, seed=6, dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    return d


@pytest.mark.parametrize("qtype", [None, "q8_0"])
def test_text_encoder_forward_entries(host_lib, text_ckpt, monkeypatch, qtype):
    """ace_ggml_text_encoder_forward / _masked / _layers / _embeddings vs oracle/text_oracle.py
    (causal attention, key mask, layer cap with and without the final norm)."""
    from oracle import text_oracle as to
    if qtype:
        monkeypatch.setenv("ACE_GGML_QWEN_WEIGHT_QTYPE", qtype)
    br = bridge(host_lib)
    br.load_text_encoder(text_ckpt)
    W = to.TextWeights(text_ckpt, qtype=qtype)
    if qtype:
        W = engine_view(W)
    rng = np.random.default_rng(12)
    ids = rng.integers(0, 1000, 37).astype(np.int32)
    np.testing.assert_array_equal(br.text_encoder_embeddings(ids), to.forward_text_encoder_embeddings(W, ids))
    ref, floor = to.forward_with_floor(W, ids)
    got = br.text_encoder_forward(ids)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    mask = np.ones(37, np.int32)
    mask[30:] = 0
    ref, floor = to.forward_with_floor(W, ids, mask)
    assert rel(br.text_encoder_forward(ids, mask), ref) <= max(1e-3, 1.5 * floor)
    ref, floor = to.forward_with_floor(W, ids, None, 1, True)   # capped: no final norm
    assert rel(br.text_encoder_forward(ids, None, n_layers=1), ref) <= max(1e-3, 1.5 * floor)
    br.close()


def test_text_encoder_causality_and_errors(host_lib, text_ckpt):
    import ctypes
    br = bridge(host_lib)
    out = np.zeros((4, 256), np.float32)
    ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    ids = np.array([1, 2, 3, 4], np.int32)
    assert br.lib.ace_ggml_text_encoder_forward(br.ctx, ip(ids), 4, fp(out), out.nbytes) == 1
    assert br._last_error() == "text encoder not loaded"
    assert br.lib.ace_ggml_load_text_encoder(br.ctx, b"/nonexistent") == 3
    br.load_text_encoder(text_ckpt)
    assert br.lib.ace_ggml_text_encoder_forward(br.ctx, ip(ids), 4, fp(out), out.nbytes - 4) == 2
    assert br._last_error() == "output buffer too small"
    assert br.lib.ace_ggml_text_encoder_forward(br.ctx, ip(ids), 0, fp(out), out.nbytes) == 2
    bad = np.array([1, 2, 1000, 4], np.int32)
    assert br.lib.ace_ggml_text_encoder_forward(br.ctx, ip(bad), 4, fp(out), out.nbytes) == 2
    assert br._last_error() == "token id out of range"
    # causal: a prefix's states do not depend on later tokens
    rng = np.random.default_rng(13)
    a = rng.integers(0, 1000, 20).astype(np.int32)
    b = a.copy()
    b[15:] = rng.integers(0, 1000, 5)
    np.testing.assert_array_equal(br.text_encoder_forward(a)[:15], br.text_encoder_forward(b)[:15])
    br.close()


# ---------------------------------------------------------------- end-to-end generate entries
def test_generate_entries_end_to_end(host_lib, cond_ckpt, text_ckpt):
    """ace_ggml_generate_audio_simple / _style_lyric_simple / _style_lyric_timbre_simple (text encoder ->
    condition -> silence context -> 8-step Euler loop -> windowed VAE decode) vs oracle/pipeline_oracle.py."""
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    from oracle import pipeline_oracle as po
    from oracle.dit_oracle import DitWeights
    from oracle.text_oracle import TextWeights
    from oracle.vae_oracle import VaeWeights
    vd = tempfile.mkdtemp(prefix="acemi_hegv_")
    write_vae_checkpoint(vd, VAE_TINY_CONFIG, seed=1)
    br = bridge(host_lib)
    br.load_dit(cond_ckpt)
    br.load_vae(vd)
    br.load_text_encoder(text_ckpt)
    DW, VW, TW = DitWeights(cond_ckpt), VaeWeights(vd), TextWeights(text_ckpt)
    rng = np.random.default_rng(14)
    style, lyric = rng.integers(0, 1000, 9), rng.integers(0, 1000, 12)
    refer = rng.standard_normal((1, 10, 64)).astype(np.float32)
    hop = br.hop_length
    cases = [dict(token_ids=style), dict(style_ids=style, lyric_ids=lyric),
             dict(style_ids=style, lyric_ids=lyric, refer=refer)]
    for i, kw in enumerate(cases):
        # > 128: chunked silence encode + windowed decode (300: three equal 128-frame windows decoded
        # as one batch, then the 96- and 76-frame edge windows)
        seq_len = 300 if i == 2 else 30
        got = br.generate_audio(seq_len, shift=3.0, seed=11 + i, **kw)
        if "token_ids" in kw:
            enc = po.forward_text_encoder_layers_for_simple(TW, style)
            ref, _ = po.generate_from_encoder(DW, VW, enc, np.ones(len(enc), np.int32), seq_len, 3.0, 11 + i, hop, 2)
        else:
            ref, _ = po.generate_style_lyric_timbre(DW, VW, TW, kw.get("style_ids"), kw.get("lyric_ids"),
                                                    kw.get("refer"), seq_len, 3.0, 11 + i, hop, 2)
        if seq_len <= 128:  # one decode; tiny VAE strides (2, 3) make it <= seq_len * hop samples, rest zero
            assert got.shape == (seq_len * hop, 2) and len(ref) <= seq_len * hop, (got.shape, ref.shape)
            assert not got[len(ref):].any()
        else:               # windowed: as many samples as the trimmed windows hold
            assert got.shape == ref.shape, (got.shape, ref.shape)
        assert rel(got[:len(ref)], ref) < 2e-2, (i, rel(got[:len(ref)], ref))
    br.close()


@pytest.mark.parametrize("quant", ["Q4", "F16"])
def test_text_encoder_gguf(host_lib, text_ckpt, quant):
    """model.gguf next to config.json (resolve_gguf_path, qwen_model.cpp:46-72): types kept, a
    quantized embed_tokens table dequantized for get_rows."""
    from acestep_mi355x.synthetic import write_gguf
    from oracle import text_oracle as to
    d = tempfile.mkdtemp(prefix="acemi_hetg_")
    shutil.copy(os.path.join(text_ckpt, "config.json"), d)
    path = write_gguf(os.path.join(text_ckpt, "model.safetensors"), os.path.join(d, "model.gguf"), quant=quant,
                      arch="qwen3")
    br = bridge(host_lib)
    br.load_text_encoder(d)
    W = engine_view(to.TextWeights(d, gguf=path))
    ids = np.random.default_rng(15).integers(0, 1000, 25).astype(np.int32)
    np.testing.assert_array_equal(br.text_encoder_embeddings(ids), to.forward_text_encoder_embeddings(W, ids))
    ref, floor = to.forward_with_floor(W, ids)
    assert rel(br.text_encoder_forward(ids), ref) <= max(1e-3, 1.5 * floor)
    br.close()


def test_generate_context_options(host_lib, cond_ckpt, text_ckpt, monkeypatch):
    """ACE_GGML_SILENCE_LATENT_F32 (frames past the file repeat its last frame) and
    ACE_GGML_USE_SILENCE_CONTEXT=0 (zero context) reach the sampler as the reference builds them."""
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    from oracle import pipeline_oracle as po
    from oracle.dit_oracle import DitWeights, forward_dit
    from oracle.text_oracle import TextWeights
    from oracle.vae_oracle import VaeWeights, decode
    vd = tempfile.mkdtemp(prefix="acemi_hegc_")
    write_vae_checkpoint(vd, VAE_TINY_CONFIG, seed=1)
    br = bridge(host_lib)
    br.load_dit(cond_ckpt)
    br.load_vae(vd)
    br.load_text_encoder(text_ckpt)
    DW, VW, TW = DitWeights(cond_ckpt), VaeWeights(vd), TextWeights(text_ckpt)
    ids = np.random.default_rng(16).integers(0, 1000, 6)
    enc = po.forward_text_encoder_layers_for_simple(TW, ids)
    seq_len = 20
    sil = np.random.default_rng(17).standard_normal((7, 64)).astype(np.float32)
    f = os.path.join(vd, "silence.f32")
    sil.tofile(f)

    def run_oracle(ctx):
        xt = po.reference_noise(5, seq_len * 64).reshape(seq_len, 64)
        sched = po.shift_schedule(1.0)
        for i, t in enumerate(sched):
            v = forward_dit(DW, xt, ctx, enc, None, np.ones(len(enc), np.int32), seq_len, len(enc), t, t)
            xt = (xt - v * (t if i + 1 == len(sched) else np.float32(t - sched[i + 1]))).astype(np.float32)
        return decode(VW, xt)

    monkeypatch.setenv("ACE_GGML_SILENCE_LATENT_F32", f)
    got = br.generate_audio(seq_len, shift=1.0, seed=5, token_ids=ids)
    ctx = np.ones((seq_len, 128), np.float32)
    ctx[:, :64] = sil[np.minimum(np.arange(seq_len), 6)]
    ref = run_oracle(ctx)
    assert rel(got[:len(ref)], ref) < 2e-2
    monkeypatch.setenv("ACE_GGML_USE_SILENCE_CONTEXT", "0")
    got = br.generate_audio(seq_len, shift=1.0, seed=5, token_ids=ids)
    ref = run_oracle(np.zeros((seq_len, 128), np.float32))
    assert rel(got[:len(ref)], ref) < 2e-2
    br.close()


def test_dit_forward_layer_cap_with_fused_cross_kv(host_lib, tiny_ckpt, monkeypatch):
    """ACE_GGML_DIT_MAX_LAYERS=1: the fused cross-k|v GEMM covers only the first layer's rows (ld of the
    k|v buffer = n_layers * 2kd), then the cache is reused by a full-depth forward of the sampler."""
    from oracle.dit_oracle import DitWeights, forward_with_floor
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", "1")
    br = bridge(host_lib)
    br.load_dit(tiny_ckpt)
    h, c, e = inputs(19, 40, 11)
    got = br.dit_forward_tfirst(h, c, e, None, None, 0.9, 0.9)
    ref, floor = forward_with_floor(DitWeights(tiny_ckpt), h, c, e, None, None, 40, 11, 0.9, 0.9, max_layers=1)
    assert rel(got, ref) <= max(1e-3, 1.5 * floor), (rel(got, ref), floor)
    br.close()


def test_eval_quant_tool_on_tiny_models(host_lib, cond_ckpt, text_ckpt):
    """tools/eval_quant.py (the reference's FP-vs-quantized acceptance metrics) end to end on the tiny
    models: identical FP runs give zero error, Q8_0 stays close, Q4_K further away."""
    import importlib.util
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    spec = importlib.util.spec_from_file_location("eval_quant", os.path.join(os.path.dirname(__file__), "..", "tools",
                                                                             "eval_quant.py"))
    eq = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(eq)
    vd = tempfile.mkdtemp(prefix="acemi_heq_")
    write_vae_checkpoint(vd, VAE_TINY_CONFIG, seed=1)
    rows = eq.run(cond_ckpt, vd, text_ckpt, 0.8, ["q8_0", "q4_k"], style_tokens=5, lyric_tokens=7, lib=host_lib,
                  vocab=1000)
    r8, r4 = rows[1], rows[2]
    assert r8["cosine"] > 0.99 and r8["snr_db"] > 20, r8
    assert r4["rmse"] > r8["rmse"], (r4, r8)
    m = eq.metrics(np.ones((300, 2)), np.ones((300, 2)))
    assert m["mae"] == 0 and m["lsd"] == 0 and m["cosine"] == pytest.approx(1.0)
