"""GPU parity of the individual gfx950 kernels (through the C-ABI self-test entries)
against an fp32 numpy reference of the same op on the same (already rounded) inputs."""
import numpy as np
import pytest

from oracle.ggml_numerics import bf16_bits_to_f32, f32_to_bf16_bits, round_f16

pytestmark = pytest.mark.gpu


def _capi():
    from acestep_mi355x import capi
    return capi


def _bits(x, act):
    if act == 0:
        return f32_to_bf16_bits(x)
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def _vals(bits, act):
    if act == 0:
        return bf16_bits_to_f32(bits)
    return bits.view(np.float16).astype(np.float32)


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (127, 256, 384), (300, 1024, 256), (1000, 384, 2048),
                                   (4100, 128, 128)])
def test_gemm_store_f32(act, M, N, K):
    rng = np.random.default_rng(M + N + K + act)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), act)
    w = _bits((rng.standard_normal((N, K)) * 0.05).astype(np.float32), act)
    bias = rng.standard_normal(N).astype(np.float32)
    got = _capi().kernel_gemm(a, w, act_type=act, epi=0, bias=bias)
    ref = (_vals(a, act).astype(np.float64) @ _vals(w, act).astype(np.float64).T + bias).astype(np.float32)
    scale = np.abs(_vals(a, act)).astype(np.float64) @ np.abs(_vals(w, act)).astype(np.float64).T
    assert np.all(np.abs(got - ref) <= 2e-6 * scale + 1e-6), np.max(np.abs(got - ref) / (scale + 1e-6))


def test_gemm_asymmetric_identity():
    """A = I (padded), W asymmetric: catches a transposed C write (guide §3)."""
    M, N, K = 128, 128, 128
    a = np.eye(M, K, dtype=np.float32)
    w = (np.arange(N)[:, None] * 1000 + np.arange(K)[None, :]).astype(np.float32) / 4096.0
    got = _capi().kernel_gemm(_bits(a, 0), _bits(w, 0), act_type=0, epi=0)
    np.testing.assert_array_equal(got, _vals(_bits(w, 0), 0).T[:M, :N])


@pytest.mark.parametrize("act", [0, 1])
def test_gemm_swiglu_epilogue(act):
    M, I, K = 200, 256, 512
    rng = np.random.default_rng(11)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), act)
    g = (rng.standard_normal((I, K)) * 0.05).astype(np.float32)
    u = (rng.standard_normal((I, K)) * 0.05).astype(np.float32)
    # 16-row interleave [g0..15, u0..15, g16..31, ...] (runtime/model.cpp)
    wi = np.empty((2 * I, K), np.float32)
    for r in range(2 * I):
        grp, w16 = divmod(r, 32)
        wi[r] = (g if w16 < 16 else u)[grp * 16 + (w16 % 16)]
    wb = _bits(wi, act)
    got = _vals(_capi().kernel_gemm(a, wb, act_type=act, epi=4), act)
    av = _vals(a, act).astype(np.float64)
    gv = av @ _vals(_bits(g, act), act).astype(np.float64).T
    uv = av @ _vals(_bits(u, act), act).astype(np.float64).T
    ref = (gv / (1 + np.exp(-gv))) * uv
    ulp = 2.0 ** (-8 if act == 0 else -11)
    np.testing.assert_allclose(got, ref, rtol=ulp, atol=1e-5)


def _attn_ref(q, kv, hq, hkv, window, kmask, scale, rnd=round_f16):
    B, nq, _ = q.shape
    nk = kv.shape[1]
    D = 128
    qh = rnd(q).reshape(B, nq, hq, D)
    k = rnd(kv[:, :, :hkv * D]).reshape(B, nk, hkv, D)
    v = rnd(kv[:, :, hkv * D:]).reshape(B, nk, hkv, D)
    out = np.zeros((B, nq, hq, D), np.float64)
    rep = hq // hkv
    for b in range(B):
        allow = np.ones((nq, nk), bool)
        if window > 0:
            allow &= np.abs(np.arange(nq)[:, None] - np.arange(nk)[None, :]) <= window
        if kmask is not None:
            allow &= kmask[b][None, :] != 0
        for h in range(hq):
            s = qh[b, :, h].astype(np.float64) @ k[b, :, h // rep].astype(np.float64).T * scale
            s = np.where(allow, s, -np.inf)
            m = s.max(axis=1, keepdims=True)
            p = np.exp(s - m)
            p /= p.sum(axis=1, keepdims=True)
            out[b, :, h] = p @ v[b, :, h // rep].astype(np.float64)
    return out.reshape(B, nq, hq * D)


MODES = {"split": dict(split=True), "pvsplit": dict(split=True, pv_split=True), "fast": dict(split=False),
         "f8c": dict(split=True, pv_split=True, f8=True), "pv8": dict(split=False, pv_split=True, f8=True)}


def _check_attn(got, q, kv, hq, hkv, window, kmask, scale, mode):
    """Bounds per precision mode: "pvsplit" (~22-bit operands everywhere) shows only the bf16 rounding of
    the output; "split" (~22-bit Q.K, fp16 P and V) adds the fp16 rounding of P and V, at most 2^-11 of
    max|v| per output; "fast" has fp16 scores too."""
    f32 = lambda x: np.asarray(x, np.float32)
    if mode in ("fast", "pv8"):  # fp16 Q.K operands (pv8: P.V at f8c precision, inside the same bound)
        ref = _attn_ref(q, kv, hq, hkv, window, kmask, scale)
        err = np.abs(got - ref)
        assert np.all(err <= 2.0 ** -8 * np.abs(ref) + 2e-3), float(err.max())
        return ref
    ref = _attn_ref(q, kv, hq, hkv, window, kmask, scale, rnd=f32)
    err = np.abs(got - ref)
    vmax = float(np.abs(kv[:, :, hkv * 128:]).max())
    # f8c: the correction products at e4m3 precision leave ~2^-15 relative per product (2^-13 of max|v| is slack)
    tol = 2.0 ** -8 * np.abs(ref) + {"pvsplit": 1e-5, "f8c": 2.0 ** -13 * vmax}.get(mode, 2.0 ** -10 * vmax)
    assert np.all(err <= tol), float((err - tol).max())
    mism = np.mean(got != bf16_bits_to_f32(f32_to_bf16_bits(ref.astype(np.float32))))
    # pvsplit (~2^-22 operands: <1 % of the outputs round to another bf16 than the f32 reference) and f8c (~2^-15
    # correction products: ~3.3 % measured) are much closer to the f32 reference than a single-fp16 evaluation
    assert mism < {"pvsplit": 0.01, "f8c": 0.05}.get(mode, 0.25), mism
    return ref


@pytest.mark.parametrize("B,hq,hkv,nq,nk,window,masked", [
    (1, 2, 1, 64, 64, 0, False),
    (2, 4, 2, 200, 200, 0, False),
    (1, 4, 2, 333, 333, 16, False),
    (2, 16, 8, 300, 77, 0, True),
    (1, 2, 2, 130, 130, 128, True),
    (1, 4, 1, 97, 500, 0, False),
    (1, 2, 1, 1100, 1100, 0, False),   # >= 16 key tiles on a small grid: two-way key split + merge
    (1, 2, 1, 150, 1500, 0, True),
    # 376 blocks on 256 CUs (the 240 s grid at 18 key tiles): hi/lo modes run one round of whole blocks and split
    # only the remaining 120 (tail split + tail merge); fp16 (two blocks per CU) splits every block
    (1, 16, 8, 3000, 1100, 0, True),
])
@pytest.mark.parametrize("mode", list(MODES))
def test_attention_vs_fp64(B, hq, hkv, nq, nk, window, masked, mode):
    rng = np.random.default_rng(B * 1000 + nq + nk)
    q = rng.standard_normal((B, nq, hq * 128)).astype(np.float32) * 2.0
    kv = rng.standard_normal((B, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
    kmask = None
    if masked:
        kmask = (rng.random((B, nk)) > 0.3).astype(np.int32)
        kmask[:, 0] = 1
    scale = 1.0 / np.sqrt(128.0)
    got = _capi().kernel_attention(q, kv, hq, hkv, window=window, kmask=kmask, scale=scale, **MODES[mode])
    _check_attn(got, q, kv, hq, hkv, window, kmask, scale, mode)


ATTN_CASES = [(1, 2, 1, 64, 64, 0, False), (2, 16, 8, 300, 77, 0, True), (1, 2, 2, 130, 130, 128, True),
              (1, 4, 1, 97, 500, 0, False), (1, 2, 1, 150, 1500, 0, True), (1, 16, 8, 3000, 1100, 0, True),
              (1, 16, 8, 3000, 3000, 128, False), (2, 16, 8, 1500, 1500, 0, True)]


@pytest.mark.parametrize("B,hq,hkv,nq,nk,window,masked", ATTN_CASES)
@pytest.mark.parametrize("kh", [0, 1])
def test_attention_f8c_both_kernels(B, hq, hkv, nq, nk, window, masked, kh):
    """f8c through each of its kernels on every range length (the default policy picks attn_kh_kernel -- two waves
    per SIMD, query group x key half, pair merge through LDS -- only for >= 16 key tiles): same fp64 bound, and the
    two kernels within the f8c bound of each other."""
    capi = _capi()
    rng = np.random.default_rng(B * 1000 + nq + nk + window)
    q = rng.standard_normal((B, nq, hq * 128)).astype(np.float32) * 2.0
    kv = rng.standard_normal((B, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
    kmask = None
    if masked:
        kmask = (rng.random((B, nk)) > 0.3).astype(np.int32)
        kmask[:, 0] = 1
    scale = 1.0 / np.sqrt(128.0)
    capi.kernel_attn_kh(kh)
    try:
        got = capi.kernel_attention(q, kv, hq, hkv, window=window, kmask=kmask, scale=scale, **MODES["f8c"])
    finally:
        capi.kernel_attn_kh(-1)
    _check_attn(got, q, kv, hq, hkv, window, kmask, scale, "f8c")


@pytest.mark.parametrize("mode", list(MODES))
def test_attention_fully_masked_row_is_nan(mode):
    """ggml soft_max of an all -inf row gives NaN (acestep_dit_model.cpp:1245); so does the kernel."""
    q = np.ones((1, 8, 128), np.float32)
    kv = np.ones((1, 8, 256), np.float32)
    got = _capi().kernel_attention(q, kv, 1, 1, window=0, kmask=np.zeros((1, 8), np.int32), **MODES[mode])
    assert np.isnan(got).all()
    # same through the key-split path (every part fully masked -> merge 0/0)
    q = np.ones((1, 8, 128), np.float32)
    kv = np.ones((1, 1100, 256), np.float32)
    got = _capi().kernel_attention(q, kv, 1, 1, window=0, kmask=np.zeros((1, 1100), np.int32), **MODES[mode])
    assert np.isnan(got).all()


def test_attention_split_handles_small_values():
    """lo parts of small operands are fp16 subnormals: check they are not flushed."""
    rng = np.random.default_rng(3)
    q = rng.standard_normal((1, 64, 128)).astype(np.float32) * 3
    kv = rng.standard_normal((1, 64, 256)).astype(np.float32)
    kv[:, :, 128:] *= 1e-3
    got = _capi().kernel_attention(q, kv, 1, 1, split=True, pv_split=True)
    ref = _attn_ref(q, kv, 1, 1, 0, None, 1 / np.sqrt(128), rnd=lambda x: np.asarray(x, np.float32))
    assert np.all(np.abs(got - ref) <= 2.0 ** -8 * np.abs(ref) + 1e-4 * np.abs(ref).max())
    # with flushed lo parts V would carry only fp16 precision and ~10% of outputs would round
    # to a different bf16 than the f32 reference
    mism = np.mean(got != bf16_bits_to_f32(f32_to_bf16_bits(ref.astype(np.float32))))
    assert mism < 0.02, mism


@pytest.mark.parametrize("nk", [700, 1100])
@pytest.mark.parametrize("mode", list(MODES))
def test_attention_running_max_moves_mid_sequence(nk, mode):
    """Scores that keep growing along the keys (and one spike on an odd tile) move the running max by
    more than the lazy-rescale threshold on many tiles: the tile loop leaves, rescales O and l, and
    resumes on even and odd tiles alike."""
    rng = np.random.default_rng(nk + len(mode))
    hq, hkv, nq = 2, 1, 96
    q = rng.standard_normal((1, nq, hq * 128)).astype(np.float32)
    kv = rng.standard_normal((1, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
    ramp = np.linspace(0.2, 20.0, nk).astype(np.float32)
    kv[0, :, :128] *= ramp[:, None]
    kv[0, 64 * 5 + 17, :128] = 4.0 * q[0, :, :128].mean(axis=0)  # spike in tile 5
    scale = 1.0 / np.sqrt(128.0)
    got = _capi().kernel_attention(q, kv, hq, hkv, window=0, kmask=None, scale=scale, **MODES[mode])
    _check_attn(got, q, kv, hq, hkv, 0, None, scale, mode)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 204, 207, 208, 210, 211,
                                     212, 307, 409, 413, 414])
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (300, 512, 128), (1000, 768, 2048), (513, 256, 6144)])
def test_gemm_all_variants(variant, M, N, K):
    """Every GEMM kernel variant (128x128 / 256x256 / 256x128 / 192x128 / 192x256 / 64x64 / 64x128, the
    single-stage, double-buffered and 3-/4-stage LDS rings, and
    split-K over 2..4 blocks per tile: variant + 100 * S), incl. M edges and K = 1, 2 and many tiles
    (pipeline prologue/epilogue paths; split-K falls back to the automatic tile below 2 K-tiles per part)."""
    capi = _capi()
    if N % 256 and variant % 100 in (2, 5, 10, 11):
        pytest.skip("256-wide tiles need N % 256 == 0")
    rng = np.random.default_rng(variant * 7 + M)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), 0)
    w = _bits((rng.standard_normal((N, K)) * 0.05).astype(np.float32), 0)
    capi.gemm_variant(variant)
    try:
        got = capi.kernel_gemm(a, w, act_type=0, epi=0)
        wi = w.copy()
        got_sw = capi.kernel_gemm(a, wi, act_type=0, epi=4)
    finally:
        capi.gemm_variant(-1)
    av, wv = _vals(a, 0).astype(np.float64), _vals(w, 0).astype(np.float64)
    ref = av @ wv.T
    scale = np.abs(av) @ np.abs(wv).T
    assert np.all(np.abs(got - ref) <= 2e-6 * scale + 1e-6)
    # SwiGLU epilogue on the same accumulators: columns 32g..32g+15 gate, 32g+16.. up
    g = ref.reshape(M, N // 32, 2, 16)[:, :, 0, :].reshape(M, N // 2)
    u = ref.reshape(M, N // 32, 2, 16)[:, :, 1, :].reshape(M, N // 2)
    sw = (g / (1 + np.exp(-g))) * u
    np.testing.assert_allclose(_vals(got_sw, 0), sw, rtol=2.0 ** -8, atol=1e-4)


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 204, 207, 210, 211, 213,
                                     215, 408])
@pytest.mark.parametrize("epi", [2, 3])
@pytest.mark.parametrize("M,N,K", [(300, 512, 128), (1000, 768, 2048), (9001, 512, 256)])
def test_gemm_residual_epilogues(variant, epi, M, N, K):
    """x += A.W^T (* gate[n]) in place (the o / cross-o / down projections), every tile incl. the 8-wave
    ones whose epilogue preloads x in chunks of 16-row groups, with M edges."""
    capi = _capi()
    if N % 256 and variant % 100 in (2, 5, 10, 11):
        pytest.skip("256-wide tiles need N % 256 == 0")
    rng = np.random.default_rng(variant * 13 + epi + M)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), 0)
    w = _bits((rng.standard_normal((N, K)) * 0.05).astype(np.float32), 0)
    x = rng.standard_normal((M, N)).astype(np.float32)
    gate = rng.standard_normal(N).astype(np.float32) if epi == 2 else None
    capi.gemm_variant(variant)
    try:
        got = capi.kernel_gemm(a, w, act_type=0, epi=epi, bias=gate, x=x)
    finally:
        capi.gemm_variant(-1)
    av, wv = _vals(a, 0).astype(np.float64), _vals(w, 0).astype(np.float64)
    acc = av @ wv.T
    scale = np.abs(av) @ np.abs(wv).T
    g = gate.astype(np.float64) if epi == 2 else np.ones(N)
    ref = x.astype(np.float64) + acc * g
    assert np.all(np.abs(got - ref) <= (2e-6 * scale + 1e-6) * np.abs(g) + 2e-7 * np.abs(ref))


@pytest.mark.parametrize("variant", [18])
@pytest.mark.parametrize("M,N,K", [(3000, 2048, 2048), (777, 384, 192), (5, 128, 64)])
def test_gemm_tiles_bit_identical(variant, M, N, K):
    """The warp-specialized 192x128 tile (one barrier per k-tile, loader waves) accumulates every element in the
    same k order as the double-buffered 192x128 tile (4): identical bits, store and residual."""
    capi = _capi()
    rng = np.random.default_rng(M + K)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), 0)
    w = _bits((rng.standard_normal((N, K)) * 0.05).astype(np.float32), 0)
    x = rng.standard_normal((M, N)).astype(np.float32)
    gate = rng.standard_normal(N).astype(np.float32)
    outs = {}
    for v in (4, variant):
        capi.gemm_variant(v)
        try:
            outs[v] = (capi.kernel_gemm(a, w, act_type=0, epi=0), capi.kernel_gemm(a, w, act_type=0, epi=2, bias=gate, x=x))
        finally:
            capi.gemm_variant(-1)
    np.testing.assert_array_equal(outs[variant][0], outs[4][0])
    np.testing.assert_array_equal(outs[variant][1], outs[4][1])


def test_attention_key_split_with_one_part_fully_masked():
    """Key split: the first part sees only masked keys (m = -inf, l = 0) and must get weight 0."""
    rng = np.random.default_rng(77)
    B, hq, hkv, nq, nk = 1, 2, 1, 100, 1500
    q = rng.standard_normal((B, nq, hq * 128)).astype(np.float32) * 2.0
    kv = rng.standard_normal((B, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
    kmask = np.ones((B, nk), np.int32)
    kmask[:, :1000] = 0
    scale = 1.0 / np.sqrt(128.0)
    for mode in ("split", "pvsplit", "f8c", "pv8"):
        got = _capi().kernel_attention(q, kv, hq, hkv, window=0, kmask=kmask, scale=scale, **MODES[mode])
        _check_attn(got, q, kv, hq, hkv, 0, kmask, scale, mode)


@pytest.mark.parametrize("nk", [566, 600])
@pytest.mark.parametrize("mode", list(MODES))
def test_attention_short_range_four_way_split(nk, mode):
    """Short key ranges on a grid of at most a quarter round are split in four parts by default (launch_attention,
    mode 0): 9 / 10 key tiles give parts of 3, 3, 3, 0 / 3, 3, 3, 1 tiles -- an EMPTY last part (n = 0) -- and the
    key mask below leaves the first part with no visible key (m = -inf, l = 0).  Against the fp64 reference."""
    rng = np.random.default_rng(nk)
    B, hq, hkv, nq = 1, 2, 1, 100  # 2 blocks of 64 queries
    q = rng.standard_normal((B, nq, hq * 128)).astype(np.float32) * 2.0
    kv = rng.standard_normal((B, nk, 2 * hkv * 128)).astype(np.float32) * 0.3
    kmask = (rng.random((B, nk)) > 0.3).astype(np.int32)
    kmask[:, :3 * 64] = 0  # part 0 fully masked
    kmask[:, 3 * 64] = 1
    scale = 1.0 / np.sqrt(128.0)
    got = _capi().kernel_attention(q, kv, hq, hkv, window=0, kmask=kmask, scale=scale, **MODES[mode])
    _check_attn(got, q, kv, hq, hkv, 0, kmask, scale, mode)


@pytest.mark.parametrize("variant", [204, 207, 211, 212, 307, 408])
def test_gemm_splitk_deterministic(variant):
    """Split-K: the last block of a tile adds the parts in K order, so repeated launches (with the per-tile
    ticket counters carried over between launches of different tile counts) give identical bits, equal to
    the fp32 sum of the S partial products in K order to within the MFMA accumulation rounding."""
    capi = _capi()
    rng = np.random.default_rng(variant)
    outs = []
    for M, N, K in [(3000, 2048, 2048), (700, 512, 1024), (3000, 2048, 2048)]:
        a = _bits(rng.standard_normal((M, K)).astype(np.float32), 0) if not outs or M != 3000 else a0
        w = _bits((rng.standard_normal((N, K)) * 0.05).astype(np.float32), 0) if not outs or M != 3000 else w0
        if not outs:
            a0, w0 = a, w
        capi.gemm_variant(variant)
        try:
            outs.append(capi.kernel_gemm(a, w, act_type=0, epi=0))
            outs.append(capi.kernel_gemm(a, w, act_type=0, epi=0))
        finally:
            capi.gemm_variant(-1)
        np.testing.assert_array_equal(outs[-1], outs[-2])
        av, wv = _vals(a, 0).astype(np.float64), _vals(w, 0).astype(np.float64)
        assert np.all(np.abs(outs[-1] - av @ wv.T) <= 2e-6 * (np.abs(av) @ np.abs(wv).T) + 1e-6)
    np.testing.assert_array_equal(outs[0], outs[4])


# ---------------------------------------------------------------- run-to-run identity of the product kernels
# The round-5 MFMA operand hazard showed as launch-dependent wrong column groups; the static audit
# (tests/test_mfma_war_audit.py) finds no unguarded pair in a two-wave kernel.  These tests are its dynamic side: the
# product picks at the 240 s shapes (M = 3000) launched repeatedly must give identical bits every time.
@pytest.mark.parametrize("name,N,K,epi", [("o / cross-o (gated residual)", 2048, 2048, 2),
                                          ("down (gated residual)", 2048, 6144, 2),
                                          ("gate|up (SwiGLU)", 12288, 2048, 4), ("qkv-shaped store", 4096, 2048, 0)])
def test_product_gemm_picks_run_to_run_identical(name, N, K, epi):
    capi = _capi()
    M = 3000
    rng = np.random.default_rng(N + K)
    a = _bits(rng.standard_normal((M, K)).astype(np.float32), 0)
    w = _bits((rng.standard_normal((N, K)) * 0.02).astype(np.float32), 0)
    x = rng.standard_normal((M, N)).astype(np.float32) if epi == 2 else None
    gate = rng.standard_normal(N).astype(np.float32) if epi == 2 else None
    outs = [capi.kernel_gemm(a, w, act_type=0, epi=epi, bias=gate, x=x) for _ in range(6)]
    for i, o in enumerate(outs[1:], 1):
        assert np.array_equal(o.view(np.uint32) if o.dtype == np.float32 else o,
                              outs[0].view(np.uint32) if outs[0].dtype == np.float32 else outs[0]), (name, i)


@pytest.mark.parametrize("kh", [-1, 0, 1])
@pytest.mark.parametrize("window", [0, 128])
def test_product_attention_run_to_run_identical(window, kh):
    """f8c (the DiT default) at the 240 s self-attention shape: full layers (tail split + merge) and sliding ones, through
    the default policy and each kernel forced (attn_kh_kernel runs two waves per SIMD: the operand-overwrite hazard's
    condition, audited statically by tests/test_mfma_war_audit.py)."""
    rng = np.random.default_rng(5 + window)
    q = rng.standard_normal((1, 3000, 16 * 128)).astype(np.float32)
    kv = rng.standard_normal((1, 3000, 2 * 8 * 128)).astype(np.float32) * 0.5
    _capi().kernel_attn_kh(kh)
    try:
        outs = [_capi().kernel_attention(q, kv, 16, 8, window=window, scale=1 / np.sqrt(128.0), **MODES["f8c"])
                for _ in range(5)]
    finally:
        _capi().kernel_attn_kh(-1)
    for i, o in enumerate(outs[1:], 1):
        assert np.array_equal(o.view(np.uint32), outs[0].view(np.uint32)), (window, i)
