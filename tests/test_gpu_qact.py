"""GPU parity of the ggml-faithful quantized-activation mode (ACE_MI_QUANT_ACT=q8, kernels/gemm_a8.hip).

ggml's mul_mat against a quantized weight converts the f32 activations to Q8_0 / Q8_K blocks and takes integer
dot products per block (oracle/ggml_numerics.py convert_activation + mul_mat; ggml-metal-embed.metal:3110-3128).
Checked here:
  * the activation quantizers bit for bit against the oracle's restatement (q, d and the Q8_K block sums);
  * the integer-dot GEMM against an fp64 product of the same dequantized blocks (its f32 sum of exact per-block
    integer dots differs from fp64 by f32 rounding only), with each epilogue the mode uses;
Whole DiT forwards in this mode against the oracle WITH ggml's activation quantization (within 1.5x the oracle's own
floor) are test_gpu_quant.py::test_quantized_full_width_vs_ggml_semantics and
test_gpu_configs.py::test_quantized_configs_full_width."""
import numpy as np
import pytest


pytestmark = pytest.mark.gpu


def _capi():
    from acestep_mi355x import capi
    return capi


def _deq(w_blocks, qtype):
    from oracle import ggml_numerics as g
    return {"q8_0": lambda r: g.dequantize_q8_0(*g.unpack_q8_0(r)), "q4_k": g.dequantize_q4_k,
            "q6_k": g.dequantize_q6_k}[qtype](w_blocks).astype(np.float64)


def _act_blocks(x, qtype):
    """oracle activation blocks: (q int8 [M][K], d per 32-value block [K/32][M], block sums [K/32][M] or None)"""
    from oracle import ggml_numerics as g
    M, K = x.shape
    if qtype == "q8_0":
        d, q = g.quantize_q8_0_activations(x)
        return q.reshape(M, K), d.astype(np.float32).T, None
    d, q = g.quantize_q8_k_activations(x)
    q = q.reshape(M, K)
    d32 = np.repeat(d, 8, axis=1).T
    bs = q.reshape(M, K // 32, 32).astype(np.int64).sum(axis=2).astype(np.float32).T
    return q, d32, bs


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("M,N,K", [(1, 128, 256), (77, 256, 512), (300, 384, 2048), (129, 128, 6144)])
def test_gemm_a8_matches_block_integer_dot(qtype, M, N, K):
    capi = _capi()
    rng = np.random.default_rng(M * 7 + K + len(qtype))
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[:, :32] *= 40.0  # a block of large values, all-zero blocks, exact ties of the largest |x| (the first wins)
    if K >= 512:
        x[:, 256:288] = 0.0
        x[0, 300], x[0, 301] = 100.0, -100.0
    if K >= 1024 and M > 1:
        x[1, 512:768] = 0.0
    x[0, 40], x[0, 41] = 3.0, -3.0
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = capi.quantize(w, qtype)
    out, q, s, bs = capi.kernel_gemm_a8(x, blocks, qtype)
    qr, dr, bsr = _act_blocks(x, qtype)
    np.testing.assert_array_equal(q, qr)
    np.testing.assert_array_equal(s, dr)
    if bsr is not None:
        np.testing.assert_array_equal(bs, bsr)
    xa = (qr.reshape(M, K // 32, 32).astype(np.float64) * dr.T[:, :, None]).reshape(M, K)
    ref = xa @ _deq(blocks, qtype).T
    mag = np.abs(xa) @ np.abs(_deq(blocks, qtype)).T
    err = np.abs(out - ref)
    assert np.all(err <= 5e-6 * mag + 1e-30), float(np.max(err / (mag + 1e-30)))


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (77, 256, 128), (129, 384, 2048), (300, 128, 6144), (3000, 2048, 2048),
                                   (2048, 8192, 128)])
@pytest.mark.parametrize("epi", [0, 3, 7])
def test_gemm_a8_bf16_mfma_form_is_bit_identical(M, N, K, epi):
    """Q8_0 on the bf16 MFMA (gemm_a8s_kernel: each block's integer dot is exact in f32 from bf16(q) operands, the
    default for K % 64 == 0) against the i8-MFMA kernel: the same integer dots, scales and f32 order -> the same bits,
    with every epilogue the comparison covers; both tile widths (128 for grids of >= one round of two workgroups per
    CU, e.g. 2048 x 8192; 64 below that)."""
    capi = _capi()
    rng = np.random.default_rng(M + N + K + epi)
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[:, :32] *= 40.0
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    blocks = capi.quantize(w, "q8_0")
    b = rng.standard_normal(N).astype(np.float32)
    x0 = rng.standard_normal((M, N)).astype(np.float32) if epi == 3 else None
    outs = []
    try:
        for mode in (0, 1):
            capi.kernel_gemm_a8_mode(mode)
            outs.append(capi.kernel_gemm_a8(x, blocks, "q8_0", epi=epi, bias=None if epi == 7 else b, x0=x0))
    finally:
        capi.kernel_gemm_a8_mode(-1)
    for i0, i1 in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(np.asarray(i0).view(np.uint8), np.asarray(i1).view(np.uint8))


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k"])
def test_gemm_a8_epilogues(qtype):
    """bias store, residual with bias (x + (acc + b): ggml adds the bias to the mul_mat result), SwiGLU in f32"""
    capi = _capi()
    rng = np.random.default_rng(5)
    M, N, K = 200, 256, 512
    x = rng.standard_normal((M, K)).astype(np.float32)
    w = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    blocks = capi.quantize(w, qtype)
    qr, dr, _ = _act_blocks(x, qtype)
    xa = (qr.reshape(M, K // 32, 32).astype(np.float64) * dr.T[:, :, None]).reshape(M, K)
    ref = xa @ _deq(blocks, qtype).T
    got, *_ = capi.kernel_gemm_a8(x, blocks, qtype, epi=0, bias=b)
    np.testing.assert_allclose(got, ref + b, rtol=1e-5, atol=1e-5)
    x0 = rng.standard_normal((M, N)).astype(np.float32)
    got, *_ = capi.kernel_gemm_a8(x, blocks, qtype, epi=3, bias=b, x0=x0)
    np.testing.assert_allclose(got, x0 + (ref + b), rtol=1e-5, atol=1e-5)
    got, *_ = capi.kernel_gemm_a8(x, blocks, qtype, epi=7)
    gcols = np.concatenate([np.arange(grp * 32, grp * 32 + 16) for grp in range(N // 32)])
    g, u = ref[:, gcols], ref[:, gcols + 16]
    np.testing.assert_allclose(got, g / (1.0 + np.exp(-g)) * u, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
def test_qact_tiny_with_masks_vs_ggml_semantics(tiny_ckpt, monkeypatch, qtype):
    """The tiny model in ACE_MI_QUANT_ACT=q8 with a key-padding mask, an encoder mask, odd T and r != t: against the
    oracle with ggml's Q8_0 / Q8_K activation quantization -- every block format, the masked attention's f32-output
    path and the t - r timestep branch.  rel-L2 bound only (max(1e-3, 1.5 x floor)): at this size the 1e-7
    perturbation floor is a count of a few discrete q flips (Q8_K: often none, floor 7e-7), so its element-wise
    statistic is no scale for an implementation whose f32 order differs at 1e-6; the element-wise bound is held at
    full width (test_gpu_quant.py / test_gpu_configs.py)."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    from test_gpu_forward import check
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", qtype)
    monkeypatch.setenv("ACE_MI_QUANT_ACT", "q8")
    rng = np.random.default_rng(41)
    T, L = 301, 20
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, 256)).astype(np.float32)
    mask = np.ones(T, np.int32)
    mask[280:] = 0
    emask = np.ones(L, np.int32)
    emask[15:] = 0
    br = GGMLCAPIBridge()
    br.load_dit(tiny_ckpt)
    got = br.dit_forward_tfirst(h, c, e, mask, emask, 0.7, 0.4)
    br.close()
    ref, floor, _ = forward_with_floor_stats(DitWeights(tiny_ckpt, qtype=qtype), h, c, e, mask, emask, T, L, 0.7, 0.4)
    check(got, ref, floor, f"tiny {qtype} ACE_MI_QUANT_ACT=q8 with masks (ggml semantics)")


def test_qact_sampling_loop_equals_per_step_forwards(tiny_ckpt, monkeypatch):
    """ace_mi_dit_sample_ex in ACE_MI_QUANT_ACT=q8 (timestep rows of every step precomputed in one pass, cross K/V
    recomputed) equals per-step batched forwards + the same f32 Euler updates, bit for bit, at B = 2."""
    import torch
    from acestep_mi355x.capi import GGMLCAPIBridge
    monkeypatch.setenv("ACE_GGML_DIT_WEIGHT_QTYPE", "q8_0")
    monkeypatch.setenv("ACE_MI_QUANT_ACT", "q8")
    rng = np.random.default_rng(43)
    B, T, L = 2, 90, 12
    sched = np.array([1.0, 0.8, 0.45], np.float32)
    dev = torch.device("cuda:0")
    x0 = torch.from_numpy(rng.standard_normal((B, T, 64)).astype(np.float32)).to(dev)
    dc = torch.from_numpy(rng.standard_normal((B, T, 128)).astype(np.float32)).to(dev)
    de = torch.from_numpy(rng.standard_normal((B, L, 256)).astype(np.float32)).to(dev)
    br = GGMLCAPIBridge()
    br.load_dit(tiny_ckpt)
    xt = x0.clone()
    torch.cuda.synchronize()
    br.dit_sample_ex_device(B, T, L, xt.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, list(sched), cache_cross=False)
    br.synchronize()
    loop = xt.cpu().numpy()
    x = x0.clone()
    v = torch.empty_like(x)
    for i, t in enumerate(sched):
        tt = torch.full((B,), float(t), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        br.dit_forward_batched_device(B, T, L, x.data_ptr(), dc.data_ptr(), de.data_ptr(), 0, 0, tt.data_ptr(),
                                      tt.data_ptr(), v.data_ptr(), 0)
        br.synchronize()
        dt = np.float32(t) if i + 1 == len(sched) else np.float32(np.float32(t) - np.float32(sched[i + 1]))
        x = x - v * float(dt)
    torch.cuda.synchronize()
    br.close()
    np.testing.assert_array_equal(loop, x.cpu().numpy())
