"""Online weight quantization (ACE_GGML_DIT_WEIGHT_QTYPE, acestep_dit_model.cpp:27-45,156-192).

The loader's C++ encoders (runtime/quant.cpp, reached through ace_mi_quantize — a host-only entry,
no GPU needed) must produce the same ggml block bytes as the oracle restatement of
quantize_row_{q8_0,q4_K,q6_K}_ref, and their dequantization must equal the oracle's.  The Q8_0 and
Q4_K layouts/dequant are pinned to the Metal text in the reference tree (test_oracle.py); Q6_K's
layout is checked here against the reference's Metal dequantizer restated independently
(ggml-metal-embed.metal:3477-3507).
"""
import numpy as np
import pytest

from oracle import ggml_numerics as g


def _capi():
    from acestep_mi355x import capi
    return capi


def _weights(seed, rows, cols, kind):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((rows, cols)).astype(np.float32)
    if kind == "small":
        w *= 0.02
    elif kind == "edge":
        w[0] = 0.0                              # all-zero blocks
        w[1, : cols // 2] = 0.5                 # constant blocks
        w[2] = np.round(w[2] * 4) / 4           # exact ties for the round-half cases
        w[3, :32] = 0.0
        w[4] = 1e-20                            # below GROUP_MAX_EPS (Q6_K zero block)
        w[5] = np.abs(w[5])                     # all-positive: Q4_K min clamps to 0
        w[6] = -np.abs(w[6])
        w[7, ::7] *= 1000.0                     # outliers
    return w


ORACLE = {
    "q8_0": lambda w: g.pack_q8_0(*g.quantize_q8_0_weights(w)),
    "q4_k": g.quantize_q4_k_weights,
    "q6_k": g.quantize_q6_k_weights,
}
DEQ = {
    "q8_0": lambda raw: g.dequantize_q8_0(*g.unpack_q8_0(raw)),
    "q4_k": g.dequantize_q4_k,
    "q6_k": g.dequantize_q6_k,
}


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("kind", ["small", "unit", "edge"])
def test_loader_encoder_matches_oracle_bytes(qtype, kind):
    w = _weights(hash((qtype, kind)) % 1000, 64, 1024, kind)
    ref = ORACLE[qtype](w)
    got = _capi().quantize(w, qtype)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), int(np.count_nonzero(got != ref))
    np.testing.assert_array_equal(_capi().dequantize(got, qtype), DEQ[qtype](got))


@pytest.mark.parametrize("qtype,rel", [("q8_0", 0.01), ("q6_k", 0.03), ("q4_k", 0.12)])
def test_quantization_error_is_format_sized(qtype, rel):
    w = _weights(3, 32, 2048, "small")
    y = DEQ[qtype](_capi().quantize(w, qtype))
    err = np.sqrt(np.mean((y - w) ** 2)) / np.sqrt(np.mean(w * w))
    assert err < rel, err


def test_quantize_rejects_bad_row_length():
    capi = _capi()
    with pytest.raises(ValueError):
        capi.quantize(np.zeros((2, 48), np.float32), "q8_0")
    with pytest.raises(ValueError):
        capi.quantize(np.zeros((2, 384), np.float32), "q4_k")   # 384 % 256 != 0 -> stays dense in the loader


def _metal_dequant_q6_k(raw):
    """dequantize_q6_K of ggml-metal-embed.metal:3477-3507, restated: 16 chunks of 16 values (il),
    low nibbles from ql, high bits from qh by masks/shifts, y = d*sc*q - d*sc*32."""
    rows, nb, _ = raw.shape
    out = np.empty((rows, nb * 256), np.float64)
    for r in range(rows):
        for b in range(nb):
            blk = raw[r, b]
            ql = blk[0:128].view(np.uint16)
            qh = blk[128:192].view(np.uint16)
            sc = blk[192:208].view(np.int8)
            d = float(blk[208:210].view(np.float16)[0])
            for il in range(16):
                qlp = ql[32 * (il // 8) + 16 * ((il // 2) & 1) + 8 * (il & 1):]
                qhp = qh[16 * (il // 8) + 8 * (il & 1):]
                s = float(sc[(il % 2) + 2 * (il // 2)])
                j = (il // 2) & 3
                kmask1 = [0x03030303, 0x0C0C0C0C, 0x30303030, 0xC0C0C0C0][j]
                kmask2 = 0x0F0F0F0F if j <= 1 else 0xF0F0F0F0
                shr_h = 2 if j > 2 else 0
                shl_h = 0 if j > 1 else (2 if j > 0 else 4)
                shr_l = 4 if j > 1 else 0
                vals = []
                for i in range(4):
                    low = (int(qlp[2 * i]) | (int(qlp[2 * i + 1]) << 16)) & kmask2
                    high = (int(qhp[2 * i]) | (int(qhp[2 * i + 1]) << 16)) & kmask1
                    q = (((high << shl_h) & 0xFFFFFFFF) >> shr_h) | (low >> shr_l)
                    for k in range(4):
                        vals.append(d * s * ((q >> (8 * k)) & 0xFF) - d * s * 32.0)
                # chunk il covers 16 consecutive output values of the 256-block
                out[r, b * 256 + 16 * il: b * 256 + 16 * il + 16] = vals
    return out


def test_q6_k_layout_matches_metal_dequantizer():
    w = _weights(5, 4, 512, "unit")
    raw = g.quantize_q6_k_weights(w)
    ours = g.dequantize_q6_k(raw).astype(np.float64)
    metal = _metal_dequant_q6_k(raw)
    np.testing.assert_allclose(ours, metal, rtol=1e-6, atol=1e-6 * np.abs(metal).max())
