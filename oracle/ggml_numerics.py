"""ggml-cpu numeric semantics restated in numpy — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

ggml 0.9.5 (the reference's absent submodule, `acestep_ggml/third_party/ggml`,
version from `acestep_ggml/build_metal/CMakeCache.txt`) is not in the container.
Its published algorithms are restated here:

* `mul_mat(W, x)` converts the f32 activation `x` to the weight type's
  `vec_dot_type` before the dot product and accumulates in f32:
  BF16 -> bf16 (round-to-nearest-even), F16 -> fp16, Q8_0 -> Q8_0 blocks,
  Q4_K -> Q8_K blocks, F32 -> f32 (no rounding).  Call sites:
  `acestep_dit_model.cpp:1194-1196,1257,1295-1302,1381,1412,1528-1531,1551`.
* Q8_0 block = {fp16 d; int8 qs[32]} (34 B / 32 weights),
  `ggml-metal-embed.metal:222-227`; quantize d = amax/127, q = round(x/d)
  (`:3110-3128`); dequant q*d (`:3328-3339`).
* Q4_K super-block = {fp16 d, fp16 dmin, u8 scales[12], u8 qs[128]}
  (144 B / 256 weights), `:298-309`; 6-bit scale/min unpack + dequant
  `:3429-3451`.  The Q4_K *encoder* (`make_qkx2_quants`, ggml-quants.c) is not
  in the container: it is restated from the published ggml source below and
  is **parity unpinned** (GPU kernels are checked on identical packed bytes).
"""
from __future__ import annotations

import numpy as np

QK8_0 = 32
QK_K = 256


# --------------------------------------------------------------------------
# bf16 / fp16 rounding
# --------------------------------------------------------------------------
def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """ggml_compute_fp32_to_bf16: round-to-nearest-even on the f32 bits, NaN kept quiet."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    nan = (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    r = (u + (np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1)))) >> np.uint32(16)
    r = np.where(nan, (u >> np.uint32(16)) | np.uint32(64), r)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def round_bf16(x: np.ndarray) -> np.ndarray:
    return bf16_bits_to_f32(f32_to_bf16_bits(x))


def round_f16(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float32)


# --------------------------------------------------------------------------
# Q8_0
# --------------------------------------------------------------------------
def quantize_q8_0_weights(w: np.ndarray):
    """quantize_row_q8_0_ref (ggml_quantize_chunk path used by `try_quantize_matrix`,
    acestep_dit_model.cpp:156-192): per 32-block d = amax/127, id = 1/d,
    q = roundf(x*id) (round half away from zero), d stored as fp16.
    Returns (d fp16 [rows, nb], qs int8 [rows, nb, 32])."""
    w = np.asarray(w, dtype=np.float32)
    rows, k = w.shape
    assert k % QK8_0 == 0
    blk = w.reshape(rows, k // QK8_0, QK8_0)
    amax = np.max(np.abs(blk), axis=2)
    d = (amax / np.float32(127.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    x0 = blk * idv[:, :, None]
    ax = np.abs(x0)
    fl = np.floor(ax)
    q = (np.sign(x0) * (fl + ((ax - fl) >= np.float32(0.5)))).astype(np.int8)  # roundf, exact
    return d.astype(np.float16), q


def dequantize_q8_0(d: np.ndarray, q: np.ndarray) -> np.ndarray:
    rows, nb = d.shape
    return (q.astype(np.float32) * d.astype(np.float32)[:, :, None]).reshape(rows, nb * QK8_0)


def quantize_q8_0_activations(x: np.ndarray):
    """x86 `quantize_row_q8_0` (AVX2 path, the vec_dot_type conversion of src1 in
    mul_mat against Q8_0 weights): d = amax/127 stored fp16, id = 127/amax,
    q = round-half-even(x*id).  Returns (d fp16, qs int8)."""
    x = np.asarray(x, dtype=np.float32)
    rows, k = x.shape
    blk = x.reshape(rows, k // QK8_0, QK8_0)
    amax = np.max(np.abs(blk), axis=2).astype(np.float32)
    d = (amax / np.float32(127.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(amax != 0, np.float32(127.0) / amax, np.float32(0.0)).astype(np.float32)
    q = np.rint(blk * idv[:, :, None]).astype(np.int8)
    return d.astype(np.float16), q


def q8_0_activation_roundtrip(x: np.ndarray) -> np.ndarray:
    d, q = quantize_q8_0_activations(x)
    return dequantize_q8_0(d, q)


def pack_q8_0(d: np.ndarray, q: np.ndarray) -> np.ndarray:
    """Byte image of block_q8_0 rows: [rows, nb, 34] uint8 (fp16 d little-endian, then 32 x int8)."""
    rows, nb = d.shape
    out = np.empty((rows, nb, 34), dtype=np.uint8)
    out[:, :, 0:2] = d.astype("<f2").view(np.uint8).reshape(rows, nb, 2)
    out[:, :, 2:] = q.view(np.uint8)
    return out


def unpack_q8_0(raw: np.ndarray):
    raw = np.asarray(raw, dtype=np.uint8)
    d = raw[..., 0:2].copy().view("<f2")[..., 0]
    q = raw[..., 2:].copy().view(np.int8)
    return d.astype(np.float16), q


# --------------------------------------------------------------------------
# Q4_K (weights) and Q8_K (activations for Q4_K weights)
# --------------------------------------------------------------------------
def _nearest_int(f):
    # ggml nearest_int: round-half-even via the 12582912 magic constant
    return np.rint(np.asarray(f, dtype=np.float32)).astype(np.int32)


def _seqsum(a: np.ndarray) -> np.ndarray:
    """Row sums in float32 accumulated left to right, like ggml's scalar `for` loops
    (np.sum would use pairwise summation and round differently)."""
    return np.add.accumulate(np.asarray(a, dtype=np.float32), axis=1, dtype=np.float32)[:, -1]


def _make_qkx2_quants(x, weights, nmax=15, rmin=-1.0, rdelta=0.1, nstep=20):
    """Vectorised make_qkx2_quants(n=32, use_mad=false) over a batch of sub-blocks.
    x, weights: [S, 32] f32.  Returns (scale [S], the_min [S] (= -min), L [S,32])."""
    x = x.astype(np.float32)
    w = weights.astype(np.float32)
    mn = np.minimum(np.min(x, axis=1), np.float32(0.0))
    mx = np.max(x, axis=1)
    sum_w = _seqsum(w)
    sum_x = _seqsum(w * x)
    flat = mx == mn
    rng_ = np.where(flat, np.float32(1.0), mx - mn).astype(np.float32)
    iscale = (np.float32(nmax) / rng_).astype(np.float32)
    scale = (np.float32(1.0) / iscale).astype(np.float32)
    L = np.clip(_nearest_int(iscale[:, None] * (x - mn[:, None])), 0, nmax)
    diff = scale[:, None] * L.astype(np.float32) + mn[:, None] - x
    best = _seqsum(w * (diff * diff))
    best_min = mn.copy()
    for i_s in range(nstep + 1):
        # ggml updates `min` in place when a better fit is found, so later search points use the
        # current best min in both the range (max - min) and the offset (x - min)
        rng_cur = np.where(flat, np.float32(1.0), mx - best_min).astype(np.float32)
        isc = ((np.float32(rmin) + np.float32(rdelta) * np.float32(i_s) + np.float32(nmax)) / rng_cur).astype(np.float32)
        La = np.clip(_nearest_int(isc[:, None] * (x - best_min[:, None])), 0, nmax).astype(np.float32)
        sum_l = _seqsum(w * La)
        sum_l2 = _seqsum(w * La * La)
        sum_xl = _seqsum(w * La * x)
        D = sum_w * sum_l2 - sum_l * sum_l
        ok = D > 0
        Ds = np.where(ok, D, np.float32(1.0))
        this_scale = (sum_w * sum_xl - sum_x * sum_l) / Ds
        this_min = (sum_l2 * sum_x - sum_l * sum_xl) / Ds
        pos = this_min > 0
        this_min = np.where(pos, np.float32(0.0), this_min)
        this_scale = np.where(pos, sum_xl / np.where(sum_l2 != 0, sum_l2, np.float32(1.0)), this_scale)
        d2 = this_scale[:, None] * La + this_min[:, None] - x
        mad = _seqsum(w * (d2 * d2))
        better = ok & (mad < best)
        L = np.where(better[:, None], La.astype(np.int32), L)
        best = np.where(better, mad, best)
        scale = np.where(better, this_scale, scale).astype(np.float32)
        best_min = np.where(better, this_min, best_min).astype(np.float32)
    scale = np.where(flat, np.float32(0.0), scale)
    best_min = np.where(flat, mn, best_min)
    L = np.where(flat[:, None], 0, L)
    return scale.astype(np.float32), (-best_min).astype(np.float32), L


def quantize_q4_k_weights(w: np.ndarray) -> np.ndarray:
    """quantize_row_q4_K_ref (no imatrix).  Returns packed bytes [rows, nb, 144]."""
    w = np.asarray(w, dtype=np.float32)
    rows, k = w.shape
    assert k % QK_K == 0
    nb = k // QK_K
    x = w.reshape(rows * nb, 8, 32)
    sub = x.reshape(-1, 32)
    av_x = np.sqrt(_seqsum(sub * sub) / np.float32(32.0)).astype(np.float32)
    weights = av_x[:, None] + np.abs(sub)
    scales, mins, L0 = _make_qkx2_quants(sub, weights)
    scales = scales.reshape(-1, 8)
    mins = mins.reshape(-1, 8)
    max_scale = np.maximum(np.max(scales, axis=1), np.float32(0.0))
    max_min = np.maximum(np.max(mins, axis=1), np.float32(0.0))
    inv_scale = np.where(max_scale > 0, np.float32(63.0) / np.where(max_scale > 0, max_scale, 1), 0).astype(np.float32)
    inv_min = np.where(max_min > 0, np.float32(63.0) / np.where(max_min > 0, max_min, 1), 0).astype(np.float32)
    ls = np.minimum(_nearest_int(inv_scale[:, None] * scales), 63).astype(np.uint8)
    lm = np.minimum(_nearest_int(inv_min[:, None] * mins), 63).astype(np.uint8)
    sc = np.zeros((rows * nb, 12), dtype=np.uint8)
    sc[:, 0:4] = ls[:, 0:4]
    sc[:, 4:8] = lm[:, 0:4]
    sc[:, 8:12] = (ls[:, 4:8] & 0xF) | ((lm[:, 4:8] & 0xF) << 4)
    sc[:, 0:4] |= (ls[:, 4:8] >> 4) << 6
    sc[:, 4:8] |= (lm[:, 4:8] >> 4) << 6
    d = (max_scale / np.float32(63.0)).astype(np.float16)
    dmin = (max_min / np.float32(63.0)).astype(np.float16)
    scv, mv = _q4k_scale_min(sc)
    dd = d.astype(np.float32)[:, None] * scv.astype(np.float32)
    dm = dmin.astype(np.float32)[:, None] * mv.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        Lq = _nearest_int((x + dm[:, :, None]) / np.where(dd != 0, dd, 1)[:, :, None])
    Lq = np.clip(Lq, 0, 15).astype(np.uint8)
    # `if (!d) continue;` keeps make_qkx2_quants' L for that sub-block
    Lq = np.where((dd != 0)[:, :, None], Lq, L0.reshape(-1, 8, 32)).astype(np.uint8).reshape(rows * nb, 256)
    qs = np.empty((rows * nb, 128), dtype=np.uint8)
    for j in range(4):
        qs[:, 32 * j:32 * j + 32] = Lq[:, 64 * j:64 * j + 32] | (Lq[:, 64 * j + 32:64 * j + 64] << 4)
    out = np.empty((rows * nb, 144), dtype=np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dmin.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = sc
    out[:, 16:] = qs
    return out.reshape(rows, nb, 144)


def _q4k_scale_min(sc: np.ndarray):
    """get_scale_min_k4 for j = 0..7 (ggml-metal-embed.metal:3429-3432 restated)."""
    scv = np.empty(sc.shape[:-1] + (8,), dtype=np.uint8)
    mv = np.empty_like(scv)
    scv[..., 0:4] = sc[..., 0:4] & 63
    mv[..., 0:4] = sc[..., 4:8] & 63
    scv[..., 4:8] = (sc[..., 8:12] & 0xF) | ((sc[..., 0:4] >> 6) << 4)
    mv[..., 4:8] = (sc[..., 8:12] >> 4) | ((sc[..., 4:8] >> 6) << 4)
    return scv, mv


def dequantize_q4_k(raw: np.ndarray) -> np.ndarray:
    """dequantize_row_q4_K: y = d*sc*q - dmin*m per 32-sub-block (`:3435-3451`)."""
    raw = np.asarray(raw, dtype=np.uint8)
    rows, nb, _ = raw.shape
    r = raw.reshape(rows * nb, 144)
    d = r[:, 0:2].copy().view("<f2")[:, 0].astype(np.float32)
    dmin = r[:, 2:4].copy().view("<f2")[:, 0].astype(np.float32)
    scv, mv = _q4k_scale_min(r[:, 4:16])
    qs = r[:, 16:]
    q = np.empty((rows * nb, 256), dtype=np.float32)
    for j in range(4):
        q[:, 64 * j:64 * j + 32] = (qs[:, 32 * j:32 * j + 32] & 0xF)
        q[:, 64 * j + 32:64 * j + 64] = (qs[:, 32 * j:32 * j + 32] >> 4)
    d1 = (d[:, None] * scv.astype(np.float32)).astype(np.float32)
    m1 = (dmin[:, None] * mv.astype(np.float32)).astype(np.float32)
    y = d1[:, :, None] * q.reshape(-1, 8, 32) - m1[:, :, None]
    return y.reshape(rows, nb * 256).astype(np.float32)


def quantize_q8_k_activations(x: np.ndarray):
    """quantize_row_q8_K_ref: per 256-block iscale = -127/max (max = signed value of
    largest magnitude, the first one on ties), q = min(127, nearest_int(iscale*x)),
    d = 1/iscale (f32); an all-zero block is d = 0, q = 0.  Returns (d f32 [rows, nb], q int8 [rows, nb, 256])."""
    x = np.asarray(x, dtype=np.float32)
    rows, k = x.shape
    blk = x.reshape(rows, k // QK_K, QK_K)
    idx = np.argmax(np.abs(blk), axis=2)
    mxv = np.take_along_axis(blk, idx[:, :, None], axis=2)[:, :, 0]
    zero = mxv == 0
    iscale = np.where(zero, np.float32(0.0), np.float32(-127.0) / np.where(zero, 1, mxv)).astype(np.float32)
    q = np.minimum(_nearest_int(iscale[:, :, None] * blk), 127).astype(np.int8)
    d = np.where(zero, np.float32(0.0), np.float32(1.0) / np.where(zero, 1, iscale)).astype(np.float32)
    return d, q


def q8_k_activation_roundtrip(x: np.ndarray) -> np.ndarray:
    d, q = quantize_q8_k_activations(x)
    rows = d.shape[0]
    return (q.astype(np.float32) * d[:, :, None]).reshape(rows, -1).astype(np.float32)


# --------------------------------------------------------------------------
# Q6_K (weights; activations -> Q8_K like Q4_K)
# --------------------------------------------------------------------------
GROUP_MAX_EPS = np.float32(1e-15)


def _make_qx_quants_rmse1(x: np.ndarray, nmax: int = 32):
    """make_qx_quants(n=16, nmax, x, L, rmse_type=1, qw=NULL) over a batch of sub-blocks
    (ggml-quants.c, restated): weights w = x*x, sequential float sums, 18-point scale search.
    Returns (scale [S] f32, L [S,16] in 0..2*nmax-1)."""
    x = np.asarray(x, dtype=np.float32)
    S, n = x.shape
    ax = np.abs(x)
    # first index of the largest |x| (strict '>' scan from i = 0)
    imax = np.argmax(ax, axis=1)
    amax = ax[np.arange(S), imax]
    mx = x[np.arange(S), imax]
    zero = amax < GROUP_MAX_EPS
    mxs = np.where(zero, np.float32(1.0), mx).astype(np.float32)
    w = x * x

    def quant(iscale):
        lf = _nearest_int(iscale[:, None] * x)
        return np.clip(lf, -nmax, nmax - 1)

    iscale = (np.float32(-nmax) / mxs).astype(np.float32)
    l = quant(iscale)
    L = (l + nmax).astype(np.int32)
    lf = l.astype(np.float32)
    sumlx = _seqsum(w * x * lf)
    suml2 = _seqsum(w * lf * lf)
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.where(suml2 != 0, sumlx / np.where(suml2 != 0, suml2, 1), np.float32(0.0)).astype(np.float32)
    best = (scale * sumlx).astype(np.float32)
    for i_s in range(-9, 10):
        if i_s == 0:
            continue
        isc = (-(np.float32(nmax) + np.float32(0.1) * np.float32(i_s)) / mxs).astype(np.float32)
        l2 = quant(isc)
        lf2 = l2.astype(np.float32)
        slx = _seqsum(w * x * lf2)
        sl2 = _seqsum(w * lf2 * lf2)
        better = (sl2 > 0) & (slx * slx > best * sl2)
        L = np.where(better[:, None], l2 + nmax, L)
        with np.errstate(divide="ignore", invalid="ignore"):
            sc2 = (slx / np.where(sl2 != 0, sl2, 1)).astype(np.float32)
        scale = np.where(better, sc2, scale).astype(np.float32)
        best = np.where(better, (sc2 * slx).astype(np.float32), best).astype(np.float32)
    scale = np.where(zero, np.float32(0.0), scale).astype(np.float32)
    L = np.where(zero[:, None], 0, L)
    return scale, L


def quantize_q6_k_weights(w: np.ndarray) -> np.ndarray:
    """quantize_row_q6_K_ref (no imatrix), restated from the published ggml source
    (parity unpinned; block layout {ql[128], qh[64], int8 scales[16], fp16 d} =
    ggml-metal-embed.metal:329-338).  Returns packed bytes [rows, nb, 210]."""
    w = np.asarray(w, dtype=np.float32)
    rows, k = w.shape
    assert k % QK_K == 0
    nb = k // QK_K
    x = w.reshape(rows * nb, 16, 16)
    scales, L0 = _make_qx_quants_rmse1(x.reshape(-1, 16))
    scales = scales.reshape(-1, 16)
    L0 = L0.reshape(-1, 16, 16)
    ab = np.abs(scales)
    imax = np.argmax(ab, axis=1)
    max_abs = ab[np.arange(len(ab)), imax]
    max_scale = scales[np.arange(len(ab)), imax]
    zero = max_abs < GROUP_MAX_EPS
    iscale = np.where(zero, np.float32(0.0), np.float32(-128.0) / np.where(zero, 1, max_scale)).astype(np.float32)
    with np.errstate(divide="ignore"):
        d = np.where(zero, np.float32(0.0), np.float32(1.0) / np.where(zero, 1, iscale)).astype(np.float16)
    sc = np.minimum(_nearest_int(iscale[:, None] * scales), 127).astype(np.int8)
    dd = d.astype(np.float32)[:, None] * sc.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        lq = _nearest_int(x / np.where(dd != 0, dd, 1)[:, :, None])
    lq = np.clip(lq, -32, 31) + 32
    L = np.where((dd != 0)[:, :, None], lq, L0).astype(np.uint8).reshape(-1, 256)
    ql = np.zeros((len(L), 128), dtype=np.uint8)
    qh = np.zeros((len(L), 64), dtype=np.uint8)
    for h in range(2):
        j = 128 * h
        Lh = L[:, j:j + 128]
        q1, q2, q3, q4 = Lh[:, 0:32], Lh[:, 32:64], Lh[:, 64:96], Lh[:, 96:128]
        ql[:, 64 * h:64 * h + 32] = (q1 & 0xF) | ((q3 & 0xF) << 4)
        ql[:, 64 * h + 32:64 * h + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
        qh[:, 32 * h:32 * h + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    out = np.zeros((len(L), 210), dtype=np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[zero] = 0  # memset(&y[i], 0, sizeof(block_q6_K))
    return out.reshape(rows, nb, 210)


def dequantize_q6_k(raw: np.ndarray) -> np.ndarray:
    """dequantize_row_q6_K: y = d * sc[l/16] * (q - 32) with q = ql nibble | qh 2 bits << 4."""
    raw = np.asarray(raw, dtype=np.uint8)
    rows, nb, _ = raw.shape
    r = raw.reshape(rows * nb, 210)
    ql, qh = r[:, 0:128], r[:, 128:192]
    sc = r[:, 192:208].copy().view(np.int8).astype(np.float32)
    d = r[:, 208:210].copy().view("<f2")[:, 0].astype(np.float32)
    q = np.empty((len(r), 256), dtype=np.float32)
    for h in range(2):
        a, b, hh = ql[:, 64 * h:64 * h + 32], ql[:, 64 * h + 32:64 * h + 64], qh[:, 32 * h:32 * h + 32]
        base = 128 * h
        q[:, base + 0:base + 32] = ((a & 0xF) | (((hh >> 0) & 3) << 4)).astype(np.float32) - 32
        q[:, base + 32:base + 64] = ((b & 0xF) | (((hh >> 2) & 3) << 4)).astype(np.float32) - 32
        q[:, base + 64:base + 96] = ((a >> 4) | (((hh >> 4) & 3) << 4)).astype(np.float32) - 32
        q[:, base + 96:base + 128] = ((b >> 4) | (((hh >> 6) & 3) << 4)).astype(np.float32) - 32
    ds = (d[:, None] * sc).astype(np.float32)  # d * sc[is] first, then * q (float)
    y = ds[:, :, None] * q.reshape(-1, 16, 16)
    return y.reshape(rows, nb * 256).astype(np.float32)


# --------------------------------------------------------------------------
# Weight container with ggml storage semantics
# --------------------------------------------------------------------------
class GgmlWeight:
    """A 2-D ggml weight W [out][in] (ggml ne0 = in).  `values` are the f32 values
    ggml reads (dequantized for quant types); `wtype` selects the vec_dot_type."""

    def __init__(self, values: np.ndarray, wtype: str, raw=None):
        self.values = np.ascontiguousarray(values, dtype=np.float32)
        self.wtype = wtype
        self.raw = raw

    @property
    def shape(self):
        return self.values.shape


def convert_activation(x: np.ndarray, wtype: str) -> np.ndarray:
    if wtype == "bf16":
        return round_bf16(x)
    if wtype == "f16":
        return round_f16(x)
    if wtype == "q8_0":
        return q8_0_activation_roundtrip(x)
    if wtype in ("q4_k", "q6_k"):
        return q8_k_activation_roundtrip(x)
    if wtype == "f32":
        return np.asarray(x, dtype=np.float32)
    raise ValueError(wtype)


# Test-only knob: relative perturbation applied to every f32 product result -- each mul_mat output and, in the
# DiT oracle, the attention scores Q.K^T and the P.V output -- as independent per-element noise
# y * (1 + p * N(0, 1)).  A different f32 summation order changes a dot product by ~1e-7 relative with no
# correlation between elements, so the output's spread under this noise is the floor any
# non-bit-identical implementation of the same graph sits on.  (Round 2 scaled every mul_mat coherently by
# (1 + p): the RMSNorms cancel a coherent scale, and the attention products were not perturbed at all, which
# under-states the floor where the softmax is peaked.)  PERTURB_RNG is re-seeded by the floor helpers.
MULMAT_PERTURB = 0.0
PERTURB_RNG = np.random.default_rng(0)


def perturb(y: np.ndarray) -> np.ndarray:
    """y with the MULMAT_PERTURB noise applied (identity when the knob is 0)."""
    if not MULMAT_PERTURB:
        return y
    noise = PERTURB_RNG.standard_normal(y.shape)
    return (y.astype(np.float64) * (1.0 + MULMAT_PERTURB * noise)).astype(np.float32)


def mul_mat(w: GgmlWeight, x: np.ndarray) -> np.ndarray:
    """ggml_mul_mat(W, x) -> x_conv @ W^T with f32 accumulation."""
    xa = convert_activation(np.asarray(x, dtype=np.float32), w.wtype)
    y = np.matmul(xa, w.values.T).astype(np.float32)
    return perturb(y)


# Optional block encoder (values [rows][K] f32, qtype) -> packed ggml blocks, used by make_weight instead of
# the numpy encoders below.  The tests set it to the product library's C++ encoder (acestep_mi355x.capi.
# quantize) for large K-quant checkpoints, where the numpy make_qkx2_quants search takes minutes: the two
# encoders are byte-identical (tests/test_quant_cpu.py), and the dequantization stays this module's.
QUANTIZER = None


def make_weight(f32_values: np.ndarray, src_dtype: str, qtype: str | None) -> GgmlWeight:
    """`load_tensor_2d_transposed` + `try_quantize_matrix` (acestep_dit_model.cpp:156-192,228-277):
    quantize when a qtype is requested and in_dim % block == 0, else keep the file dtype."""
    v = np.asarray(f32_values, dtype=np.float32)
    if QUANTIZER is not None and qtype in ("q4_k", "q6_k") and v.shape[1] % QK_K == 0:
        raw = np.asarray(QUANTIZER(v, qtype), dtype=np.uint8)
        deq = dequantize_q4_k(raw) if qtype == "q4_k" else dequantize_q6_k(raw)
        return GgmlWeight(deq.reshape(v.shape), qtype, raw=raw)
    if qtype == "q8_0" and v.shape[1] % QK8_0 == 0:
        d, q = quantize_q8_0_weights(v)
        return GgmlWeight(dequantize_q8_0(d, q), "q8_0", raw=pack_q8_0(d, q))
    if qtype == "q4_k" and v.shape[1] % QK_K == 0:
        raw = quantize_q4_k_weights(v)
        return GgmlWeight(dequantize_q4_k(raw), "q4_k", raw=raw)
    if qtype == "q6_k" and v.shape[1] % QK_K == 0:
        raw = quantize_q6_k_weights(v)
        return GgmlWeight(dequantize_q6_k(raw), "q6_k", raw=raw)
    wt = {"BF16": "bf16", "F16": "f16", "F32": "f32"}[src_dtype]
    return GgmlWeight(v, wt)
