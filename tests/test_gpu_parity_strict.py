"""Discriminating parity at full width ("Next round" item 1).

* Peaked attention.  The synthetic checkpoints' q_norm / k_norm weights are ~1, so post-norm logits
  q.k/sqrt(128) are ~N(0, 1): a near-uniform softmax in which fp16 score errors average out.  Trained
  checkpoints have logits of tens.  `qk_norm_scale = 3` multiplies those norm weights (synthetic.py), giving
  logits with |s| up to ~40 and a row maximum of ~30 (top-1 probability ~0.7, ~2 effective keys: asserted
  below from the oracle's own q / k), and the 240 s forward (T = 6000, N = 3000, L = 512, 2 layers: one
  sliding, one full) is checked against the oracle -- whose attention is f32 like ggml's
  (`ggml_mul_mat_set_prec(kq, GGML_PREC_F32)`, acestep_dit_model.cpp:1238-1251) -- in every attention
  precision mode of the engine: fp16 operands, `split` (hi/lo fp16 Q.K, fp16 P.V) and `f32` (hi/lo both).
* One layer.  Depth amplifies the bf16 activation-rounding floor; after one full-width layer
  it has not accumulated yet, so the north-star bound is asserted literally there wherever the oracle's own
  floor leaves room for it (rel-L2 <= max(1e-3, floor)), for a sliding and a full-attention first layer, with
  and without peaked logits, in the fp16 (default) and f32 attention modes.
* Negative control.  ACE_MI_TEST_FAULT (test-only engine hook of the self-test library, restated in the oracle as
  dit_oracle.FAULT) adds 0.015 to one 16 x 128 tile of the residual after layer 1's o-projection -- one row
  group of one GEMM output tile, a ~4 % error on 16 of 3000 tokens.  The rel-L2 bound absorbs it (the test
  asserts that it does); the element-wise bound max|d| / rms <= 2.5 x its floor must catch it.
"""
import math
import os

import numpy as np
import pytest

from test_gpu_forward import MAXABS_K, REL_L2, check, maxabs_rms, rel_errors

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

T240, L240 = 6000, 512
QK_SCALE = 3.0
FAULT = (1, 1500, 512, 0.015)
_REFS = {}


def _inputs(seed=1234, T=T240, L=L240):
    rng = np.random.default_rng(seed)
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = np.concatenate([rng.standard_normal((T, 64)), np.ones((T, 64))], axis=1).astype(np.float32)
    e = rng.standard_normal((L, 2048)).astype(np.float32)
    return h, c, e


def _ckpt(scale, layer_types=None):
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    kw = dict(num_hidden_layers=2)
    if layer_types:
        kw["layer_types"] = layer_types
    return cached_checkpoint(make_config(**kw), seed=0, backend="torch", qk_norm_scale=scale)


def _oracle(d, layers, t=0.9):
    """(ref, floor_l2, floor_maxabs) of the oracle at 240 s, cached per (checkpoint, layers)."""
    from oracle.dit_oracle import DitWeights, forward_with_floor_stats
    key = (d, layers, t)
    if key not in _REFS:
        h, c, e = _inputs()
        _REFS[key] = forward_with_floor_stats(DitWeights(d), h, c, e, None, None, T240, L240, t, t,
                                              max_layers=layers)
    return _REFS[key]


def _gpu(d, layers, monkeypatch, precision=None, fault=None, t=0.9):
    from acestep_mi355x.capi import GGMLCAPIBridge, selftest_library_path
    monkeypatch.setenv("ACE_GGML_DIT_MAX_LAYERS", str(layers))
    if precision:
        monkeypatch.setenv("ACE_MI_ATTN_PRECISION", precision)
    else:
        monkeypatch.delenv("ACE_MI_ATTN_PRECISION", raising=False)
    if fault:
        monkeypatch.setenv("ACE_MI_TEST_FAULT", ",".join(str(v) for v in fault))
    else:
        monkeypatch.delenv("ACE_MI_TEST_FAULT", raising=False)
    h, c, e = _inputs()
    # the fault hook is read by the self-test library only (runtime/test_hooks.cpp)
    br = GGMLCAPIBridge(lib_path=selftest_library_path()) if fault else GGMLCAPIBridge()
    try:
        br.load_dit(d)
        return br.dit_forward_tfirst(h, c, e, None, None, t, t)
    finally:
        br.close()


def _logit_stats(d, layer=1, t=0.9):
    """Pre-softmax self-attention logits of `layer`'s weights (q head 0 vs its kv head, every 25th query) on
    the 240 s inputs' proj_in output, from the oracle's own pieces: (max |s|, mean row max, mean top-1
    probability).  Post-norm logits scale with the q/k norm weights, not with the block input."""
    from oracle.dit_oracle import DitWeights, apply_rope_neox, mul_mat, rms_norm, rope_tables, timestep_forward
    W = DitWeights(d)
    cfg = W.cfg
    h, c, _ = _inputs()
    Np = T240 // 2
    x = mul_mat(W.proj_in_w, np.concatenate([c, h], axis=1).reshape(Np, 2 * cfg.in_channels)) + W.proj_in_b
    _, pt = timestep_forward(W.time_embed["time_embed"], t)
    _, pr = timestep_forward(W.time_embed["time_embed_r"], np.float32(0.0))
    Ly = W.layers[layer]
    mod = Ly["table"] + pt + pr
    n = rms_norm(x, Ly["self_attn_norm"], cfg.rms_norm_eps) * (mod[1] + 1) + mod[0]
    q = rms_norm(mul_mat(Ly["self_attn"]["q"], n).reshape(Np, 16, 128), Ly["self_attn"]["q_norm"], cfg.rms_norm_eps)
    k = rms_norm(mul_mat(Ly["self_attn"]["k"], n).reshape(Np, 8, 128), Ly["self_attn"]["k_norm"], cfg.rms_norm_eps)
    cs, sn = rope_tables(Np, 128, cfg.rope_theta)
    q, k = apply_rope_neox(q, cs, sn), apply_rope_neox(k, cs, sn)
    s = (q[::25, 0] @ k[:, 0].T) / math.sqrt(128)
    p = np.exp(s - s.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    return float(np.abs(s).max()), float(s.max(1).mean()), float(p.max(1).mean())


def test_peaked_regime_is_peaked():
    """The peaked checkpoint really is in the trained-model regime (|logit| of tens, a few dominant keys);
    the default checkpoint is not.  Oracle arithmetic only (numpy)."""
    smax, rowmax, top1 = _logit_stats(_ckpt(QK_SCALE))
    print(f"peaked (qk_norm x{QK_SCALE}): max|s|={smax:.1f} mean row max={rowmax:.1f} top-1 p={top1:.3f}")
    assert smax >= 30 and rowmax >= 20 and top1 >= 0.5
    smax1, rowmax1, top11 = _logit_stats(_ckpt(1.0))
    print(f"default: max|s|={smax1:.1f} mean row max={rowmax1:.1f} top-1 p={top11:.3f}")
    assert smax1 < 8 and top11 < 0.05


@pytest.mark.parametrize("precision", ["fp16", "split", "f32", "f8c", "pv8"])
def test_peaked_attention_240s_two_layers(monkeypatch, precision):
    """240 s, full width, 2 layers, peaked logits, each attention precision mode vs the f32 oracle."""
    d = _ckpt(QK_SCALE)
    ref, floor, fmax = _oracle(d, 2)
    got = _gpu(d, 2, monkeypatch, precision)
    check(got, ref, floor, f"peaked 240 s 2 layers, attention {precision}", fmax)


@pytest.mark.parametrize("precision", ["fp16", "split", "f32", "f8c", "pv8"])
@pytest.mark.parametrize("peaked", [False, True], ids=["default", "peaked"])
@pytest.mark.parametrize("first", ["sliding_attention", "full_attention"])
def test_one_layer_literal_bound(monkeypatch, first, peaked, precision):
    """One full-width layer at 240 s, before depth amplifies the bf16 activation-rounding floor: the element-wise
    and L2 bounds against the floor, and the north-star literal rel-L2 <= 1e-3 wherever the oracle's own spread
    under 1e-7 summation noise (the floor) leaves room for it -- measured: at one layer that spread is already
    ~1.1e-3 (default logits) and ~3.7e-3 (peaked), i.e. no f32 re-implementation of the graph can be held to a
    literal 1e-3 there; the test asserts the floor itself so that statement stays checked."""
    other = "full_attention" if first == "sliding_attention" else "sliding_attention"
    d = _ckpt(QK_SCALE if peaked else 1.0, [first, other])
    ref, floor, fmax = _oracle(d, 1)
    got = _gpu(d, 1, monkeypatch, precision)
    tag = f"1 layer ({first}, {'peaked' if peaked else 'default'}, attention {precision}) 240 s"
    l2 = check(got, ref, floor, tag, fmax)
    print(f"{tag}: literal 1e-3 {'met' if l2 <= REL_L2 else 'not met'} (rel_l2 {l2:.3e}, oracle floor {floor:.3e})")
    assert l2 <= max(REL_L2, floor), (l2, floor)
    assert floor >= (2.5e-3 if peaked else 0.8e-3), floor  # the claim in the docstring
def test_fault_injection_is_caught(monkeypatch):
    """Negative control: one corrupted 16 x 128 tile of one GEMM output passes the rel-L2 bound but fails the
    element-wise bound; the oracle with the same fault restated agrees with the faulted GPU output."""
    from oracle import dit_oracle
    d = _ckpt(1.0)
    ref, floor, fmax = _oracle(d, 2)
    clean = _gpu(d, 2, monkeypatch)
    check(clean, ref, floor, "negative control: clean run", fmax)
    bad = _gpu(d, 2, monkeypatch, fault=FAULT)
    l2, _ = rel_errors(bad, ref)
    ma = maxabs_rms(bad, ref)
    print(f"faulted: rel_l2={l2:.3e} (bound {max(REL_L2, 1.5 * floor):.3e}) maxabs/rms={ma:.3e} "
          f"(bound {MAXABS_K * fmax:.3e}, ratio {ma / fmax:.2f})")
    assert l2 <= max(REL_L2, 1.5 * floor), "the L2 bound alone would have caught it: raise the control's subtlety"
    with pytest.raises(AssertionError):
        check(bad, ref, floor, "negative control: faulted run", fmax)
    # the faulted GPU output is the oracle's faulted output (so the check fails because of the fault only)
    h, c, e = _inputs()
    dit_oracle.FAULT = FAULT
    try:
        fref = dit_oracle.forward_dit(dit_oracle.DitWeights(d), h, c, e, None, None, T240, L240, 0.9, 0.9,
                                      max_layers=2)
    finally:
        dit_oracle.FAULT = None
    check(bad, fref, floor, "faulted GPU vs faulted oracle", fmax)
