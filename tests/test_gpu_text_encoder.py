"""GPU parity of the Qwen3 text encoder through the reference ABI
(ace_ggml_load_text_encoder, ace_ggml_text_encoder_forward[_masked|_layers|_embeddings]) against
oracle/text_oracle.py, and the causal mode of the attention kernel against an fp64 reference."""
import tempfile

import numpy as np
import pytest

from test_gpu_forward import check

pytestmark = pytest.mark.gpu


def _causal_ref(q, kv, hq, hkv, kmask, scale):
    B, nq, _ = q.shape
    D = 128
    k = kv[:, :, :hkv * D].reshape(B, nq, hkv, D).astype(np.float64)
    v = kv[:, :, hkv * D:].reshape(B, nq, hkv, D).astype(np.float64)
    qh = q.reshape(B, nq, hq, D).astype(np.float64)
    out = np.zeros((B, nq, hq, D))
    allow = np.tril(np.ones((nq, nq), bool))
    for b in range(B):
        al = allow & (kmask[b][None, :] != 0) if kmask is not None else allow
        for h in range(hq):
            s = np.where(al, qh[b, :, h] @ k[b, :, h * hkv // hq].T * scale, -np.inf)
            p = np.exp(s - s.max(axis=1, keepdims=True))
            out[b, :, h] = (p / p.sum(axis=1, keepdims=True)) @ v[b, :, h * hkv // hq]
    return out.reshape(B, nq, hq * D)


@pytest.mark.parametrize("B,hq,hkv,n,masked", [(1, 2, 1, 64, False), (2, 16, 8, 300, False), (1, 4, 2, 257, True),
                                              (1, 4, 1, 31, False)])
def test_causal_attention_kernel(B, hq, hkv, n, masked):
    from acestep_mi355x import capi
    rng = np.random.default_rng(n + hq)
    q = rng.standard_normal((B, n, hq * 128)).astype(np.float32) * 2.0
    kv = rng.standard_normal((B, n, 2 * hkv * 128)).astype(np.float32) * 0.3
    kmask = None
    if masked:
        kmask = (rng.random((B, n)) > 0.3).astype(np.int32)
        kmask[:, 0] = 1
    scale = 1.0 / np.sqrt(128.0)
    got = capi.kernel_attention(q, kv, hq, hkv, kmask=kmask, scale=scale, split=True, causal=True)
    ref = _causal_ref(q, kv, hq, hkv, kmask, scale)
    err = np.abs(got - ref)
    assert np.all(err <= 2.0 ** -8 * np.abs(ref) + 1e-5), float(err.max())


@pytest.fixture(scope="module")
def text_ckpt():
    from acestep_mi355x.synthetic import TEXT_TINY_CONFIG, text_tensor_specs, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_gt_")
    write_checkpoint(d, TEXT_TINY_CONFIG, seed=6, dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    return d


@pytest.fixture(scope="module")
def text_bridge(text_ckpt):
    from acestep_mi355x.capi import GGMLCAPIBridge
    br = GGMLCAPIBridge()
    br.load_text_encoder(text_ckpt)
    yield br
    br.close()


@pytest.mark.parametrize("n", [1, 37, 200])
def test_text_encoder_forward(text_ckpt, text_bridge, n):
    from oracle import text_oracle as to
    W = to.TextWeights(text_ckpt)
    ids = np.random.default_rng(n).integers(0, 1000, n).astype(np.int32)
    np.testing.assert_array_equal(text_bridge.text_encoder_embeddings(ids), to.forward_text_encoder_embeddings(W, ids))
    ref, floor = to.forward_with_floor(W, ids)
    check(text_bridge.text_encoder_forward(ids), ref, floor, f"text n={n}")
    if n > 8:
        mask = np.ones(n, np.int32)
        mask[n - 5:] = 0
        ref, floor = to.forward_with_floor(W, ids, mask)
        check(text_bridge.text_encoder_forward(ids, mask), ref, floor, f"text masked n={n}")
        ref, floor = to.forward_with_floor(W, ids, None, 1, True)
        check(text_bridge.text_encoder_forward(ids, None, n_layers=1), ref, floor, f"text 1 layer n={n}")


def test_text_encoder_prefix_causality(text_bridge):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 1000, 150).astype(np.int32)
    b = a.copy()
    b[140:] = rng.integers(0, 1000, 10)
    np.testing.assert_array_equal(text_bridge.text_encoder_forward(a)[:140], text_bridge.text_encoder_forward(b)[:140])
