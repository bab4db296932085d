"""CPU: the text-encoder oracle (oracle/text_oracle.py) pinned against transformers' Qwen3Model -- the model the reference's
own parity harness compares its ggml text encoder with (acestep_ggml/tools/compare_text_encoder.py:133-183).

tests/golden/text_encoder_qwen3.npz holds Qwen3Model's float64 hidden states on the synthetic tiny text checkpoint
(tests/golden/make_text_encoder_fixture.py).  Two checks per case:
  * the restatement's graph: with the weights taken as F32 (ggml then rounds no activation, so the oracle computes the
    same real-number function as the float64 model) it must agree to f32 accuracy -- any misread of the graph (RoPE
    pairing, q/k-norm placement, GQA grouping, causal / padding mask, final norm) shows up as O(1) error;
  * ggml's own BF16 arithmetic (activations rounded to bf16 before each mul_mat): reported with the harness's metrics
    (mean |d|, max |d|, per-token cosine) and bounded, since that distance is what the GPU text encoder's test
    (tests/test_gpu_text_encoder.py) holds the device to."""
import hashlib
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "text_encoder_qwen3.npz")
CASES = ["full37", "full200", "masked37", "masked200", "layer1_37", "layer1_200"]


@pytest.fixture(scope="module")
def fixture_and_weights():
    from acestep_mi355x.synthetic import TEXT_TINY_CONFIG, text_tensor_specs, write_checkpoint
    from oracle import text_oracle as to
    z = np.load(FIX)
    d = tempfile.mkdtemp(prefix="acemi_te_pin_")
    write_checkpoint(d, TEXT_TINY_CONFIG, seed=int(z["seed"]), dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    with open(os.path.join(d, "model.safetensors"), "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == str(z["sha256"]), "synthetic text checkpoint changed: regenerate"
    return z, to.TextWeights(d), d


def as_f32(W):
    """the same (bf16-exact) weight values declared F32: ggml rounds no activation for F32 weights"""
    import copy
    from oracle.ggml_numerics import GgmlWeight
    W2 = copy.deepcopy(W)
    for L in W2.layers:
        for grp in ("self_attn", "mlp"):
            for k, v in L[grp].items():
                if isinstance(v, GgmlWeight):
                    L[grp][k] = GgmlWeight(v.values, "f32")
    return W2


def run(to, W, z, case):
    ids = z[f"{case}/ids"]
    mask = z[f"{case}/mask"] if f"{case}/mask" in z.files else None
    if case.startswith("layer1"):
        return to.forward_text_encoder_layers(W, ids, None, 1, True)
    return to.forward_text_encoder_layers(W, ids, mask)


def metrics(got, ref):
    got64, ref64 = got.astype(np.float64), ref.astype(np.float64)
    l2 = float(np.linalg.norm(got64 - ref64) / np.linalg.norm(ref64))
    cos = [float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b))) for a, b in zip(got64, ref64)]
    return l2, float(np.mean(np.abs(got64 - ref64))), float(np.max(np.abs(got64 - ref64))), float(np.min(cos))


@pytest.mark.parametrize("case", CASES)
def test_text_oracle_graph_matches_qwen3model(fixture_and_weights, case):
    from oracle import text_oracle as to
    z, W, _ = fixture_and_weights
    got = run(to, as_f32(W), z, case)
    l2, mae, mx, cmin = metrics(got, z[f"{case}/out"])
    print(f"{case}: F32 restatement vs Qwen3Model(float64) rel_l2={l2:.2e} mae={mae:.2e} max={mx:.2e} cos_min={cmin:.9f}")
    assert l2 < 2e-6, l2


@pytest.mark.parametrize("case", CASES)
def test_text_oracle_ggml_bf16_arithmetic_vs_qwen3model(fixture_and_weights, case):
    from oracle import text_oracle as to
    z, W, _ = fixture_and_weights
    got = run(to, W, z, case)
    l2, mae, mx, cmin = metrics(got, z[f"{case}/out"])
    print(f"{case}: ggml BF16 semantics vs Qwen3Model(float64) rel_l2={l2:.2e} mae={mae:.2e} max={mx:.2e} "
          f"cos_min={cmin:.7f}")
    assert l2 < 1e-2 and cmin > 0.9999, (l2, cmin)
