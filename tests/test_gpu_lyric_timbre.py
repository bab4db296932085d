"""GPU parity of the condition encoders through the C-ABI: lyric encoder, batched
timbre encoder, text projector and the packed encoder_hidden_states of ace_mi_build_condition against
oracle/cond_oracle.py (same bound as the DiT: rel_l2 <= max(1e-3, 1.5 x the oracle's own
perturbation floor), cos >= 0.99999)."""
import tempfile

import numpy as np
import pytest

from test_gpu_forward import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cond_ckpt():
    from acestep_mi355x.synthetic import TINY_COND_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_gc_")
    write_checkpoint(d, TINY_COND_CONFIG, seed=4, dtype="BF16")
    return d


@pytest.fixture(scope="module")
def cond_bridge(cond_ckpt):
    from acestep_mi355x.capi import GGMLCAPIBridge
    br = GGMLCAPIBridge()
    br.load_dit(cond_ckpt)
    yield br
    br.close()


@pytest.mark.parametrize("n", [1, 45, 300])
def test_lyric_encoder(cond_ckpt, cond_bridge, n):
    from oracle import cond_oracle as co
    from oracle.dit_oracle import DitWeights
    x = np.random.default_rng(n).standard_normal((n, 256)).astype(np.float32)
    ref, floor = co.encode_with_floor(co.forward_lyric_encoder, DitWeights(cond_ckpt), x)
    check(cond_bridge.lyric_encode(x), ref, floor, f"lyric n={n}")


def test_timbre_encoder_batched(cond_ckpt, cond_bridge):
    from oracle import cond_oracle as co
    from oracle.dit_oracle import DitWeights
    W = DitWeights(cond_ckpt)
    refer = np.random.default_rng(5).standard_normal((3, 150, 64)).astype(np.float32)
    got = cond_bridge.timbre_encode(refer)
    for i in range(3):
        ref, floor = co.encode_with_floor(co.forward_timbre_encoder, W, refer[i])
        check(got[i], ref, floor, f"timbre {i}")


def test_build_condition(cond_ckpt, cond_bridge):
    from oracle import cond_oracle as co
    from oracle.dit_oracle import DitWeights
    W = DitWeights(cond_ckpt)
    rng = np.random.default_rng(6)
    sty = rng.standard_normal((20, 256)).astype(np.float32)
    lyr = rng.standard_normal((60, 256)).astype(np.float32)
    refer = rng.standard_normal((2, 40, 64)).astype(np.float32)
    enc, mask = cond_bridge.build_condition(sty, lyr, refer)
    ref, mref = co.build_condition(W, sty, lyr, refer, text_hidden=256)
    _, floor = co.encode_with_floor(co.forward_lyric_encoder, W, lyr)
    assert np.array_equal(mask, mref)
    check(enc, ref, floor, "build_condition")
    np.testing.assert_allclose(cond_bridge.text_project(sty), co.project_tokens_linear(W, sty), rtol=2e-5, atol=1e-5)
