"""oracle/cond_oracle.py on the CPU: the packing rule of ace_pack_sequences_single_batch
(acestep_ggml.cpp:1729-1801), the assembly order of the encoder_hidden_states
(acestep_ggml.cpp:2507-2548) and the encoder forwards' structural properties.  No reference fixture
covers the condition encoders, so their numerics are "parity unpinned" beyond the shared DiT pieces
(attention / rms_norm / mul_mat), which the DiT golden vectors pin."""
import tempfile

import numpy as np
import pytest

from oracle import cond_oracle as co


def test_pack_sequences_moves_valid_rows_first_stably():
    h1 = np.arange(4, dtype=np.float32)[:, None] * np.ones((1, 3), np.float32)
    h2 = (10 + np.arange(3, dtype=np.float32))[:, None] * np.ones((1, 3), np.float32)
    h, m = co.pack_sequences_single_batch(h1, np.array([1, 0, 1, 0]), h2, np.array([0, 1, 1]))
    assert h[:, 0].tolist() == [0, 2, 11, 12, 1, 3, 10]
    assert m.tolist() == [1, 1, 1, 1, 0, 0, 0]
    h, m = co.pack_sequences_single_batch(None, None, h2, np.array([1, 1, 0]))
    assert h[:, 0].tolist() == [10, 11, 12] and m.tolist() == [1, 1, 0]   # one side empty: returned as is


@pytest.fixture(scope="module")
def cond_weights():
    from acestep_mi355x.synthetic import TINY_COND_CONFIG, write_checkpoint
    from oracle.dit_oracle import DitWeights
    d = tempfile.mkdtemp(prefix="acemi_cond_")
    write_checkpoint(d, TINY_COND_CONFIG, seed=4, dtype="BF16")
    return DitWeights(d)


def test_condition_order_lyric_timbre_style(cond_weights):
    W = cond_weights
    rng = np.random.default_rng(1)
    sty = rng.standard_normal((5, 256)).astype(np.float32)
    lyr = rng.standard_normal((7, 256)).astype(np.float32)
    refer = rng.standard_normal((2, 6, 64)).astype(np.float32)
    enc, mask = co.build_condition(W, sty, lyr, refer, text_hidden=256)
    assert enc.shape == (14, 256) and mask.tolist() == [1] * 14
    np.testing.assert_array_equal(enc[:7], co.forward_lyric_encoder(W, lyr))
    np.testing.assert_array_equal(enc[7], co.forward_timbre_encoder(W, refer[0]))
    np.testing.assert_array_equal(enc[9:], co.project_tokens_linear(W, sty))


def test_timbre_token_is_first_row_of_the_full_pass(cond_weights):
    """forward_timbre_encoder keeps token 0 of the normed output; attention mixes all tokens, so the
    first row depends on the later frames too."""
    W = cond_weights
    rng = np.random.default_rng(2)
    r = rng.standard_normal((9, 64)).astype(np.float32)
    t = co.forward_timbre_encoder(W, r)
    r2 = r.copy()
    r2[-1] += 1.0
    assert t.shape == (256,) and not np.array_equal(t, co.forward_timbre_encoder(W, r2))


def test_lyric_projection_falls_back_to_text_projector(cond_weights):
    """proj_w = lyric_embed_w ? lyric_embed_w : text_projector_w (no bias), :1577-1578; neither -> failure."""
    import copy
    W = copy.copy(cond_weights)
    W.lyric = dict(cond_weights.lyric, embed=None, embed_b=None)
    x = np.random.default_rng(3).standard_normal((4, 256)).astype(np.float32)
    y = co.forward_lyric_encoder(W, x)
    np.testing.assert_array_equal(y, co.encoder_blocks(W, W.lyric, co.project_tokens_linear(W, x)))
    W.text_proj = None
    with pytest.raises(co.EncoderFailed):
        co.forward_lyric_encoder(W, x)


def test_reference_noise_restatement_matches_the_library_stream():
    """oracle.pipeline_oracle.reference_noise (std::mt19937 + std::normal_distribution<float> restated)
    equals the stream the generate entries draw (ace_mi_reference_noise: host code, no GPU)."""
    from acestep_mi355x import capi
    from oracle.pipeline_oracle import reference_noise
    for seed in (0, 42, -7, 2 ** 31 - 1):
        np.testing.assert_array_equal(capi.reference_noise(seed, 3001), reference_noise(seed, 3001))


def test_shift_schedule_picks_the_nearest_turbo_table():
    from oracle.pipeline_oracle import shift_schedule
    assert shift_schedule(1.0)[1] == np.float32(0.875)
    assert shift_schedule(2.4)[1] == np.float32(0.9333333333)
    assert shift_schedule(2.5)[1] == np.float32(0.9333333333)   # tie d2 == d3 -> s2 (d2 <= d3 first)
    assert shift_schedule(7.0)[7] == np.float32(0.3)
