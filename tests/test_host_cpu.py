"""Host-side logic without a GPU: the decoder.forward hook plumbing (with a recording fake bridge),
shard assignment, and the synthetic checkpoint format."""
import json
import os
import struct
import tempfile
import types

import numpy as np
import pytest
import torch

from acestep_mi355x import hook
from acestep_mi355x.sampler import shard_indices
from acestep_mi355x.synthetic import TINY_CONFIG, tensor_specs, write_checkpoint


class FakeBridge:
    """Records host-path calls; returns hidden + t so results are checkable."""

    def __init__(self):
        self.calls = []

    def dit_forward_tfirst(self, hs, ctx, enc, am, eam, t, r):
        self.calls.append(dict(hs=hs.copy(), ctx=ctx.copy(), enc=enc.copy(), am=am.copy(), eam=eam.copy(), t=t, r=r))
        return hs + np.float32(t)


def make_handler():
    dec = types.SimpleNamespace()
    dec.forward = lambda **kw: ("original", kw)
    return types.SimpleNamespace(model=types.SimpleNamespace(decoder=dec))


def test_hook_replaces_decoder_forward_and_marks_handler():
    h = make_handler()
    br = FakeBridge()
    hook.install_dit_backend(h, br)
    assert h._ggml_dit_backend == "mi355x-capi" and h._ggml_dit_decoder_forward_hooked
    B, T, L = 3, 10, 4
    hs = torch.randn(B, T, 64, dtype=torch.bfloat16)
    ctx = torch.randn(B, T, 128)
    enc = torch.randn(B, L, 32)
    am = torch.ones(B, T, dtype=torch.long)
    am[1, 7:] = 0
    t = torch.tensor([1.0, 0.5, 0.25])
    out = h.model.decoder.forward(hidden_states=hs, timestep=t, timestep_r=t, attention_mask=am,
                                  encoder_hidden_states=enc, encoder_attention_mask=None, context_latents=ctx,
                                  past_key_values="pkv", output_attentions=True)
    pred, pkv, attn = out
    assert pkv == "pkv" and attn is None and pred.dtype == torch.bfloat16 and pred.shape == (B, T, 64)
    assert len(br.calls) == B
    for b, c in enumerate(br.calls):
        assert c["t"] == pytest.approx(float(t[b])) and c["r"] == pytest.approx(float(t[b]))
        np.testing.assert_array_equal(c["am"], (am[b] > 0).numpy().astype(np.int32))
        np.testing.assert_array_equal(c["eam"], np.ones(L, np.int32))
        np.testing.assert_array_equal(c["hs"], hs[b].float().numpy())
    np.testing.assert_allclose(pred.float().numpy(), (hs.float() + t[:, None, None]).to(torch.bfloat16).float().numpy())


def test_hook_scalar_timestep_and_non3d_passthrough():
    h = make_handler()
    br = FakeBridge()
    hook.install_dit_backend(h, br)
    hs = torch.zeros(2, 4, 64)
    out = h.model.decoder.forward(hidden_states=hs, timestep=torch.tensor(0.3), timestep_r=0.3,
                                  attention_mask=None, encoder_hidden_states=torch.zeros(2, 3, 8),
                                  encoder_attention_mask=None, context_latents=torch.zeros(2, 4, 128))
    assert len(out) == 2 and [c["t"] for c in br.calls] == pytest.approx([0.3, 0.3])
    res = h.model.decoder.forward(hidden_states=torch.zeros(4, 64), timestep=0.3, timestep_r=0.3,
                                  attention_mask=None, encoder_hidden_states=None, encoder_attention_mask=None,
                                  context_latents=None)
    assert res[0] == "original"


@pytest.mark.parametrize("B,W", [(1, 1), (8, 8), (8, 3), (5, 2), (16, 8)])
def test_shards_partition_the_batch(B, W):
    seen = sorted(b for r in range(W) for b in shard_indices(B, W, r))
    assert seen == list(range(B))
    sizes = [len(shard_indices(B, W, r)) for r in range(W)]
    assert max(sizes) - min(sizes) <= 1


def test_synthetic_checkpoint_format():
    with tempfile.TemporaryDirectory() as d:
        write_checkpoint(d, TINY_CONFIG, seed=3)
        cfg = json.load(open(os.path.join(d, "config.json")))
        assert cfg["layer_types"] == ["sliding_attention", "full_attention"]
        with open(os.path.join(d, "model.safetensors"), "rb") as f:
            (n,) = struct.unpack("<Q", f.read(8))
            header = json.loads(f.read(n))
        specs = list(tensor_specs(TINY_CONFIG))
        assert set(header) == {s[0] for s in specs}
        for name, shape, _ in specs:
            assert header[name]["shape"] == list(shape) and header[name]["dtype"] == "BF16"
        assert os.path.getsize(os.path.join(d, "model.safetensors")) == 8 + n + max(
            v["data_offsets"][1] for v in header.values())


def test_text_encoder_hook_routes_rows_through_the_bridge():
    """install_text_encoder_backend mirrors _install_ggml_text_encoder_backend
    (scripts/run_non_ggml_real_case.py:406-428): one bridge call per row, stacked, moved to the
    handler's device/dtype."""
    calls = []

    class TB:
        def text_forward_full(self, ids, hidden):
            calls.append(("full", ids.tolist(), hidden))
            return np.tile(ids[:, None].astype(np.float32), (1, hidden))

        def text_forward_embeddings(self, ids, hidden):
            calls.append(("emb", ids.tolist(), hidden))
            return -np.tile(ids[:, None].astype(np.float32), (1, hidden))

    h = types.SimpleNamespace(text_encoder=types.SimpleNamespace(config=types.SimpleNamespace(hidden_size=8)),
                              device="cpu", dtype=torch.bfloat16)
    hook.install_text_encoder_backend(h, TB())
    out = h.infer_text_embeddings(torch.tensor([[1, 2, 3], [4, 5, 6]]))
    assert out.shape == (2, 3, 8) and out.dtype == torch.bfloat16 and float(out[1, 2, 0]) == 6.0
    lyr = h.infer_lyric_embeddings([[7, 8]])
    assert lyr.shape == (1, 2, 8) and float(lyr[0, 1, 3]) == -8.0
    assert [c[0] for c in calls] == ["full", "full", "emb"] and calls[0][1:] == ([1, 2, 3], 8)
