"""GGUF export/import path (acestep_dit_model.cpp:47-99,492-718; export_safetensors_to_gguf.py:154-281):
the synthetic exporter's files read back by the oracle's independent GGUF reader, with the
reference's type rules (>= 2-D tensors whose last dim is a block multiple quantized, rest F16; conv
weights converted to F32 by the loader)."""
import os
import shutil
import tempfile

import numpy as np
import pytest

from oracle import ggml_numerics as g
from oracle.dit_oracle import DitWeights, read_gguf, read_safetensors


@pytest.fixture(scope="module")
def tiny_dir():
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_gguf_")
    write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
    return d


@pytest.mark.parametrize("quant,gt", [("Q8", 8), ("Q4", 12), ("Q6", 14), ("F16", 1)])
def test_gguf_export_types_and_values(tiny_dir, quant, gt):
    from acestep_mi355x.synthetic import write_gguf
    path = os.path.join(tempfile.mkdtemp(), "model.gguf")
    write_gguf(os.path.join(tiny_dir, "model.safetensors"), path, quant=quant)
    st = read_safetensors(os.path.join(tiny_dir, "model.safetensors"))
    gg = read_gguf(path)
    assert set(gg) == set(st)
    blk = {8: 32, 12: 256, 14: 256, 1: 1}[gt]
    for name, (dt, shape, v) in st.items():
        t, ne, raw = gg[name]
        assert list(reversed(ne)) == list(shape)
        quantized = gt != 1 and len(shape) >= 2 and shape[-1] % blk == 0
        assert t == (gt if quantized else 1), name
    # a quantized matrix decodes to the oracle's quantization of the same values
    name = "decoder.layers.0.mlp.down_proj.weight"
    t, ne, raw = gg[name]
    w = st[name][2].reshape(ne[1], ne[0]).astype(np.float32)
    ref = g.make_weight(w, "BF16", {8: "q8_0", 12: "q4_k", 14: "q6_k", 1: None}[gt])
    if gt != 1:
        assert bytes(ref.raw.tobytes()) == raw
    else:
        np.testing.assert_array_equal(np.frombuffer(raw, "<f2").astype(np.float32).reshape(w.shape),
                                      w.astype(np.float16).astype(np.float32))


def test_gguf_weights_follow_reference_types(tiny_dir):
    from acestep_mi355x.synthetic import write_gguf
    path = os.path.join(tempfile.mkdtemp(), "model.gguf")
    write_gguf(os.path.join(tiny_dir, "model.safetensors"), path, quant="Q8")
    W = DitWeights(tiny_dir, gguf=path)
    assert W.proj_in_w.wtype == "f32" and W.proj_out_w.wtype == "f32"      # conv weights -> F32
    assert W.layers[0]["mlp"]["down"].wtype == "q8_0"
    assert W.condition_w.wtype == "q8_0"
    # 1-D tensors were exported F16: the loaded f32 values are fp16-exact
    v = W.layers[0]["self_attn_norm"]
    np.testing.assert_array_equal(v, v.astype(np.float16).astype(np.float32))
