"""Weight-loader layouts checked on the CPU: runtime/{model,vae,quant,gguf}.cpp are compiled with the
host compiler against stub HIP memory functions (tests/host/loader_dump.cpp), load checkpoints exactly
as ace_ggml_load_dit / ace_ggml_load_vae do, and every device buffer is compared with the layout the
kernels assume, built here from the oracle's view of the same files."""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT
from oracle import ggml_numerics as g
from oracle.dit_oracle import read_safetensors

CSRC = os.path.join(ROOT, "ace-step-1.5-ggml_amd", "csrc")
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.fixture(scope="module")
def dumper():
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    out = os.path.join(tempfile.mkdtemp(prefix="acemi_ld_"), "loader_dump")
    srcs = [os.path.join(ROOT, "tests", "host", "loader_dump.cpp")] + [
        os.path.join(CSRC, "runtime", f) for f in ("json.cpp", "gguf.cpp", "quant.cpp", "model.cpp", "vae.cpp")]
    subprocess.run([CLANG, "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I" + CSRC,
                    "-ffp-contract=off", "-pthread", "-Wno-unused-result", *srcs, "-o", out], check=True)
    return out


def run_dump(dumper, kind, model_dir, env=None):
    out = tempfile.mkdtemp(prefix="acemi_dump_")
    e = dict(os.environ)
    for k in ("ACE_GGML_DIT_WEIGHT_QTYPE", "ACE_GGML_WEIGHT_QTYPE", "ACE_GGML_DIT_GGUF", "ACE_GGML_DIT_GGUF_PATH"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([dumper, kind, model_dir, out], env=e, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    idx = {}
    for line in open(os.path.join(out, "index.txt")):
        parts = line.split()
        idx[parts[0]] = parts[1:]
    return out, idx


def load_w(out, idx, name):
    fmt, rows, cols = (int(x) for x in idx[name][1:4])
    q = np.fromfile(os.path.join(out, name + ".q.bin"), np.uint8)
    sp = os.path.join(out, name + ".s.bin")
    s = np.fromfile(sp, np.float32) if os.path.exists(sp) else None
    return fmt, rows, cols, q, s


def to_planes(qtype, raw, rows, cols):
    """runtime/quant.h plane layout from ggml block bytes [rows][nb][bb]."""
    if qtype == "q8_0":
        d, q = g.unpack_q8_0(raw)
        return q.reshape(rows, cols).view(np.uint8).ravel(), d.astype(np.float32).ravel()
    if qtype == "q6_k":
        vals = g.dequantize_q6_k(raw)  # only for the scale check; q from the bit layout below
        r = raw.reshape(-1, 210)
        ql, qh = r[:, 0:128], r[:, 128:192]
        q = np.empty((len(r), 256), np.int16)
        for h in range(2):
            a, b, hh = ql[:, 64 * h:64 * h + 32], ql[:, 64 * h + 32:64 * h + 64], qh[:, 32 * h:32 * h + 32]
            base = 128 * h
            q[:, base:base + 32] = (a & 0xF) | (((hh >> 0) & 3) << 4)
            q[:, base + 32:base + 64] = (b & 0xF) | (((hh >> 2) & 3) << 4)
            q[:, base + 64:base + 96] = (a >> 4) | (((hh >> 4) & 3) << 4)
            q[:, base + 96:base + 128] = (b >> 4) | (((hh >> 6) & 3) << 4)
        sc = r[:, 192:208].copy().view(np.int8).astype(np.float32)
        d = r[:, 208:210].copy().view("<f2")[:, 0].astype(np.float32)
        return (q - 32).astype(np.int8).view(np.uint8).ravel(), (d[:, None] * sc).astype(np.float32).ravel()
    # q4_k
    r = raw.reshape(-1, 144)
    d = r[:, 0:2].copy().view("<f2")[:, 0].astype(np.float32)
    dmin = r[:, 2:4].copy().view("<f2")[:, 0].astype(np.float32)
    scv, mv = g._q4k_scale_min(r[:, 4:16])
    qs = r[:, 16:]
    vals = np.empty((len(r), 256), np.uint8)
    for j in range(4):
        vals[:, 64 * j:64 * j + 32] = qs[:, 32 * j:32 * j + 32] & 0xF
        vals[:, 64 * j + 32:64 * j + 64] = qs[:, 32 * j:32 * j + 32] >> 4
    v8 = vals.reshape(-1, 8, 32)
    kk = np.array([8 * (i // 4) + (i % 4) for i in range(16)])
    nib = (v8[:, :, kk] | (v8[:, :, kk + 4] << 4)).astype(np.uint8)
    s = np.stack([(d[:, None] * scv.astype(np.float32)), (dmin[:, None] * mv.astype(np.float32))], axis=-1)
    return nib.ravel(), s.astype(np.float32).ravel()


def bits16(st, name):
    dt, shape, v = st[name]
    assert dt == "BF16"
    return g.f32_to_bf16_bits(v.reshape(shape).astype(np.float32))


@pytest.fixture(scope="module")
def tiny():
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_ldt_")
    write_checkpoint(d, TINY_CONFIG, seed=3, dtype="BF16")
    return d, TINY_CONFIG


def test_dense_bf16_layouts(dumper, tiny):
    d, cfg = tiny
    out, idx = run_dump(dumper, "dit", d)
    st = read_safetensors(os.path.join(d, "model.safetensors"))
    H, I, P, Cin, A = cfg["hidden_size"], cfg["intermediate_size"], cfg["patch_size"], cfg["in_channels"], 64
    fmt, rows, cols, q, _ = load_w(out, idx, "l1.qkv")
    assert fmt == 0
    p = "decoder.layers.1.self_attn."
    exp = np.concatenate([bits16(st, p + "q_proj.weight"), bits16(st, p + "k_proj.weight"),
                          bits16(st, p + "v_proj.weight")])
    np.testing.assert_array_equal(q.view(np.uint16).reshape(rows, cols), exp)
    # gate|up interleaved in groups of 16 rows
    gate = bits16(st, "decoder.layers.0.mlp.gate_proj.weight")
    up = bits16(st, "decoder.layers.0.mlp.up_proj.weight")
    fmt, rows, cols, q, _ = load_w(out, idx, "l0.gu")
    gu = q.view(np.uint16).reshape(rows, cols)
    for r in range(2 * I):
        grp, w = divmod(r, 32)
        src = gate if w < 16 else up
        np.testing.assert_array_equal(gu[r], src[grp * 16 + w % 16])
    # proj_in [H][P*Cin]: column k*Cin + c = w[o][c][k]
    w = bits16(st, "decoder.proj_in.1.weight").reshape(H, Cin, P)
    fmt, rows, cols, q, _ = load_w(out, idx, "proj_in")
    np.testing.assert_array_equal(q.view(np.uint16).reshape(rows, cols), w.transpose(0, 2, 1).reshape(H, P * Cin))
    # proj_out [(o + k*A)][H] = w[i][o][k]
    w = bits16(st, "decoder.proj_out.1.weight").reshape(H, A, P)
    fmt, rows, cols, q, _ = load_w(out, idx, "proj_out")
    np.testing.assert_array_equal(q.view(np.uint16).reshape(rows, cols), w.transpose(2, 1, 0).reshape(P * A, H))
    tables = np.fromfile(os.path.join(out, "tables.bin"), np.float32).reshape(cfg["num_hidden_layers"], 6, H)
    np.testing.assert_array_equal(tables[1], st["decoder.layers.1.scale_shift_table"][2].reshape(6, H))


@pytest.mark.parametrize("qtype", ["q8_0", "q4_k", "q6_k"])
def test_online_quantized_planes(dumper, tiny, qtype):
    d, cfg = tiny
    out, idx = run_dump(dumper, "dit", d, {"ACE_GGML_DIT_WEIGHT_QTYPE": qtype})
    st = read_safetensors(os.path.join(d, "model.safetensors"))
    H = cfg["hidden_size"]
    wf = {"q8_0": 2, "q4_k": 3, "q6_k": 4}[qtype]
    for name, key in (("l0.down", "decoder.layers.0.mlp.down_proj.weight"),
                      ("cond", "decoder.condition_embedder.weight")):
        fmt, rows, cols, q, s = load_w(out, idx, name)
        assert fmt == wf
        v = st[key][2].reshape(rows, cols).astype(np.float32)
        raw = g.make_weight(v, "BF16", qtype).raw
        eq, es = to_planes(qtype, raw, rows, cols)
        np.testing.assert_array_equal(q, eq)
        np.testing.assert_array_equal(s, es)
    # proj_in (in-dim 384): Q8_0 quantizes it, the K-quants keep it bf16 (in % 256 != 0)
    assert int(idx["proj_in"][1]) == (2 if qtype == "q8_0" else 0)
    # AdaLN table: cast_f32 of the quantized table = dequant(quant(t))
    tables = np.fromfile(os.path.join(out, "tables.bin"), np.float32).reshape(cfg["num_hidden_layers"], 6, H)
    t0 = st["decoder.layers.0.scale_shift_table"][2].reshape(6, H).astype(np.float32)
    np.testing.assert_array_equal(tables[0], g.make_weight(t0, "BF16", qtype).values)
    # timestep GEMV weights: bf16(dequant(quant(w)))
    w1 = st["decoder.time_embed.linear_1.weight"][2].reshape(H, 256).astype(np.float32)
    exp = g.f32_to_bf16_bits(g.make_weight(w1, "BF16", qtype).values)
    np.testing.assert_array_equal(np.fromfile(os.path.join(out, "te0.w1.bin"), np.uint16).reshape(H, 256), exp)


@pytest.mark.parametrize("quant", ["Q8", "Q4", "F16"])
def test_gguf_source(dumper, tiny, quant):
    from acestep_mi355x.synthetic import write_gguf
    d, cfg = tiny
    dd = tempfile.mkdtemp(prefix="acemi_ldg_")
    shutil.copy(os.path.join(d, "config.json"), dd)
    path = write_gguf(os.path.join(d, "model.safetensors"), os.path.join(dd, "model.gguf"), quant=quant)
    out, idx = run_dump(dumper, "dit", dd, {"ACE_GGML_DIT_WEIGHT_QTYPE": "q6_k"})  # ignored for GGUF
    from oracle.dit_oracle import read_gguf
    gg = read_gguf(path)
    H = cfg["hidden_size"]
    qtype = {"Q8": "q8_0", "Q4": "q4_k", "F16": None}[quant]
    fmt, rows, cols, q, s = load_w(out, idx, "l0.down")
    gt, ne, raw = gg["decoder.layers.0.mlp.down_proj.weight"]
    if qtype:
        bb = {"q8_0": 34, "q4_k": 144}[qtype]
        eq, es = to_planes(qtype, np.frombuffer(raw, np.uint8).reshape(rows, -1, bb), rows, cols)
        np.testing.assert_array_equal(q, eq)
        np.testing.assert_array_equal(s, es)
    else:
        assert fmt == 1
        np.testing.assert_array_equal(q.view(np.uint16), np.frombuffer(raw, np.uint16))
    # proj_in / proj_out become F32 weights: the fp16 triple [hi | lo | hi]
    for name in ("proj_in", "proj_out"):
        fmt, rows, cols, q, _ = load_w(out, idx, name)
        assert fmt == 5
        t = q.view(np.float16).reshape(rows, 3, cols).astype(np.float32)
        np.testing.assert_array_equal(t[:, 0], t[:, 2])
        assert np.all(np.abs(t[:, 1]) <= np.abs(t[:, 0]) * 2.0 ** -10 + 1e-30)
    gt, ne, raw = gg["decoder.proj_in.1.weight"]        # F16 [H][Cin][P] -> [H][P*Cin], k*Cin + c
    w = np.frombuffer(raw, "<f2").astype(np.float32).reshape(H, cfg["in_channels"], cfg["patch_size"])
    fmt, rows, cols, q, _ = load_w(out, idx, "proj_in")
    hi = q.view(np.float16).reshape(rows, 3, cols)[:, 0].astype(np.float32)
    np.testing.assert_array_equal(hi, w.transpose(0, 2, 1).reshape(rows, cols))
    assert idx["act"][0] == ("1" if quant == "F16" else "0")


@pytest.fixture(scope="module")
def tiny_vae_dir():
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_ldv_")
    write_vae_checkpoint(d, VAE_TINY_CONFIG, seed=2)
    return d


def test_vae_layouts(dumper, tiny_vae_dir):
    from oracle.vae_oracle import VaeWeights
    out, idx = run_dump(dumper, "vae", tiny_vae_dir)
    W = VaeWeights(tiny_vae_dir)
    assert idx["hop"] == ["6"]

    def w16(name):
        return np.fromfile(os.path.join(out, name + ".w.bin"), np.float16).astype(np.float32)

    # conv: [Cout][K][Cin] of the folded fp16 weight
    w = W.conv1["w"]
    np.testing.assert_array_equal(w16("decoder.conv1").reshape(w.shape[0], w.shape[2], w.shape[1]),
                                  w.transpose(0, 2, 1))
    ru = W.blocks[1]["res"][2]
    w = ru["conv1"]["w"]
    np.testing.assert_array_equal(w16("decoder.block.1.res_unit3.conv1").reshape(w.shape[0], 7, w.shape[1]),
                                  w.transpose(0, 2, 1))
    assert idx["decoder.block.1.res_unit3.conv1"][4:7] == ["7", "9", "27"]   # taps, dil, pad
    # conv_t: [s*Cout][2][Cin] with [r*Cout+co][tap][ci] = w[ci][co][r + tap*s]
    blk = W.blocks[0]
    s = blk["stride"]
    w = blk["conv_t1"]["w"]
    cin, cout, _ = w.shape
    got = w16("decoder.block.0.conv_t1").reshape(s, cout, 2, cin)
    for r in range(s):
        for tap in range(2):
            np.testing.assert_array_equal(got[r, :, tap, :], w[:, :, r + tap * s].T)
    ea = np.fromfile(os.path.join(out, "decoder.block.0.res_unit1.snake2.ea.bin"), np.float32)
    np.testing.assert_allclose(ea, np.exp(W.blocks[0]["res"][0]["snake2"]["alpha"]), rtol=1e-6)
    # encoder conv1: 2 audio channels zero-padded to 64
    e = W.enc["conv1"]["w"]
    got = w16("encoder.conv1").reshape(e.shape[0], 7, 64)
    np.testing.assert_array_equal(got[:, :, :2], e.transpose(0, 2, 1))
    assert not got[:, :, 2:].any()
    assert idx["encoder.block.1.conv1"][4:8] == ["6", "1", "2", "3"]            # taps 2s, dil, pad ceil(s/2), stride
