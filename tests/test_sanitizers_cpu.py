"""The runtime under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; GPU sanitizers are
not available on the pool): tests/host/asan_driver.cpp drives every C-ABI entry family over the
host-emulated kernels, where "device" buffers are host allocations, so under-sized workspaces, loader
over-reads and bad staging offsets are reported by the sanitizer."""
import os
import shutil
import subprocess
import json
import struct
import tempfile

import pytest

from hostlib import CLANG, CSRC, ROOT, RUNTIME


def test_runtime_under_asan_ubsan():
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    from acestep_mi355x.synthetic import (TEXT_TINY_CONFIG, TINY_COND_CONFIG, VAE_TINY_CONFIG, text_tensor_specs,
                                          write_checkpoint, write_gguf, write_vae_checkpoint)
    work = tempfile.mkdtemp(prefix="acemi_asan_")
    dit, vae, text, gg = (os.path.join(work, n) for n in ("dit", "vae", "text", "gguf"))
    write_checkpoint(dit, TINY_COND_CONFIG, seed=4, dtype="BF16")
    write_vae_checkpoint(vae, VAE_TINY_CONFIG, seed=1)
    write_checkpoint(text, TEXT_TINY_CONFIG, seed=6, dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    os.makedirs(gg)
    shutil.copy(os.path.join(dit, "config.json"), gg)
    write_gguf(os.path.join(dit, "model.safetensors"), os.path.join(gg, "model.gguf"), quant="Q8")
    bad = []
    for kind in ("short", "reversed", "past_eof"):
        d = os.path.join(work, "bad_" + kind)
        os.makedirs(d)
        shutil.copy(os.path.join(dit, "config.json"), d)
        _write_malformed(os.path.join(dit, "model.safetensors"), os.path.join(d, "model.safetensors"), kind)
        bad.append(d)
    exe = os.path.join(work, "asan_driver")
    srcs = [os.path.join(CSRC, "runtime", f) for f in RUNTIME] + [
        os.path.join(ROOT, "tests", "host", "kernel_emul.cpp"), os.path.join(ROOT, "tests", "host", "asan_driver.cpp")]
    subprocess.run([CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I" + CSRC,
                    "-ffp-contract=off", "-pthread", "-Wno-unused-result", *srcs, "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, dit, vae, text, gg, *bad], capture_output=True, text=True, timeout=900, env=env)
    print(r.stdout[-2000:], r.stderr[-6000:])
    assert r.returncode == 0, r.stderr[-6000:]
    assert "0 failures" in r.stdout


def _write_malformed(src: str, dst: str, kind: str) -> None:
    """Copy of a safetensors file whose first tensor's data_offsets are corrupted: "short" (fewer bytes
    than its shape), "reversed" (end < begin) or "past_eof" (end beyond the file)."""
    with open(src, "rb") as f:
        raw = f.read()
    hlen = struct.unpack("<Q", raw[:8])[0]
    header = json.loads(raw[8:8 + hlen])
    data = raw[8 + hlen:]
    name = next(k for k in header if k != "__metadata__")
    b, e = header[name]["data_offsets"]
    header[name]["data_offsets"] = {"short": [b, e - 2], "reversed": [e, b],
                                    "past_eof": [b, len(data) + 64]}[kind]
    hj = json.dumps(header, separators=(",", ":")).encode()
    hj += b" " * ((8 - len(hj) % 8) % 8)
    with open(dst, "wb") as f:
        f.write(struct.pack("<Q", len(hj)) + hj + data)
