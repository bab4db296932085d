"""Build (once per source content) the host-emulation library: the product's runtime/*.cpp linked with
tests/host/kernel_emul.cpp, every launch_* restated as host loops (see test_host_emul.py)."""
import hashlib
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ace-step-1.5-ggml_amd", "csrc")
CLANG = "/opt/rocm/llvm/bin/clang++"
RUNTIME = ("json.cpp", "gguf.cpp", "quant.cpp", "model.cpp", "blocks.cpp", "engine.cpp", "engine_qact.cpp", "text_encoder.cpp", "vae.cpp",
           "abi.cpp", "cond.cpp", "text.cpp", "generate.cpp", "util_abi.cpp", "selftest.cpp", "test_hooks.cpp")


def build_host_lib() -> str:
    srcs = [os.path.join(CSRC, "runtime", f) for f in RUNTIME] + [os.path.join(ROOT, "tests", "host", "kernel_emul.cpp")]
    h = hashlib.sha1(" ".join(RUNTIME).encode())
    for d in (os.path.join(CSRC, "runtime"), CSRC, os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "host")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".cpp", ".h")):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(f.encode() + fh.read())
    out_dir = os.path.join(tempfile.gettempdir(), "acemi_hostlib_" + h.hexdigest()[:16])
    out = os.path.join(out_dir, "libacestep_mi355x_host.so")
    if not os.path.exists(out):
        os.makedirs(out_dir, exist_ok=True)
        tmp = out + f".{os.getpid()}.tmp"
        subprocess.run([CLANG, "-std=c++17", "-O2", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-I" + CSRC, "-ffp-contract=off", "-pthread", "-Wno-unused-result", "-Wl,-Bsymbolic", *srcs,
                        "-o", tmp], check=True)
        os.replace(tmp, out)
    return out
