"""MI355X-native ACE-Step 1.5 DiT denoising engine (host side).

The compute path is `lib/libacestep_mi355x.so`: hand-written gfx950 HIP
kernels behind the reference's own C-ABI (`include/acestep_ggml.h`) plus the
MI355X extensions (`include/acestep_mi355x.h`).  This package only binds it:

* :mod:`.capi`      ctypes bindings + ``GGMLCAPIBridge`` (same surface as the
  reference bridge, scripts/run_non_ggml_real_case.py:135-354)
* :mod:`.hook`      ``install_dit_backend`` — the ``decoder.forward`` drop-in
  (scripts/run_non_ggml_real_case.py:445-538), device pointers, batched
* :mod:`.sampler`   Euler turbo sampling, batch-sharded over ranks (RCCL)
* :mod:`.schedule`  turbo timestep schedules (acestep/mlx_dit/generate.py:14-72)
* :mod:`.synthetic` synthetic checkpoints with the real tensor names/shapes

There is no CPU fallback: if the shared library is missing, importing
:mod:`.capi` raises.
"""
import os

PACKAGE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PACKAGE_DIR, "lib", "libacestep_mi355x.so")

CSRC_DIR = os.path.join(os.path.dirname(PACKAGE_DIR), "csrc")


def source_hash() -> str:
    """sha256 (16 hex digits) over the library's sources (csrc/**, Makefile, include/*.h): the build stamp that
    profiles/pmc_traffic.json carries, so bench.py uses counter data only when it came from the same kernels."""
    import hashlib
    h = hashlib.sha256()
    inc = os.path.join(os.path.dirname(os.path.dirname(PACKAGE_DIR)), "include")
    files = []
    for root in (CSRC_DIR, inc):
        for dp, _, fns in os.walk(root):
            files += [os.path.join(dp, f) for f in fns if f.endswith((".hip", ".h", ".cpp", "Makefile"))]
    for f in sorted(files, key=lambda x: os.path.relpath(x, os.path.dirname(CSRC_DIR))):
        h.update(os.path.relpath(f, os.path.dirname(CSRC_DIR)).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


__all__ = ["PACKAGE_DIR", "LIB_PATH", "CSRC_DIR", "source_hash"]
