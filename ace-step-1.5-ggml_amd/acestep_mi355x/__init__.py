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

__all__ = ["PACKAGE_DIR", "LIB_PATH"]
