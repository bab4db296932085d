"""Generate tests/golden/dit_tiny.npz: seeded inputs + oracle outputs of the DiT forward
on the TINY synthetic checkpoint (acestep_mi355x.synthetic.TINY_CONFIG, seed 0, BF16).

The expected outputs come from the oracle restatement (oracle/dit_oracle.py); the
real ggml DiT cannot be built here, so this fixture pins the oracle
against regressions and gives the GPU tests committed vectors ("parity unpinned"
against real ggml).  Regenerate with:  python tests/golden/make_dit_fixture.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))

from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint  # noqa: E402
from oracle.dit_oracle import DitWeights, forward_dit  # noqa: E402

# (name, T, L, timestep, timestep_r, frame-mask zeros, enc-mask zeros)
CASES = [
    ("base", 40, 9, 0.75, 0.75, None, None),
    ("odd_T_masks", 37, 12, 0.5, 0.0, (30, 37), (10, 12)),
    ("t1_r0", 64, 5, 1.0, 0.3, None, (2, 3)),
    ("no_enc", 24, 0, 0.3, 0.3, None, None),
]


def case_inputs(name, T, L, seed):
    rng = np.random.default_rng(seed)
    hidden = rng.standard_normal((T, 64), dtype=np.float32)
    context = rng.standard_normal((T, 128), dtype=np.float32)
    enc = rng.standard_normal((max(L, 1), TINY_CONFIG["hidden_size"]), dtype=np.float32)[:L]
    return hidden, context, enc


def build(out_path):
    with tempfile.TemporaryDirectory() as d:
        write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
        W = DitWeights(d)
        arrays = {}
        for i, (name, T, L, t, r, mz, ez) in enumerate(CASES):
            hidden, context, enc = case_inputs(name, T, L, 1234 + i)
            mask = None
            if mz is not None:
                mask = np.ones(T, dtype=np.int32)
                mask[mz[0]:mz[1]] = 0
            emask = None
            if ez is not None:
                emask = np.ones(L, dtype=np.int32)
                emask[ez[0]:ez[1]] = 0
            out = forward_dit(W, hidden, context, enc if L > 0 else None, mask, emask, T, L, t, r)
            arrays[f"{name}/hidden"] = hidden
            arrays[f"{name}/context"] = context
            arrays[f"{name}/enc"] = enc
            arrays[f"{name}/mask"] = mask if mask is not None else np.zeros(0, np.int32)
            arrays[f"{name}/enc_mask"] = emask if emask is not None else np.zeros(0, np.int32)
            arrays[f"{name}/meta"] = np.array([T, L, t, r], dtype=np.float64)
            arrays[f"{name}/out"] = out
    np.savez_compressed(out_path, **arrays)


if __name__ == "__main__":
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dit_tiny.npz")
    build(p)
    print("wrote", p)
