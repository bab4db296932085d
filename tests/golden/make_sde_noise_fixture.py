"""Writes tests/golden/sde_noise_seed7.json: the SDE re-noise draws of acestep_mi355x.sampler.sde_noise for seed 7,
items [0, 3], 2 draws of (T = 4, C = 3) -- pins the seed -> noise mapping (item b: torch CPU generator seeded
with seed * 1000003 + b), an intentional deviation from the reference's one (bsz, T, C) MLX draw per step."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))

from acestep_mi355x.sampler import sde_noise  # noqa: E402

x = sde_noise(2, [0, 3], 4, 3, 7, "cpu")
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sde_noise_seed7.json"), "w", encoding="utf-8") as f:
    json.dump({"seed": 7, "items": [0, 3], "n_draws": 2, "T": 4, "C": 3,
               "values": [float(v) for v in x.reshape(-1).tolist()]}, f, indent=0)
