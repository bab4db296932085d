"""Generate tests/golden/schedule_cases.json by importing the REFERENCE's own
`acestep.mlx_dit.generate.get_timestep_schedule` (acestep/mlx_dit/generate.py:33-72;
its module imports only numpy at top level).  Run in the build container where
/root/reference exists:

    PYTHONPATH=/root/reference python tests/golden/make_schedule_fixture.py

The fixture pins both this repo's schedule (`acestep_mi355x.schedule`) and the
oracle; the reference itself never travels to the GPU box.
"""
import json
import os

from acestep.mlx_dit.generate import get_timestep_schedule  # reference code

CASES = [
    {"shift": 1.0, "timesteps": None},
    {"shift": 2.0, "timesteps": None},
    {"shift": 3.0, "timesteps": None},
    {"shift": 2.4, "timesteps": None},
    {"shift": 1.49, "timesteps": None},
    {"shift": 7.0, "timesteps": None},
    {"shift": 0.0, "timesteps": None},
    {"shift": 3.0, "timesteps": [0.97, 0.5, 0.2, 0.0]},
    {"shift": 3.0, "timesteps": [1.0, 0.8, 0.6, 0.4, 0.2, 0.0, 0.0]},
    {"shift": 3.0, "timesteps": [0.0]},
    {"shift": 1.0, "timesteps": [round(1.0 - i / 25.0, 4) for i in range(25)]},
]

if __name__ == "__main__":
    out = []
    for c in CASES:
        out.append({**c, "expected": get_timestep_schedule(c["shift"], c["timesteps"])})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schedule_cases.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)
