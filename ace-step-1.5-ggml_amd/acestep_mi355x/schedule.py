"""Turbo timestep schedules of ACE-Step 1.5.

Restates `get_timestep_schedule` (acestep/mlx_dit/generate.py:14-72) and the C
sampler's `ace_get_shift_schedule` (acestep_ggml/cpp/acestep_ggml.cpp:1484-1500):
8-step tables for shift 1/2/3, shift snapped to the nearest valid value, custom
timesteps snapped to the nearest VALID_TIMESTEPS entry (trailing zeros dropped,
at most 20).  Also the linear "N-step" schedule with shift used for the 27/60
step benchmark configs (t_i = 1 - i/S, t' = s*t / (1 + (s-1)*t),
acestep/inference.py:70).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

VALID_SHIFTS = [1.0, 2.0, 3.0]

VALID_TIMESTEPS = [
    1.0, 0.9545454545454546, 0.9333333333333333, 0.9, 0.875,
    0.8571428571428571, 0.8333333333333334, 0.7692307692307693, 0.75,
    0.6666666666666666, 0.6428571428571429, 0.625, 0.5454545454545454,
    0.5, 0.4, 0.375, 0.3, 0.25, 0.2222222222222222, 0.125,
]

SHIFT_TIMESTEPS = {
    1.0: [1.0, 0.875, 0.75, 0.625, 0.5, 0.375, 0.25, 0.125],
    2.0: [1.0, 0.9333333333333333, 0.8571428571428571, 0.7692307692307693,
          0.6666666666666666, 0.5454545454545454, 0.4, 0.2222222222222222],
    3.0: [1.0, 0.9545454545454546, 0.9, 0.8333333333333334, 0.75,
          0.6428571428571429, 0.5, 0.3],
}


def get_timestep_schedule(shift: float = 3.0, timesteps: Optional[Sequence[float]] = None) -> List[float]:
    if timesteps is not None:
        ts = list(timesteps)
        while ts and ts[-1] == 0:
            ts.pop()
        if ts:
            ts = ts[:20]
            return [min(VALID_TIMESTEPS, key=lambda x, t=t: abs(x - t)) for t in ts]
    s = min(VALID_SHIFTS, key=lambda x: abs(x - shift))
    return list(SHIFT_TIMESTEPS[s])


def shifted_linear_schedule(steps: int, shift: float = 3.0) -> List[float]:
    """t_i = 1 - i/steps (i < steps), mapped by t' = shift*t / (1 + (shift-1)*t)."""
    out = []
    for i in range(steps):
        t = 1.0 - i / steps
        out.append(shift * t / (1.0 + (shift - 1.0) * t))
    return out
