"""Turbo schedules vs the golden vectors produced by the reference's own Python
(`acestep.mlx_dit.generate.get_timestep_schedule`, tests/golden/make_schedule_fixture.py)."""
import json
import os

import numpy as np

from conftest import GOLDEN
from acestep_mi355x.schedule import SHIFT_TIMESTEPS, get_timestep_schedule, shifted_linear_schedule


def test_schedule_matches_reference_vectors():
    with open(os.path.join(GOLDEN, "schedule_cases.json"), encoding="utf-8") as f:
        cases = json.load(f)
    assert len(cases) >= 10
    for c in cases:
        assert get_timestep_schedule(c["shift"], c["timesteps"]) == c["expected"], c


def test_c_sampler_tables_are_f32_truncations():
    # acestep_ggml.cpp:1485-1487 stores the same tables as float literals
    c3 = [1.0, 0.9545454545454, 0.9, 0.8333333333333, 0.75, 0.6428571429, 0.5, 0.3]
    np.testing.assert_array_equal(np.float32(SHIFT_TIMESTEPS[3.0]), np.float32(c3))


def test_shifted_linear_schedule():
    s = shifted_linear_schedule(27, 3.0)
    assert len(s) == 27 and s[0] == 1.0
    assert all(a > b for a, b in zip(s, s[1:]))
    t = 1 - 5 / 27
    assert abs(s[5] - 3 * t / (1 + 2 * t)) < 1e-12
