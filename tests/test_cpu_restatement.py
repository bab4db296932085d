"""The C++/OpenMP restatement of the ggml CPU forward (oracle/cpu/dit_cpu.cpp, bench.py's cpu_baseline)
against the numpy oracle: the two restatements of forward_dit agree to the oracle's own
summation-order floor (1e-6 perturbation spread; the C++ side sums in another order, streams the
softmax and uses the C library's expf), for BF16 and F16 weights, masks and sliding windows."""
import tempfile

import numpy as np
import pytest


@pytest.fixture(scope="module")
def cpu_lib():
    from oracle import cpu_restatement as cr
    try:
        cr.build()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"g++ build of the CPU restatement failed: {e}")
    return cr


@pytest.mark.parametrize("dtype", ["BF16", "F16"])
@pytest.mark.parametrize("masked", [False, True])
def test_cpu_restatement_matches_oracle(cpu_lib, dtype, masked):
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    from oracle.dit_oracle import DitWeights, forward_with_floor
    d = tempfile.mkdtemp(prefix="acemi_cpu_")
    write_checkpoint(d, TINY_CONFIG, seed=0, dtype=dtype)
    W = DitWeights(d)
    cd = cpu_lib.CpuDit(W)
    rng = np.random.default_rng(3)
    T, L = 301, 20
    h = rng.standard_normal((T, 64)).astype(np.float32)
    c = rng.standard_normal((T, 128)).astype(np.float32)
    e = rng.standard_normal((L, 256)).astype(np.float32)
    m = em = None
    if masked:
        m = np.ones(T, np.int32)
        m[290:] = 0
        em = np.ones(L, np.int32)
        em[15:] = 0
    ref, floor = forward_with_floor(W, h, c, e, m, em, T, L, 0.7, 0.4, perturb=1e-6)
    got = cd.forward(h, c, e, m, em, T, L, 0.7, 0.4)
    cd.close()
    l2 = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    print(f"cpu restatement {dtype} masked={masked} ({cpu_lib.isa_name()}): rel_l2={l2:.3e} floor={floor:.3e}")
    assert np.isfinite(got).all() and l2 <= 2.0 * floor, (l2, floor)
