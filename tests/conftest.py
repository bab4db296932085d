"""Test setup: make the product package and the oracle importable; register markers.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, C-ABI
library load/exports, gloo multi-process sharding.  `-m gpu` runs on an MI355X
and calls the HIP path through the C-ABI.
"""
import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ace-step-1.5-ggml_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def tiny_ckpt():
    """A random-init TINY_CONFIG DiT checkpoint (bf16 safetensors + config.json)."""
    from acestep_mi355x.synthetic import TINY_CONFIG, write_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_tiny_")
    write_checkpoint(d, TINY_CONFIG, seed=0, dtype="BF16")
    return d


@pytest.fixture(scope="module")
def tiny_bridge(tiny_ckpt):
    """The C-ABI bridge with the tiny DiT loaded (GPU tests only)."""
    from acestep_mi355x.capi import GGMLCAPIBridge
    br = GGMLCAPIBridge(n_threads=1, compute_buffer_mb=0)
    br.load_dit(tiny_ckpt)
    yield br
    br.close()
