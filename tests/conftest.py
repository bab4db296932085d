"""Test setup: make the product package and the oracle importable; register markers.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, C-ABI
library load/exports, gloo multi-process sharding.  `-m gpu` runs on an MI355X
and calls the HIP path through the C-ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ace-step-1.5-ggml_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")
