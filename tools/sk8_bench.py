"""Micro-benchmark of the split-K ping-pong tiles (variants 210 / 211) against the current picks at the 240 s DiT
shapes (M = 3000): TFLOP/s per (shape, variant, epilogue) as JSON lines.  GPU only; tools, not tests."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

M = int(os.environ.get("M", "3000"))
shapes = {"o": (2048, 2048), "down": (2048, 6144), "qkv": (4096, 2048), "gate_up": (12288, 2048)}
variants = [int(v) for v in os.environ.get("VARIANTS", "-1,7,11,211,10,210").split(",")]
for name, (N, K) in shapes.items():
    for epi in (0, 2):
        row = {"M": M, "shape": name, "epi": epi}
        for v in variants:
            try:
                ms = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=30)
                row[str(v)] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
            except RuntimeError as e:
                row[str(v)] = str(e)[:40]
        print(json.dumps(row), flush=True)
