"""Epilogue cost of the N = 2048 DiT projections: TFLOP/s of the engine GEMM per (shape, epilogue,
variant) on the GPU box (EPI_STORE_F32 0, EPI_STORE_ACT 1, EPI_RESID_GATED 2, EPI_RESID 3)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

for name, M, N, K in [("o/cross 240s", 3000, 2048, 2048), ("down 240s", 3000, 2048, 6144)]:
    for epi in (0, 1, 2, 3):
        row = {"shape": name, "epi": epi}
        for v in (1, 4, 6, 7):
            ms = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=20)
            row[f"v{v}"] = round(2.0 * M * N * K / (ms / 1e3) / 1e12, 1)
        print(json.dumps(row), flush=True)
