"""GEMM micro-benchmark on the GPU box: TFLOP/s per (shape, variant) of the engine GEMM."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

SHAPES = [  # (name, M, N, K, epi)
    ("gate_up 240s", 3000, 12288, 2048, 4),
    ("down 240s", 3000, 2048, 6144, 2),
    ("qkv 240s", 3000, 4096, 2048, 0),
    ("o/cross 240s", 3000, 2048, 2048, 2),
    ("gate_up bs8", 24000, 12288, 2048, 4),
    ("square 4096", 4096, 4096, 4096, 0),
    ("square 8192", 8192, 8192, 8192, 0),
]
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "3"])]
qtypes = sys.argv[2].split(",") if len(sys.argv) > 2 else [""]
for qt in qtypes:
    for name, M, N, K, epi in SHAPES:
        if qt and M > 8192:
            continue
        row = {"shape": name, "MNK": [M, N, K], "weights": qt or "bf16"}
        for v in variants:
            if v in (2, 5) and N % 256:
                continue
            if qt and v == 6:
                continue
            if qt:
                ms = capi.bench_gemm_q(M, N, K, qt, variant=v, epi=epi, iters=20)
            else:
                ms = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=20)
            row[f"v{v}"] = round(2.0 * M * N * K / (ms / 1e3) / 1e12, 1)
        print(json.dumps(row), flush=True)
