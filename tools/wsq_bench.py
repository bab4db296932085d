"""Warp-specialized dequant-fused GEMM (variant 25) at the DiT block shapes, M = 3000 (GPU box): TFLOP/s of the
dense default pick, the dense warp-specialized tile (variant 18) and variant 25 for Q8_0 / Q4_K weights.
Usage: python tools/wsq_bench.py [M] [label] -> one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
label = sys.argv[2] if len(sys.argv) > 2 else ""
for name, N, K, epi in [("gate_up", 12288, 2048, 4), ("qkv", 4096, 2048, 0), ("down", 2048, 6144, 2),
                        ("o", 2048, 2048, 2)]:
    fl = 2.0 * M * N * K
    tf = lambda ms: round(fl / (ms / 1e3) / 1e12, 1)  # noqa: E731
    row = {"label": label, "M": M, "shape": name, "dense": tf(capi.bench_gemm(M, N, K, epi=epi, iters=20)),
           "dense_v18": tf(capi.bench_gemm(M, N, K, variant=18, epi=epi, iters=20))}
    for qt in ("q8_0", "q4_k"):
        for v in (-1, 25):
            row[f"{qt}_v{v}"] = tf(capi.bench_gemm_q(M, N, K, qt, variant=v, epi=epi, iters=20))
    print(json.dumps(row), flush=True)
