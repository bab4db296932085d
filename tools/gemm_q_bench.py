"""Quantized vs dense GEMM at the DiT block shapes (GPU box): TFLOP/s of the dense bf16 kernel, the register-dequant
Q8_0 / Q4_K kernel (automatic tile or forced variants) and the staged path (dequant launch + dense GEMM) at the 240 s
(M = 3000), 60 s (M = 750) and 10 s (M = 125) token counts.  Usage: python tools/gemm_q_bench.py [M,...] [v,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

ms = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["3000", "750", "125"])]
vs = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["-1"])]
for M in ms:
    for name, N, K, epi in [("gate_up", 12288, 2048, 4), ("qkv", 4096, 2048, 0), ("down", 2048, 6144, 2),
                            ("o", 2048, 2048, 2)]:
        fl = 2.0 * M * N * K
        row = {"M": M, "shape": name, "dense_bf16": round(fl / (capi.bench_gemm(M, N, K, epi=epi, iters=20) / 1e3) / 1e12, 1)}
        for qt in ("q8_0", "q4_k"):
            for v in vs:
                try:
                    t = capi.bench_gemm_q(M, N, K, qt, variant=v, epi=epi, iters=20)
                    row[f"{qt}_v{v}"] = round(fl / (t / 1e3) / 1e12, 1)
                    row[f"{qt}_v{v}_us"] = round(t * 1e3, 2)
                except RuntimeError as e:
                    row[f"{qt}_v{v}"] = str(e)[:40]
        print(json.dumps(row), flush=True)
