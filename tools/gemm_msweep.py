"""GEMM tile choice vs M (batch items x 3000 tokens): TFLOP/s of each variant at the DiT block shapes on the
GPU box.  Usage: python tools/gemm_msweep.py 2,4,7,10,11 [3000,6000,12000,24000]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
ms = [int(m) for m in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["3000", "6000", "12000", "24000"])]
for M in ms:
    for name, N, K, epi in [("gate_up", 12288, 2048, 4), ("qkv", 4096, 2048, 0), ("down", 2048, 6144, 2),
                            ("o", 2048, 2048, 2)]:
        row = {"M": M, "shape": name}
        for v in variants:
            if v in (2, 5, 10, 11) and N % 256:
                continue
            t = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=20)
            row[f"v{v}"] = round(2.0 * M * N * K / (t / 1e3) / 1e12, 1)
        print(json.dumps(row), flush=True)
