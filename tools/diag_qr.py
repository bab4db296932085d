"""Register-dequant GEMM correctness matrix (round-3 diagnostic, GPU box): every (format, variant, shape) twice
against the fp64 product of the same bf16 operands; prints max error / tolerance and run-to-run identity."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
sys.path.insert(0, ROOT)
from acestep_mi355x import capi  # noqa: E402
from oracle import ggml_numerics as g  # noqa: E402
from oracle.ggml_numerics import bf16_bits_to_f32, f32_to_bf16_bits  # noqa: E402

for qt in ("q8_0", "q4_k", "q6_k"):
    for (M, N, K) in [(1, 256, 256), (64, 128, 256), (300, 512, 512), (1000, 256, 2048)]:
        rng = np.random.default_rng(M + K)
        a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
        w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
        blocks = capi.quantize(w, qt)
        deq = {"q8_0": lambda r: g.dequantize_q8_0(*g.unpack_q8_0(r)), "q4_k": g.dequantize_q4_k,
               "q6_k": g.dequantize_q6_k}[qt](blocks)
        wv = g.round_bf16(deq).astype(np.float64)
        av = bf16_bits_to_f32(a).astype(np.float64)
        ref, scale = av @ wv.T, np.abs(av) @ np.abs(wv).T
        row = []
        for v in (1, 20, 22, 23, 122, 123, 222, 223):
            if v >= 100 and K // 64 < 2 * (v // 100):
                continue
            try:
                o1 = capi.kernel_gemm_q(a, blocks, qt, epi=0, variant=v)
                o2 = capi.kernel_gemm_q(a, blocks, qt, epi=0, variant=v)
            except RuntimeError as e:
                row.append(f"v{v}:ERR")
                continue
            err = float(np.max(np.abs(o1 - ref) / (2e-6 * scale + 1e-6)))
            bad_cols = np.nonzero(np.max(np.abs(o1 - ref) / (2e-6 * scale + 1e-6), axis=0) > 1)[0]
            row.append(f"v{v}:{err:.2g}{'' if np.array_equal(o1, o2) else '(nondet)'}"
                       + (f"[cols {bad_cols[:4].tolist()}..{len(bad_cols)}]" if len(bad_cols) else ""))
        print(qt, (M, N, K), " ".join(row), flush=True)
