"""Diagnostic (GPU box): the 8-wave register-dequant tile (variant 21) with Q4_K weights, forced past the picker
(variant | 0x10000), against the fp64 product of the same bf16 operands -- which rows / columns / k-tiles are wrong."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT, os.path.join(ROOT, "tests")]
from acestep_mi355x import capi  # noqa: E402
from oracle.ggml_numerics import f32_to_bf16_bits  # noqa: E402
from test_gpu_quant import _q_ref  # noqa: E402


def main():
    for qtype in ("q4_k", "q8_0", "q6_k"):
        for (M, N, K) in [(192, 256, 256), (192, 256, 512), (384, 512, 256), (1000, 256, 2048)]:
            rng = np.random.default_rng(M + N + K)
            a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
            w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
            blocks = capi.quantize(w, qtype)
            ref, scale = _q_ref(a, blocks, qtype)
            for v in [v for v in [int(x) for x in os.environ.get("VARIANTS", "20,21,22,23").split(",")] for _ in range(int(os.environ.get("REPS", "1")))]:
                got = capi.kernel_gemm_q(a, blocks, qtype, epi=0, variant=v | 0x10000)
                bad = np.abs(got - ref) > 2e-6 * scale + 1e-6
                rows, cols = np.nonzero(bad)
                msg = f"{qtype} v{v} M={M} N={N} K={K}: bad {int(bad.sum())}/{bad.size}"
                if bad.any():
                    cm = np.unique(cols % 256)
                    msg += (f" cols%256 {cm[:12].tolist()}{'...' if len(cm) > 12 else ''} (n={len(cm)})"
                            f" col-waves {np.unique((cols % 256) // 32).tolist()} rows%192 n={len(np.unique(rows % 192))}"
                            f" lane16 {np.unique(cols % 16).tolist()} max rel {float(np.max((np.abs(got - ref) / (np.broadcast_to(scale, got.shape) + 1e-6))[bad])):.3g}")
                print(msg, flush=True)


if __name__ == "__main__":
    main()
