"""Attention kernel micro-benchmark at the DiT's 240 s shapes (one JSON line per case): ms per launch and
the algorithmic rate (4*nq*nk_eff*D*Hq FLOP, bf16-equivalent; the split mode issues 3x the MFMAs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]
from acestep_mi355x import capi  # noqa: E402

CASES = [  # name, B, hq, hkv, nq, nk, window, masked
    ("self_full 240s", 1, 16, 8, 3000, 3000, 0, False),
    ("self_sliding 240s", 1, 16, 8, 3000, 3000, 128, False),
    ("cross 240s", 1, 16, 8, 3000, 512, 0, False),
    ("cross 240s masked", 1, 16, 8, 3000, 512, 0, True),
    ("self_full 60s", 1, 16, 8, 750, 750, 0, False),
    ("self_full 240s bs8", 8, 16, 8, 3000, 3000, 0, False),
]


def main():
    only = os.environ.get("ATTN_CASE")  # e.g. "self_full 240s" (one mode, ATTN_MODE or split) for a PMC pass
    only_mode = os.environ.get("ATTN_MODE", "split")
    modes_env = os.environ.get("ATTN_MODES")  # e.g. "f8c" or "f8c,fp16": these modes for every case
    for name, B, hq, hkv, nq, nk, win, masked in CASES:
        if only and name != only:
            continue
        modes = {"split": (True, False, False), "pvsplit": (True, True, False), "fast": (False, False, False),
                 "f8c": (True, True, True), "pv8": (False, True, True)}
        for mode, (split, pvs, f8) in modes.items():
            if only and mode != only_mode:
                continue
            if modes_env and mode not in modes_env.split(","):
                continue
            ms = capi.bench_attention(B, hq, hkv, nq, nk, win, split=split, masked=masked, iters=10, pv_split=pvs,
                                      f8=f8)
            nk_eff = min(nk, 2 * win + 1) if win else nk
            flop = 4.0 * B * nq * nk_eff * 128 * hq
            print(json.dumps({"case": name, "mode": mode, "kh": os.environ.get("ACE_MI_ATTN_KH", "1"), "ms": round(ms, 4),
                              "tflops_alg": round(flop / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
