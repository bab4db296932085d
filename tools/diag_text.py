"""GPU diagnostic: bisect the Qwen3 text-encoder forward (layers 0..2, with/without final norm) against
the oracle, for a few sequence lengths."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]
import numpy as np

from acestep_mi355x.capi import GGMLCAPIBridge
from acestep_mi355x.synthetic import TEXT_TINY_CONFIG, text_tensor_specs, write_checkpoint
from oracle import text_oracle as to


def rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b.astype(np.float64)), 1e-30))


def main():
    d = tempfile.mkdtemp(prefix="acemi_dt_")
    write_checkpoint(d, TEXT_TINY_CONFIG, seed=6, dtype="BF16", specs=text_tensor_specs(TEXT_TINY_CONFIG))
    W = to.TextWeights(d)
    br = GGMLCAPIBridge()
    br.load_text_encoder(d)
    for n in (1, 37, 200):
        ids = np.random.default_rng(n).integers(0, 1000, n).astype(np.int32)
        for nl, fn in ((0, False), (0, True), (1, False), (2, False), (2, True)):
            got = br.text_encoder_forward(ids, None, n_layers=nl, apply_final_norm=fn)
            ref = to.forward_text_encoder_layers(W, ids, None, nl, fn)
            bad = np.argwhere(np.abs(got - ref) > 1e-2 * (np.abs(ref) + 1e-3))
            rows = np.unique(bad[:, 0]) if len(bad) else []
            print(f"n={n} layers={nl} final_norm={fn}: rel={rel(got, ref):.3e} |got|={np.linalg.norm(got):.3e} "
                  f"|ref|={np.linalg.norm(ref):.3e} bad_rows={list(rows)[:20]} nbad={len(bad)}", flush=True)
        got = br.text_encoder_forward(ids)
        ref = to.forward_text_encoder_layers(W, ids)
        print(f"n={n} plain entry: rel={rel(got, ref):.3e}", flush=True)
    br.close()


if __name__ == "__main__":
    main()
