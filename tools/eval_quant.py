"""Quantized-DiT quality check on the end-to-end pipeline, the acceptance the reference uses for
Q8_0 / Q6_K / Q4_K weights (acestep_ggml/tools/eval_quant_style_lyric_pipeline.py:232-260): the same
style + lyric request and seed through ace_ggml_generate_audio_style_lyric_simple with FP and with
online-quantized DiT weights (ACE_GGML_DIT_WEIGHT_QTYPE), compared sample-wise (MAE, RMSE, peak
|diff|, cosine, SNR) and spectrally (log-spectral distance of the mono mix, 1024-point Hann STFT, hop
256, log10 magnitudes).

usage: python tools/eval_quant.py --dit DIR --vae DIR --text DIR [--seconds 10] [--variants q8_0,q6_k,q4_k]
       (without checkpoint dirs: full-size synthetic weights, as tools/bench_generate.py)
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]


def stft_logmag(x, n_fft=1024, hop=256, eps=1e-8):
    """log10 |rfft(hann * frame)| per frame; short inputs are zero padded to one frame."""
    x = np.asarray(x, np.float32)
    if x.size < n_fft:
        x = np.pad(x, (0, n_fft - x.size))
    n = 1 + (x.size - n_fft) // hop
    idx = np.arange(n)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = x[idx] * np.hanning(n_fft).astype(np.float32)
    return np.log10(np.abs(np.fft.rfft(frames, axis=1)).astype(np.float32) + eps)


def metrics(ref, cur):
    a = np.asarray(ref, np.float32).reshape(-1)
    b = np.asarray(cur, np.float32).reshape(-1)
    n = min(a.size, b.size)
    a, b = a[:n], b[:n]
    d = b - a
    mono = lambda x: np.asarray(x, np.float32) if np.ndim(x) == 1 else np.mean(np.asarray(x, np.float32), axis=1)
    la, lb = stft_logmag(mono(ref)), stft_logmag(mono(cur))
    m = min(len(la), len(lb))
    return {"mae": float(np.mean(np.abs(d))), "rmse": float(np.sqrt(np.mean(d * d))),
            "peak_abs_diff": float(np.max(np.abs(d))),
            "cosine": float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-12)),
            "snr_db": float(10.0 * math.log10((np.mean(a * a) + 1e-12) / (np.mean(d * d) + 1e-12))),
            "lsd": float(np.mean(np.sqrt(np.mean((la[:m] - lb[:m]) ** 2, axis=1))))}


def run(dit, vae, text, seconds, variants, seed=42, style_tokens=64, lyric_tokens=256, lib=None, vocab=None):
    from acestep_mi355x.capi import GGMLCAPIBridge
    rng = np.random.default_rng(0)
    vocab = vocab or 151669
    style, lyric = rng.integers(0, vocab, style_tokens), rng.integers(0, vocab, lyric_tokens)
    seq_len = int(round(seconds * 25))
    out, results = {}, []
    for v in ["fp"] + list(variants):
        if v == "fp":
            os.environ.pop("ACE_GGML_DIT_WEIGHT_QTYPE", None)
        else:
            os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = v
        t0 = time.perf_counter()
        br = GGMLCAPIBridge(lib_path=lib)
        br.load_dit(dit)
        br.load_vae(vae)
        br.load_text_encoder(text)
        t1 = time.perf_counter()
        out[v] = br.generate_audio(seq_len, shift=3.0, seed=seed, style_ids=style, lyric_ids=lyric)
        t2 = time.perf_counter()
        br.close()
        row = {"variant": v, "load_s": round(t1 - t0, 3), "infer_s": round(t2 - t1, 3)}
        if v != "fp":
            row.update({k: round(x, 6) for k, x in metrics(out["fp"], out[v]).items()})
        results.append(row)
    os.environ.pop("ACE_GGML_DIT_WEIGHT_QTYPE", None)
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dit")
    ap.add_argument("--vae")
    ap.add_argument("--text")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--variants", default="q8_0,q6_k,q4_k")
    args = ap.parse_args()
    dit, vae, text = args.dit, args.vae, args.text
    if not (dit and vae and text):
        import tempfile
        from acestep_mi355x.synthetic import (COND_KEYS, TEXT_FULL_CONFIG, VAE_FULL_CONFIG, cached_checkpoint,
                                              make_config, write_vae_checkpoint)
        dit = cached_checkpoint(make_config(**COND_KEYS), seed=0, backend="torch")
        text = cached_checkpoint(TEXT_FULL_CONFIG, seed=0, backend="torch", kind="text")
        vae = os.path.join(os.environ.get("ACE_MI_SYNTH_DIR") or tempfile.gettempdir(), "acestep_mi355x_vae_full")
        if not os.path.exists(os.path.join(vae, "diffusion_pytorch_model.safetensors")):
            write_vae_checkpoint(vae, VAE_FULL_CONFIG, seed=0)
    for row in run(dit, vae, text, args.seconds, [v for v in args.variants.split(",") if v]):
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
