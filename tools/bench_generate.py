"""End-to-end text-to-audio timing on one MI355X: ace_ggml_generate_audio_style_lyric_simple with
full-size synthetic weights (Qwen3-0.6B text encoder, 24-layer DiT with lyric/timbre encoders,
Oobleck VAE), the reference's own end-to-end entry (acestep_ggml.cpp:2576) whose CPU timings are
in SURVEY §8d (quant_eval summary: 17.3 s FP for the style+lyric pipeline on an Apple arm64 CPU,
sequence length not recorded).

Usage: python tools/bench_generate.py [--seconds 10 240] [--runs 3]   (prints one JSON line per length)
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, nargs="+", default=[10.0, 240.0])
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--style-tokens", type=int, default=64)
    ap.add_argument("--lyric-tokens", type=int, default=256)
    args = ap.parse_args()
    import numpy as np
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.synthetic import (COND_KEYS, TEXT_FULL_CONFIG, VAE_FULL_CONFIG, cached_checkpoint,
                                          make_config, write_vae_checkpoint)
    t0 = time.perf_counter()
    dit = cached_checkpoint(make_config(**COND_KEYS), seed=0, backend="torch")
    text = cached_checkpoint(TEXT_FULL_CONFIG, seed=0, backend="torch", kind="text")
    vae = os.path.join(os.environ.get("ACE_MI_SYNTH_DIR") or tempfile.gettempdir(), "acestep_mi355x_vae_full")
    if not os.path.exists(os.path.join(vae, "diffusion_pytorch_model.safetensors")):
        write_vae_checkpoint(vae, VAE_FULL_CONFIG, seed=0)
    print(f"# checkpoints ready in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    br = GGMLCAPIBridge()
    br.load_dit(dit)
    br.load_vae(vae)
    br.load_text_encoder(text)
    rng = np.random.default_rng(0)
    style = rng.integers(0, TEXT_FULL_CONFIG["vocab_size"], args.style_tokens)
    lyric = rng.integers(0, TEXT_FULL_CONFIG["vocab_size"], args.lyric_tokens)
    for sec in args.seconds:
        seq_len = int(round(sec * 25))
        br.generate_audio(seq_len, shift=3.0, seed=1, style_ids=style, lyric_ids=lyric)  # warm-up
        times = []
        for r in range(args.runs):
            t = time.perf_counter()
            audio = br.generate_audio(seq_len, shift=3.0, seed=1 + r, style_ids=style, lyric_ids=lyric)
            times.append(time.perf_counter() - t)
        print(json.dumps({"metric": "generate_audio_style_lyric_simple infer_s", "audio_seconds": sec,
                          "latent_frames": seq_len, "infer_s_median": round(sorted(times)[len(times) // 2], 4),
                          "infer_s_all": [round(x, 4) for x in times], "samples": int(audio.shape[0]),
                          "finite": bool(np.isfinite(audio).all()), "style_tokens": args.style_tokens,
                          "lyric_tokens": args.lyric_tokens, "weights": "synthetic bf16, real shapes",
                          "reference_cpu_s": {"FP, Apple arm64 CPU, seq_len unknown (SURVEY 8d)": 17.303}}), flush=True)
    br.close()


if __name__ == "__main__":
    main()
