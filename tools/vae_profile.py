"""VAE decoder roofline evidence: the Oobleck decode (acestep_vae_model.cpp:957-1002) of one
long latent sequence on one MI355X, per conv stage.

  python tools/vae_profile.py --frames 6000 [--runs 3]            -> one JSON line: whole-decode time + TFLOP/s
  python tools/vae_profile.py --summarize <kernel_trace.csv> --frames 6000
                                                                 -> per-stage TFLOP/s from a rocprofv3 trace

The launch plan below restates VaeEngine::decode's order (runtime/vae.cpp): conv1, then per decoder block the
ConvTranspose1d and three residual units (k7 dilated conv, k1 conv; one fused launch at 128 channels), all as
conv_gemm_kernel launches, then the VALU conv_out.  Algorithmic FLOPs per launch = 2 * (output rows) * Cout * taps * Cin (the transposed conv:
two taps per output sample).  Under rocprofv3 --kernel-trace the tool decodes once (warm) then `--runs` more
times; the summary takes the last run's conv_gemm_kernel dispatches in order and joins them with the plan.
"""
import argparse
import csv
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT]
FP16_PEAK_TFLOPS = 2500.0


def plan(cfg, frames):
    """[(stage, M, N, K, flops)] of the conv_gemm launches of one decode, plus conv_out."""
    ch, lat = cfg["decoder_channels"], cfg["decoder_input_channels"]
    strides = list(reversed(cfg["downsampling_ratios"]))
    cm = [1] + list(cfg["channel_multiples"])
    n = len(strides)
    out = []
    L = frames
    c0 = ch * cm[-1]
    out.append(("conv1 k7 %d->%d" % (lat, c0), L, c0, 7 * lat, 2.0 * L * c0 * 7 * lat))
    for i, s in enumerate(strides):
        cin, cout = ch * cm[n - i], ch * cm[n - i - 1]
        pad = (s + 1) // 2
        full = (L + 1) * s
        Lo = full - 2 * pad if 0 < full - 2 * pad < full else full
        out.append((f"block{i} convT x{s} {cin}->{cout}", L + 1, s * cout, 2 * cin, 2.0 * Lo * cout * 2 * cin))
        L = Lo
        for j in range(3):
            if cout == 128:  # one launch: k1 fused into the k7 conv's tile (ConvGemmArgs::W2)
                out.append((f"block{i} res{j} k7+k1 {cout} (fused)", L, cout, 8 * cout, 2.0 * L * cout * 8 * cout))
                continue
            out.append((f"block{i} res{j} k7 {cout}", L, cout, 7 * cout, 2.0 * L * cout * 7 * cout))
            out.append((f"block{i} res{j} k1 {cout}", L, cout, cout, 2.0 * L * cout * cout))
    out.append((f"conv_out k7 {ch}->{cfg['audio_channels']} (VALU)", L, cfg["audio_channels"], 7 * ch,
                2.0 * L * cfg["audio_channels"] * 7 * ch))
    return out


def summarize(trace, cfg, frames, runs):
    rows = list(csv.DictReader(open(trace)))
    conv = [r for r in rows if "conv_gemm_kernel" in r["Kernel_Name"]]
    outk = [r for r in rows if "conv_out_kernel" in r["Kernel_Name"]]
    p = plan(cfg, frames)
    n_conv = len(p) - 1
    conv = conv[-n_conv:]
    outk = outk[-1:]
    stages = []
    tot_f = tot_t = 0.0
    for (name, M, N, K, fl), r in zip(p[:-1] + p[-1:], conv + outk):
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        stages.append({"stage": name, "M": M, "N": N, "K": K, "gflop": round(fl / 1e9, 2), "us": round(dt * 1e6, 1),
                       "tflops": round(fl / dt / 1e12, 1), "frac_of_fp16_peak": round(fl / dt / 1e12 / FP16_PEAK_TFLOPS, 3)})
        tot_f += fl
        tot_t += dt
    return {"metric": "VAE decode per-stage rate (rocprofv3 kernel trace)", "frames": frames,
            "audio_seconds": frames * 1920 / 48000.0, "total_gflop": round(tot_f / 1e9, 1),
            "kernel_ms": round(tot_t * 1e3, 3), "tflops": round(tot_f / tot_t / 1e12, 1),
            "frac_of_fp16_peak": round(tot_f / tot_t / 1e12 / FP16_PEAK_TFLOPS, 3), "stages": stages}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=6000)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--summarize", default="")
    args = ap.parse_args()
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG, write_vae_checkpoint
    cfg = VAE_FULL_CONFIG
    if args.summarize:
        print(json.dumps(summarize(args.summarize, cfg, args.frames, args.runs)))
        return
    import torch
    from acestep_mi355x.capi import GGMLCAPIBridge
    vae = os.path.join(os.environ.get("ACE_MI_SYNTH_DIR") or tempfile.gettempdir(), "acestep_mi355x_vae_full")
    if not os.path.exists(os.path.join(vae, "diffusion_pytorch_model.safetensors")):
        write_vae_checkpoint(vae, cfg, seed=0)
    br = GGMLCAPIBridge()
    br.load_vae(vae)
    n_out = br.vae_out_len(args.frames)
    g = torch.Generator().manual_seed(0)
    lat = torch.randn((args.frames, cfg["decoder_input_channels"]), generator=g).cuda()
    out = torch.empty((n_out, cfg["audio_channels"]), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    br.vae_decode_device(lat.data_ptr(), args.frames, out.data_ptr())
    br.synchronize()
    times = []
    for _ in range(args.runs):
        t = time.perf_counter()
        br.vae_decode_device(lat.data_ptr(), args.frames, out.data_ptr())
        br.synchronize()
        times.append(time.perf_counter() - t)
    fl = sum(x[4] for x in plan(cfg, args.frames))
    best = min(times)
    print(json.dumps({"metric": "VAE decode (one sequence, device buffers)", "frames": args.frames,
                      "audio_seconds": args.frames * 1920 / 48000.0, "samples": n_out, "gflop": round(fl / 1e9, 1),
                      "s_min": round(best, 4), "s_all": [round(x, 4) for x in times],
                      "tflops": round(fl / best / 1e12, 1), "finite": bool(torch.isfinite(out).all().item())}))
    br.close()


if __name__ == "__main__":
    main()
