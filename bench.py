#!/usr/bin/env python3
"""Benchmark: ACE-Step 1.5 DiT denoising steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]: Q8_0 weights by default, `--qtype bf16` for bf16; see DESIGN.md "Measurement"):
240 s of audio = T = 6000 latent frames at 25 Hz (the DiT's frame rate; "5Hz" in
BASELINE.json is the LM code rate) -> N = 3000 patch tokens, encoder
length L = 512, full 24-layer DiT with synthetic bf16 weights of the real
architecture, 27-step shifted-linear (shift 3) Euler sampling.  One "step" = one
DiT forward over the local batch + the Euler update, all on the GPU, run by the
library's device-side generation loop (ace_mi_dit_sample_ex) with the encoder-side
cross-attention K/V recomputed every step like the ggml C sampler (--cross-cache
reuses them like the reference Python/MLX sampler does).

Multi-GPU (one process per GPU, torchrun): the batch is sharded across ranks
(weak scaling, `--batch-per-gpu` items each); rank 0 broadcasts the conditioning
once over RCCL before the timed region; no collective inside it.

Prints ONE JSON line on rank 0 (driver contract), with `roofline` for the
dominant kernel (the MLP gate|up GEMM, measured with HIP events on the launch
stream) and `cpu_baseline` (oracle/cpu/dit_cpu.cpp, the C++/OpenMP restatement of ggml's CPU
forward_dit, on the host cores: one 240 s forward plus the configs[0] 10 s F16 forward).

Extra lines beside the headline (one GPU only; each the same 27-step schedule, timed the same way):
  hook_line        the reference pipeline's drop-in path: a Python Euler loop over torch ROCm tensors calling
                   the installed `decoder.forward` (acestep_mi355x.hook, scripts/run_non_ggml_real_case.py:
                   460-533) once per step, as model.generate_audio does
  qact_line        the headline loop in the ggml-faithful quantized-activation mode (ACE_MI_QUANT_ACT=q8)
  attn_{fp16,split,f32}_line  the headline loop in each attention precision (fp16 operands; hi/lo Q.K; hi/lo Q.K and
                   P.V = ggml's F32 kq / kqv), each with its per-kernel attention time per step
  line_bs          the metric's bs = 2, 4, 8 per GPU at 240 s (item-steps/s, block-linear fraction of peak)
  line_config4     BASELINE configs[4] per GPU: Q4_K 60-step 600 s sample + windowed VAE decode of the result
  bf16_line        the same workload with bf16 weights (+ its own hook_line)
  line_60s         BASELINE configs[1]: 60 s (T = 1500), bs = 1, bf16 weights
  line_600s        BASELINE configs[4]'s DiT sequence on one GPU: 600 s (T = 15000, N = 7500), bs = 1, bf16 weights
  line_10s         10 s (T = 250, configs[0]'s shape) forward rate with the headline weights and with bf16
  lowmem_line      quantized weights with ACE_MI_QUANT_STAGE_SCOPE=layer (planes + one 117 MB bf16 slot,
                   expanded before every layer of every step) and its device-memory footprint
  fused_line       quantized weights with ACE_MI_QUANT_STAGED=0: every quantized block linear through the
                   dequant-fused GEMMs (no bf16 weight image), its memory and per-GEMM launch times
`memory` reports the device bytes taken by the weights (after load_dit) and by the workspace (after the timed
run; with the default `model` scope it holds the bf16 images of the quantized block weights).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
sys.path.insert(0, ROOT)
from acestep_mi355x import source_hash  # noqa: E402  (build stamp of the kernel sources)

METRIC = "DiT denoising steps/sec (240s@5Hz latent, bs=1..8) + single-step ms; 1/2/4/8 GPU"
# DiT attention operand precision of the headline (the engine's default; ACE_MI_BENCH_ATTN overrides for A/B runs):
# "fp16" single fp16 operands, "split" hi/lo fp16 Q.K, "f32" hi/lo Q.K and P.V (ggml's F32 kq / kqv,
# acestep_dit_model.cpp:1238-1251)
HEADLINE_ATTN = os.environ.get("ACE_MI_BENCH_ATTN", "f8c")
ATTN_DESC = {"fp16": "fp16-operand f32-accumulate attention",
             "split": "split attention (hi/lo fp16 Q.K, fp16 P.V, f32 accumulate)",
             "f32": "f32-faithful attention (hi/lo fp16 Q.K and P.V, f32 accumulate)",
             "f8c": "f32-class attention (hi/lo Q.K and P.V: hi x hi fp16, correction products block-scaled e4m3, "
                    "f32 accumulate)",
             "pv8": "fp16 Q.K with f32-class P.V (hi x hi fp16 + block-scaled e4m3 corrections, f32 accumulate)"}
BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16/fp16 MFMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=27)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--batch-per-gpu", type=int, default=1)
    ap.add_argument("--enc-len", type=int, default=512)
    ap.add_argument("--sample-steps", type=int, default=27)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--cross-cache", action="store_true",
                    help="reuse cross-attention K/V across steps (MLXCrossAttentionCache); off = ggml C sampler")
    ap.add_argument("--qtype", default="q8_0", choices=["bf16", "q8_0", "q4_k", "q6_k"],
                    help="DiT weights: online quantization (ACE_GGML_DIT_WEIGHT_QTYPE) or bf16; the default is "
                         "BASELINE configs[2] (240 s, bs=1, Q8_0 dequant-fused matmul)")
    ap.add_argument("--no-bf16-line", action="store_true",
                    help="skip the bf16-weight run that is reported beside a quantized line")
    ap.add_argument("--no-extra-lines", action="store_true",
                    help="skip hook_line / attn_split_line / line_10s / line_60s")
    ap.add_argument("--emulate", action="store_true",
                    help="TEST MODE: the multi-rank code path on CPU (gloo, the host-emulated library of tests/, "
                         "tiny config); its numbers are not a measurement")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if args.emulate:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)

    def sync():
        if not args.emulate:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.sampler import Conditioning, broadcast_conditioning, shard_indices
    from acestep_mi355x.schedule import shifted_linear_schedule
    from acestep_mi355x.synthetic import cached_checkpoint, make_config

    if args.emulate:
        from acestep_mi355x.synthetic import TINY_CONFIG
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from hostlib import build_host_lib  # test infrastructure: the CPU restatement of every launch_*
        cfg = TINY_CONFIG
        lib_path = build_host_lib() if rank == 0 else None
        barrier()
        lib_path = lib_path or build_host_lib()
    else:
        cfg = make_config()
        lib_path = None
    # rank 0 writes the synthetic checkpoint, the others wait for it
    if rank == 0:
        ckpt = cached_checkpoint(cfg, seed=0, backend="torch")
    barrier()
    if rank != 0:
        ckpt = cached_checkpoint(cfg, seed=0, backend="torch")

    if args.qtype == "bf16":
        args.qtype = ""
    def dev_used():
        if args.emulate:
            return 0
        free, total = torch.cuda.mem_get_info(dev)
        return total - free

    set_weights(args.qtype)
    mem0 = dev_used()
    br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
    br.load_dit(ckpt)
    br.set_attn_precision(HEADLINE_ATTN)
    mem_weights = dev_used() - mem0
    stage_scope = os.environ.get("ACE_MI_QUANT_STAGE_SCOPE", "model")
    if not args.qtype:
        wdesc = "bf16"
    elif os.environ.get("ACE_MI_QUANT_STAGED", "1") == "0":
        wdesc = f"{args.qtype.upper()} dequant-fused GEMM (bf16 MFMA)"
    else:
        wdesc = (f"{args.qtype.upper()} (staged dequant to bf16 images, scope {stage_scope}; bf16 MFMA)")
    info = br.info

    T = int(round(args.seconds * 25))        # 25 Hz latent frames
    L = args.enc_len
    b_loc = args.batch_per_gpu
    B = b_loc * world
    audio, ctxd, H = info.audio_dim, info.in_channels - info.audio_dim, info.hidden_size
    shapes = dict(B=B, T=T, L=L, audio=audio, ctx=ctxd, H=H, mask=False, enc_mask=False)
    cond = None
    if rank == 0:
        g = torch.Generator().manual_seed(1234)
        noise = torch.randn((B, T, audio), generator=g)
        src = torch.randn((B, T, audio), generator=g)
        context = torch.cat([src, torch.ones((B, T, ctxd - audio))], dim=-1)  # silence latent | chunk mask
        enc = torch.randn((B, L, H), generator=g)
        cond = Conditioning(noise=noise, context=context, enc=enc)
    sync()
    cond = broadcast_conditioning(cond, shapes, dev)
    items = shard_indices(B, world, rank)
    idx = torch.tensor(items, device=dev)
    xt = cond.noise.index_select(0, idx).contiguous()
    ctx = cond.context.index_select(0, idx).contiguous()
    enc = cond.enc.index_select(0, idx).contiguous()
    sync()  # the library runs on its own stream: inputs complete before the warmup reads them
    sched = shifted_linear_schedule(args.sample_steps, 3.0)
    stream = 0 if args.emulate else torch.cuda.current_stream().cuda_stream

    def run(first, k, inp=None, bridge=None):
        """k denoising steps of the schedule (cyclic) in ONE device-side generation-loop call
        (ace_mi_dit_sample_ex): per step one batched DiT forward + the Euler update, both HIP kernels.
        Cross-attention K/V are recomputed every step (as the ggml C sampler does) unless
        --cross-cache asks for the reference Python/MLX sampler's cache."""
        x_, c_, e_, T_ = inp if inp is not None else (xt, ctx, enc, T)
        sch = [sched[(first + i) % len(sched)] for i in range(k)]
        (bridge or br).dit_sample_ex_device(x_.shape[0], T_, L, x_.data_ptr(), c_.data_ptr(), e_.data_ptr(), 0, 0, sch,
                                            cache_cross=args.cross_cache, stream=stream)

    def timed(fn, k=args.steps, w=args.warmup):
        """seconds for k steps of fn(first, k) after w warmup steps (single GPU: synchronised around)"""
        if w > 0:
            fn(0, w)
        sync()
        t_0 = time.perf_counter()
        fn(w, k)
        sync()
        return time.perf_counter() - t_0

    def line(units, seconds, what):
        return {"value": round(units / seconds, 3), "unit": "steps/s", "ms_per_step": round(1000.0 * seconds /
                                                                                            args.steps, 3),
                "workload": what}

    def small_inputs(T_):
        g_ = torch.Generator(device=dev).manual_seed(T_)
        x_ = torch.randn((1, T_, audio), generator=g_, device=dev)
        c_ = torch.cat([torch.randn((1, T_, audio), generator=g_, device=dev),
                        torch.ones((1, T_, ctxd - audio), device=dev)], dim=-1).contiguous()
        e_ = torch.randn((1, L, H), generator=g_, device=dev)
        sync()
        return x_, c_, e_, T_

    def hook_runner(bridge, x_, c_, e_, T_):
        """model.generate_audio's loop (acestep/handler.py:2827 via the ggml decoder hook): per step the installed
        decoder.forward on torch tensors, then x <- x - v * dt as torch ops on the current stream"""
        import types
        from acestep_mi355x.hook import install_dit_backend
        handler = types.SimpleNamespace(model=types.SimpleNamespace(decoder=types.SimpleNamespace(forward=None)))
        install_dit_backend(handler, bridge)
        dec = handler.model.decoder
        state = {"x": x_.clone()}

        def fn(first, k):
            x = state["x"]
            for i in range(k):
                j = (first + i) % len(sched)
                t_ = torch.full((x.shape[0],), float(sched[j]), dtype=torch.float32, device=dev)
                v_, _ = dec.forward(hidden_states=x, timestep=t_, timestep_r=t_, attention_mask=None,
                                    encoder_hidden_states=e_, encoder_attention_mask=None, context_latents=c_)
                dt = sched[j] if j + 1 == len(sched) else sched[j] - sched[j + 1]
                x = x - v_ * float(dt)
            state["x"] = x
        return fn

    if args.warmup > 0:
        run(0, args.warmup)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    rank_elapsed = [elapsed]
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        gathered = [torch.zeros_like(el) for _ in range(world)]
        dist.all_gather(gathered, el)
        rank_elapsed = [float(g.item()) for g in gathered]
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
    # conditioning broadcast to every rank before the timed region (f32 noise, context, encoder states)
    bcast_bytes = 4 * B * (T * audio + T * ctxd + L * H)
    finite = bool(torch.isfinite(xt).all().item())
    memory = {"weights_bytes": mem_weights, "workspace_bytes": dev_used() - mem0 - mem_weights,
              "stage_scope": stage_scope if args.qtype else None}

    # ---- per-kernel timing (HIP events on the launch stream, one event pair per launch)
    breakdown = {}
    roofline = None
    roofline_attn = None
    roofline_gemm = None
    if not args.no_profile:
        br.profile_enable(True)
        br.profile_reset()
        # one generation-loop call of the timed region's length (per-call work such as the staged dequant of
        # quantized weights is then spread over its steps exactly as in the timed run)
        nprof = args.steps
        run(0, nprof)
        sync()
        prof = br.profile_get()
        br.profile_enable(False)
        for name, ms, cnt in prof:
            breakdown[name] = {"ms_per_step": round(ms / nprof, 4), "launches_per_step": round(cnt / nprof, 3),
                               "avg_us": round(1000.0 * ms / max(cnt, 1), 2)}
        gu = [p for p in prof if p[0] == "gemm_gate_up"]
        roofline_gu = None
        if gu:
            name, ms, cnt = gu[0]
            M = b_loc * ((T + 1) // 2)
            flops = 2.0 * M * (2 * info.intermediate_size) * info.hidden_size
            avg_s = ms / cnt / 1000.0
            ach = flops / avg_s / 1e12
            roofline_gu = {"kernel": f"gemm_gate_up (MLP gate|up, {wdesc} weights, bf16 MFMA, SwiGLU epilogue)",
                           "bound": "mfma",
                           "achieved": round(ach, 1), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / BF16_PEAK_TFLOPS, 4),
                           "traffic": pmc_traffic(T, L, b_loc, args.qtype or "bf16", "gate_up"),
                           "flops_per_launch": flops, "avg_launch_us": round(avg_s * 1e6, 2),
                           "ms_per_step": round(ms / nprof, 4),
                           "shape_MNK": [M, 2 * info.intermediate_size, info.hidden_size]}
        frac = block_linear_frac(prof, nprof, T, b_loc, info)
        if frac is not None:
            breakdown["_dit_block_linears"] = {"tflops": round(frac * BF16_PEAK_TFLOPS, 1), "frac_of_bf16_peak": frac}
        roofline_attn = attention_roofline(prof, nprof, T, L, b_loc, info)
        if roofline_attn is not None:
            roofline_attn["traffic"] = pmc_traffic(T, L, b_loc, args.qtype or "bf16", "attention")
        # `roofline` names the dominant kernel of the step (the most GPU time per step: the f8c attention operator or
        # the gate|up GEMM); the other one stays in its own field
        cands = [r for r in (roofline_attn, roofline_gu) if r is not None]
        if cands:
            roofline = max(cands, key=lambda r: r["ms_per_step"])
        roofline_gemm = roofline_gu

    extras = {}
    single = world == 1 and not args.emulate
    if single and not args.no_extra_lines:
        # ---- the reference pipeline's drop-in path with the headline weights
        extras["hook_line"] = line(B * args.steps, timed(hook_runner(br, xt, ctx, enc, T)),
                                   "the headline workload through the installed decoder.forward hook: a Python "
                                   "Euler loop on torch tensors, one hook call per step (model.generate_audio)")
        # ---- every attention precision: steps/s of the headline loop + per-kernel attention time per step
        modes = {}
        for mode in ("fp16", "split", "f32", "f8c", "pv8"):
            br.set_attn_precision(mode)
            el_m = elapsed if mode == HEADLINE_ATTN else timed(run)
            entry = line(B * args.steps, el_m, f"the headline loop with {ATTN_DESC[mode]}")
            if not args.no_profile:
                entry["attention"] = attention_breakdown(br, run, args.steps, sync)
            modes[mode] = entry
        br.set_attn_precision(HEADLINE_ATTN)
        extras["attn_split_line"] = modes["split"]
        extras["attn_f32_line"] = modes["f32"]
        extras["attn_fp16_line"] = modes["fp16"]
        extras["attn_f8c_line"] = modes["f8c"]
        extras["attn_pv8_line"] = modes["pv8"]
        # ---- 10 s forward rate (configs[0]'s shape) with the headline weights
        in10 = small_inputs(250)
        extras["line_10s"] = {"weights": args.qtype or "bf16", **line(args.steps, timed(lambda f, k: run(f, k, in10)),
                                                                       "10 s (T = 250, N = 125 tokens, L = 512), bs = 1:"
                                                                       " DiT forwards + Euler per s")}

    # ---- low-memory quantized mode: one shared 117 MB bf16 slot expanded before every layer of every step
    if args.qtype and single and not args.no_extra_lines and stage_scope != "layer":
        br.close()
        os.environ["ACE_MI_QUANT_STAGE_SCOPE"] = "layer"
        m0 = dev_used()
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
        br.load_dit(ckpt)
        mw = dev_used() - m0
        el_lm = timed(run)
        extras["lowmem_line"] = {**line(B * args.steps, el_lm,
                                        "the headline loop with ACE_MI_QUANT_STAGE_SCOPE=layer: quantized planes + one "
                                        "shared bf16 slot expanded before every layer of every step"),
                                 "weights_bytes": mw, "workspace_bytes": dev_used() - m0 - mw}
        os.environ.pop("ACE_MI_QUANT_STAGE_SCOPE", None)
    # ---- dequant-fused quantized GEMMs (ACE_MI_QUANT_STAGED=0): no bf16 image of any block weight; the
    #      quantized bytes are expanded inside the GEMM (register-dequant / warp-specialized tiles, gemm_q.hip)
    if args.qtype and single and not args.no_extra_lines and os.environ.get("ACE_MI_QUANT_STAGED", "1") != "0":
        br.close()
        os.environ["ACE_MI_QUANT_STAGED"] = "0"
        m0 = dev_used()
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
        br.load_dit(ckpt)
        mw = dev_used() - m0
        el_fu = timed(run)
        extras["fused_line"] = {**line(B * args.steps, el_fu,
                                       "the headline loop with ACE_MI_QUANT_STAGED=0: dequant-fused GEMMs for every "
                                       "quantized block linear (no bf16 weight images)"),
                                "weights_bytes": mw, "workspace_bytes": dev_used() - m0 - mw}
        if not args.no_profile:
            br.profile_enable(True)
            br.profile_reset()
            run(0, args.steps)
            sync()
            prof_f = br.profile_get()
            br.profile_enable(False)
            frac = block_linear_frac(prof_f, args.steps, T, b_loc, info)
            if frac is not None:
                extras["fused_line"]["dit_block_linears_frac_of_bf16_peak"] = frac
            extras["fused_line"]["gemm_us_per_launch"] = {n: round(1000.0 * ms / max(c, 1), 2) for n, ms, c in prof_f
                                                           if n.startswith("gemm_")}
        os.environ.pop("ACE_MI_QUANT_STAGED", None)
    # ---- ggml's own quantized arithmetic (ACE_MI_QUANT_ACT=q8, the parity mode): Q8 activation blocks, integer
    #      block dots, f32 activations between the linears, f32-precision attention
    if args.qtype and single and not args.no_extra_lines and os.environ.get("ACE_MI_QUANT_ACT", "bf16") == "bf16":
        br.close()
        os.environ["ACE_MI_QUANT_ACT"] = "q8"
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
        br.load_dit(ckpt)
        el_qa = timed(run)
        extras["qact_line"] = line(B * args.steps, el_qa,
                                   "the headline loop with ACE_MI_QUANT_ACT=q8: ggml's quantized arithmetic (Q8_0 "
                                   "activation blocks, exact per-block integer dots on the bf16 MFMA from bf16(q) "
                                   "operands, f32 activations, f32-precision attention)")
        if not args.no_profile:
            br.profile_enable(True)
            br.profile_reset()
            run(0, args.steps)
            sync()
            prof_q = br.profile_get()
            br.profile_enable(False)
            frac = block_linear_frac(prof_q, args.steps, T, b_loc, info)
            if frac is not None:
                extras["qact_line"]["dit_block_linears_frac_of_bf16_peak"] = frac
            extras["qact_line"]["us_per_launch"] = {n: round(1000.0 * ms / max(c, 1), 2) for n, ms, c in prof_q}
        os.environ.pop("ACE_MI_QUANT_ACT", None)
    # ---- the same workload with bf16 weights, reported beside a quantized line (single GPU only)
    bf16_line = None
    if args.qtype and single and not args.no_bf16_line:
        br.close()
        set_weights("")
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
        m0 = dev_used()
        br.load_dit(ckpt)
        mw = dev_used() - m0
        el_bf16 = timed(run)
        bf16_line = line(B * args.steps, el_bf16, "the same 240 s bs=1 sampling loop with bf16 weights (no quantization)")
        bf16_line["weights_bytes"] = mw
        if not args.no_profile:
            br.profile_enable(True)
            br.profile_reset()
            run(0, args.steps)
            sync()
            prof_b = br.profile_get()
            br.profile_enable(False)
            frac = block_linear_frac(prof_b, args.steps, T, b_loc, info)
            if frac is not None:
                bf16_line["dit_block_linears_frac_of_bf16_peak"] = frac
            gu = [p for p in prof_b if p[0] == "gemm_gate_up"]
            if gu:
                bf16_line["gate_up_avg_launch_us"] = round(1000.0 * gu[0][1] / gu[0][2], 2)
        if not args.no_extra_lines:
            bf16_line["hook_line"] = line(B * args.steps, timed(hook_runner(br, xt, ctx, enc, T)),
                                          "bf16 weights through the decoder.forward hook")
            in10 = small_inputs(250)
            extras["line_10s"]["bf16"] = line(args.steps, timed(lambda f, k: run(f, k, in10)),
                                              "10 s forward rate with bf16 weights")
            q = extras["line_10s"]["value"] / max(extras["line_10s"]["bf16"]["value"], 1e-9)
            extras["line_10s"]["ratio_vs_bf16"] = round(q, 3)
    if single and not args.no_extra_lines and (not args.qtype or bf16_line is not None):
        # ---- BASELINE configs[1]: 60 s, bs = 1, bf16 weights (the bridge holds bf16 weights here)
        in60 = small_inputs(1500)
        extras["line_60s"] = line(args.steps, timed(lambda f, k: run(f, k, in60)),
                                  "BASELINE configs[1]: DiT 27-step sample, 60 s (T = 1500, N = 750), bs = 1, bf16")
        if not args.no_profile:
            br.profile_enable(True)
            br.profile_reset()
            run(0, args.steps, in60)
            sync()
            prof60 = br.profile_get()
            br.profile_enable(False)
            extras["line_60s"]["dit_block_linears_frac_of_bf16_peak"] = block_linear_frac(prof60, args.steps, 1500, 1,
                                                                                           info)
            extras["line_60s"]["breakdown_ms_per_step"] = {n: round(ms / args.steps, 4) for n, ms, _ in prof60}
        # ---- BASELINE configs[4]'s DiT sequence (its 4 items sharded one per GPU): 600 s, bs = 1, bf16
        in600 = small_inputs(15000)
        extras["line_600s"] = line(args.steps, timed(lambda f, k: run(f, k, in600)),
                                   "configs[4]'s DiT sequence on one GPU: 27-step sample, 600 s (T = 15000, N = 7500), "
                                   "bs = 1, bf16 (configs[4] itself: 60 steps, Q4_K, one item per GPU)")
        del in600

    if single and not args.no_extra_lines:
        # ---- the metric's bs = 2, 4, 8 per GPU at 240 s with the headline weights (reload them: the bridge above
        # may hold bf16 weights now)
        br.close()
        set_weights(args.qtype)
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
        br.load_dit(ckpt)
        br.set_attn_precision(HEADLINE_ATTN)
        extras["line_bs"] = batch_lines(br, run, timed, torch, dev, T, L, audio, ctxd, H, args, info, sync)
        br.close()
        # ---- BASELINE configs[4]'s per-GPU work: Q4_K, 60-step DiT sample of 600 s + windowed VAE decode
        extras["line_config4"] = config4_line(ckpt, lib_path, local, torch, dev, L, audio, ctxd, H, sync)
        br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)

    # ---- CPU baseline: the C++/OpenMP restatement of ggml's CPU forward_dit on the host cores
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and os.environ.get("ACE_MI_CPU_BASELINE", "1") != "0":
        try:
            cpu = cpu_baseline(ckpt, T, L, args.qtype or None)
        except Exception as e:  # noqa: BLE001  (reported, never fatal)
            cpu = {"value": None, "error": str(e)[:200]}

    if rank == 0:
        ms_per_step = 1000.0 * elapsed / args.steps
        value = B * args.steps / elapsed
        line = {
            "metric": METRIC if not args.emulate else "EMULATED (host CPU restatement, tiny config): not a measurement",
            "value": round(value, 3),
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: random N(0,0.02) bf16 weights with the real DiT tensor names/shapes; "
                    "N(0,1) latents/conditioning",
            "config": {
                "workload": ("BASELINE configs[2]: " if (args.qtype == "q8_0" and args.seconds == 240.0 and b_loc == 1)
                             else "") + f"DiT {args.sample_steps}-step sample, {args.seconds:g} s audio "
                            f"(T={T} latent frames @25 Hz, N={(T + 1) // 2} tokens), enc_len={L}, "
                            f"bs={b_loc}/GPU, {wdesc} weights, {ATTN_DESC[HEADLINE_ATTN]}",
                "attention_precision": HEADLINE_ATTN,
                "weights": args.qtype or "bf16",
                "sampler": "ace_mi_dit_sample_ex (device loop: batched DiT forward + Euler kernel per step)",
                "cross_attention_cache": bool(args.cross_cache),
                "model": "ACE-Step 1.5 DiT (24 layers, hidden 2048, MLP 6144, 16/8 heads)",
                "seconds": args.seconds, "latent_frames": T, "tokens": (T + 1) // 2, "enc_len": L,
                "batch_per_gpu": b_loc, "global_batch": B, "seq_len": T,
                "parallelism": f"dp{world} (batch-sharded, RCCL broadcast of conditioning)",
            },
            "finite": finite,
            "memory": memory,
            "ranks": {"elapsed_s": [round(v, 5) for v in rank_elapsed], "broadcast_bytes_per_rank": bcast_bytes,
                      "items_per_rank": [len(shard_indices(B, world, r)) for r in range(world)]},
            "roofline": roofline,
            "roofline_attention": roofline_attn,
            "roofline_gemm": roofline_gemm,
            "build": source_hash(),
            "bf16_line": bf16_line,
            **extras,
            "cpu_baseline": cpu,
            "breakdown": breakdown,
        }
        print(json.dumps(line), flush=True)
    br.close()
    if world > 1:
        dist.destroy_process_group()


def attention_breakdown(br, run, steps, sync):
    """per-kernel attention time of one generation-loop call (HIP events on the launch stream), per step"""
    br.profile_enable(True)
    br.profile_reset()
    run(0, steps)
    sync()
    prof = br.profile_get()
    br.profile_enable(False)
    out = {}
    tot = 0.0
    for name, ms, cnt in prof:
        if name.startswith("attn_"):
            out[name] = {"avg_us": round(1000.0 * ms / max(cnt, 1), 2), "ms_per_step": round(ms / steps, 4)}
            tot += ms / steps
    out["total_ms_per_step"] = round(tot, 4)
    return out


def batch_lines(br, run, timed, torch, dev, T, L, audio, ctxd, H, args, info, sync):
    """item-steps/s of the 240 s loop at bs = 2, 4, 8 items per GPU (one batched forward per step) with the DiT
    block linears' fraction of the bf16 MFMA peak"""
    out = {}
    for b in (2, 4, 8):
        g = torch.Generator(device=dev).manual_seed(100 + b)
        x_ = torch.randn((b, T, audio), generator=g, device=dev)
        c_ = torch.cat([torch.randn((b, T, audio), generator=g, device=dev),
                        torch.ones((b, T, ctxd - audio), device=dev)], dim=-1).contiguous()
        e_ = torch.randn((b, L, H), generator=g, device=dev)
        sync()
        inp = (x_, c_, e_, T)
        el = timed(lambda f, k: run(f, k, inp))
        ent = {"value": round(b * args.steps / el, 3), "unit": "item-steps/s", "ms_per_step": round(1000.0 * el / args.steps, 3),
               "batch_per_gpu": b, "workload": f"240 s (T = {T}), bs = {b} per GPU, headline weights and attention"}
        if not args.no_profile:
            br.profile_enable(True)
            br.profile_reset()
            run(0, args.steps, inp)
            sync()
            prof = br.profile_get()
            br.profile_enable(False)
            ent["dit_block_linears_frac_of_bf16_peak"] = block_linear_frac(prof, args.steps, T, b, info)
        out[f"bs{b}"] = ent
        del x_, c_, e_, inp
    return out


def config4_line(ckpt, lib_path, local, torch, dev, L, audio, ctxd, H, sync):
    """BASELINE configs[4] per GPU (its bs = 4 over 4 GPUs is one item per GPU): Q4_K DiT weights, a 60-step
    shifted-linear (shift 3) sample of 600 s (T = 15000 frames, N = 7500 tokens) in one device-loop call, then
    the reference's windowed VAE decode of the result (ACE_GGML_VAE_CHUNK_FRAMES default 128, overlap 32,
    acestep_ggml.cpp:2114-2229) through the installed tiled_decode hook on the same GPU.  Synthetic weights
    (DiT N(0, 0.02), VAE weight-normed N(0, 1)); wall time of each stage with the stream synchronised around it."""
    import tempfile
    import types
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.hook import install_vae_backend
    from acestep_mi355x.schedule import shifted_linear_schedule
    from acestep_mi355x.synthetic import VAE_FULL_CONFIG, write_vae_checkpoint
    T, steps = 15000, 60
    set_weights("q4_k")
    br = GGMLCAPIBridge(device=local, lib_path=lib_path) if lib_path else GGMLCAPIBridge(device=local)
    try:
        br.load_dit(ckpt)
        br.set_attn_precision(HEADLINE_ATTN)
        vdir = os.path.join(tempfile.gettempdir(), "acestep_mi355x_synth", "vae_full_f32_seed0")
        if not os.path.exists(os.path.join(vdir, "diffusion_pytorch_model.safetensors")):
            write_vae_checkpoint(vdir, VAE_FULL_CONFIG, seed=0)
        br.load_vae(vdir)
        g = torch.Generator(device=dev).manual_seed(4)
        x_ = torch.randn((1, T, audio), generator=g, device=dev)
        c_ = torch.cat([torch.randn((1, T, audio), generator=g, device=dev),
                        torch.ones((1, T, ctxd - audio), device=dev)], dim=-1).contiguous()
        e_ = torch.randn((1, L, H), generator=g, device=dev)
        sched = shifted_linear_schedule(steps, 3.0)
        stream = torch.cuda.current_stream().cuda_stream
        x_w = x_.clone()
        br.dit_sample_ex_device(1, T, L, x_w.data_ptr(), c_.data_ptr(), e_.data_ptr(), 0, 0, sched[:2], stream=stream)
        sync()
        t0 = time.perf_counter()
        br.dit_sample_ex_device(1, T, L, x_.data_ptr(), c_.data_ptr(), e_.data_ptr(), 0, 0, sched, stream=stream)
        sync()
        t_dit = time.perf_counter() - t0
        handler = types.SimpleNamespace()
        install_vae_backend(handler, br, chunk_size_default=128, overlap_default=32)
        lat = x_.transpose(1, 2).contiguous()                       # [1, 64, T]
        handler.tiled_decode(lat[:, :, :256], offload_wav_to_cpu=False)  # warm the decoder's workspace
        sync()
        t0 = time.perf_counter()
        wav = handler.tiled_decode(lat, offload_wav_to_cpu=False)
        sync()
        t_vae = time.perf_counter() - t0
        finite = bool(torch.isfinite(wav).all().item()) and bool(torch.isfinite(x_).all().item())
        n_samples = int(wav.shape[-1])
        total = t_dit + t_vae
        return {"value": round(1.0 / total, 4), "unit": "items/s", "seconds_per_item": round(total, 3),
                "dit_s": round(t_dit, 3), "dit_steps_per_s": round(steps / t_dit, 3), "vae_decode_s": round(t_vae, 3),
                "audio_samples": n_samples, "audio_seconds": round(n_samples / 48000.0, 2),
                "realtime_factor": round(n_samples / 48000.0 / total, 1), "finite": finite, "weights": "q4_k",
                "workload": "configs[4] per GPU: Q4_K DiT 60-step sample of 600 s (T = 15000, N = 7500, L = 512, bs 1) "
                            "+ windowed VAE decode (128-frame windows, 32-frame overlap) through the tiled_decode hook"}
    finally:
        br.close()
        set_weights("")


def set_weights(qtype):
    """ACE_GGML_DIT_WEIGHT_QTYPE for the next load_dit: online quantization, or none (bf16 as stored)."""
    if qtype:
        os.environ["ACE_GGML_DIT_WEIGHT_QTYPE"] = qtype
    else:
        os.environ.pop("ACE_GGML_DIT_WEIGHT_QTYPE", None)
        os.environ.pop("ACE_GGML_WEIGHT_QTYPE", None)


def block_linear_frac(prof, nprof, T, b_loc, info):
    """DiT block linears (qkv, o, cross q/o, gate|up, down: F_lin of SURVEY §8(d) without the cross K/V) per
    step over their HIP-event time, as a fraction of the 2.5 PFLOP/s dense bf16 MFMA peak."""
    M = b_loc * ((T + 1) // 2)
    H_, I_ = info.hidden_size, info.intermediate_size
    qd, kd = info.num_heads * info.head_dim, info.num_kv_heads * info.head_dim
    per_layer = 2.0 * M * H_ * ((qd + 2 * kd) + qd + qd + qd + 2 * I_) + 2.0 * M * I_ * H_
    lin_ms = sum(p[1] for p in prof if p[0] in ("gemm_qkv", "gemm_o", "gemm_cross_q", "gemm_cross_o",
                                                  "gemm_gate_up", "gemm_down")) / nprof
    if lin_ms <= 0:
        return None
    return round(per_layer * info.num_layers / (lin_ms / 1000.0) / 1e12 / BF16_PEAK_TFLOPS, 4)


def attention_roofline(prof, nprof, T, L, b_loc, info):
    """The attention operator (the headline precision's kernel + its key-split merge, one HIP-event pair per layer)
    against the dense fp16/bf16 MFMA peak: algorithmic FLOP per launch = 4 * (query, key) pairs inside the mask *
    head_dim * q heads (Q.K^T and P.V; SURVEY §8(d) F_attn), per class -- full layers (every key), sliding layers
    (|q - k| <= window) and cross attention (L encoder keys) -- and over the whole step."""
    N = (T + 1) // 2
    w = max(int(info.sliding_window), 0)
    pairs_sliding = sum(min(N - 1, q + w) - max(0, q - w) + 1 for q in range(N)) if w > 0 else N * N
    per_pair = 4.0 * info.head_dim * info.num_heads * b_loc
    classes = {"attn_self_full": per_pair * N * N, "attn_self_sliding": per_pair * pairs_sliding,
               "attn_cross": per_pair * N * L}
    out, tot_flops, tot_ms = {}, 0.0, 0.0
    for name, ms, cnt in prof:
        if name not in classes or cnt <= 0:
            continue
        avg_s = ms / cnt / 1000.0
        ach = classes[name] / avg_s / 1e12
        out[name] = {"flops_per_launch": classes[name], "avg_launch_us": round(avg_s * 1e6, 2), "launches": cnt,
                     "achieved": round(ach, 1), "frac": round(ach / BF16_PEAK_TFLOPS, 4)}
        tot_flops += classes[name] * cnt
        tot_ms += ms
    if not out:
        return None
    ach = tot_flops / (tot_ms / 1000.0) / 1e12
    return {"kernel": f"attention ({ATTN_DESC[HEADLINE_ATTN]}; operator time incl. its key-split merge)", "bound": "mfma",
            "achieved": round(ach, 1), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / BF16_PEAK_TFLOPS, 4),
            "ms_per_step": round(tot_ms / nprof, 4), "classes": out}


def pmc_traffic(T, L, b_loc, weights, kernel):
    """HBM bytes per launch of `kernel` ("gate_up" or "attention") from the committed PMC summary
    (tools/gpu_pmc.sh -> tools/pmc_summary.py -> profiles/pmc_traffic.json) -- only when that summary was collected on
    the same workload (its "config": T / enc_len / batch_per_gpu / weights) AND from the same kernel sources (its
    "build" = acestep_mi355x.source_hash() of this tree); None otherwise."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(path, "r", encoding="utf-8") as f:
            d = json.load(f)
        c = d["config"]
        if (c["latent_frames"], c["enc_len"], c["batch_per_gpu"], c["weights"]) != (T, L, b_loc, weights):
            return None
        if d.get("build") != source_hash():
            return None
        return float(d[kernel]["hbm_bytes"])
    except (OSError, KeyError, ValueError, TypeError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo", "r", encoding="utf-8") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ckpt, T, L, qtype=None):
    """The acestep_ggml CPU path, restated in C++/OpenMP (oracle/cpu/dit_cpu.cpp: ggml-cpu's precision
    rules, vdpbf16ps / vcvtph2ps dot products, streamed f32 attention) because ggml itself cannot be built
    (SURVEY §8c), timed on the host cores: one full 24-layer forward of the bench workload (steps/s =
    1 / seconds) and BASELINE configs[0] (10 s, F16 weights, bs = 1).  Bench infrastructure only."""
    from acestep_mi355x.synthetic import cached_checkpoint, make_config
    from oracle import cpu_restatement as cr
    from oracle.dit_oracle import DitWeights
    import numpy as np
    cr.build()
    threads = int(os.environ.get("OMP_NUM_THREADS") or (os.cpu_count() or 1))

    def one(ckpt_dir, T_, L_, seed):
        cd = cr.CpuDit(DitWeights(ckpt_dir))
        rng = np.random.default_rng(seed)
        h = rng.standard_normal((T_, 64)).astype(np.float32)
        c = np.concatenate([rng.standard_normal((T_, 64)), np.ones((T_, 64))], axis=1).astype(np.float32)
        e = rng.standard_normal((L_, cd.cfg.hidden_size)).astype(np.float32)
        t0 = time.perf_counter()
        out = cd.forward(h, c, e, None, None, T_, L_, 0.9, 0.9)
        sec = time.perf_counter() - t0
        cd.close()
        return sec, bool(np.isfinite(out).all())

    sec, finite = one(ckpt, T, L, 1234)
    c0 = cached_checkpoint(make_config(), seed=0, dtype="F16", backend="torch")
    sec0, finite0 = one(c0, 250, 512, 1234)
    return {"value": round(1.0 / sec, 5), "unit": "steps/s", "cores": threads, "kind": "port",
            "impl": "restatement-cpp (oracle/cpu/dit_cpu.cpp, OpenMP, " + cr.isa_name() + ")",
            "cpu": _cpu_model(), "seconds_per_step": round(sec, 3), "finite": finite and finite0,
            "sample": f"1 full 24-layer DiT forward, T={T}, L={L}, bs=1, bf16 weights (ggml CPU precision rules; "
                      f"GPU line: {qtype or 'bf16'}), attention streamed (a lower bound on ggml's materialised scores)",
            "configs0": {"workload": "acestep_ggml CPU DiT single forward, 10 s (T=250), L=512, bs=1, F16 weights",
                         "seconds_per_forward": round(sec0, 3), "steps_per_s": round(1.0 / sec0, 4)}}


if __name__ == "__main__":
    main()
