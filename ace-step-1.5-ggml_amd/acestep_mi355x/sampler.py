"""Batch-sharded diffusion sampling across the GPUs of one node.

The reference samples batch items serially on one host thread
(scripts/run_non_ggml_real_case.py:518-527; C sampler acestep_ggml.cpp:2042-2086).
Each item's whole denoising loop is independent, so here rank k owns
items {b : b % world == k}: rank 0 broadcasts the per-request conditioning
(encoder states, masks, context latents, initial noise) once over RCCL/xGMI, every
rank runs its shard's Euler loop on its own GPU with no data-path collective, and
the final latents are gathered back to rank 0.  No tensor parallelism.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU node,
"gloo" for the CPU tests; world_size 1 needs no process group at all.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


def dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_indices(global_batch: int, world: int, rank: int) -> List[int]:
    """Items owned by `rank`: b % world == rank (round-robin keeps shards within one item)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return [b for b in range(global_batch) if b % world == rank]


@dataclass
class Conditioning:
    """Per-request inputs of the sampling loop for the whole (global) batch."""
    noise: torch.Tensor                 # [B][T][audio] f32 initial x_t
    context: torch.Tensor               # [B][T][ctx] f32 (silence latent | chunk mask)
    enc: torch.Tensor                   # [B][L][H] f32 encoder hidden states
    enc_mask: Optional[torch.Tensor] = None   # [B][L] int32
    mask: Optional[torch.Tensor] = None       # [B][T] int32


def broadcast_conditioning(cond: Optional[Conditioning], shapes: dict, device, src: int = 0) -> Conditioning:
    """Rank `src` holds `cond`; every rank returns a full copy on `device`.  `shapes` (known to all
    ranks from the request) gives B, T, L, audio, ctx, H and which masks exist."""
    rank, world = dist_info()
    B, T, L = shapes["B"], shapes["T"], shapes["L"]
    audio, ctx, H = shapes["audio"], shapes["ctx"], shapes["H"]

    def buf(shape, dtype, have):
        if rank == src:
            return have.to(device=device, dtype=dtype).contiguous()
        return torch.empty(shape, dtype=dtype, device=device)

    out = Conditioning(
        noise=buf((B, T, audio), torch.float32, cond.noise if cond else None),
        context=buf((B, T, ctx), torch.float32, cond.context if cond else None),
        enc=buf((B, L, H), torch.float32, cond.enc if cond else None),
        enc_mask=buf((B, L), torch.int32, cond.enc_mask if cond else None) if shapes.get("enc_mask") else None,
        mask=buf((B, T), torch.int32, cond.mask if cond else None) if shapes.get("mask") else None,
    )
    if world > 1:
        for t in (out.noise, out.context, out.enc, out.enc_mask, out.mask):
            if t is not None:
                dist.broadcast(t, src=src)
    return out


def gather_latents(x_local: torch.Tensor, global_batch: int, dst: int = 0) -> Optional[torch.Tensor]:
    """Collect every rank's [b_local][...] shard into [B][...] (item order restored) on `dst`: final
    latents [b][T][C], or decoded audio [b][channels][samples] (every item of one request has the same
    shape).  One `gather` of ceil(B/W) items per rank."""
    rank, world = dist_info()
    if world == 1:
        return x_local
    n_max = (global_batch + world - 1) // world
    pad = torch.zeros((n_max,) + tuple(x_local.shape[1:]), dtype=x_local.dtype, device=x_local.device)
    pad[: x_local.shape[0]] = x_local
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, parts, dst=dst)
    if rank != dst:
        return None
    out = torch.empty((global_batch,) + tuple(x_local.shape[1:]), dtype=x_local.dtype, device=x_local.device)
    for r in range(world):
        for j, b in enumerate(shard_indices(global_batch, world, r)):
            out[b] = parts[r][j]
    return out


def _sync(t: torch.Tensor) -> None:
    """Order torch's pending work on `t` before the library reads it (its own stream); host tensors
    (the host-emulated library of the CPU tests) need nothing."""
    if t.is_cuda:
        torch.cuda.current_stream().synchronize()


def euler_sample_local(bridge, cond: Conditioning, items: Sequence[int], schedule: Sequence[float],
                       stream: int = 0) -> torch.Tensor:
    """Run the ODE loop (acestep_ggml.cpp:2056-2086) for `items` on this rank's GPU through
    `ace_mi_dit_sample`; returns x0 [len(items)][T][audio]."""
    idx = torch.tensor(list(items), dtype=torch.long, device=cond.noise.device)
    xt = cond.noise.index_select(0, idx).contiguous()
    ctx = cond.context.index_select(0, idx).contiguous()
    enc = cond.enc.index_select(0, idx).contiguous()
    em = cond.enc_mask.index_select(0, idx).contiguous() if cond.enc_mask is not None else None
    mk = cond.mask.index_select(0, idx).contiguous() if cond.mask is not None else None
    B, T, _ = xt.shape
    L = enc.shape[1]
    _sync(xt)
    bridge.dit_sample_device(B, T, L, xt.data_ptr(), ctx.data_ptr(), enc.data_ptr(),
                             mk.data_ptr() if mk is not None else 0, em.data_ptr() if em is not None else 0,
                             list(schedule), stream)
    bridge.synchronize()
    return xt


def sde_noise(n_draws: int, items: Sequence[int], T: int, C: int, seed: Optional[int], device) -> torch.Tensor:
    """SDE re-noise draws [n_draws][len(items)][T][C] for this rank's `items` only: item b draws from its own
    generator seeded from (seed, b), so every item gets an independent stream (as generate.py:187 draws one
    (bsz, T, C) normal per step) that does not depend on the world size or on which rank owns it, and a rank
    draws and moves nothing but its own slice.  Drawn on the CPU (the same stream on every backend) and moved
    to `device`.  seed None -> fresh nondeterministic seeds (every rank must then be given an explicit seed to
    agree).  Intentional deviation: the reference draws one (bsz, T, C) normal per step from MLX's generator
    (generate.py:187), which cannot be reproduced here; this per-item mapping (seed * 1000003 + b) is pinned by
    tests/golden/sde_noise_seed7.json."""
    out = torch.empty((n_draws, len(items), T, C), dtype=torch.float32)
    for k, b in enumerate(items):
        g = torch.Generator()
        if seed is None:
            g.seed()
        else:
            g.manual_seed((int(seed) * 1000003 + int(b)) % (1 << 63))
        out[:, k] = torch.randn((n_draws, T, C), generator=g, dtype=torch.float32)
    return out.to(device)


def generate_local(bridge, cond: Conditioning, items: Sequence[int], schedule: Sequence[float],
                   infer_method: str = "ode", seed: Optional[int] = None, cover_steps: int = -1,
                   cond_non_cover: Optional[Conditioning] = None, cache_cross: bool = True,
                   stream: int = 0) -> torch.Tensor:
    """The reference generation loop (acestep/mlx_dit/generate.py:143-199) for this rank's `items`
    through `ace_mi_dit_sample_ex`: ODE or SDE stepping, the audio-cover switch to non-cover
    conditions from step `cover_steps` on, and the cross-attention cache.  SDE re-noise draws come
    from `sde_noise` (one generator for the global batch; the MLX draws cannot be reproduced)."""
    dev = cond.noise.device
    if len(items) == 0:  # more ranks than items: this rank idles (and still joins the gather)
        return cond.noise[:0].clone()
    idx = torch.tensor(list(items), dtype=torch.long, device=dev)
    sel = lambda t: t.index_select(0, idx).contiguous() if t is not None else None
    xt = sel(cond.noise)
    ctx, enc, em, mk = sel(cond.context), sel(cond.enc), sel(cond.enc_mask), sel(cond.mask)
    ctx_nc = sel(cond_non_cover.context) if cond_non_cover is not None else None
    enc_nc = sel(cond_non_cover.enc) if cond_non_cover is not None else None
    B, T, C = xt.shape
    L = enc.shape[1]
    noise = None
    if infer_method == "sde" and len(schedule) > 1:
        noise = sde_noise(len(schedule) - 1, list(items), T, C, seed, dev).contiguous()
    elif infer_method not in ("ode", "sde"):
        raise ValueError(infer_method)
    _sync(xt)
    ptr = lambda t: t.data_ptr() if t is not None else 0
    bridge.dit_sample_ex_device(B, T, L, xt.data_ptr(), ptr(ctx), ptr(enc), ptr(mk), ptr(em), list(schedule),
                                sde=infer_method == "sde", d_noise=ptr(noise), cover_steps=cover_steps,
                                d_context_nc=ptr(ctx_nc), d_enc_nc=ptr(enc_nc), cache_cross=cache_cross,
                                stream=stream)
    bridge.synchronize()
    return xt


def decode_local(bridge, x0_local: torch.Tensor, chunk_size: int = 32, overlap: int = 8) -> torch.Tensor:
    """VAE-decode this rank's final latents x0 [b][T][C] -> audio [b][channels][samples] on its own GPU,
    with the reference's windowed plan (run_non_ggml_real_case.py:550-659, chunk 32 / overlap 8
    defaults :889-890) through ace_mi_vae_decode_device (the 600 s pipeline decodes on
    every rank, then gathers audio)."""
    from .hook import tiled_out_len, vae_decode_torch
    if x0_local.shape[0] == 0:
        return x0_local.new_empty((0, bridge.audio_channels, tiled_out_len(bridge, x0_local.shape[1], chunk_size, overlap)))
    return vae_decode_torch(bridge, x0_local.transpose(1, 2), chunk_size, overlap)


def generate_and_decode(bridge, cond: Conditioning, global_batch: int, schedule: Sequence[float],
                        infer_method: str = "ode", seed: Optional[int] = None, chunk_size: int = 32,
                        overlap: int = 8, dst: int = 0) -> Optional[torch.Tensor]:
    """Full batch-sharded pipeline of BASELINE configs[4] on this rank: its items' DiT sampling loop, its
    items' VAE decode, then the audio of every item gathered to `dst` in item order
    ([B][channels][samples] there, None elsewhere).  No collective inside either loop."""
    rank, world = dist_info()
    items = shard_indices(global_batch, world, rank)
    x0 = generate_local(bridge, cond, items, schedule, infer_method=infer_method, seed=seed)
    audio = decode_local(bridge, x0, chunk_size, overlap)
    return gather_latents(audio.contiguous(), global_batch, dst=dst)
