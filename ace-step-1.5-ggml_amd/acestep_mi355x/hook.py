"""`decoder.forward` drop-in for the ACE-Step Python pipeline.

Mirrors `_install_ggml_dit_backend` (scripts/run_non_ggml_real_case.py:445-538): it
replaces `dit_handler.model.decoder.forward` with a function of the same keyword
signature (hidden_states, timestep, timestep_r, attention_mask,
encoder_hidden_states, encoder_attention_mask, context_latents, use_cache,
past_key_values, ..., output_attentions) returning `(pred, past_key_values[, None])`,
and marks the handler with `_ggml_dit_backend` / `_ggml_dit_decoder_forward_hooked`
(read by acestep/handler.py:2740-2746).

Unlike the reference hook (device->host copy, serial per-item ctypes calls, host->device
copy every step, :502-529), tensors already on the GPU are handed over as device
pointers on torch's current stream and the whole batch runs in one call
(`ace_mi_dit_forward_batched`, <= 8 items per launch).  CPU tensors go through the
reference host-pointer entry `ace_ggml_dit_forward`, one item at a time; both paths
compute on the MI355X.
"""
from __future__ import annotations

import types
from typing import Any

import numpy as np

MAX_BATCH_PER_CALL = 8


def _timesteps(ts, bsz: int, device, torch):
    """timestep(_r) as a float32 [bsz] tensor on `device` (tensor scalar/[B], list or float)."""
    if isinstance(ts, torch.Tensor):
        t = ts.detach().to(device=device, dtype=torch.float32).reshape(-1)
        if t.numel() == 1:
            t = t.expand(bsz)
        return t.contiguous()
    if isinstance(ts, (list, tuple)):
        return torch.tensor([float(x) for x in ts], dtype=torch.float32, device=device)
    return torch.full((bsz,), float(ts), dtype=torch.float32, device=device)


def _mask(m, shape, device, torch):
    if m is None:
        return None
    return (m.detach().to(device) > 0).to(torch.int32).reshape(shape).contiguous()


def dit_forward_torch(bridge, hidden_states, timestep, timestep_r, attention_mask, encoder_hidden_states,
                      encoder_attention_mask, context_latents):
    """One batched DiT step on torch tensors; returns pred with hidden_states' dtype/device."""
    import torch

    hs = hidden_states.detach()
    bsz, seq_len, audio = hs.shape
    dev = hs.device
    ctx = context_latents.detach().to(device=dev, dtype=torch.float32).contiguous()
    enc = encoder_hidden_states.detach().to(device=dev, dtype=torch.float32).contiguous()
    x = hs.to(dtype=torch.float32).contiguous()
    am = _mask(attention_mask, (bsz, seq_len), dev, torch)
    eam = _mask(encoder_attention_mask, (bsz, enc.shape[1]), dev, torch)
    t = _timesteps(timestep, bsz, dev, torch)
    r = _timesteps(timestep_r, bsz, dev, torch)
    enc_len = int(enc.shape[1])
    if dev.type == "cuda":
        out = torch.empty((bsz, seq_len, audio), dtype=torch.float32, device=dev)
        with _OrderedCall(bridge, dev) as stream:
            for b0 in range(0, bsz, MAX_BATCH_PER_CALL):
                b1 = min(bsz, b0 + MAX_BATCH_PER_CALL)
                n = b1 - b0
                bridge.dit_forward_batched_device(
                    n, seq_len, enc_len, x[b0:b1].data_ptr(), ctx[b0:b1].data_ptr(),
                    enc[b0:b1].data_ptr() if enc_len > 0 else 0,
                    am[b0:b1].data_ptr() if am is not None else 0,
                    eam[b0:b1].data_ptr() if eam is not None else 0,
                    t[b0:b1].data_ptr(), r[b0:b1].data_ptr(), out[b0:b1].data_ptr(), stream)
        return out.to(hidden_states.dtype)
    # host tensors: reference host-pointer ABI, one item per call (compute still on the GPU)
    out_np = np.empty((bsz, seq_len, audio), dtype=np.float32)
    am_np = am.numpy() if am is not None else np.ones((bsz, seq_len), np.int32)
    eam_np = eam.numpy() if eam is not None else np.ones((bsz, enc_len), np.int32)
    for b in range(bsz):
        out_np[b] = bridge.dit_forward_tfirst(x[b].numpy(), ctx[b].numpy(), enc[b].numpy(), am_np[b], eam_np[b],
                                              float(t[b]), float(r[b]))
    return torch.from_numpy(out_np).to(dev).to(hidden_states.dtype)


def install_dit_backend(dit_handler: Any, bridge) -> None:
    """Replace dit_handler.model.decoder.forward with the MI355X engine."""
    decoder = dit_handler.model.decoder
    original_forward = decoder.forward

    def decoder_forward_mi355x(self, hidden_states, timestep, timestep_r, attention_mask, encoder_hidden_states,
                               encoder_attention_mask, context_latents, use_cache=None, past_key_values=None,
                               cache_position=None, position_ids=None, output_attentions=False,
                               return_hidden_states=None, custom_layers_config=None, enable_early_exit=False,
                               **flash_attn_kwargs):
        if hidden_states is None or hidden_states.dim() != 3:
            return original_forward(hidden_states=hidden_states, timestep=timestep, timestep_r=timestep_r,
                                    attention_mask=attention_mask, encoder_hidden_states=encoder_hidden_states,
                                    encoder_attention_mask=encoder_attention_mask, context_latents=context_latents,
                                    use_cache=use_cache, past_key_values=past_key_values,
                                    cache_position=cache_position, position_ids=position_ids,
                                    output_attentions=output_attentions, return_hidden_states=return_hidden_states,
                                    custom_layers_config=custom_layers_config,
                                    enable_early_exit=enable_early_exit, **flash_attn_kwargs)
        pred = dit_forward_torch(bridge, hidden_states, timestep, timestep_r, attention_mask, encoder_hidden_states,
                                 encoder_attention_mask, context_latents)
        outputs = (pred, past_key_values)
        if output_attentions:
            outputs += (None,)
        return outputs

    decoder.forward = types.MethodType(decoder_forward_mi355x, decoder)
    setattr(dit_handler, "_ggml_dit_backend", "mi355x-capi")
    setattr(dit_handler, "_ggml_dit_decoder_forward_hooked", True)


def _tile_plan(T: int, chunk_size: int, overlap: int):
    """Windows of the reference tiled decode (run_non_ggml_real_case.py:597-611): returns
    (stride, [(core_start, core_end, win_start, win_end)])."""
    max_overlap = max(0, (chunk_size // 2) - 1)
    if overlap > max_overlap:
        overlap = max_overlap
    stride = chunk_size - 2 * overlap
    if stride <= 0:
        overlap = max(0, chunk_size // 4)
        stride = chunk_size - 2 * overlap
        if stride <= 0:
            stride, overlap = max(1, chunk_size), 0
    steps = -(-T // stride)
    plan = []
    for i in range(steps):
        cs = i * stride
        ce = min(cs + stride, T)
        plan.append((cs, ce, max(0, cs - overlap), min(T, ce + overlap)))
    return plan


HIP_STREAM_LEGACY = 1  # hipStreamLegacy: the legacy default stream, which torch's default stream is


class _OrderedCall:
    """Order one library call on device tensors against torch's current stream: the library runs on that
    stream, so both sides are in stream order with no host synchronisation.  torch's default stream has
    handle 0, which the C-ABI reads as "the context's own stream" (include/acestep_mi355x.h), so it is handed
    over as hipStreamLegacy, the same legacy default stream under its explicit handle."""

    def __init__(self, bridge, dev):
        import torch
        self.bridge = bridge
        # host tensors (the host-emulated library of the CPU tests) are ordered by program order
        ts = torch.cuda.current_stream(dev) if torch.device(dev).type == "cuda" else None
        self.stream = (ts.cuda_stream or HIP_STREAM_LEGACY) if ts is not None else 0

    def __enter__(self):
        return self.stream

    def __exit__(self, *exc):
        return False


def _trim(bridge, n: int, cs: int, ce: int, ws: int, we: int):
    """(samples of a window of n frames, leading trim, trailing trim) of the reference tiled decode."""
    total = bridge.vae_out_len(n)
    up = float(total) / float(max(1, n))
    return total, int(round((cs - ws) * up)), int(round((we - ce) * up))


def tiled_out_len(bridge, T: int, chunk_size: int, overlap: int) -> int:
    """Samples per item that vae_decode_torch returns for T latent frames (no decode)."""
    plan = [(0, T, 0, T)] if T <= chunk_size else _tile_plan(T, chunk_size, overlap)
    n = 0
    for cs, ce, ws, we in plan:
        total, ts, te = _trim(bridge, we - ws, cs, ce, ws, we)
        n += (total - te if te > 0 else total) - ts
    return n


def vae_decode_torch(bridge, latents_bct, chunk_size: int, overlap: int):
    """latents [B, C, T] (ROCm tensor) -> audio [B, channels, samples] on the same device, decoding
    each window with ace_mi_vae_decode_device on torch's current stream (no host round trip).
    Windowing and trimming are those of the reference tiled decode, so outputs match it."""
    import torch
    B, C, T = latents_bct.shape
    dev = latents_bct.device
    lat = latents_bct.detach().to(torch.float32)
    outs = []
    plan = [(0, T, 0, T)] if T <= chunk_size else _tile_plan(T, chunk_size, overlap)
    for b in range(B):
        parts = []
        for cs, ce, ws, we in plan:
            win = lat[b, :, ws:we].transpose(0, 1).contiguous()        # [frames, C]
            n = we - ws
            total, ts, te = _trim(bridge, n, cs, ce, ws, we)
            wav = torch.empty((total, bridge.audio_channels), dtype=torch.float32, device=dev)
            with _OrderedCall(bridge, dev) as stream:
                bridge.vae_decode_device(win.data_ptr(), n, wav.data_ptr(), stream)
            parts.append(wav[ts:wav.shape[0] - te if te > 0 else wav.shape[0]])
        outs.append(torch.cat(parts, dim=0).transpose(0, 1))            # [channels, samples]
    return torch.stack(outs, dim=0)


def install_vae_backend(dit_handler: Any, bridge, chunk_size_default: int = 32, overlap_default: int = 8) -> None:
    """Replace dit_handler.tiled_decode (the `_install_ggml_vae_backend` seam,
    scripts/run_non_ggml_real_case.py:541-659) with the MI355X VAE decoder."""

    def tiled_decode_mi355x(self, latents, chunk_size=None, overlap=None, offload_wav_to_cpu=None):
        import torch
        if not isinstance(latents, torch.Tensor):
            raise TypeError(f"latents must be torch.Tensor, got {type(latents)!r}")
        if latents.dim() != 3:
            raise ValueError(f"latents must have shape [B,C,T], got {tuple(latents.shape)}")
        cs = int(chunk_size) if chunk_size is not None and int(chunk_size) > 0 else int(chunk_size_default)
        ov = int(overlap) if overlap is not None else int(overlap_default)
        x = latents if latents.is_cuda else latents.to("cuda")
        out = vae_decode_torch(bridge, x, cs, max(0, ov))
        if offload_wav_to_cpu is None and hasattr(self, "_should_offload_wav_to_cpu"):
            offload_wav_to_cpu = self._should_offload_wav_to_cpu()
        return out.cpu() if offload_wav_to_cpu else out

    dit_handler.tiled_decode = types.MethodType(tiled_decode_mi355x, dit_handler)
    setattr(dit_handler, "_ggml_vae_backend", "mi355x-capi")


def install_text_encoder_backend(dit_handler: Any, bridge) -> None:
    """`_install_ggml_text_encoder_backend` (scripts/run_non_ggml_real_case.py:406-428): route
    `dit_handler.infer_text_embeddings` / `infer_lyric_embeddings` through the GPU text encoder
    (ace_ggml_text_encoder_forward / _embeddings), one call per row as the reference does."""
    import torch

    hidden_dim = int(dit_handler.text_encoder.config.hidden_size)

    def _rows(ids):
        if not isinstance(ids, torch.Tensor):
            ids = torch.tensor(ids, dtype=torch.long)
        return ids.detach().cpu().numpy().astype(np.int32, copy=False)

    def infer_text_embeddings_mi355x(self, text_token_idss):
        out = np.stack([bridge.text_forward_full(r, hidden_dim) for r in _rows(text_token_idss)], axis=0)
        return torch.from_numpy(out).to(self.device).to(self.dtype)

    def infer_lyric_embeddings_mi355x(self, lyric_token_ids):
        out = np.stack([bridge.text_forward_embeddings(r, hidden_dim) for r in _rows(lyric_token_ids)], axis=0)
        return torch.from_numpy(out).to(self.device).to(self.dtype)

    dit_handler.infer_text_embeddings = types.MethodType(infer_text_embeddings_mi355x, dit_handler)
    dit_handler.infer_lyric_embeddings = types.MethodType(infer_lyric_embeddings_mi355x, dit_handler)
