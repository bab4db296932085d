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
        stream = torch.cuda.current_stream(dev).cuda_stream
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
