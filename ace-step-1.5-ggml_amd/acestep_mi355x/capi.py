"""ctypes bindings of libacestep_mi355x.so.

`GGMLCAPIBridge` keeps the reference bridge's surface
(scripts/run_non_ggml_real_case.py:135-354: constructor args, `load_dit`,
`dit_forward_tfirst`, `close`, RuntimeError "<where> failed: <last_error>
(status=N)") so reference callers switch by pointing `lib_path` at this
library.  The MI355X extensions (`dit_forward_batched_device`,
`dit_sample_device`) take raw device pointers (e.g. torch ROCm
`tensor.data_ptr()`) and keep everything on the GPU.
"""
from __future__ import annotations

import atexit
import ctypes
import os
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

from . import LIB_PATH

ACE_GGML_OK = 0
ACE_GGML_ERR = 1
ACE_GGML_ERR_INVALID_ARG = 2
ACE_GGML_ERR_IO = 3
ACE_GGML_ERR_UNSUPPORTED = 4

# Every symbol declared in include/acestep_ggml.h and include/acestep_mi355x.h.
EXPORTED_SYMBOLS = (
    "ace_ggml_create", "ace_ggml_destroy", "ace_ggml_last_error", "ace_ggml_load_dit", "ace_ggml_dit_forward",
    "ace_mi_create_on_device", "ace_mi_dit_get_info", "ace_mi_dit_forward_batched", "ace_mi_dit_sample",
    "ace_mi_dit_sample_ex",
    "ace_mi_profile_enable", "ace_mi_dit_set_attn_precision", "ace_mi_profile_reset", "ace_mi_profile_get", "ace_mi_probe_gemm",
    "ace_mi_synchronize",
    "ace_mi_gemm_variant", "ace_ggml_load_vae", "ace_ggml_vae_get_info", "ace_ggml_vae_decode",
    "ace_mi_vae_out_len", "ace_mi_vae_decode_device", "ace_ggml_vae_encode", "ace_mi_vae_enc_out_len",
    "ace_mi_vae_encode_device", "ace_mi_quantize", "ace_mi_dequantize",
    "ace_mi_cond_get_info", "ace_mi_text_project", "ace_mi_lyric_encode", "ace_mi_timbre_encode",
    "ace_mi_build_condition", "ace_ggml_load_lm", "ace_ggml_load_text_encoder", "ace_ggml_text_encoder_forward",
    "ace_ggml_text_encoder_forward_masked", "ace_ggml_text_encoder_forward_embeddings",
    "ace_ggml_text_encoder_forward_layers", "ace_ggml_generate_audio_simple", "ace_ggml_generate_audio_style_lyric_simple",
    "ace_ggml_generate_audio_style_lyric_timbre_simple", "ace_mi_reference_noise",
)

# Every symbol declared in include/acestep_mi355x_selftest.h: the TEST library (libacestep_mi355x_selftest.so = the
# product objects + the kernel self-test / micro-benchmark entries); the product library does not export them.
SELFTEST_SYMBOLS = ("ace_mi_kernel_gemm", "ace_mi_kernel_attention", "ace_mi_bench_attention", "ace_mi_bench_gemm",
                    "ace_mi_kernel_gemm_q", "ace_mi_kernel_dequant", "ace_mi_bench_gemm_q", "ace_mi_kernel_gemm_a8",
                    "ace_mi_kernel_gemm_a8_mode", "ace_mi_kernel_attn_kh")

# qtype codes of ace_mi_quantize & co. (names as parse_quant_type, acestep_dit_model.cpp:27-37)
QTYPES = {"q8_0": 1, "q4_k": 2, "q6_k": 3}


class AceInitParams(ctypes.Structure):
    _fields_ = [
        ("n_threads", ctypes.c_int32),
        ("use_metal", ctypes.c_int32),
        ("compute_buffer_bytes", ctypes.c_size_t),
    ]


class AceMiDitInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "hidden_size", "intermediate_size", "num_layers", "num_heads", "num_kv_heads", "head_dim",
        "patch_size", "in_channels", "audio_dim", "sliding_window", "act_type", "device")] + [
        ("weight_bytes", ctypes.c_int64)]


class AceMiCondInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "hidden_size", "lyric_in_dim", "timbre_in_dim", "text_projector_in", "has_lyric_encoder", "lyric_layers",
        "has_timbre_encoder", "timbre_layers")]


_LIB = None


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load and bind the shared library (raises if it was not built: there is no fallback)."""
    global _LIB
    p = path or os.environ.get("ACE_MI_LIB") or LIB_PATH
    if _LIB is not None and path is None:
        return _LIB
    if not os.path.exists(p):
        raise RuntimeError(f"libacestep_mi355x.so not found at {p}: run __graft_entry__.build() / make -C "
                           "ace-step-1.5-ggml_amd/csrc")
    # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME
    # libamdhip64.so.7).  Loading torch first makes this library bind to that
    # already-loaded runtime, so torch device pointers and our kernels share it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    vp, i32, f32, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float, ctypes.c_size_t
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int32)
    lib.ace_ggml_create.argtypes = [ctypes.POINTER(AceInitParams), ctypes.POINTER(vp)]
    lib.ace_ggml_create.restype = ctypes.c_int
    lib.ace_mi_create_on_device.argtypes = [ctypes.POINTER(AceInitParams), i32, ctypes.POINTER(vp)]
    lib.ace_mi_create_on_device.restype = ctypes.c_int
    lib.ace_ggml_destroy.argtypes = [vp]
    lib.ace_ggml_destroy.restype = None
    lib.ace_ggml_last_error.argtypes = [vp]
    lib.ace_ggml_last_error.restype = ctypes.c_char_p
    lib.ace_ggml_load_dit.argtypes = [vp, ctypes.c_char_p]
    lib.ace_ggml_load_dit.restype = ctypes.c_int
    lib.ace_ggml_dit_forward.argtypes = [vp, fp, fp, fp, ip, ip, i32, i32, f32, f32, fp, sz]
    lib.ace_ggml_dit_forward.restype = ctypes.c_int
    lib.ace_mi_dit_get_info.argtypes = [vp, ctypes.POINTER(AceMiDitInfo)]
    lib.ace_mi_dit_get_info.restype = ctypes.c_int
    lib.ace_mi_dit_forward_batched.argtypes = [vp, i32, vp, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp]
    lib.ace_mi_dit_forward_batched.restype = ctypes.c_int
    lib.ace_mi_dit_sample.argtypes = [vp, i32, vp, vp, vp, vp, vp, i32, i32, fp, i32, vp]
    lib.ace_mi_dit_sample.restype = ctypes.c_int
    lib.ace_mi_dit_sample_ex.argtypes = [vp, i32, vp, vp, vp, vp, vp, i32, i32, fp, i32, i32, vp, i32, vp, vp, i32, vp]
    lib.ace_mi_dit_sample_ex.restype = ctypes.c_int
    lib.ace_mi_profile_enable.argtypes = [vp, i32]
    lib.ace_mi_dit_set_attn_precision.argtypes = [vp, i32]
    lib.ace_mi_dit_set_attn_precision.restype = ctypes.c_int
    lib.ace_mi_profile_enable.restype = ctypes.c_int
    lib.ace_mi_profile_reset.argtypes = [vp]
    lib.ace_mi_profile_reset.restype = ctypes.c_int
    lib.ace_mi_profile_get.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_double), ip, i32, ip]
    lib.ace_mi_profile_get.restype = ctypes.c_int
    lib.ace_mi_probe_gemm.argtypes = [vp, i32, i32, i32]
    lib.ace_mi_probe_gemm.restype = ctypes.c_int
    lib.ace_mi_synchronize.argtypes = [vp]
    lib.ace_mi_synchronize.restype = ctypes.c_int
    lib.ace_mi_gemm_variant.argtypes = [i32]
    lib.ace_mi_gemm_variant.restype = ctypes.c_int
    i64, u8p = ctypes.c_int64, ctypes.POINTER(ctypes.c_uint8)
    lib.ace_ggml_load_vae.argtypes = [vp, ctypes.c_char_p]
    lib.ace_ggml_load_vae.restype = ctypes.c_int
    lib.ace_ggml_vae_get_info.argtypes = [vp, ip, ip, ip]
    lib.ace_ggml_vae_get_info.restype = ctypes.c_int
    lib.ace_ggml_vae_decode.argtypes = [vp, fp, i32, fp, sz]
    lib.ace_ggml_vae_decode.restype = ctypes.c_int
    lib.ace_mi_vae_out_len.argtypes = [vp, i32, ctypes.POINTER(i64)]
    lib.ace_mi_vae_out_len.restype = ctypes.c_int
    lib.ace_mi_vae_decode_device.argtypes = [vp, vp, i32, vp, vp]
    lib.ace_mi_vae_decode_device.restype = ctypes.c_int
    lib.ace_ggml_vae_encode.argtypes = [vp, fp, i32, fp, sz]
    lib.ace_ggml_vae_encode.restype = ctypes.c_int
    lib.ace_mi_vae_enc_out_len.argtypes = [vp, i32, ctypes.POINTER(i64)]
    lib.ace_mi_vae_enc_out_len.restype = ctypes.c_int
    lib.ace_mi_vae_encode_device.argtypes = [vp, vp, i32, vp, vp]
    lib.ace_mi_vae_encode_device.restype = ctypes.c_int
    lib.ace_mi_quantize.argtypes = [i32, fp, i64, i64, u8p, sz]
    lib.ace_mi_quantize.restype = ctypes.c_int64
    lib.ace_mi_dequantize.argtypes = [i32, u8p, i64, i64, fp]
    lib.ace_mi_dequantize.restype = ctypes.c_int
    for name in ("ace_ggml_load_lm", "ace_ggml_load_text_encoder"):
        getattr(lib, name).argtypes = [vp, ctypes.c_char_p]
        getattr(lib, name).restype = ctypes.c_int
    lib.ace_ggml_text_encoder_forward.argtypes = [vp, ip, i32, fp, sz]
    lib.ace_ggml_text_encoder_forward.restype = ctypes.c_int
    lib.ace_ggml_text_encoder_forward_masked.argtypes = [vp, ip, ip, i32, fp, sz]
    lib.ace_ggml_text_encoder_forward_masked.restype = ctypes.c_int
    lib.ace_ggml_text_encoder_forward_embeddings.argtypes = [vp, ip, i32, fp, sz]
    lib.ace_ggml_text_encoder_forward_embeddings.restype = ctypes.c_int
    lib.ace_ggml_text_encoder_forward_layers.argtypes = [vp, ip, ip, i32, i32, i32, fp, sz]
    lib.ace_ggml_text_encoder_forward_layers.restype = ctypes.c_int
    lib.ace_ggml_generate_audio_simple.argtypes = [vp, ip, i32, i32, f32, i32, fp, sz, ip, ip]
    lib.ace_ggml_generate_audio_simple.restype = ctypes.c_int
    lib.ace_ggml_generate_audio_style_lyric_simple.argtypes = [vp, ip, i32, ip, i32, i32, f32, i32, fp, sz, ip, ip]
    lib.ace_ggml_generate_audio_style_lyric_simple.restype = ctypes.c_int
    lib.ace_ggml_generate_audio_style_lyric_timbre_simple.argtypes = [vp, ip, i32, ip, i32, fp, ip, i32, i32, i32, f32,
                                                                      i32, fp, sz, ip, ip]
    lib.ace_ggml_generate_audio_style_lyric_timbre_simple.restype = ctypes.c_int
    lib.ace_mi_reference_noise.argtypes = [i32, i64, fp]
    lib.ace_mi_reference_noise.restype = ctypes.c_int
    lib.ace_mi_cond_get_info.argtypes = [vp, ctypes.POINTER(AceMiCondInfo)]
    lib.ace_mi_cond_get_info.restype = ctypes.c_int
    lib.ace_mi_text_project.argtypes = [vp, fp, i32, i32, fp, sz]
    lib.ace_mi_text_project.restype = ctypes.c_int
    lib.ace_mi_lyric_encode.argtypes = [vp, fp, i32, fp, sz]
    lib.ace_mi_lyric_encode.restype = ctypes.c_int
    lib.ace_mi_timbre_encode.argtypes = [vp, fp, ip, i32, i32, fp, sz]
    lib.ace_mi_timbre_encode.restype = ctypes.c_int
    lib.ace_mi_build_condition.argtypes = [vp, fp, i32, fp, i32, i32, fp, ip, i32, i32, fp, sz, ip, sz, ip]
    lib.ace_mi_build_condition.restype = ctypes.c_int
    if path is None:
        _LIB = lib
    return lib


_SELFTEST = None


def selftest_library_path() -> str:
    """Path of the TEST library (a superset of the product ABI that also reads the test-only environment hooks,
    runtime/test_hooks.cpp)."""
    return os.environ.get("ACE_MI_SELFTEST_LIB") or os.path.join(os.path.dirname(LIB_PATH), "libacestep_mi355x_selftest.so")


def load_selftest_library() -> ctypes.CDLL:
    """The TEST library (kernel self-tests / micro-benchmarks, include/acestep_mi355x_selftest.h), built beside the
    product library by the same make; the product library is loaded first (one HIP runtime per process)."""
    global _SELFTEST
    if _SELFTEST is not None:
        return _SELFTEST
    load_library()
    p = selftest_library_path()
    if not os.path.exists(p):
        raise RuntimeError(f"libacestep_mi355x_selftest.so not found at {p}: make -C ace-step-1.5-ggml_amd/csrc")
    lib = ctypes.CDLL(p)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int32)
    u16p, u8p = ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint8)
    u16p = ctypes.POINTER(ctypes.c_uint16)
    lib.ace_mi_kernel_gemm.argtypes = [i32, i32, i32, i32, i32, u16p, u16p, fp, fp, u16p]
    lib.ace_mi_kernel_gemm.restype = ctypes.c_int
    lib.ace_mi_kernel_attention.argtypes = [i32, i32, i32, i32, i32, i32, f32, i32, fp, fp, ip, fp]
    lib.ace_mi_kernel_attention.restype = ctypes.c_int
    lib.ace_mi_bench_gemm.argtypes = [i32, i32, i32, i32, i32, i32, i32, fp]
    lib.ace_mi_bench_attention.argtypes = [i32, i32, i32, i32, i32, i32, i32, i32, fp]
    lib.ace_mi_bench_attention.restype = ctypes.c_int
    lib.ace_mi_bench_gemm.restype = ctypes.c_int
    lib.ace_mi_kernel_gemm_q.argtypes = [i32, i32, i32, i32, i32, i32, u16p, u8p, fp, fp, u16p]
    lib.ace_mi_kernel_gemm_q.restype = ctypes.c_int
    lib.ace_mi_kernel_dequant.argtypes = [i32, i32, i32, u8p, u16p]
    lib.ace_mi_kernel_dequant.restype = ctypes.c_int
    lib.ace_mi_bench_gemm_q.argtypes = [i32, i32, i32, i32, i32, i32, i32, fp]
    lib.ace_mi_bench_gemm_q.restype = ctypes.c_int
    i8p = ctypes.POINTER(ctypes.c_int8)
    lib.ace_mi_kernel_gemm_a8.argtypes = [i32, i32, i32, i32, i32, fp, u8p, fp, fp, i8p, fp, fp]
    lib.ace_mi_kernel_gemm_a8.restype = ctypes.c_int
    lib.ace_mi_kernel_gemm_a8_mode.argtypes = [i32]
    lib.ace_mi_kernel_gemm_a8_mode.restype = ctypes.c_int
    lib.ace_mi_kernel_attn_kh.argtypes = [i32]
    lib.ace_mi_kernel_attn_kh.restype = ctypes.c_int
    _SELFTEST = lib
    return lib


def _fptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _iptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


class GGMLCAPIBridge:
    """Drop-in for the reference GGMLCAPIBridge (DiT part) backed by the MI355X library."""

    ACE_GGML_OK = ACE_GGML_OK

    def __init__(self, lib_path: Optional[Path] = None, n_threads: int = 0, compute_buffer_mb: int = 0,
                 use_metal: bool = False, device: Optional[int] = None):
        self.lib_path = str(lib_path) if lib_path else LIB_PATH
        self.lib = load_library(None if lib_path is None else str(lib_path))
        self.ctx = ctypes.c_void_p()
        self.closed = False
        self.use_metal = bool(use_metal)
        params = AceInitParams(n_threads=int(n_threads), use_metal=1 if use_metal else 0,
                               compute_buffer_bytes=int(compute_buffer_mb) * 1024 * 1024)
        if device is None:
            st = self.lib.ace_ggml_create(ctypes.byref(params), ctypes.byref(self.ctx))
        else:
            st = self.lib.ace_mi_create_on_device(ctypes.byref(params), int(device), ctypes.byref(self.ctx))
        self._ensure_ok(st, "ace_ggml_create")
        atexit.register(self.close)
        self.info: Optional[AceMiDitInfo] = None
        self.audio_channels = 0
        self.hop_length = 0
        self.latent_channels = 0

    # -- reference surface -------------------------------------------------
    def _last_error(self) -> str:
        msg = self.lib.ace_ggml_last_error(self.ctx)
        return msg.decode("utf-8", errors="replace") if msg else "unknown error"

    def _ensure_ok(self, status: int, where: str) -> None:
        if status != self.ACE_GGML_OK:
            raise RuntimeError(f"{where} failed: {self._last_error()} (status={status})")

    def close(self) -> None:
        if not self.closed and self.ctx:
            self.lib.ace_ggml_destroy(self.ctx)
            self.closed = True

    def load_dit(self, model_dir) -> None:
        st = self.lib.ace_ggml_load_dit(self.ctx, str(model_dir).encode("utf-8"))
        self._ensure_ok(st, "ace_ggml_load_dit")
        info = AceMiDitInfo()
        self._ensure_ok(self.lib.ace_mi_dit_get_info(self.ctx, ctypes.byref(info)), "ace_mi_dit_get_info")
        self.info = info

    def dit_forward_tfirst(self, hidden_states_tfirst, context_latents_tfirst, encoder_hidden_states_tfirst,
                           attention_mask, encoder_attention_mask, timestep: float, timestep_r: float) -> np.ndarray:
        """[T, D], [T, Ctx], [L, H], [T] int32, [L] int32 -> vt [T, D] float32 (host buffers)."""
        hs = np.ascontiguousarray(hidden_states_tfirst, dtype=np.float32)
        ctx = np.ascontiguousarray(context_latents_tfirst, dtype=np.float32)
        enc = np.ascontiguousarray(encoder_hidden_states_tfirst, dtype=np.float32)
        am = None if attention_mask is None else np.ascontiguousarray(attention_mask, dtype=np.int32)
        eam = None if encoder_attention_mask is None else np.ascontiguousarray(encoder_attention_mask, dtype=np.int32)
        if hs.ndim != 2 or ctx.ndim != 2 or enc.ndim != 2:
            raise ValueError("dit inputs must be 2D arrays [T,D]/[T,Ctx]/[L,H]")
        seq_len = int(hs.shape[0])
        enc_len = int(enc.shape[0])
        out = np.empty_like(hs, dtype=np.float32)
        st = self.lib.ace_ggml_dit_forward(self.ctx, _fptr(hs), _fptr(ctx), _fptr(enc), _iptr(am), _iptr(eam),
                                           seq_len, enc_len, float(timestep), float(timestep_r), _fptr(out),
                                           out.nbytes)
        self._ensure_ok(st, "ace_ggml_dit_forward")
        return out

    def load_vae(self, model_dir) -> None:
        """ace_ggml_load_vae + ace_ggml_vae_get_info (run_non_ggml_real_case.py:243-253)."""
        self._ensure_ok(self.lib.ace_ggml_load_vae(self.ctx, str(model_dir).encode("utf-8")), "ace_ggml_load_vae")
        lat, aud, hop = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        st = self.lib.ace_ggml_vae_get_info(self.ctx, ctypes.byref(lat), ctypes.byref(aud), ctypes.byref(hop))
        self._ensure_ok(st, "ace_ggml_vae_get_info")
        self.latent_channels, self.audio_channels, self.hop_length = int(lat.value), int(aud.value), int(hop.value)

    def vae_decode_tfirst(self, latents_tfirst) -> np.ndarray:
        """latents [T, C] f32 -> audio [T*hop, channels] f32 (host buffers; :283-305)."""
        if self.audio_channels <= 0 or self.hop_length <= 0:
            raise RuntimeError("VAE not initialized in ggml bridge")
        lat = np.ascontiguousarray(latents_tfirst, dtype=np.float32)
        n_frames = int(lat.shape[0])
        out_samples = n_frames * self.hop_length
        out = np.empty((out_samples * self.audio_channels,), dtype=np.float32)
        st = self.lib.ace_ggml_vae_decode(self.ctx, _fptr(lat), n_frames, _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_ggml_vae_decode")
        return out.reshape(out_samples, self.audio_channels)

    def vae_encode_tfirst(self, audio_tfirst) -> np.ndarray:
        """audio [samples, channels] f32 -> latent mean [samples // hop, latent_channels] (host buffers)."""
        if self.latent_channels <= 0 or self.hop_length <= 0:
            raise RuntimeError("VAE not initialized in ggml bridge")
        a = np.ascontiguousarray(audio_tfirst, dtype=np.float32)
        n = int(a.shape[0])
        out = np.empty((n // self.hop_length, self.latent_channels), dtype=np.float32)
        st = self.lib.ace_ggml_vae_encode(self.ctx, _fptr(a), n, _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_ggml_vae_encode")
        return out

    # -- Qwen3 text encoder (acestep_ggml.h:41-94; the reference's ctypes callers are
    #    acestep_ggml/tools/compare_text_encoder.py and run_style_lyric_pipeline.py) ----------------
    def load_text_encoder(self, model_dir) -> None:
        st = self.lib.ace_ggml_load_text_encoder(self.ctx, str(model_dir).encode("utf-8"))
        self._ensure_ok(st, "ace_ggml_load_text_encoder")
        with open(os.path.join(str(model_dir) if not str(model_dir).endswith(".gguf")
                               else os.path.dirname(str(model_dir)), "config.json"), "r", encoding="utf-8") as f:
            import json
            self.text_hidden = int(json.load(f)["hidden_size"])

    def text_encoder_forward(self, token_ids, attention_mask=None, n_layers: Optional[int] = None,
                             apply_final_norm: bool = True) -> np.ndarray:
        """Causal Qwen3 forward: ids [n] -> hidden states [n, hidden] (the _layers entry when n_layers is
        given, _masked with a mask, the plain entry otherwise)."""
        ids = np.ascontiguousarray(token_ids, dtype=np.int32)
        am = None if attention_mask is None else np.ascontiguousarray(attention_mask, dtype=np.int32)
        out = np.empty((ids.shape[0], self.text_hidden), np.float32)
        if n_layers is not None:
            st = self.lib.ace_ggml_text_encoder_forward_layers(self.ctx, _iptr(ids), _iptr(am), ids.shape[0],
                                                               int(n_layers), 1 if apply_final_norm else 0,
                                                               _fptr(out), out.nbytes)
        elif am is not None:
            st = self.lib.ace_ggml_text_encoder_forward_masked(self.ctx, _iptr(ids), _iptr(am), ids.shape[0],
                                                               _fptr(out), out.nbytes)
        else:
            st = self.lib.ace_ggml_text_encoder_forward(self.ctx, _iptr(ids), ids.shape[0], _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_ggml_text_encoder_forward")
        return out

    # reference GGMLCAPIBridge names (scripts/run_non_ggml_real_case.py:255-281)
    def text_forward_full(self, token_ids, hidden_dim: int) -> np.ndarray:
        ids = np.ascontiguousarray(token_ids, dtype=np.int32)
        out = np.empty((ids.shape[0] * int(hidden_dim),), np.float32)
        st = self.lib.ace_ggml_text_encoder_forward(self.ctx, _iptr(ids), ids.shape[0], _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_ggml_text_encoder_forward")
        return out.reshape(ids.shape[0], int(hidden_dim))

    def text_forward_embeddings(self, token_ids, hidden_dim: int) -> np.ndarray:
        ids = np.ascontiguousarray(token_ids, dtype=np.int32)
        out = np.empty((ids.shape[0] * int(hidden_dim),), np.float32)
        st = self.lib.ace_ggml_text_encoder_forward_embeddings(self.ctx, _iptr(ids), ids.shape[0], _fptr(out),
                                                               out.nbytes)
        self._ensure_ok(st, "ace_ggml_text_encoder_forward_embeddings")
        return out.reshape(ids.shape[0], int(hidden_dim))

    def text_encoder_embeddings(self, token_ids) -> np.ndarray:
        ids = np.ascontiguousarray(token_ids, dtype=np.int32)
        out = np.empty((ids.shape[0], self.text_hidden), np.float32)
        st = self.lib.ace_ggml_text_encoder_forward_embeddings(self.ctx, _iptr(ids), ids.shape[0], _fptr(out),
                                                               out.nbytes)
        self._ensure_ok(st, "ace_ggml_text_encoder_forward_embeddings")
        return out

    # -- end-to-end generation (acestep_ggml.h:110-152; reference caller:
    #    acestep_ggml/tools/run_unified_prompt_style_lyric_timbre.py) ------------------------------------
    def generate_audio(self, seq_len: int, shift: float = 3.0, seed: int = 0, token_ids=None, style_ids=None,
                       lyric_ids=None, refer=None, refer_order_mask=None) -> np.ndarray:
        """audio [samples, channels]: ace_ggml_generate_audio_simple when token_ids is given, else the
        style/lyric(/timbre) entry."""
        if self.audio_channels <= 0 or self.hop_length <= 0:
            raise RuntimeError("VAE not initialized in ggml bridge")
        out = np.empty((int(seq_len) * self.hop_length * self.audio_channels,), np.float32)
        ns, nc = ctypes.c_int32(0), ctypes.c_int32(0)
        arr = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.int32)
        if token_ids is not None:
            ids = arr(token_ids)
            st = self.lib.ace_ggml_generate_audio_simple(self.ctx, _iptr(ids), len(ids), int(seq_len), float(shift),
                                                         int(seed), _fptr(out), out.nbytes, ctypes.byref(ns),
                                                         ctypes.byref(nc))
        else:
            si, li = arr(style_ids), arr(lyric_ids)
            n_s = 0 if si is None else len(si)
            n_l = 0 if li is None else len(li)
            if refer is None:
                st = self.lib.ace_ggml_generate_audio_style_lyric_simple(
                    self.ctx, _iptr(si), n_s, _iptr(li), n_l, int(seq_len), float(shift), int(seed), _fptr(out),
                    out.nbytes, ctypes.byref(ns), ctypes.byref(nc))
            else:
                rf = np.ascontiguousarray(refer, dtype=np.float32)
                om = arr(refer_order_mask)
                st = self.lib.ace_ggml_generate_audio_style_lyric_timbre_simple(
                    self.ctx, _iptr(si), n_s, _iptr(li), n_l, _fptr(rf), _iptr(om), int(rf.shape[0]),
                    int(rf.shape[1]), int(seq_len), float(shift), int(seed), _fptr(out), out.nbytes,
                    ctypes.byref(ns), ctypes.byref(nc))
        self._ensure_ok(st, "ace_ggml_generate_audio")
        return out[: ns.value * nc.value].reshape(ns.value, nc.value)

    # -- condition encoders (include/acestep_mi355x.h; acestep_ggml.cpp:1624-1899, :2414-2556) -------
    def cond_info(self) -> AceMiCondInfo:
        info = AceMiCondInfo()
        self._ensure_ok(self.lib.ace_mi_cond_get_info(self.ctx, ctypes.byref(info)), "ace_mi_cond_get_info")
        return info

    def text_project(self, states) -> np.ndarray:
        """encoder.text_projector: [n, in] -> [n, H]."""
        x = np.ascontiguousarray(states, dtype=np.float32)
        out = np.empty((x.shape[0], self.cond_info().hidden_size), np.float32)
        st = self.lib.ace_mi_text_project(self.ctx, _fptr(x), int(x.shape[0]), int(x.shape[1]), _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_mi_text_project")
        return out

    def lyric_encode(self, lyric_embeds) -> np.ndarray:
        """Lyric encoder: token embeddings [n, text_hidden] -> [n, H]."""
        x = np.ascontiguousarray(lyric_embeds, dtype=np.float32)
        out = np.empty((x.shape[0], self.cond_info().hidden_size), np.float32)
        st = self.lib.ace_mi_lyric_encode(self.ctx, _fptr(x), int(x.shape[0]), _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_mi_lyric_encode")
        return out

    def timbre_encode(self, refer, order_mask=None) -> np.ndarray:
        """Timbre encoder: references [n_refer, refer_len, timbre_in] -> [n_refer, H]."""
        x = np.ascontiguousarray(refer, dtype=np.float32)
        om = None if order_mask is None else np.ascontiguousarray(order_mask, dtype=np.int32)
        out = np.empty((x.shape[0], self.cond_info().hidden_size), np.float32)
        st = self.lib.ace_mi_timbre_encode(self.ctx, _fptr(x), _iptr(om), int(x.shape[0]), int(x.shape[1]),
                                           _fptr(out), out.nbytes)
        self._ensure_ok(st, "ace_mi_timbre_encode")
        return out

    def build_condition(self, style_states=None, lyric_embeds=None, refer=None, refer_order_mask=None,
                        text_hidden: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """(encoder_hidden_states [len, H], encoder_attention_mask [len]) from text-encoder style states,
        lyric token embeddings and timbre references."""
        ss = None if style_states is None else np.ascontiguousarray(style_states, dtype=np.float32)
        le = None if lyric_embeds is None else np.ascontiguousarray(lyric_embeds, dtype=np.float32)
        rf = None if refer is None else np.ascontiguousarray(refer, dtype=np.float32)
        om = None if refer_order_mask is None else np.ascontiguousarray(refer_order_mask, dtype=np.int32)
        ns = 0 if ss is None else int(ss.shape[0])
        nl = 0 if le is None else int(le.shape[0])
        nr, rl = (0, 0) if rf is None else (int(rf.shape[0]), int(rf.shape[1]))
        if text_hidden is None:
            text_hidden = int(ss.shape[1]) if ss is not None else (int(le.shape[1]) if le is not None else 0)
        H = self.cond_info().hidden_size
        cap = max(ns + nl + nr, 1)
        enc = np.empty((cap, H), np.float32)
        mask = np.empty(cap, np.int32)
        n = ctypes.c_int32(0)
        st = self.lib.ace_mi_build_condition(self.ctx, _fptr(ss), ns, _fptr(le), nl, int(text_hidden), _fptr(rf),
                                             _iptr(om), nr, rl, _fptr(enc), enc.nbytes, _iptr(mask), mask.nbytes,
                                             ctypes.byref(n))
        self._ensure_ok(st, "ace_mi_build_condition")
        return enc[: n.value].copy(), mask[: n.value].copy()

    # -- MI355X extensions ---------------------------------------------------
    def vae_enc_out_len(self, n_samples: int) -> int:
        n = ctypes.c_int64(0)
        st = self.lib.ace_mi_vae_enc_out_len(self.ctx, int(n_samples), ctypes.byref(n))
        self._ensure_ok(st, "ace_mi_vae_enc_out_len")
        return int(n.value)

    def vae_encode_device(self, d_audio: int, n_samples: int, d_out: int, stream: int = 0) -> None:
        st = self.lib.ace_mi_vae_encode_device(self.ctx, d_audio, int(n_samples), d_out, stream or None)
        self._ensure_ok(st, "ace_mi_vae_encode_device")

    def vae_out_len(self, n_frames: int) -> int:
        n = ctypes.c_int64(0)
        self._ensure_ok(self.lib.ace_mi_vae_out_len(self.ctx, int(n_frames), ctypes.byref(n)), "ace_mi_vae_out_len")
        return int(n.value)

    def vae_decode_device(self, d_latents: int, n_frames: int, d_out: int, stream: int = 0) -> None:
        st = self.lib.ace_mi_vae_decode_device(self.ctx, d_latents, int(n_frames), d_out, stream or None)
        self._ensure_ok(st, "ace_mi_vae_decode_device")

    def dit_forward_batched_device(self, batch: int, seq_len: int, enc_len: int, d_hidden: int, d_context: int,
                                   d_enc: int, d_mask: int, d_enc_mask: int, d_t: int, d_r: int, d_out: int,
                                   stream: int = 0) -> None:
        st = self.lib.ace_mi_dit_forward_batched(self.ctx, int(batch), d_hidden or None, d_context or None,
                                                 d_enc or None, d_mask or None, d_enc_mask or None, int(seq_len),
                                                 int(enc_len), d_t, d_r, d_out, stream or None)
        self._ensure_ok(st, "ace_mi_dit_forward_batched")

    def dit_sample_device(self, batch: int, seq_len: int, enc_len: int, d_xt: int, d_context: int, d_enc: int,
                          d_mask: int, d_enc_mask: int, schedule: List[float], stream: int = 0) -> None:
        sched = np.ascontiguousarray(schedule, dtype=np.float32)
        st = self.lib.ace_mi_dit_sample(self.ctx, int(batch), d_xt, d_context or None, d_enc or None,
                                        d_mask or None, d_enc_mask or None, int(seq_len), int(enc_len),
                                        _fptr(sched), int(sched.shape[0]), stream or None)
        self._ensure_ok(st, "ace_mi_dit_sample")

    def dit_sample_ex_device(self, batch: int, seq_len: int, enc_len: int, d_xt: int, d_context: int, d_enc: int,
                             d_mask: int, d_enc_mask: int, schedule: List[float], sde: bool = False, d_noise: int = 0,
                             cover_steps: int = -1, d_context_nc: int = 0, d_enc_nc: int = 0,
                             cache_cross: bool = True, stream: int = 0) -> None:
        """The MLX/PyTorch generation loop on the device (ace_mi_dit_sample_ex)."""
        sched = np.ascontiguousarray(schedule, dtype=np.float32)
        st = self.lib.ace_mi_dit_sample_ex(self.ctx, int(batch), d_xt, d_context or None, d_enc or None,
                                           d_mask or None, d_enc_mask or None, int(seq_len), int(enc_len),
                                           _fptr(sched), int(sched.shape[0]), 1 if sde else 0, d_noise or None,
                                           int(cover_steps), d_context_nc or None, d_enc_nc or None,
                                           1 if cache_cross else 0, stream or None)
        self._ensure_ok(st, "ace_mi_dit_sample_ex")

    def synchronize(self) -> None:
        self._ensure_ok(self.lib.ace_mi_synchronize(self.ctx), "ace_mi_synchronize")

    def set_attn_precision(self, mode: str) -> None:
        """DiT attention operand precision for subsequent forwards: "fp16", "split", "f32", "f8c" or "pv8"
        (include/acestep_mi355x.h, ace_mi_dit_set_attn_precision)."""
        code = {"fp16": 0, "split": 1, "f32": 2, "f8c": 3, "pv8": 4}[mode]
        self._ensure_ok(self.lib.ace_mi_dit_set_attn_precision(self.ctx, code), "ace_mi_dit_set_attn_precision")

    def profile_enable(self, on: bool) -> None:
        self._ensure_ok(self.lib.ace_mi_profile_enable(self.ctx, 1 if on else 0), "ace_mi_profile_enable")

    def profile_reset(self) -> None:
        self._ensure_ok(self.lib.ace_mi_profile_reset(self.ctx), "ace_mi_profile_reset")

    def profile_get(self) -> List[Tuple[str, float, int]]:
        cap = 64
        names = ctypes.create_string_buffer(8192)
        ms = (ctypes.c_double * cap)()
        counts = (ctypes.c_int32 * cap)()
        n = ctypes.c_int32(0)
        self._ensure_ok(self.lib.ace_mi_profile_get(self.ctx, names, 8192, ms, counts, cap, ctypes.byref(n)),
                        "ace_mi_profile_get")
        raw = names.raw.split(b"\0")
        return [(raw[i].decode(), float(ms[i]), int(counts[i])) for i in range(min(n.value, cap))]

    def probe_gemm(self, which: int, m_rows: int, iters: int) -> None:
        self._ensure_ok(self.lib.ace_mi_probe_gemm(self.ctx, int(which), int(m_rows), int(iters)),
                        "ace_mi_probe_gemm")


# ---- kernel self-test wrappers (GPU parity tests) ----------------------------
def kernel_gemm(a_bits: np.ndarray, w_bits: np.ndarray, act_type: int = 0, epi: int = 0,
                bias: Optional[np.ndarray] = None, x: Optional[np.ndarray] = None) -> np.ndarray:
    """a_bits [M][K], w_bits [N][K] uint16 words; epi 0 -> f32 [M][N], epi 4 -> uint16 [M][N/2];
    epi 3 / 2 -> f32 x + C (* gate) with x [M][N] f32 and, for epi 2, the gate [N] passed as `bias`."""
    lib = load_selftest_library()
    a = np.ascontiguousarray(a_bits, dtype=np.uint16)
    w = np.ascontiguousarray(w_bits, dtype=np.uint16)
    M, K = a.shape
    N = w.shape[0]
    u16p = ctypes.POINTER(ctypes.c_uint16)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    if epi in (2, 3):
        out = np.array(x, dtype=np.float32, order="C", copy=True)
        st = lib.ace_mi_kernel_gemm(act_type, epi, M, N, K, a.ctypes.data_as(u16p), w.ctypes.data_as(u16p),
                                    _fptr(b), _fptr(out), None)
    elif epi == 0:
        out = np.empty((M, N), dtype=np.float32)
        st = lib.ace_mi_kernel_gemm(act_type, epi, M, N, K, a.ctypes.data_as(u16p), w.ctypes.data_as(u16p),
                                    _fptr(b), _fptr(out), None)
    else:
        out = np.empty((M, N // 2), dtype=np.uint16)
        st = lib.ace_mi_kernel_gemm(act_type, epi, M, N, K, a.ctypes.data_as(u16p), w.ctypes.data_as(u16p),
                                    _fptr(b), None, out.ctypes.data_as(u16p))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_kernel_gemm failed (status={st})")
    return out


def kernel_attention(q: np.ndarray, kv: np.ndarray, hq: int, hkv: int, window: int = 0,
                     kmask: Optional[np.ndarray] = None, scale: Optional[float] = None,
                     split: bool = True, causal: bool = False, pv_split: bool = False, f8: bool = False) -> np.ndarray:
    """q [B][nq][hq*128] f32, kv [B][nk][2*hkv*128] f32 -> out [B][nq][hq*128] f32 (bf16-rounded).
    split: hi/lo fp16 Q.K; pv_split: hi/lo fp16 P.V too (both = the fully f32-faithful mode); f8 (with both):
    the f8c mode (fp8 correction products); f8 with pv_split and not split: the pv8 mode (fp16 Q.K, f8c P.V)."""
    lib = load_selftest_library()
    q = np.ascontiguousarray(q, dtype=np.float32)
    kv = np.ascontiguousarray(kv, dtype=np.float32)
    B, nq, _ = q.shape
    nk = kv.shape[1]
    km = None if kmask is None else np.ascontiguousarray(kmask, dtype=np.int32)
    out = np.empty_like(q)
    sc = float(scale) if scale is not None else 1.0 / np.sqrt(128.0)
    st = lib.ace_mi_kernel_attention(B, hq, hkv, nq, nk, int(window), sc, (1 if split else 0) | (2 if causal else 0)
                                     | (8 if pv_split else 0) | (16 if f8 else 0), _fptr(q), _fptr(kv),
                                     _iptr(km), _fptr(out))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_kernel_attention failed (status={st})")
    return out


def bench_attention(B: int, hq: int, hkv: int, nq: int, nk: int, window: int = 0, split: bool = True,
                    causal: bool = False, masked: bool = False, iters: int = 20, pv_split: bool = False,
                    f8: bool = False) -> float:
    """Average ms per launch of the engine's attention kernel on pseudo-random operands (GPU)."""
    lib = load_selftest_library()
    ms = ctypes.c_float(0.0)
    flags = (1 if split else 0) | (2 if causal else 0) | (4 if masked else 0) | (8 if pv_split else 0) | \
        (16 if f8 else 0)
    st = lib.ace_mi_bench_attention(B, hq, hkv, nq, nk, int(window), flags, iters, ctypes.byref(ms))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_bench_attention failed (status={st})")
    return float(ms.value)


def bench_gemm(M: int, N: int, K: int, variant: int = -1, epi: int = 0, act_type: int = 0, iters: int = 20) -> float:
    """Average ms per launch of the engine GEMM on random operands (GPU)."""
    lib = load_selftest_library()
    ms = ctypes.c_float(0.0)
    st = lib.ace_mi_bench_gemm(act_type, epi, variant, M, N, K, iters, ctypes.byref(ms))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_bench_gemm failed (status={st})")
    return float(ms.value)


_BLOCK = {"q8_0": (32, 34), "q4_k": (256, 144), "q6_k": (256, 210)}


def quantize(x: np.ndarray, qtype: str) -> np.ndarray:
    """The loader's ggml block encoder on host rows: f32 [rows][cols] -> uint8 [rows][nb][block bytes]."""
    lib = load_library()
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, cols = x.shape
    qk, bb = _BLOCK[qtype]
    out = np.empty((rows, cols // qk, bb), dtype=np.uint8)
    n = lib.ace_mi_quantize(QTYPES[qtype], _fptr(x), rows, cols, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                            out.nbytes)
    if n != out.nbytes:
        raise ValueError(f"ace_mi_quantize failed ({qtype}, cols={cols})")
    return out


def dequantize(raw: np.ndarray, qtype: str) -> np.ndarray:
    lib = load_library()
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    rows, nb, _ = raw.shape
    cols = nb * _BLOCK[qtype][0]
    out = np.empty((rows, cols), dtype=np.float32)
    st = lib.ace_mi_dequantize(QTYPES[qtype], raw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), rows, cols,
                               _fptr(out))
    if st != ACE_GGML_OK:
        raise ValueError(f"ace_mi_dequantize failed (status={st})")
    return out


def kernel_dequant(w_blocks: np.ndarray, qtype: str) -> np.ndarray:
    """Staged dequant kernel: ggml block bytes [N][nb][bb] -> bf16 words [N][K] of bf16(dequant(W))."""
    lib = load_selftest_library()
    w = np.ascontiguousarray(w_blocks, dtype=np.uint8)
    N, nb = w.shape[0], w.shape[1]
    K = nb * _BLOCK[qtype][0]
    out = np.empty((N, K), dtype=np.uint16)
    st = lib.ace_mi_kernel_dequant(QTYPES[qtype], N, K, w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_kernel_dequant failed (status={st})")
    return out


def kernel_gemm_q(a_bits: np.ndarray, w_blocks: np.ndarray, qtype: str, epi: int = 0, variant: int = -1,
                  bias: Optional[np.ndarray] = None, x: Optional[np.ndarray] = None) -> np.ndarray:
    """Dequant-fused GEMM: a_bits bf16 words [M][K], w_blocks ggml block bytes [N][nb][bb].  epi 2 / 3: returns
    x + acc (* bias as the per-column gate for 2)."""
    lib = load_selftest_library()
    a = np.ascontiguousarray(a_bits, dtype=np.uint16)
    w = np.ascontiguousarray(w_blocks, dtype=np.uint8)
    M, K = a.shape
    N = w.shape[0]
    u16p = ctypes.POINTER(ctypes.c_uint16)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    if epi in (0, 2, 3):
        out = np.ascontiguousarray(x, dtype=np.float32).copy() if epi in (2, 3) else np.empty((M, N), np.float32)
        st = lib.ace_mi_kernel_gemm_q(QTYPES[qtype], epi, variant, M, N, K, a.ctypes.data_as(u16p),
                                      w.ctypes.data_as(u8p), _fptr(b), _fptr(out), None)
    else:
        out = np.empty((M, N // 2), dtype=np.uint16)
        st = lib.ace_mi_kernel_gemm_q(QTYPES[qtype], epi, variant, M, N, K, a.ctypes.data_as(u16p),
                                      w.ctypes.data_as(u8p), _fptr(b), None, out.ctypes.data_as(u16p))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_kernel_gemm_q failed (status={st})")
    return out


def kernel_gemm_a8(x: np.ndarray, w_blocks: np.ndarray, qtype: str, epi: int = 0, bias: Optional[np.ndarray] = None,
                   x0: Optional[np.ndarray] = None):
    """ggml-faithful quantized-activation GEMM (ACE_MI_QUANT_ACT=q8): x f32 [M][K] quantized on the device, then the
    integer-dot GEMM against ggml block rows w_blocks [N][nb][bb].  epi 0: acc (+ bias); 3: x0 + (acc + bias);
    7: silu(g) * u.  Returns (out, q int8 [M][K], s f32 [K/32][M], bsum f32 [K/32][M])."""
    lib = load_selftest_library()
    xa = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w_blocks, dtype=np.uint8)
    M, K = xa.shape
    N = w.shape[0]
    ncol = N // 2 if epi == 7 else N
    out = np.ascontiguousarray(x0, dtype=np.float32).copy() if epi == 3 else np.empty((M, ncol), np.float32)
    q = np.empty((M, K), np.int8)
    s = np.empty((K // 32, M), np.float32)
    bs = np.empty((K // 32, M), np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    st = lib.ace_mi_kernel_gemm_a8(QTYPES[qtype], epi, M, N, K, _fptr(xa), w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                   _fptr(b), _fptr(out), q.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), _fptr(s),
                                   _fptr(bs))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_kernel_gemm_a8 failed (status={st})")
    return out, q, s, bs


def bench_gemm_q(M: int, N: int, K: int, qtype: str, variant: int = -1, epi: int = 0, iters: int = 20) -> float:
    lib = load_selftest_library()
    ms = ctypes.c_float(0.0)
    st = lib.ace_mi_bench_gemm_q(QTYPES[qtype], epi, variant, M, N, K, iters, ctypes.byref(ms))
    if st != ACE_GGML_OK:
        raise RuntimeError(f"ace_mi_bench_gemm_q failed (status={st})")
    return float(ms.value)


def reference_noise(seed: int, n: int) -> np.ndarray:
    """x_T of the reference generator (std::mt19937 + std::normal_distribution<float>), host code."""
    out = np.empty(int(n), np.float32)
    if load_library().ace_mi_reference_noise(int(seed), int(n), _fptr(out)) != ACE_GGML_OK:
        raise RuntimeError("ace_mi_reference_noise failed")
    return out


def gemm_variant(variant: int) -> None:
    lib = load_library()
    if lib.ace_mi_gemm_variant(int(variant)) != ACE_GGML_OK:
        raise ValueError(variant)


def kernel_attn_kh(mode: int) -> None:
    """f8c attention kernel of this process: -1 environment / default policy, 0 attn2 (one wave per SIMD), 1 attn_kh."""
    if load_selftest_library().ace_mi_kernel_attn_kh(int(mode)) != ACE_GGML_OK:
        raise ValueError(mode)


def kernel_gemm_a8_mode(mode: int) -> None:
    """Q8_0 GEMM form of the q8 mode in this process: -1 environment / default (bf16 MFMA), 0 i8 MFMA, 1 bf16 MFMA."""
    if load_selftest_library().ace_mi_kernel_gemm_a8_mode(int(mode)) != ACE_GGML_OK:
        raise ValueError(mode)
