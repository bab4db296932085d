"""ctypes driver of oracle/cpu/dit_cpu.cpp, the C++/OpenMP restatement of the acestep_ggml CPU DiT forward
-- TEST / BENCH INFRASTRUCTURE ONLY (see oracle/__init__.py): bench.py's `cpu_baseline` times it and
tests/test_cpu_restatement.py checks it against the numpy oracle (dit_oracle.forward_dit).

The weights come from the numpy oracle's loader (dit_oracle.DitWeights: load_model_from_dir,
acestep_dit_model.cpp:753-1088), so both restatements read the checkpoint the same way; BF16 / F16
matrices are handed over as their 16-bit values.  Quantized weights are not restated here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from .ggml_numerics import f32_to_bf16_bits

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu")
LIB = os.path.join(HERE, "libdit_cpu.so")

# dit_cpu.cpp enums
M_PROJ_IN, M_COND, M_PROJ_OUT, M_TE_W1, M_TE_W2, M_TE_WP = range(6)
M_SQ, M_SK, M_SV, M_SO, M_CQ, M_CK, M_CV, M_CO, M_GATE, M_UP, M_DOWN = range(6, 17)
(V_PROJ_IN_B, V_COND_B, V_PROJ_OUT_B, V_NORM_OUT, V_OUT_TABLE, V_TE_B1, V_TE_B2, V_TE_BP, V_SA_NORM, V_CA_NORM,
 V_MLP_NORM, V_SQN, V_SKN, V_CQN, V_CKN, V_TABLE) = range(16)

_lib = None


def build() -> str:
    """make -C oracle/cpu (g++, seconds); returns the library path."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        f, i, p = ctypes.c_float, ctypes.c_int, ctypes.c_void_p
        lib.dcpu_create.restype = p
        lib.dcpu_create.argtypes = [i, i, i, i, i, i, i, i, i, i, f, f, p]
        lib.dcpu_destroy.argtypes = [p]
        lib.dcpu_matrix.argtypes = [p, i, i, i, p, i, i]
        lib.dcpu_vector.argtypes = [p, i, i, p, i]
        lib.dcpu_forward.argtypes = [p, p, p, p, p, p, i, i, f, f, i, p]
        lib.dcpu_isa.restype = i
        _lib = lib
    return _lib


def isa_name() -> str:
    return {2: "avx512+avx512bf16", 1: "avx512", 0: "scalar"}[load().dcpu_isa()]


class CpuDit:
    """One loaded model of the C++ restatement.  `W` is a dit_oracle.DitWeights with BF16 / F16 weights."""

    def __init__(self, W):
        lib = load()
        c = W.cfg
        self.cfg = c
        self._keep = []
        sliding = np.array([1 if L["sliding"] else 0 for L in W.layers], np.int32)
        self.h = lib.dcpu_create(c.hidden_size, c.intermediate_size, len(W.layers), c.num_attention_heads,
                                 c.num_key_value_heads, c.head_dim, c.patch_size, c.in_channels,
                                 c.audio_acoustic_hidden_dim, c.sliding_window, c.rms_norm_eps, c.rope_theta,
                                 sliding.ctypes.data)
        self._keep.append(sliding)

        def mat(mid, layer, gw):
            if gw.wtype == "bf16":
                bits, t = f32_to_bf16_bits(gw.values), 0
            elif gw.wtype == "f16":
                bits, t = gw.values.astype(np.float16).view(np.uint16), 1
            else:
                raise ValueError(f"CPU restatement: weight type {gw.wtype} not restated")
            bits = np.ascontiguousarray(bits, dtype=np.uint16)
            rows, cols = bits.shape
            if lib.dcpu_matrix(self.h, mid, layer, t, bits.ctypes.data, rows, cols) != 0:
                raise ValueError("dcpu_matrix: shape")

        def vec(vid, layer, v):
            v = np.ascontiguousarray(np.asarray(v, np.float32).reshape(-1))
            lib.dcpu_vector(self.h, vid, layer, v.ctypes.data, v.size)

        mat(M_PROJ_IN, -1, W.proj_in_w)
        vec(V_PROJ_IN_B, -1, W.proj_in_b)
        mat(M_COND, -1, W.condition_w)
        vec(V_COND_B, -1, W.condition_b)
        mat(M_PROJ_OUT, -1, W.proj_out_w)
        vec(V_PROJ_OUT_B, -1, W.proj_out_b)
        vec(V_NORM_OUT, -1, W.norm_out)
        vec(V_OUT_TABLE, -1, W.out_table)
        for e, tag in enumerate(("time_embed", "time_embed_r")):
            tw = W.time_embed[tag]
            for mid, vid, k in ((M_TE_W1, V_TE_B1, "1"), (M_TE_W2, V_TE_B2, "2"), (M_TE_WP, V_TE_BP, "p")):
                mat(mid, e, tw["w" + k])
                vec(vid, e, tw["b" + k])
        for li, L in enumerate(W.layers):
            sa, ca, mlp = L["self_attn"], L["cross_attn"], L["mlp"]
            for mid, gw in ((M_SQ, sa["q"]), (M_SK, sa["k"]), (M_SV, sa["v"]), (M_SO, sa["o"]), (M_CQ, ca["q"]),
                            (M_CK, ca["k"]), (M_CV, ca["v"]), (M_CO, ca["o"]), (M_GATE, mlp["gate"]),
                            (M_UP, mlp["up"]), (M_DOWN, mlp["down"])):
                mat(mid, li, gw)
            for vid, v in ((V_SA_NORM, L["self_attn_norm"]), (V_CA_NORM, L["cross_attn_norm"]),
                           (V_MLP_NORM, L["mlp_norm"]), (V_SQN, sa["q_norm"]), (V_SKN, sa["k_norm"]),
                           (V_CQN, ca["q_norm"]), (V_CKN, ca["k_norm"]), (V_TABLE, L["table"])):
                vec(vid, li, v)

    def forward(self, hidden, context, enc, mask, enc_mask, T: int, L: int, t: float, r: float,
                max_layers: int = 0) -> np.ndarray:
        """forward_dit for one sample (same arguments as dit_oracle.forward_dit) -> [T][64] f32."""
        c = self.cfg
        arr = lambda x, dt: None if x is None else np.ascontiguousarray(np.asarray(x, dt))
        h, cx, e = arr(hidden, np.float32), arr(context, np.float32), arr(enc, np.float32)
        m, em = arr(mask, np.int32), arr(enc_mask, np.int32)
        out = np.empty((T, c.audio_acoustic_hidden_dim), np.float32)
        ptr = lambda x: None if x is None else x.ctypes.data
        load().dcpu_forward(self.h, ptr(h), ptr(cx), ptr(e), ptr(m), ptr(em), T, L, float(t), float(r),
                            int(max_layers or 0), out.ctypes.data)
        return out

    def close(self):
        if self.h:
            load().dcpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
