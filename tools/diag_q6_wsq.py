import os, sys, numpy as np
sys.path[:0] = ["ace-step-1.5-ggml_amd", ".", "tests"]
from acestep_mi355x import capi
from oracle.ggml_numerics import f32_to_bf16_bits, bf16_bits_to_f32
from test_gpu_quant import _q_ref
for qt in ("q6_k", "q4_k", "q8_0"):
    for (M, N, K, epi) in [(3000, 2048, 6144, 0), (3000, 1024, 2048, 0), (3000, 512, 2048, 4), (1500, 2048, 2048, 0)]:
        rng = np.random.default_rng(M + N + K)
        a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
        w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
        blocks = capi.quantize(w, qt)
        ref, scale = _q_ref(a, blocks, qt)
        for v in (25, 20):
            got = capi.kernel_gemm_q(a, blocks, qt, epi=epi, variant=v)
            if epi == 4:
                got = bf16_bits_to_f32(got)
                I = N // 2
                gcols = np.concatenate([np.arange(g * 32, g * 32 + 16) for g in range(I // 16)])
                gv, uv = ref[:, gcols], ref[:, gcols + 16]
                sw = gv / (1.0 + np.exp(-gv)) * uv
                err = np.max(np.abs(got - sw) / (np.abs(sw).max()))
                print(qt, v, M, N, K, epi, "swiglu max rel", err, flush=True)
            else:
                bad = np.abs(got - ref) > 2e-6 * scale + 1e-6
                print(qt, v, M, N, K, epi, "bad", int(bad.sum()), "of", bad.size, flush=True)
