"""GPU diagnostic for the dequant-fused GEMM: A = identity (bf16 one-hot rows), so out[k][n] is the
kernel's view of bf16(dequant(W))[n][k].  Prints which (n, k) entries differ from the host dequant,
per qtype / tile variant, over repeated launches (determinism)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np

from acestep_mi355x import capi
from oracle import ggml_numerics as g
from oracle.ggml_numerics import f32_to_bf16_bits

DEQ = {"q8_0": lambda r: g.dequantize_q8_0(*g.unpack_q8_0(r)), "q4_k": g.dequantize_q4_k, "q6_k": g.dequantize_q6_k}


def main():
    print("lib:", os.environ.get("ACE_MI_LIB", "default"), flush=True)
    K, N = 512, 256
    rng = np.random.default_rng(5)
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    a = f32_to_bf16_bits(np.eye(K, dtype=np.float32))
    for qtype in ("q8_0", "q4_k", "q6_k"):
        blocks = capi.quantize(w, qtype)
        want = g.round_bf16(DEQ[qtype](blocks)).astype(np.float32)  # [N][K]
        for variant in (1, 2, 3, 4, 5, 7):
            prev = None
            for rep in range(3):
                got = capi.kernel_gemm_q(a, blocks, qtype, epi=0, variant=variant).T  # [N][K]
                bad = np.argwhere(got != want)
                same = prev is not None and np.array_equal(prev, got)
                prev = got
                msg = f"{qtype} v{variant} rep{rep}: bad={len(bad)} same_as_prev={same}"
                if len(bad):
                    ns, ks = np.unique(bad[:, 0]), np.unique(bad[:, 1])
                    n0, k0 = bad[0]
                    msg += (f" n[{len(ns)}]={ns[:24].tolist()} k[{len(ks)}]={ks[:24].tolist()}"
                            f" e.g. got={got[n0, k0]:.6g} want={want[n0, k0]:.6g}"
                            f" nearest_equal_k={[int(x) for x in np.where(want[n0] == got[n0, k0])[0][:4]]}")
                    # fp-rounding-only mismatch?  (differences of one bf16 ulp)
                    rel = np.abs(got[bad[:, 0], bad[:, 1]] - want[bad[:, 0], bad[:, 1]]) / np.maximum(
                        np.abs(want[bad[:, 0], bad[:, 1]]), 1e-30)
                    msg += f" max_rel={rel.max():.3g} median_rel={np.median(rel):.3g}"
                    if rep == 0:
                        from collections import Counter
                        nk = Counter((int(n) % 32, int(k) % 64) for n, k in bad)
                        kt = Counter(int(k) // 64 for _, k in bad)
                        # stale-value hypotheses: the value two tiles earlier / the other K half
                        vals = got[bad[:, 0], bad[:, 1]]
                        st2 = np.mean(vals == want[bad[:, 0], np.maximum(bad[:, 1] - 128, 0)])
                        msg += f"\n   (n%32,k%64)={sorted(nk.items())[:40]}\n   tiles={sorted(kt.items())} stale2={st2:.2f}"
                print(msg, flush=True)




def stress(reps=20):
    """The failing shape of the parity suite (M=129, N=768, K=6144), repeated: count bad launches."""
    from test_gpu_quant import _q_ref  # noqa
    M, N, K = 129, 768, 6144
    rng = np.random.default_rng(1)
    a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    for qtype in ("q4_k", "q6_k", "q8_0"):
        blocks = capi.quantize(w, qtype)
        ref, scale = _q_ref(a, blocks, qtype)
        for variant in (1, 2, 3, 4, 5, 7):
            nbad = 0
            worst = 0.0
            for _ in range(reps):
                got = capi.kernel_gemm_q(a, blocks, qtype, epi=0, variant=variant)
                e = np.abs(got - ref) / (scale + 1e-6)
                worst = max(worst, float(e.max()))
                nbad += int(np.any(np.abs(got - ref) > 2e-6 * scale + 1e-6))
            print(f"stress {qtype} v{variant}: bad launches {nbad}/{reps} worst={worst:.3g}", flush=True)


if __name__ == "__main__":
    main()
    stress(int(os.environ.get("STRESS_REPS", "20")))
