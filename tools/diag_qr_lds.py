"""Diagnostic (GPU box, ACEMI_QR_DIAG build via tools/build_ab.sh qrdiag "-DACEMI_QR_DIAG" gemm_q): what the
register-dequant kernel's lanes actually read from LDS.  Every lane stores its q words and scales of every k-tile as
first read, and the same LDS words re-read after the tile's MFMAs.  All blocks of one column tile read the same
weight bytes, so the per-(k-tile, lane) majority over blocks is the expected value: a first read that differs from it
while the re-read agrees is a DMA that landed late; both wrong is a DMA that wrote the wrong place (or was overwritten)."""
import ctypes
import os
import sys
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ace-step-1.5-ggml_amd"), ROOT, os.path.join(ROOT, "tests")]
from acestep_mi355x import capi  # noqa: E402
from oracle.ggml_numerics import f32_to_bf16_bits  # noqa: E402
from test_gpu_quant import _q_ref  # noqa: E402

W = 24  # words per lane per k-tile


def main():
    st = capi.load_selftest_library()
    rd = st.ace_mi_qr_diag_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rd.restype = ctypes.c_int
    reps = int(os.environ.get("REPS", "3"))
    for qtype in ("q4_k", "q8_0"):
        for v, nw in ((21, 8), (20, 4)):
            for (M, K) in [(1000, 2048), (1500, 1024)]:
                N = 32 * nw
                rng = np.random.default_rng(M + N + K)
                a = f32_to_bf16_bits(rng.standard_normal((M, K)).astype(np.float32))
                w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
                blocks = capi.quantize(w, qtype)
                ref, scale = _q_ref(a, blocks, qtype)
                BN, BM = 32 * nw, 192
                nblk = ((M + BM - 1) // BM) * (N // BN)
                nk = K // 64
                for rep in range(reps):
                    assert rd(None, 0, 1) == 0
                    got = capi.kernel_gemm_q(a, blocks, qtype, epi=0, variant=v | 0x10000)
                    bad = np.abs(got - ref) > 2e-6 * scale + 1e-6
                    buf = np.empty(nblk * nk * nw * 64 * W, np.uint32)
                    assert rd(buf.ctypes.data, buf.size, 0) == 0
                    d = buf.reshape(nblk, nk, nw, 64, 2, 12)
                    first = d[..., :8]
                    # expected: majority over blocks (all blocks share the weights when N == BN)
                    if N == BN and nblk >= 3:
                        exp = np.sort(first.reshape(nblk, -1), axis=0)[nblk // 2].reshape(first.shape[1:])
                        wrong = first != exp[None]
                    else:
                        wrong = np.zeros(first.shape, bool)
                    # re-read vs first read (words 8..11 = q[j][0][0], q[j][1][0], sc.x, sc.z)
                    again = d[..., 8:12]
                    firstsel = first[..., [0, 2, 4, 6]]
                    changed = again != firstsel
                    msg = (f"{qtype} v{v} M={M} N={N} K={K} rep{rep}: bad outputs {int(bad.sum())}, "
                           f"wrong first reads {int(wrong.sum())}, changed on re-read {int(changed.sum())}")
                    if wrong.any():
                        b_, kt_, w_, l_, j_, k_ = np.nonzero(wrong)
                        msg += (f"\n   wrong: waves {sorted(set(w_.tolist()))} kt {sorted(set(kt_.tolist()))[:12]} "
                                f"blocks {sorted(set(b_.tolist()))} j {sorted(set(j_.tolist()))} word {sorted(set(k_.tolist()))} "
                                f"lanes {len(set(l_.tolist()))}")
                        # did the re-read match the expectation?
                        exp_sel = exp[..., [0, 2, 4, 6]]
                        again_ok = (again == exp_sel[None])
                        msg += f"\n   re-read equals expected where first read wrong: " \
                               f"{int(again_ok[wrong[..., [0, 2, 4, 6]]].sum())}/{int(wrong[..., [0, 2, 4, 6]].sum())}"
                        # is the wrong value the previous occupant of that slot (tile kt - RS)?
                        for rs in (3, 4):
                            prev_hit = 0
                            tot = 0
                            for (bb, kk, ww, ll, jj, kw) in zip(b_, kt_, w_, l_, j_, k_):
                                if kk >= rs:
                                    tot += 1
                                    prev_hit += int(first[bb, kk, ww, ll, jj, kw] == exp[kk - rs, ww, ll, jj, kw])
                            msg += f"\n   wrong value == expected of tile kt-{rs}: {prev_hit}/{tot}"
                    if bad.any():
                        rows, cols = np.nonzero(bad)
                        msg += f"\n   bad col groups {sorted(set((cols % BN // 16).tolist()))}"
                    print(msg, flush=True)


if __name__ == "__main__":
    main()
