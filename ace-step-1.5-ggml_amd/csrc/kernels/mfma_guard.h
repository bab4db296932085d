// MFMA operand write-after-read guards shared by every MFMA kernel (gemm*.hip, vae.hip, attention.hip).
// tools/audit_mfma_war.py checks the built .s for VALU writes to an in-flight MFMA's A / B registers;
// tests/test_mfma_war_audit.py fails on any such pair in a kernel that can run two waves per SIMD.
#pragma once

#include <hip/hip_runtime.h>

namespace acemi {

typedef __attribute__((ext_vector_type(4))) unsigned mfma_guard_u32x4;

// MFMA operand write-after-read guard.  On gfx950 with two waves per SIMD, a VALU that writes an A / B source register of
// an MFMA issued just before it can corrupt that product: the register-dequant tile with the kk = 1 dequant VALU
// scheduled between the kk = 0 MFMAs (hipcc pads this pair for the C operand only) gave whole wrong 16-column groups
// of waves 4-7 on some launches -- rounds 3-4's "variant 21 x Q4_K" and "64-row tile not run-to-run identical"
// anomalies.  Measured (tools/diag_v21.py, profiles/r05/qr_war/): a scheduling fence between the MFMA block and the
// VALU that follows it removes every failure; padding only the end of the tile does not.  The fence keeps hipcc from
// interleaving the two, the s_nops keep 16 wait states between the last MFMA and the first overwrite.  The same
// fence between the dequant VALU and the MFMAs that read its B fragments (read-after-write) made the split-K forms
// (223 / 423) and the residual epilogue of 21 x Q4_K exact as well (profiles/r05/qr_war/).
__device__ __forceinline__ void mfma_war_guard() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}

// The same guard for an MFMA block whose operands are register arrays (round 6, tools/audit_mfma_war.py): the fence
// keeps later instructions out of the block, and an empty asm use of every operand fragment AFTER the 16 wait states
// keeps those registers allocated until then, so no instruction that hipcc interleaves INTO the block (address VALU of
// the next LDS-DMA, epilogue setup) can be given an operand register that an earlier MFMA of the block still reads.
__device__ __forceinline__ void mfma_keep(const uint4& x) { asm volatile("" ::"v"(__builtin_bit_cast(mfma_guard_u32x4, x))); }
template <int N>
__device__ __forceinline__ void mfma_keep(const uint4 (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) mfma_keep(x[i]);
}
template <int N, int K>
__device__ __forceinline__ void mfma_keep(const uint4 (&x)[N][K]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int k = 0; k < K; ++k) mfma_keep(x[i][k]);
}
#ifndef ACEMI_NO_WAR_RETIRE
#define ACEMI_NO_WAR_RETIRE 0  // (1: A/B diagnostic builds only, tools/build_ab.sh -- the round-5 code without the retire)
#endif
template <class... F>
__device__ __forceinline__ void mfma_war_retire(const F&... frags) {
    if constexpr (ACEMI_NO_WAR_RETIRE) return;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7");
    (mfma_keep(frags), ...);
    __builtin_amdgcn_sched_barrier(0);
}

}  // namespace acemi
