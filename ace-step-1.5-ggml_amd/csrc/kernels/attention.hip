// Flash-style attention for the DiT self/cross attention (gfx950 / CDNA4).
//
// Replaces the materialised ggml graph of attention()
// (acestep_dit_model.cpp:1212-1256): kq = K.Q (F32), *1/sqrt(D), + mask,
// soft_max, V.attn, with GQA head h -> kv head h / n_rep
// (repeat_kv_interleave :1118-1130) and the additive mask of
// build_attention_mask (:1132-1173: key padding, bidirectional sliding window
// |q-k| <= w), plus the causal mask of the Qwen3 text encoder
// (qwen_model.cpp:618-637).  Scores never touch HBM; the sliding layers visit
// only the key tiles inside the window, causal blocks stop at their last query.
//
// Numerics: the reference runs attention in F32 (ggml_mul_mat_set_prec(kq, GGML_PREC_F32), acestep_dit_model.cpp:
// 1238-1251).  Four operand modes (AttnArgs split / pv_split / f8; ACE_MI_ATTN_PRECISION):
//   fp16   single fp16 operands, f32 accumulation (two workgroups per CU);
//   split  Q and K as fp16 pairs x = hi + lo (hi = fp16(x), lo = fp16(x - hi)): each score is hi*hi + hi*lo + lo*hi
//          (three v_mfma_f32_32x32x16_f16, ~22-bit operands); P.V single fp16 (P rounded to nearest, V hi);
//   f32    the same three-product form for P.V too (P hi = fp16 toward zero, lo = fp16(P - hi));
//   f8c    (the DiT default) hi x hi in fp16 as above, the correction products Kl.Qh + Kh.Ql and Vl.Ph + Vh.Pl as
//          block-scaled e4m3 MFMAs (v_mfma_scale_f32_32x32x64_f8f6f4, K = 64; the lo parts stored as fp8(2^11 lo)
//          and scaled back by the MFMA's E8M0 block scale): ~2^-15 relative per product instead of ~2^-22, at 2/3 of
//          the f32 mode's matrix-core time; meets the literal 1e-3 one-layer parity bound (tests/test_gpu_parity_strict.py).
// P is formed as exp2(s - m + PSCALE) (2^12 in the fp16 hi/lo modes so the lo part stays a normal fp16; 2^5 in f8c so P
// stays inside e4m3's range; O and l carry the same factor).
// Online softmax in f32 (exp2 domain) with a lazy running max: O and l are
// rescaled only when a row's max grows by more than 2^RESCALE_LOG2 (P then
// stays below 2^15, inside fp16), which after the first tiles is almost never.
// A row whose keys are all masked yields 0/0 = NaN exactly like ggml's
// soft_max of an all -inf row.
//
// Structure: one workgroup = 4 waves = (batch item, kv head, 128 query rows
// spread over the n_rep q heads sharing that kv head), so each K/V tile is
// staged once for all heads of the group.  Each wave owns 32 query rows and
// computes S^T = K.Q^T (swapped), so a lane holds one query's scores in
// registers: row max / sum are in-register + one cross-half shuffle.  The
// S^T accumulator registers are, after f16 packing, directly the B operand of
// O^T = V^T . P^T (the k order inside a 16-key step is permuted; V^T is stored
// with the matching permutation by the prep kernel), so P never goes through
// LDS and the per-row rescale factor is lane-local.
//
// Software pipeline (one wave per SIMD, so the wave itself must overlap its
// VALU softmax with its MFMAs): iteration i issues the MFMAs of S(i+1) while
// it turns S(i) into P(i) (exp2, row sums, fp16 hi/lo packing), then the
// MFMAs of O += V(i) P(i) while it scales and masks S(i+1) and takes its row
// max.  K and V^T tiles arrive by global_load_lds into two 2-slot rings in
// LDS: K(i+2) and V(i+1) are requested at the top of iteration i (their
// slots were last read in iteration i-1) and land by its closing barrier.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../kernels.h"
#include "lds_asm.h"

namespace acemi {
namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int D = 128;
constexpr int KT = 64;                    // keys per tile
constexpr int K_BYTES = KT * D * 2;       // 16 KiB
constexpr int V_BYTES = D * KT * 2;       // 16 KiB
constexpr float PSCALE_LOG2 = 12.0f;
constexpr float RESCALE_LOG2 = 3.0f;      // P <= 2^(12+3) = 32768 < fp16 max

// LDS rings.  K slot: [key bias (64 f32) | K hi | K lo]; V slot: [V^T hi | V^T lo].  All fragment
// reads of the K ring use a 16-bit immediate offset from a per-lane address; the V ring has its own
// base register (it starts past 64 KiB).
template <bool SPLIT, bool PVS>
struct Ring {
    static constexpr int KB = 0;
    static constexpr int K_HI = KT * 4;
    static constexpr int K_LO = K_HI + K_BYTES;
    static constexpr int KS = K_HI + (SPLIT ? 2 : 1) * K_BYTES;  // one K slot
    static constexpr int V_LO = V_BYTES;
    static constexpr int VS = (PVS ? 2 : 1) * V_BYTES;            // one V slot
    static constexpr int V0 = 2 * KS;                              // V ring start
    static constexpr int BYTES = 2 * KS + 2 * VS;
    static_assert(KS + K_LO + 32 * 256 + 255 < 65536, "K reads need 16-bit offsets");
    static_assert(VS + V_LO + 3 * 32 * 128 + 127 < 65536, "V reads need 16-bit offsets");
};

typedef u32x4_t frag;  // 8 fp16 of one MFMA operand
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;

__device__ __forceinline__ f32x16 mfma32(const frag& a, const frag& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

typedef __attribute__((ext_vector_type(8))) int v8i;
__device__ __forceinline__ v8i cat8(const frag& x, const frag& y) {
    return v8i{(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)y[0], (int)y[1], (int)y[2], (int)y[3]};
}
__device__ __forceinline__ v8i cat8(const uint32_t (&w)[8]) {
    return v8i{(int)w[0], (int)w[1], (int)w[2], (int)w[3], (int)w[4], (int)w[5], (int)w[6], (int)w[7]};
}
// f8c mode: block-scaled e4m3 x e4m3 MFMA, K = 64, with E8M0 scales (127 = 1, 116 = 2^-11) on A and B
constexpr int F8_SCALE_1 = 127;
constexpr int F8_SCALE_LO = 127 - 11;
constexpr float PSCALE_F8_LOG2 = 5.0f;  // f8c: P <= 2^(5 + RESCALE_LOG2) = 256, inside e4m3 (max 448)
// attn2_kernel: fragment reads are issued RA steps ahead of their MFMA (ring of RA + 1 fragment sets)
#ifndef ACEMI_ATTN_RA
#define ACEMI_ATTN_RA 2
#endif
constexpr int RA = ACEMI_ATTN_RA;
// attn_kh_kernel (round 6): 1 = each phase's wait-and-barrier after its 7th step, the next phase's first RA fragments read
// right behind it (0 = the barriers between the phases, A/B builds only)
#ifndef ACEMI_KH_EARLY
#define ACEMI_KH_EARLY 1
#endif
// Diagnostic ablation (A/B builds only, tools/build_ab.sh; results wrong by design): 1 = no next-tile LDS-DMA inside
// the attn2 pipeline (every tile computes on the prologue's K / V), 2 = no exp2 in the softmax finish (P = the raw
// score), 4 = no P lo formation in phase C (f8c / pv8), 8 = no workgroup barrier inside the tile loop, 16 = no wait
// for the fragment reads before each step's MFMAs (the MFMAs read whatever the registers hold); precision probes
// (results deliberately less exact, not slower): 32 = f8c without the Kh.Ql correction, 64 = without Kl.Qh
#ifndef ACEMI_ATTN_ABLATE
#define ACEMI_ATTN_ABLATE 0
#endif
constexpr int kAttnAblate = ACEMI_ATTN_ABLATE;

// The workgroup's logical block (item, kv head, query tile) and key-range part.  Uniform layout: every block in
// a.ksplit parts, XCD-aware order over all of them (the hardware deals launch index j to XCD j % 8; logical
// index (j % 8) * per + j / 8 gives each XCD one contiguous run, i.e. the blocks of one (item, kv head), whose
// K / V^T tiles they all stream, share one XCD's L2).  Tail split (a.split_from = F > 0, a multiple of 8): launch
// indices [0, F) are whole blocks 0..F-1 (one full round), the rest the two key-range halves of blocks F..n-1
// (the last, partial round split so it fills the chip), XCD-aware within each range.  Returns false for the up
// to 7 empty trailing workgroups of a range.
__device__ __forceinline__ bool attn_block(const AttnArgs& a, int n_blk, int& blk, int& part, int& parts) {
    const int x = blockIdx.x;
    auto xcd = [&](int i, int n) { return a.xcd_order ? (i & 7) * ((n + 7) >> 3) + (i >> 3) : i; };
    if (a.split_from > 0) {
        const int F = a.split_from;
        if (x < F) {
            blk = xcd(x, F);
            part = 0;
            parts = 1;
            return blk < F;
        }
        const int n2 = 2 * (n_blk - F);
        const int y = xcd(x - F, n2);
        blk = F + (y >> 1);
        part = y & 1;
        parts = 2;
        return y < n2;
    }
    const int n = n_blk * a.ksplit;
    const int y = xcd(x, n);
    blk = y / a.ksplit;
    part = y % a.ksplit;
    parts = a.ksplit;
    return y < n;
}
static_assert(RA >= 1 && 2 * RA <= 15, "lgkmcnt counts at most 15 outstanding reads");
// LDS reads issued after step p's own, i.e. those of steps p+1 .. p+RA (< n), for the counted lgkmcnt of step p
template <class F>
constexpr int reads_after(int p, int n, F reads) {
    int c = 0;
    for (int k = 1; k <= RA; ++k)
        if (p + k < n) c += reads(p + k);
    return c;
}
__device__ __forceinline__ f32x16 mfma_f8(const v8i& a, const v8i& b, f32x16 c, int sa, int sb) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

template <int OFF>
__device__ __forceinline__ frag lds_frag(uint32_t addr) {
    frag v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}

// Wait for this wave's LDS reads and tie the fragments to the wait (guide §5.7 item 1, form ii): their
// consumers stay below it, while independent VALU / MFMA work may still be scheduled across it.
template <int N>
__device__ __forceinline__ void lds_wait_tie(frag (&r)[N]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < N; ++j) asm volatile("" : "+v"(r[j]));
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

template <bool F16OUT>
__device__ __forceinline__ uint16_t to_act(float f) {
    if constexpr (F16OUT) {
        _Float16 h = (_Float16)f;
        return __builtin_bit_cast(uint16_t, h);
    } else {
        return f32_to_bf16_rne(f);
    }
}

// f(std::integral_constant<int, I>) for I = B..E-1 (compile-time LDS offsets inside the body)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// key index (within a 64-key tile) of accumulator element r of 32-key half t, for lane half h:
// the 32x32 C/D map puts rows (= keys of S^T) at 8*(r/4) + 4*h + r%4
__device__ __forceinline__ constexpr int key_of(int t, int r) { return 32 * t + (r & 3) + 8 * (r >> 2); }

// ---------------------------------------------------------------------------------------------------------------
// attn2_kernel (round 4): the operands, layouts, block decomposition and online softmax of round 3's kernel, with
// the per-tile instruction stream laid out by hand for one wave per SIMD (the hi/lo modes run one workgroup per CU):
//   phase B  S(i+1) = K(i+1) Q^T  (16 k-steps of (k-slice, 32-key half), 1 or 3 MFMAs each)  interleaved step by
//            step with the softmax finish of tile i: p = exp2(s * c - m'), the row sum and the fp16 packing of
//            one pair of scores (one v_cvt_pk_f16_f32), the K fragments read two steps ahead (counted lgkmcnt) and
//            the next tiles' LDS-DMA pieces spread over the first steps;
//   phase C  O^T += V^T(i) P^T(i)  (16 steps of (d-tile, 16-key group), 1 or 3 MFMAs) interleaved with the
//            softmax start of tile i+1: the running max over raw scores (c > 0, so max(s) * c = max(s * c)
//            exactly), V fragments read two steps ahead.
// The score scale c = scale * log2(e) is folded into the exp2 argument (one FMA per score instead of a multiply
// and a subtract); every MFMA accumulator chain starts from an inline zero; scores are consumed in place (no
// copy of S between iterations: the two tile buffers alternate by name in the 2-unrolled loop).  A
// sched_barrier after each step keeps the step's MFMAs and its VALU / LDS slice together (the compiler otherwise
// clusters all MFMAs of a phase and leaves the VALU work exposed after them).
template <bool F16OUT, bool SPLIT, bool PVS, bool KBIAS, int OCC, bool F8 = false>
__global__ void __launch_bounds__(256, OCC) attn2_kernel(AttnArgs a) {
    static_assert(SPLIT || !PVS || F8, "hi/lo fp16 P.V needs hi/lo operands");
    static_assert(!F8 || PVS, "the fp8 correction modes stage the V lo plane");
    // QC: the Q.K correction products (f8c); without SPLIT the F8 kernel is the pv8 mode (fp16 Q.K, hi/lo P.V)
    constexpr bool QC = F8 && SPLIT;
    using RG = Ring<SPLIT, PVS>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int lq = lane & 31;

    const int rep = a.Hq / a.Hkv;
    const int qpb = 128 / rep;
    const int n_qt = (a.nq + qpb - 1) / qpb;
    int bid, split, ks;  // logical block, its key-range part (AttnArgs::part) and the block's number of parts
    if (!attn_block(a, a.B * a.Hkv * n_qt, bid, split, ks)) return;
    const int qt = bid % n_qt;
    bid /= n_qt;
    const int kvh = bid % a.Hkv;
    const int b = bid / a.Hkv;
    const int waves_per_head = 4 / rep;
    const int head = kvh * rep + wid / waves_per_head;
    const int q0 = qt * qpb;
    const int qw0 = q0 + (wid % waves_per_head) * 32;
    const int qrow = qw0 + lq;

    int klo = 0, khi = a.nk;
    if (a.window > 0) {
        klo = max(0, q0 - a.window);
        khi = min(a.nk, q0 + qpb - 1 + a.window + 1);
    }
    if (a.causal) khi = min(khi, q0 + qpb);
    const int n_all = max(0, (khi + KT - 1) / KT - klo / KT);
    const int chunk = (n_all + ks - 1) / ks;
    const int kt_begin = klo / KT + split * chunk;
    const int n = max(0, min(chunk, n_all - split * chunk));

    int lo_abs = 0, hi_abs = a.nk;
    if (a.window > 0) {
        lo_abs = max(lo_abs, qrow - a.window);
        hi_abs = min(hi_abs, qrow + a.window + 1);
    }
    if (a.causal) hi_abs = min(hi_abs, qrow + 1);
    lo_abs -= 4 * h;
    hi_abs -= 4 * h;

    const uint16_t* qptr = a.q + (((int64_t)b * a.Hq + head) * a.nq_pad + qrow) * D + 8 * h;
    frag qf[8], qfl[8];
    v8i q8[4];  // QC: B operands of the correction chain, bytes [64 c + 32 h, +32) of the [hi8 | lo8] q row
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const frag*)(qptr + 16 * ks);
    if constexpr (QC) {
        const char* q8row = reinterpret_cast<const char*>(qptr - 8 * h + a.q_plane) + 32 * h;
#pragma unroll
        for (int c = 0; c < 4; ++c) q8[c] = cat8(*(const frag*)(q8row + 64 * c), *(const frag*)(q8row + 64 * c + 16));
    } else if constexpr (SPLIT) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) qfl[ks] = *(const frag*)(qptr + a.q_plane + 16 * ks);
    }

    const uint16_t* kbase = a.k + ((int64_t)b * a.Hkv + kvh) * a.nk_pad * D;
    const uint16_t* vbase = a.vt + ((int64_t)b * a.Hkv + kvh) * D * a.nk_pad;
    const float* kb = KBIAS ? a.kbias + (int64_t)b * a.nk_pad : nullptr;

    // LDS-DMA pieces of one K / V^T tile (1 KiB per wave instruction) as buffer loads: the lane part of the source
    // offset is the same for every piece (the XOR swizzle depends on the row mod 16 / d mod 16 only), so one voffset
    // register per operand; the piece and tile parts go to the scalar offset.  K piece p: hi rows
    // 4 (wid + 4 (p & 3)) + lane / 16, p >= 4 the lo plane (SPLIT); V piece p: V^T d-rows 8 (wid + 4 (p & 3)) + lane / 8,
    // p >= 4 the lo plane (PVS); the key bias: wave 0, 4 bytes per lane.
    constexpr int NPK = SPLIT ? 8 : 4;
    constexpr int NPV = PVS ? 8 : 4;
    // VL: V(i+1) is requested in phase C of iteration i and waited for before phase C of iteration i+1 (a second
    // barrier per tile), so its pieces can sit behind the phase's long MFMAs; the fp16 mode keeps one barrier
    constexpr bool VL = SPLIT || PVS;
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)kbase, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vbase, 0, 0x7fffffff, 0x00020000);
    const int krow = 4 * wid + (lane >> 4);
    const int kvoff = krow * 256 + (((lane & 15) ^ (krow & 15)) << 4);
    const int vrow = 8 * wid + (lane >> 3);
    const int vvoff = vrow * a.nk_pad * 2 + (((lane & 7) ^ ((vrow >> 1) & 7)) << 4);
    const int kplane_b = SPLIT ? (int)(a.k_plane * 2) : 0;
    const int vplane_b = PVS ? (int)(a.v_plane * 2) : 0;
    auto k_piece = [&](int slot, int kt, int p) {
        const int so = kt * (KT * D * 2) + (p & 3) * 4096 + (p >= 4 ? kplane_b : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            krs, (lds_void*)(smem + slot * RG::KS + (p >= 4 ? RG::K_LO : RG::K_HI) + (wid + 4 * (p & 3)) * 1024), 16, kvoff,
            so, 0, 0);
    };
    auto v_piece = [&](int slot, int kt, int p) {
        const int so = kt * (KT * 2) + (p & 3) * (64 * a.nk_pad) + (p >= 4 ? vplane_b : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            vrs, (lds_void*)(smem + RG::V0 + slot * RG::VS + (p >= 4 ? RG::V_LO : 0) + (wid + 4 * (p & 3)) * 1024), 16,
            vvoff, so, 0, 0);
    };
    auto bias_piece = [&](int slot, int kt) {
        if constexpr (KBIAS) {
            if (wid == 0)
                __builtin_amdgcn_global_load_lds((const void*)(kb + kt * KT + lane), (lds_void*)(smem + slot * RG::KS + RG::KB),
                                                 4, 0, 0);
        }
    };

    const int cK = h ^ (lq & 15);
    const int cV = h ^ ((lq >> 1) & 7);
    const uint32_t smem_l = lds_addr(smem);
    uint32_t kaddr[8], vaddr[4];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kaddr[ks] = smem_l + RG::K_HI + lq * 256 + (((2 * ks) ^ cK) << 4);
#pragma unroll
    for (int g = 0; g < 4; ++g) vaddr[g] = smem_l + RG::V0 + lq * 128 + (((2 * g) ^ cV) << 4);
    const uint32_t kbaddr = smem_l + RG::KB + 16 * h;
    // F8: fp8 K row (key 32 t + lq) chunks 4 c + 2 h + e, fp8 V^T row (d = 32 dt + lq) chunks 4 i + 2 h + e, swizzled
    // like the fp16 images (the same LDS-DMA pieces fill them)
    uint32_t k8a[4][2], v8a[2][2];
    if constexpr (QC) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 2; ++e) k8a[c][e] = smem_l + RG::K_LO + lq * 256 + (((4 * c + 2 * h + e) ^ (lq & 15)) << 4);
    }
    if constexpr (F8) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 2; ++e)
                v8a[i][e] = smem_l + RG::V0 + RG::V_LO + lq * 128 + (((4 * i + 2 * h + e) ^ ((lq >> 1) & 7)) << 4);
    }
    constexpr float PSC = F8 ? PSCALE_F8_LOG2 : PSCALE_LOG2;

    const float c_log2 = a.scale * 1.4426950408889634f;
    const float one_rt = a.scale / a.scale;  // exactly 1 (scale > 0), opaque to the compiler: see plo

    // ---- phase B: QK of the next tile in NB steps.  Position p runs the hi step h (k-slice ks = h / 2 of half
    // t = h % 2: fp16 hi, + lo for SPLIT) or, for F8, every third position (p % 3 == 2) the correction step
    // k = p / 3 (chunk c = k / 2 of half t = k % 2: two 16-byte reads of the fp8 row, one K = 64 fp8 MFMA)
    constexpr int NB = QC ? 24 : 16;
    struct BStep {
        bool corr;
        int idx;  // h or k
    };
    auto bstep = [](int p) constexpr -> BStep {
        if (!QC) return BStep{false, p};
        return p % 3 == 2 ? BStep{true, p / 3} : BStep{false, p - p / 3};
    };
    auto k_read = [&](auto slot_c, auto p_c, frag& x, frag& y) {
        constexpr int SLOT = decltype(slot_c)::value;
        constexpr BStep st = bstep(decltype(p_c)::value);
        constexpr int t = st.idx & 1;
        if constexpr (!st.corr) {
            constexpr int ks = st.idx >> 1;
            x = lds_frag<SLOT * RG::KS + t * 32 * 256>(kaddr[ks]);
            if constexpr (SPLIT && !F8) y = lds_frag<SLOT * RG::KS + t * 32 * 256 + RG::K_LO - RG::K_HI>(kaddr[ks]);
        } else {
            constexpr int c = st.idx >> 1;
            x = lds_frag<SLOT * RG::KS + t * 32 * 256>(k8a[c][0]);
            y = lds_frag<SLOT * RG::KS + t * 32 * 256>(k8a[c][1]);
        }
    };
    // LDS reads of QK position p
    auto rk = [](int p) constexpr { return QC ? (p % 3 == 2 ? 2 : 1) : ((SPLIT && !F8) ? 2 : 1); };
    // S(tile in K slot SLOT) into sn, interleaved with fin(p) (a softmax-finish slice) and dma(p)
    auto qk_phase = [&](auto slot_c, f32x16 (&sn)[2], auto&& fin, auto&& dma) {
        frag kh[RA + 1], kl[RA + 1];
        static_for<0, RA>([&](auto r_c) {
            constexpr int r = decltype(r_c)::value;
            if constexpr (r < NB) k_read(slot_c, r_c, kh[r], kl[r]);
        });
        static_for<0, NB>([&](auto p_c) {
            constexpr int p = decltype(p_c)::value;
            constexpr BStep st = bstep(p);
            constexpr int t = st.idx & 1;
            if constexpr (p + RA < NB)
                k_read(slot_c, std::integral_constant<int, p + RA>{}, kh[(p + RA) % (RA + 1)], kl[(p + RA) % (RA + 1)]);
            constexpr int after = reads_after(p, NB, rk);
            if constexpr (!(kAttnAblate & 16)) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(after) : "memory");
            asm volatile("" : "+v"(kh[p % (RA + 1)]));
            if constexpr (rk(p) == 2) asm volatile("" : "+v"(kl[p % (RA + 1)]));
            if constexpr (st.corr) {
                // Kl.Qh (c = 0, 1: the 2^-11 on A) + Kh.Ql (c = 2, 3: on B), e4m3 x e4m3, K = 64 per MFMA
                constexpr int c = st.idx >> 1;
                if constexpr (!((kAttnAblate & 32) && c >= 2) && !((kAttnAblate & 64) && c < 2))
                    sn[t] = mfma_f8(cat8(kh[p % (RA + 1)], kl[p % (RA + 1)]), q8[c], sn[t], c < 2 ? F8_SCALE_LO : F8_SCALE_1,
                                c < 2 ? F8_SCALE_1 : F8_SCALE_LO);
            } else {
                constexpr int ks = st.idx >> 1;
                if constexpr (ks == 0) {
                    sn[t] = mfma32(kh[p % (RA + 1)], qf[0], f32x16{});
                } else {
                    sn[t] = mfma32(kh[p % (RA + 1)], qf[ks], sn[t]);
                }
                if constexpr (SPLIT && !F8) {
                    sn[t] = mfma32(kh[p % (RA + 1)], qfl[ks], sn[t]);
                    sn[t] = mfma32(kl[p % (RA + 1)], qf[ks], sn[t]);
                }
            }
            dma(p_c);
            fin(p_c);
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    float m_run = -INFINITY;
    float l_run = 0.f;
    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;

    // softmax start of a tile (S in sn, its key bias in K slot SLOT, relative index i): KBIAS folds scale and bias
    // into sn (x = s * c + bias); masks (tiles crossing a bound only) set -inf; returns the lane's max over its 64
    // keys in the exp2 domain, combined across the two lane halves
    auto mask_tile = [&](f32x16 (&sn)[2], int i) {
        const int k0 = (kt_begin + i) * KT;
        const int lo = lo_abs - k0, hi = hi_abs - k0;
        if (__builtin_amdgcn_ballot_w64(lo > 0 || hi < 60) != 0) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int kr = key_of(t, r);
                    sn[t][r] = (kr >= lo && kr < hi) ? sn[t][r] : -INFINITY;
                }
        }
    };
    auto bias_tile = [&](auto slot_c, f32x16 (&sn)[2]) {
        if constexpr (KBIAS) {
            constexpr int SLOT = decltype(slot_c)::value;
            frag kbv[8];
            static_for<0, 8>([&](auto j_c) {
                constexpr int j = decltype(j_c)::value;
                kbv[j] = lds_frag<SLOT * RG::KS + (32 * (j / 4) + 8 * (j % 4)) * 4>(kbaddr);
            });
            lds_wait_tie(kbv);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    sn[t][r] = __builtin_fmaf(sn[t][r], c_log2, __uint_as_float(kbv[4 * t + (r >> 2)][r & 3]));
        }
    };
    auto finish_max = [&](float mraw) -> float {
        const float mx = KBIAS ? mraw : (mraw == -INFINITY ? -INFINITY : mraw * c_log2);
        return fmaxf(mx, __shfl_xor(mx, 32));
    };

    float alpha = 1.f;
    bool rescale = false;
    auto update_max = [&](float mloc) {
        const bool move = mloc > m_run + RESCALE_LOG2;
        alpha = move ? __builtin_amdgcn_exp2f(m_run - mloc) : 1.f;
        m_run = move ? mloc : m_run;
        rescale = __builtin_amdgcn_ballot_w64(move) != 0;
    };
    auto apply_rescale = [&]() {
        if (rescale) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            l_run *= alpha;
        }
    };

    f32x16 sA[2], sB[2];
    auto no_fin = [](auto) {};
    auto no_dma = [](auto) {};
    if (n > 0) {
#pragma unroll
        for (int p = 0; p < NPK; ++p) k_piece(0, kt_begin, p);
        bias_piece(0, kt_begin);
#pragma unroll
        for (int p = 0; p < NPV; ++p) v_piece(0, kt_begin, p);
        if (n > 1) {
#pragma unroll
            for (int p = 0; p < NPK; ++p) k_piece(1, kt_begin + 1, p);
            bias_piece(1, kt_begin + 1);
        }
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        qk_phase(std::integral_constant<int, 0>{}, sA, no_fin, no_dma);
        bias_tile(std::integral_constant<int, 0>{}, sA);
        mask_tile(sA, 0);
        float mr = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) mr = fmaxf(mr, sA[t][r]);
        update_max(finish_max(mr));
        apply_rescale();
        __builtin_amdgcn_s_barrier();  // every wave has read K slot 0: iteration 0 restages it
    }

    // one pipeline iteration for relative tile i: S(i) in sc (from K slot SLOT), V(i) in V slot SLOT; computes
    // S(i+1) into sn from K slot NXT
    auto iter = [&](auto slot_c, f32x16 (&sc)[2], f32x16 (&sn)[2], int i) {
        constexpr int SLOT = decltype(slot_c)::value;
        constexpr int NXT = SLOT ^ 1;
        const bool more = i + 1 < n;
        // the next tiles' DMA is issued unconditionally (no branch per piece): past the last tile it re-reads the
        // last one into the slot the next iteration would fill, which nothing reads afterwards (the garbage S of
        // the step past the end is never used)
        const int ktk = kt_begin + min(i + 2, n - 1), ktv = kt_begin + min(i + 1, n - 1);
        const float m_use = ((m_run == -INFINITY) ? 0.f : m_run) - PSC;
        const float nm = -m_use;
        float lsum = 0.f;
        frag pf[4], pfl[4];
        uint32_t ph8[8] = {}, pl8[8] = {};  // F8: fp8 P (hi) and P - f16(P) (lo), byte c = 16 t + r of the lane's keys
        // softmax finish of tile i at QK position p: pair j (elements 2j, 2j + 1 of the flattened [t][r] scores) =
        // the position's hi step
        // fp8 lo part of P pair j: P - f16(P) (exact in f32), as one mixed-precision FMA per value: fma(-f16, one, P)
        // with a run-time 1.0 (hipcc folds a literal 1 into a v_cvt_f32_f16 + v_sub pair, and an inline-asm
        // v_fma_mix_f32 costs an s_nop per use: the hazard recognizer cannot see into it)
        auto plo = [&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            constexpr int t = j >> 3, r = 2 * (j & 7);
            constexpr int fi = 2 * t + (r >> 3), fj = (r & 7) >> 1;
            int w8 = (int)pl8[j >> 1];
            typedef _Float16 h2v __attribute__((ext_vector_type(2)));
            const h2v hv = __builtin_bit_cast(h2v, (uint32_t)pf[fi][fj]);
            const float l0 = __builtin_fmaf(-(float)hv[0], one_rt, sc[t][r]);
            const float l1 = __builtin_fmaf(-(float)hv[1], one_rt, sc[t][r + 1]);
            w8 = __builtin_amdgcn_cvt_pk_fp8_f32(l0, l1, w8, (j & 1) != 0);
            asm volatile("" : "+v"(w8));
            pl8[j >> 1] = (uint32_t)w8;
        };
        // PLO_B (f8c): P's lo parts are formed on phase B's correction steps (64-cycle MFMAs with spare issue slots),
        // pairs 2k and 2k + 1 on correction step k, right after the two hi steps that formed their P; otherwise on
        // phase C's hi steps (measured: the P-lo VALU on phase C's 32-cycle steps cost 12 % of the f8c kernel)
        constexpr bool PLO_B = QC && !(kAttnAblate & 4);
        auto fin = [&](auto p_c) {
            constexpr BStep st = bstep(decltype(p_c)::value);
            constexpr int j = st.idx;
            if constexpr (st.corr && PLO_B) {
                plo(std::integral_constant<int, 2 * j>{});
                plo(std::integral_constant<int, 2 * j + 1>{});
            }
            if constexpr (!st.corr) {
                constexpr int t = j >> 3, r = 2 * (j & 7);
                float p0, p1;
                if constexpr (kAttnAblate & 2) {
                    p0 = sc[t][r];
                    p1 = sc[t][r + 1];
                } else if constexpr (KBIAS) {
                    p0 = __builtin_amdgcn_exp2f(sc[t][r] + nm);
                    p1 = __builtin_amdgcn_exp2f(sc[t][r + 1] + nm);
                } else {
                    p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[t][r], c_log2, nm));
                    p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[t][r + 1], c_log2, nm));
                }
                lsum += p0;
                lsum += p1;
                constexpr int fi = 2 * t + (r >> 3), fj = (r & 7) >> 1;
                // (the empty asm pins each result to its step: without it the IR passes sink the whole softmax
                // finish to the P.V MFMAs that consume it, i.e. after every MFMA of this phase)
                if constexpr (F8) {
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
                    const h2t hv = __builtin_convertvector((f2){p0, p1}, h2t);
                    uint32_t w = __builtin_bit_cast(uint32_t, hv);
                    int w8 = (int)ph8[j >> 1];  // (the even pair writes the low word; the high word is written next)
                    w8 = __builtin_amdgcn_cvt_pk_fp8_f32(p0, p1, w8, (j & 1) != 0);
                    asm volatile("" : "+v"(w), "+v"(w8), "+v"(lsum), "+v"(p0), "+v"(p1));
                    pf[fi][fj] = w;
                    ph8[j >> 1] = (uint32_t)w8;
                    sc[t][r] = p0;  // P itself, for the lo part formed in phase C
                    sc[t][r + 1] = p1;
                } else if constexpr (PVS) {
                    const auto h2 = __builtin_amdgcn_cvt_pkrtz(p0, p1);
                    uint32_t w = __builtin_bit_cast(uint32_t, h2);
                    uint32_t wl = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(p0 - (float)h2[0], p1 - (float)h2[1]));
                    asm volatile("" : "+v"(w), "+v"(wl), "+v"(lsum));
                    pf[fi][fj] = w;
                    pfl[fi][fj] = wl;
                } else {
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    typedef _Float16 h2t __attribute__((ext_vector_type(2)));
                    const h2t hv = __builtin_convertvector((f2){p0, p1}, h2t);
                    uint32_t w = __builtin_bit_cast(uint32_t, hv);
                    asm volatile("" : "+v"(w), "+v"(lsum));
                    pf[fi][fj] = w;
                }
            }
        };
        // next tiles' LDS-DMA: K(i+2) in phase B (F8: behind the 64-cycle correction MFMAs); V(i+1) in phase B too
        // for the fp16 mode, in phase C for the hi/lo modes (VL: waited for before the next iteration's phase C)
        auto dma = [&](auto p_c) {
            constexpr int p = decltype(p_c)::value;
            constexpr BStep st = bstep(p);
            constexpr int kp = QC ? (st.corr ? st.idx : -1) : p;  // K piece of this position
            static_assert(VL || NPK + NPV <= NB, "one DMA piece per QK step");
            if constexpr (kAttnAblate & 1) {
            } else if constexpr (kp >= 0 && kp < NPK) {
                k_piece(SLOT, ktk, kp);
                if constexpr (kp == 0) bias_piece(SLOT, ktk);
            } else if constexpr (!VL && p >= NPK && p < NPK + NPV) {
                v_piece(NXT, ktv, p - NPK);
            }
        };
        qk_phase(std::integral_constant<int, NXT>{}, sn, [&](auto j_c) { fin(j_c); }, [&](auto j_c) { dma(j_c); });
        l_run += lsum;

        // phase C: O^T += V^T(i) P^T(i) || softmax start of tile i+1, NC steps.  Position q runs the hi step hs (d-tile
        // hs / 4, 16-key group hs % 4: fp16 hi, + lo for PVS) or, for F8, a correction step (one K = 64 fp8 MFMA of
        // d-tile dt: Vl.Ph at q = 2, 5, 8, 11 (dt 0..3), Vh.Pl at q = 20..23, after every hi step has formed P's lo
        // part)
        if constexpr (VL) {  // V(i), requested in the previous iteration's phase C, landed for every wave
            if (KBIAS && wid == 0)
                wait_vmcnt<NPK + 1>();
            else
                wait_vmcnt<NPK>();
            if constexpr (!(kAttnAblate & 8)) __builtin_amdgcn_s_barrier();
        }
        bias_tile(std::integral_constant<int, NXT>{}, sn);
        mask_tile(sn, i + 1);
        float mr = -INFINITY;
        {
            constexpr int NC = F8 ? 24 : 16;
            struct CStep {
                int kind;  // 0 hi, 1 Vl.Ph, 2 Vh.Pl
                int idx;   // hs, or the d-tile
            };
            auto cstep = [](int q) constexpr -> CStep {
                if (!F8) return CStep{0, q};
                if (q >= 20) return CStep{2, q - 20};
                if (q < 12) return q % 3 == 2 ? CStep{1, q / 3} : CStep{0, q - (q + 1) / 3};
                return CStep{0, q - 4};
            };
            frag vh[RA + 1], vl[RA + 1];
            auto v_read = [&](auto q_c, frag& x, frag& y) {
                constexpr CStep st = cstep(decltype(q_c)::value);
                if constexpr (st.kind == 0) {
                    constexpr int dt = st.idx >> 2, g = st.idx & 3;
                    x = lds_frag<SLOT * RG::VS + dt * 32 * 128>(vaddr[g]);
                    if constexpr (PVS && !F8) y = lds_frag<SLOT * RG::VS + dt * 32 * 128 + RG::V_LO>(vaddr[g]);
                } else {
                    constexpr int dt = st.idx, ii = st.kind - 1;
                    x = lds_frag<SLOT * RG::VS + dt * 32 * 128>(v8a[ii][0]);
                    y = lds_frag<SLOT * RG::VS + dt * 32 * 128>(v8a[ii][1]);
                }
            };
            auto rv = [](int q) constexpr { return F8 ? ((q >= 20 || (q < 12 && q % 3 == 2)) ? 2 : 1) : (PVS ? 2 : 1); };
            // V(i+1) pieces of the hi/lo modes: F8 behind its 8 correction MFMAs, else the first NPV positions
            auto vdma = [&](auto q_c) {
                if constexpr (VL) {
                    constexpr int q = decltype(q_c)::value;
                    constexpr CStep st = cstep(q);
                    constexpr int vp = F8 ? (st.kind == 1 ? st.idx : st.kind == 2 ? 4 + st.idx : -1) : q;
                    if constexpr (vp >= 0 && vp < NPV && !(kAttnAblate & 1)) v_piece(NXT, ktv, vp);
                }
            };
            static_for<0, RA>([&](auto r_c) {
                constexpr int r = decltype(r_c)::value;
                if constexpr (r < NC) v_read(r_c, vh[r], vl[r]);
            });
            static_for<0, NC>([&](auto q_c) {
                constexpr int q = decltype(q_c)::value;
                constexpr CStep st = cstep(q);
                if constexpr (q + RA < NC)
                    v_read(std::integral_constant<int, q + RA>{}, vh[(q + RA) % (RA + 1)], vl[(q + RA) % (RA + 1)]);
                constexpr int after = reads_after(q, NC, rv);
                if constexpr (!(kAttnAblate & 16)) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(after) : "memory");
                asm volatile("" : "+v"(vh[q % (RA + 1)]));
                if constexpr (rv(q) == 2) asm volatile("" : "+v"(vl[q % (RA + 1)]));
                if constexpr (st.kind == 0) {
                    constexpr int j = st.idx;
                    constexpr int dt = j >> 2, g = j & 3;
                    o[dt] = mfma32(vh[q % (RA + 1)], pf[g], o[dt]);
                    if constexpr (PVS && !F8) {
                        o[dt] = mfma32(vh[q % (RA + 1)], pfl[g], o[dt]);
                        o[dt] = mfma32(vl[q % (RA + 1)], pf[g], o[dt]);
                    }
                    // running max of tile i+1: two scores per step
                    constexpr int t = j >> 3, r = 2 * (j & 7);
                    mr = fmaxf(mr, fmaxf(sn[t][r], sn[t][r + 1]));
                    asm volatile("" : "+v"(mr));
                    if constexpr (F8 && !PLO_B && !(kAttnAblate & 4)) plo(std::integral_constant<int, j>{});
                } else {
                    constexpr int dt = st.idx;
                    const v8i pb = st.kind == 1 ? cat8(ph8) : cat8(pl8);
                    o[dt] = mfma_f8(cat8(vh[q % (RA + 1)], vl[q % (RA + 1)]), pb, o[dt], st.kind == 1 ? F8_SCALE_LO : F8_SCALE_1,
                                    F8_SCALE_1);
                }
                vdma(q_c);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        const float mnx = finish_max(mr);
        if (more) {
            update_max(mnx);
            apply_rescale();
            // K(i+2) landed (VL: V(i+1), issued after it, may stay in flight) and every wave is done with K slot NXT
            if constexpr (VL)
                wait_vmcnt<NPV>();
            else
                wait_vmcnt<0>();
            if constexpr (!(kAttnAblate & 8)) __builtin_amdgcn_s_barrier();
        }
    };

    int i = 0;
    for (; i + 1 < n; i += 2) {
        iter(std::integral_constant<int, 0>{}, sA, sB, i);
        iter(std::integral_constant<int, 1>{}, sB, sA, i + 1);
    }
    if (i < n) iter(std::integral_constant<int, 0>{}, sA, sB, i);
    wait_vmcnt<0>();  // the re-read tiles past the end

    const float l = l_run + __shfl_xor(l_run, 32);
    if (ks > 1) {
        if (qrow < a.nq) {
            const int64_t row = ((int64_t)split * a.B + b) * a.nq + qrow;
            float* po = a.part + row * (a.Hq * D) + head * D;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *(float4*)(po + 32 * dt + 8 * g4 + 4 * h) =
                        make_float4(o[dt][4 * g4 + 0], o[dt][4 * g4 + 1], o[dt][4 * g4 + 2], o[dt][4 * g4 + 3]);
            if (h == 0)
                *(float2*)(a.part + (int64_t)a.ksplit * a.B * a.nq * a.Hq * D + (row * a.Hq + head) * 2) =
                    make_float2(m_run, l);
        }
        return;
    }
    const float inv = 1.0f / l;
    if (a.out_f32) {  // f32 rows (the quantized-activation mode: the next linear quantizes them)
        if (qrow < a.nq) {
            float* of = a.out_f32 + ((int64_t)b * a.nq + qrow) * (a.Hq * D) + head * D;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *(float4*)(of + 32 * dt + 8 * g4 + 4 * h) =
                        make_float4(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv, o[dt][4 * g4 + 2] * inv,
                                    o[dt][4 * g4 + 3] * inv);
        }
        return;
    }
    if (qrow < a.nq) {
        uint16_t* op = a.out + ((int64_t)b * a.nq + qrow) * (a.Hq * D) + head * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 32 * dt + 8 * g4 + 4 * h;
                uint2 w;
                w.x = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 0] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 1] * inv) << 16);
                w.y = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 2] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 3] * inv) << 16);
                *(uint2*)(op + d) = w;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// attn_kh_kernel (round 6): the f8c mode at two waves per SIMD.  attn2 holds a whole 64-key tile's scores and P
// operands, both ring stages and the Q planes in one wave (312 registers, so one wave per SIMD; its per-tile stream
// takes ~2.2x its MFMA time).  Here a workgroup of 8 waves runs the same block (item, kv
// head, 128 query rows) over the same LDS rings: wave w = 4 kh + wq takes query group wq's 32 rows against key half kh
// (keys [32 kh, 32 kh + 32)) of every tile -- exactly attn2's half t = kh -- with its own online softmax, and the two
// halves of a row meet once after the key loop, through LDS (the key-split merge's combination).  Per wave and tile:
//   S^T half   8 fp16 hi MFMAs + 4 block-scaled e4m3 corrections (Kl.Qh, Kh.Ql over D = 128), one accumulator;
//   O^T        8 fp16 hi MFMAs + 4 e4m3 MFMAs, each carrying BOTH P.V corrections of one d-tile in one K = 64 product:
//              K 0-31 (lanes 0-31) Vl x Ph, K 32-63 (lanes 32-63) Vh x Pl, after one permlane32_swap per P word has
//              regrouped [Ph | Pl] of the lane halves into [Ph (all 32 keys) ; Pl (all 32 keys)].  Both halves carry
//              2^11 (Vl is stored as fp8(2^11 lo) by the prep, Pl is formed as fp8(2^11 (P - f16(P))), which also keeps
//              it clear of e4m3's subnormals) and share one uniform E8M0 scale 2^-11: a VGPR scale that differs between
//              the lane halves is not applied per K block (measured, profiles/r06/attn_kh/diag_per_lane_scale_attempt.jsonl).
// The same MFMA cycles per key as attn2 at <= 256 registers, so a partner wave shares each SIMD -- measured equal in
// speed to attn2 (the issue per tile and SIMD is the same); launch_attention runs it on >= 16-tile blocks.
// Pipeline, DMA ring and masks as attn2 (phase B: S(i+1) || softmax finish of i; phase C: O += V(i) P(i) || softmax
// start of i+1), with 4 K + 4 V^T LDS-DMA pieces per wave and tile.
template <bool F16OUT, bool KBIAS>
__global__ void __launch_bounds__(512) attn_kh_kernel(AttnArgs a) {
    using RG = Ring<true, true>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kh = wid >> 2, wq = wid & 3;
    const int h = lane >> 5;
    const int lq = lane & 31;

    const int rep = a.Hq / a.Hkv;
    const int qpb = 128 / rep;
    const int n_qt = (a.nq + qpb - 1) / qpb;
    int bid, split, ks;
    if (!attn_block(a, a.B * a.Hkv * n_qt, bid, split, ks)) return;
    const int qt = bid % n_qt;
    bid /= n_qt;
    const int kvh = bid % a.Hkv;
    const int b = bid / a.Hkv;
    const int waves_per_head = 4 / rep;
    const int head = kvh * rep + wq / waves_per_head;
    const int q0 = qt * qpb;
    const int qrow = q0 + (wq % waves_per_head) * 32 + lq;

    int klo = 0, khi = a.nk;
    if (a.window > 0) {
        klo = max(0, q0 - a.window);
        khi = min(a.nk, q0 + qpb - 1 + a.window + 1);
    }
    if (a.causal) khi = min(khi, q0 + qpb);
    const int n_all = max(0, (khi + KT - 1) / KT - klo / KT);
    const int chunk = (n_all + ks - 1) / ks;
    const int kt_begin = klo / KT + split * chunk;
    const int n = max(0, min(chunk, n_all - split * chunk));

    int lo_abs = 0, hi_abs = a.nk;
    if (a.window > 0) {
        lo_abs = max(lo_abs, qrow - a.window);
        hi_abs = min(hi_abs, qrow + a.window + 1);
    }
    if (a.causal) hi_abs = min(hi_abs, qrow + 1);
    lo_abs -= 4 * h;
    hi_abs -= 4 * h;

    const uint16_t* qptr = a.q + (((int64_t)b * a.Hq + head) * a.nq_pad + qrow) * D + 8 * h;
    frag qf[8];
    v8i q8[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[j] = *(const frag*)(qptr + 16 * j);
    {
        const char* q8row = reinterpret_cast<const char*>(qptr - 8 * h + a.q_plane) + 32 * h;
#pragma unroll
        for (int c = 0; c < 4; ++c) q8[c] = cat8(*(const frag*)(q8row + 64 * c), *(const frag*)(q8row + 64 * c + 16));
    }

    const uint16_t* kbase = a.k + ((int64_t)b * a.Hkv + kvh) * a.nk_pad * D;
    const uint16_t* vbase = a.vt + ((int64_t)b * a.Hkv + kvh) * D * a.nk_pad;
    const float* kb = KBIAS ? a.kbias + (int64_t)b * a.nk_pad : nullptr;

    // LDS-DMA pieces (1 KiB per wave instruction): K piece p = hi / lo plane (p >= 2) rows 4 (wid + 8 (p & 1)) +
    // lane / 16; V^T piece p = hi / lo plane (p >= 2) d-rows 8 (wid + 8 (p & 1)) + lane / 8; the key bias: wave 0
    constexpr int NPK = 4, NPV = 4;
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)kbase, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vbase, 0, 0x7fffffff, 0x00020000);
    const int krow = 4 * wid + (lane >> 4);
    const int kvoff = krow * 256 + (((lane & 15) ^ (krow & 15)) << 4);
    const int vrow = 8 * wid + (lane >> 3);
    const int vvoff = vrow * a.nk_pad * 2 + (((lane & 7) ^ ((vrow >> 1) & 7)) << 4);
    const int kplane_b = (int)(a.k_plane * 2), vplane_b = (int)(a.v_plane * 2);
    auto k_piece = [&](int slot, int kt, int p) {
        const int so = kt * (KT * D * 2) + (p & 1) * 8192 + (p >= 2 ? kplane_b : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            krs, (lds_void*)(smem + slot * RG::KS + (p >= 2 ? RG::K_LO : RG::K_HI) + (wid + 8 * (p & 1)) * 1024), 16, kvoff,
            so, 0, 0);
    };
    auto v_piece = [&](int slot, int kt, int p) {
        const int so = kt * (KT * 2) + (p & 1) * (128 * a.nk_pad) + (p >= 2 ? vplane_b : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            vrs, (lds_void*)(smem + RG::V0 + slot * RG::VS + (p >= 2 ? RG::V_LO : 0) + (wid + 8 * (p & 1)) * 1024), 16,
            vvoff, so, 0, 0);
    };
    auto bias_piece = [&](int slot, int kt) {
        if constexpr (KBIAS) {
            if (wid == 0)
                __builtin_amdgcn_global_load_lds((const void*)(kb + kt * KT + lane), (lds_void*)(smem + slot * RG::KS + RG::KB),
                                                 4, 0, 0);
        }
    };

    // fragment addresses (slot 0; the slot is an immediate offset): K hi row 32 kh + lq, k-slice j; its fp8 row
    // [Kl8 | Kh8] chunks 4 c + 2 h + e; V^T hi d-row lq of d-tile 0, 16-key group 2 kh + g; the fp8 V^T row's
    // correction chunks 4 h + 2 e + kh (lane half 0: Vl of the half's keys, lane half 1: Vh)
    const uint32_t smem_l = lds_addr(smem);
    const int cK = h ^ (lq & 15);
    const int cV = h ^ ((lq >> 1) & 7);
    uint32_t kaddr[8], k8a[4][2], vaddr[2], v8a[2];
#pragma unroll
    for (int j = 0; j < 8; ++j) kaddr[j] = smem_l + RG::K_HI + (32 * kh + lq) * 256 + (((2 * j) ^ cK) << 4);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e)
            k8a[c][e] = smem_l + RG::K_LO + (32 * kh + lq) * 256 + (((4 * c + 2 * h + e) ^ (lq & 15)) << 4);
#pragma unroll
    for (int g = 0; g < 2; ++g) vaddr[g] = smem_l + RG::V0 + lq * 128 + (((2 * (2 * kh + g)) ^ cV) << 4);
#pragma unroll
    for (int e = 0; e < 2; ++e) v8a[e] = smem_l + RG::V0 + RG::V_LO + lq * 128 + (((4 * h + 2 * e + kh) ^ ((lq >> 1) & 7)) << 4);
    const uint32_t kbaddr = smem_l + RG::KB + 16 * h + 128 * kh;

    const float c_log2 = a.scale * 1.4426950408889634f;
    const float one_rt = a.scale / a.scale;  // exactly 1, opaque to the compiler (attn2's plo)

    // Two waves per SIMD: no VALU or LDS read may write an A / B register of an MFMA that may still be waiting for the
    // matrix pipe (tools/audit_mfma_war.py, --loads).  The first fragment of every step comes from a
    // ring of RA + 3 slots, the second one of the correction steps (every third step) from a ring of 2; every step's
    // fragments stay allocated to the end of the second step after it (the ring slots are only names: liveness is what
    // keeps hipcc from giving a just-read operand register to a new value), a correction's concatenated operand to
    // the next correction, and each phase ends with 16 wait states.
    constexpr int RX = RA + 3;
    auto keep = [](const frag& x) { asm volatile("" ::"v"(x)); };
    auto keep8 = [](const v8i& x) { asm volatile("" ::"v"(x)); };

    // phase B positions: p % 3 == 2 the correction c = p / 3 (two 16-byte reads), else the hi k-slice p - p / 3
    constexpr int NB = 12;
    auto k_read = [&](auto slot_c, auto p_c, frag& x, frag& y) {
        constexpr int SLOT = decltype(slot_c)::value;
        constexpr int p = decltype(p_c)::value;
        if constexpr (p % 3 != 2) {
            x = lds_frag<SLOT * RG::KS>(kaddr[p - p / 3]);
        } else {
            x = lds_frag<SLOT * RG::KS>(k8a[p / 3][0]);
            y = lds_frag<SLOT * RG::KS>(k8a[p / 3][1]);
        }
    };
    auto rk = [](int p) constexpr { return p % 3 == 2 ? 2 : 1; };
    // EARLY: each phase waits for the next tile's DMA and meets the other waves after its step MID (the MFMAs issued
    // before it keep the pipe busy through the barrier), and right behind that barrier reads the first RA fragments of
    // the phase that follows (V in phase B, the next iteration's K in phase C), so no phase opens on an LDS latency.
    // Those RA reads sit between the step reads: the two steps after MID count them in their lgkmcnt.  The K ones cross
    // the loop's back-edge only after they have landed and been tied (end of phase C), so no register copy of an asm-load
    // destination can run before its wait.
    constexpr bool EARLY = ACEMI_KH_EARLY;
    constexpr int MID = 6;
    auto extra = [](int p) constexpr { return (EARLY && (p == MID + 1 || p == MID + 2)) ? RA : 0; };
    frag kpre[RA], vpre[RA];
    auto qk_phase = [&](auto slot_c, f32x16& sn, auto&& fin, auto&& dma, auto&& mid, auto pre_c) {
        frag kx[RX], ky[2];
        v8i kc;  // the last correction step's concatenated A operand (hipcc may copy the two fragments into it)
        static_for<0, RA>([&](auto r_c) {
            constexpr int r = decltype(r_c)::value;
            if constexpr (decltype(pre_c)::value)
                kx[r] = kpre[r];
            else
                k_read(slot_c, r_c, kx[r], ky[0]);
        });
        static_for<0, NB>([&](auto p_c) {
            constexpr int p = decltype(p_c)::value;
            if constexpr (p + RA < NB)
                k_read(slot_c, std::integral_constant<int, p + RA>{}, kx[(p + RA) % RX], ky[((p + RA) / 3) % 2]);
            constexpr int after = reads_after(p, NB, rk) + (decltype(pre_c)::value ? extra(p) : 0);
            asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(after) : "memory");
            asm volatile("" : "+v"(kx[p % RX]));
            if constexpr (rk(p) == 2) asm volatile("" : "+v"(ky[(p / 3) % 2]));
            if constexpr (p % 3 == 2) {
                constexpr int c = p / 3;  // Kl.Qh (c = 0, 1: 2^-11 on A) + Kh.Ql (c = 2, 3: on B)
                kc = cat8(kx[p % RX], ky[(p / 3) % 2]);
                sn = mfma_f8(kc, q8[c], sn, c < 2 ? F8_SCALE_LO : F8_SCALE_1, c < 2 ? F8_SCALE_1 : F8_SCALE_LO);
            } else {
                constexpr int j = p - p / 3;
                sn = j == 0 ? mfma32(kx[p % RX], qf[0], f32x16{}) : mfma32(kx[p % RX], qf[j], sn);
            }
            dma(p_c);
            fin(p_c);
            static_for<1, 3>([&](auto d_c) {  // the fragments of the two steps before stay allocated
                constexpr int pd = p - decltype(d_c)::value;
                if constexpr (pd >= 0) {
                    keep(kx[pd % RX]);
                    if constexpr (rk(pd) == 2) keep(ky[(pd / 3) % 2]);
                }
            });
            if constexpr (p > 2) keep8(kc);
            mid(p_c);
            __builtin_amdgcn_sched_barrier(0);
        });
        asm volatile("" : "+v"(sn));  // (the phase's MFMAs stay above the wait states: IR passes sink the last ones)
        asm volatile("s_nop 7\n\ts_nop 7");
        keep(kx[(NB - 1) % RX]);
        keep(kx[(NB - 2) % RX]);
        keep(ky[((NB - 1) / 3) % 2]);
        keep8(kc);
#pragma unroll
        for (int j = 0; j < 8; ++j) keep(qf[j]);  // (the last iteration's phase B is their last use)
#pragma unroll
        for (int c = 0; c < 4; ++c) keep8(q8[c]);
        __builtin_amdgcn_sched_barrier(0);
    };

    float m_run = -INFINITY;
    float l_run = 0.f;
    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;

    auto mask_tile = [&](f32x16& sn, int i) {
        const int k0 = (kt_begin + i) * KT;
        const int lo = lo_abs - k0, hi = hi_abs - k0;
        if (__builtin_amdgcn_ballot_w64(lo > 32 * kh || hi < 32 * kh + 28) != 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kr = 32 * kh + key_of(0, r);
                sn[r] = (kr >= lo && kr < hi) ? sn[r] : -INFINITY;
            }
        }
    };
    auto bias_tile = [&](auto slot_c, f32x16& sn) {
        if constexpr (KBIAS) {
            constexpr int SLOT = decltype(slot_c)::value;
            frag kbv[4];
            static_for<0, 4>([&](auto j_c) {
                constexpr int j = decltype(j_c)::value;
                kbv[j] = lds_frag<SLOT * RG::KS + 32 * j>(kbaddr);
            });
            lds_wait_tie(kbv);
#pragma unroll
            for (int r = 0; r < 16; ++r) sn[r] = __builtin_fmaf(sn[r], c_log2, __uint_as_float(kbv[r >> 2][r & 3]));
        }
    };
    auto finish_max = [&](float mraw) -> float {
        const float mx = KBIAS ? mraw : (mraw == -INFINITY ? -INFINITY : mraw * c_log2);
        return fmaxf(mx, __shfl_xor(mx, 32));
    };
    float alpha = 1.f;
    bool rescale = false;
    auto update_max = [&](float mloc) {
        const bool move = mloc > m_run + RESCALE_LOG2;
        alpha = move ? __builtin_amdgcn_exp2f(m_run - mloc) : 1.f;
        m_run = move ? mloc : m_run;
        rescale = __builtin_amdgcn_ballot_w64(move) != 0;
    };
    auto apply_rescale = [&]() {
        if (rescale) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            l_run *= alpha;
        }
    };

    f32x16 sA, sB;
    auto no_fin = [](auto) {};
    auto no_dma = [](auto) {};
    auto pre_k = [&](auto slot_c) {  // the first RA fragments of a phase B that reads K slot SLOT (hi steps: no second read)
        static_for<0, RA>([&](auto r_c) {
            frag unused;
            k_read(slot_c, r_c, kpre[decltype(r_c)::value], unused);
        });
    };
    if (n > 0) {
#pragma unroll
        for (int p = 0; p < NPK; ++p) k_piece(0, kt_begin, p);
        bias_piece(0, kt_begin);
#pragma unroll
        for (int p = 0; p < NPV; ++p) v_piece(0, kt_begin, p);
        if (n > 1) {
#pragma unroll
            for (int p = 0; p < NPK; ++p) k_piece(1, kt_begin + 1, p);
            bias_piece(1, kt_begin + 1);
        }
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        qk_phase(std::integral_constant<int, 0>{}, sA, no_fin, no_dma, no_fin, std::false_type{});
        bias_tile(std::integral_constant<int, 0>{}, sA);
        mask_tile(sA, 0);
        float mr = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) mr = fmaxf(mr, sA[r]);
        update_max(finish_max(mr));
        apply_rescale();
        __builtin_amdgcn_s_barrier();  // every wave has read K slot 0: iteration 0 restages it
        if constexpr (EARLY) {
            pre_k(std::integral_constant<int, 1>{});
            lds_wait_tie(kpre);
        }
    }

    auto iter = [&](auto slot_c, f32x16& sc, f32x16& sn, int i) {
        constexpr int SLOT = decltype(slot_c)::value;
        constexpr int NXT = SLOT ^ 1;
        const bool more = i + 1 < n;
        const int ktk = kt_begin + min(i + 2, n - 1), ktv = kt_begin + min(i + 1, n - 1);
        const float m_use = ((m_run == -INFINITY) ? 0.f : m_run) - PSCALE_F8_LOG2;
        const float nm = -m_use;
        float lsum = 0.f;
        frag pf[2];
        uint32_t ph8[4] = {}, pl8[4] = {};  // fp8 P and P - f16(P): byte r = the lane's score r of the half
        auto plo = [&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            constexpr int r = 2 * j;
            constexpr int fi = r >> 3, fj = (r & 7) >> 1;
            int w8 = (int)pl8[j >> 1];
            typedef _Float16 h2v __attribute__((ext_vector_type(2)));
            const h2v hv = __builtin_bit_cast(h2v, (uint32_t)pf[fi][fj]);
            const float l0 = __builtin_fmaf(-(float)hv[0], one_rt, sc[r]);
            const float l1 = __builtin_fmaf(-(float)hv[1], one_rt, sc[r + 1]);
            w8 = __builtin_amdgcn_cvt_pk_fp8_f32(l0 * 2048.f, l1 * 2048.f, w8, (j & 1) != 0);  // 2^11 (P - f16(P))
            asm volatile("" : "+v"(w8));
            pl8[j >> 1] = (uint32_t)w8;
        };
        // softmax finish of tile i: hi step j forms P pair j (scores 2j, 2j + 1); correction step c forms the lo
        // parts of pairs 2c, 2c + 1 (formed by the two hi steps before it)
        auto fin = [&](auto p_c) {
            constexpr int p = decltype(p_c)::value;
            if constexpr (p % 3 == 2) {
                plo(std::integral_constant<int, 2 * (p / 3)>{});
                plo(std::integral_constant<int, 2 * (p / 3) + 1>{});
            } else {
                constexpr int j = p - p / 3;
                constexpr int r = 2 * j;
                float p0, p1;
                if constexpr (KBIAS) {
                    p0 = __builtin_amdgcn_exp2f(sc[r] + nm);
                    p1 = __builtin_amdgcn_exp2f(sc[r + 1] + nm);
                } else {
                    p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[r], c_log2, nm));
                    p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[r + 1], c_log2, nm));
                }
                lsum += p0;
                lsum += p1;
                constexpr int fi = r >> 3, fj = (r & 7) >> 1;
                typedef float f2 __attribute__((ext_vector_type(2)));
                typedef _Float16 h2t __attribute__((ext_vector_type(2)));
                const h2t hv = __builtin_convertvector((f2){p0, p1}, h2t);
                uint32_t w = __builtin_bit_cast(uint32_t, hv);
                int w8 = (int)ph8[j >> 1];
                w8 = __builtin_amdgcn_cvt_pk_fp8_f32(p0, p1, w8, (j & 1) != 0);
                asm volatile("" : "+v"(w), "+v"(w8), "+v"(lsum), "+v"(p0), "+v"(p1));
                pf[fi][fj] = w;
                ph8[j >> 1] = (uint32_t)w8;
                sc[r] = p0;
                sc[r + 1] = p1;
            }
        };
        // K(i + 2) behind phase B's correction MFMAs (the bias with the first)
        auto dma = [&](auto p_c) {
            constexpr int p = decltype(p_c)::value;
            if constexpr (p % 3 == 2) {
                k_piece(SLOT, ktk, p / 3);
                if constexpr (p == 2) bias_piece(SLOT, ktk);
            }
        };
        // phase C's V reads (defined below) and, EARLY, the mid-phase-B point: V(i), requested in the previous iteration's
        // phase C, landed for every wave (K(i + 2)'s first two pieces + the bias are the only later requests), then
        // phase C's first RA fragments
        auto v_read = [&](auto q_c, frag& x, frag& y) {
            constexpr int q = decltype(q_c)::value;
            if constexpr (q % 3 != 2) {
                constexpr int s = q - q / 3;
                x = lds_frag<SLOT * RG::VS + (s & 3) * 32 * 128>(vaddr[s >> 2]);
            } else {
                x = lds_frag<SLOT * RG::VS + (q / 3) * 32 * 128>(v8a[0]);
                y = lds_frag<SLOT * RG::VS + (q / 3) * 32 * 128>(v8a[1]);
            }
        };
        auto midB = [&](auto p_c) {
            if constexpr (EARLY && decltype(p_c)::value == MID) {
                if (KBIAS && wid == 0)
                    wait_vmcnt<3>();
                else
                    wait_vmcnt<2>();
                __builtin_amdgcn_s_barrier();
                static_for<0, RA>([&](auto r_c) {
                    frag unused;
                    v_read(r_c, vpre[decltype(r_c)::value], unused);
                });
            }
        };
        qk_phase(std::integral_constant<int, NXT>{}, sn, [&](auto j_c) { fin(j_c); }, [&](auto j_c) { dma(j_c); },
                 [&](auto j_c) { midB(j_c); }, std::integral_constant<bool, EARLY>{});
        l_run += lsum;

        if constexpr (EARLY) {
            asm volatile("" : "+v"(vpre[0]), "+v"(vpre[1]));  // landed: phase B's last steps waited for every read
        } else {
            // V(i), requested in the previous iteration's phase C, landed for every wave
            if (KBIAS && wid == 0)
                wait_vmcnt<NPK + 1>();
            else
                wait_vmcnt<NPK>();
            __builtin_amdgcn_s_barrier();
        }
        bias_tile(std::integral_constant<int, NXT>{}, sn);
        mask_tile(sn, i + 1);
        float mr = -INFINITY;
        {
            // phase C positions: q % 3 == 2 the correction of d-tile q / 3, else the hi step s = q - q / 3 (d-tile
            // s & 3, 16-key group s >> 2 of the half)
            constexpr int NC = 12;
            uint32_t pb[8];  // [Ph ; Pl] of the half's 32 keys: lane half 0 the Ph bytes, lane half 1 the Pl bytes
            frag vx[RX], vy[2];
            v8i vc;
            auto rv = [](int q) constexpr { return q % 3 == 2 ? 2 : 1; };
            static_for<0, RA>([&](auto r_c) {
                constexpr int r = decltype(r_c)::value;
                if constexpr (EARLY)
                    vx[r] = vpre[r];
                else
                    v_read(r_c, vx[r], vy[0]);
            });
            static_for<0, NC>([&](auto q_c) {
                constexpr int q = decltype(q_c)::value;
                if constexpr (q + RA < NC)
                    v_read(std::integral_constant<int, q + RA>{}, vx[(q + RA) % RX], vy[((q + RA) / 3) % 2]);
                if constexpr (q == 0) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const auto sw = __builtin_amdgcn_permlane32_swap(ph8[w], pl8[w], false, false);
                        pb[w] = sw[0];
                        pb[4 + w] = sw[1];
                    }
                }
                constexpr int after = reads_after(q, NC, rv) + extra(q);
                asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(after) : "memory");
                asm volatile("" : "+v"(vx[q % RX]));
                if constexpr (rv(q) == 2) asm volatile("" : "+v"(vy[(q / 3) % 2]));
                if constexpr (q % 3 != 2) {
                    constexpr int s = q - q / 3;
                    o[s & 3] = mfma32(vx[q % RX], pf[s >> 2], o[s & 3]);
                } else {
                    constexpr int dt = q / 3;
                    vc = cat8(vx[q % RX], vy[(q / 3) % 2]);
                    o[dt] = mfma_f8(vc, cat8(pb), o[dt], F8_SCALE_LO, F8_SCALE_1);
                }
                if constexpr (q % 3 != 2) {
                    constexpr int s = q - q / 3;
                    mr = fmaxf(mr, fmaxf(sn[2 * s], sn[2 * s + 1]));
                    asm volatile("" : "+v"(mr));
                } else {
                    v_piece(NXT, ktv, q / 3);  // V(i + 1) behind the correction MFMAs
                }
                static_for<1, 3>([&](auto d_c) {
                    constexpr int qd = q - decltype(d_c)::value;
                    if constexpr (qd >= 0) {
                        keep(vx[qd % RX]);
                        if constexpr (rv(qd) == 2) keep(vy[(qd / 3) % 2]);
                    }
                });
                if constexpr (q > 2) keep8(vc);  // (phase C's hi steps are short: held until the next correction)
                if constexpr (EARLY && q == MID) {
                    // K(i + 2) landed for every wave (V(i + 1)'s first two pieces are the later requests), then the next
                    // phase B's first fragments (K(i + 2) sits in this iteration's slot)
                    wait_vmcnt<2>();
                    __builtin_amdgcn_s_barrier();
                    pre_k(slot_c);
                }
                if constexpr (EARLY && q == NC - 1) asm volatile("" : "+v"(kpre[0]), "+v"(kpre[1]));  // landed (lgkmcnt(0))
                __builtin_amdgcn_sched_barrier(0);
            });
            // the P operands and the last fragments stay allocated through the retire (phase B rewrites pf / ph8 / pl8)
            asm volatile("" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]));
            asm volatile("s_nop 7\n\ts_nop 7");
            keep(vx[(NC - 1) % RX]);
            keep(vx[(NC - 2) % RX]);
            keep(vy[((NC - 1) / 3) % 2]);
            keep8(vc);
            keep(pf[0]);
            keep(pf[1]);
#pragma unroll
            for (int w = 0; w < 8; ++w) asm volatile("" ::"v"(pb[w]));
            __builtin_amdgcn_sched_barrier(0);
        }
        const float mnx = finish_max(mr);
        if (more) {
            update_max(mnx);
            apply_rescale();
            if constexpr (!EARLY) {
                wait_vmcnt<NPV>();  // K(i + 2) landed (V(i + 1), issued after it, may stay in flight)
                __builtin_amdgcn_s_barrier();
            }
        }
    };

    int i = 0;
    for (; i + 1 < n; i += 2) {
        iter(std::integral_constant<int, 0>{}, sA, sB, i);
        iter(std::integral_constant<int, 1>{}, sB, sA, i + 1);
    }
    if (i < n) iter(std::integral_constant<int, 0>{}, sA, sB, i);
    wait_vmcnt<0>();

    // the two key halves of each row: half 1 hands (O, m, l) to half 0 through LDS (the rings are free after the
    // barrier), half 0 combines them as the key-split merge does (weight 2^(m_k - M), 0 for a half with no key)
    float l = l_run + __shfl_xor(l_run, 32);
    __builtin_amdgcn_s_barrier();
    float4* xch = reinterpret_cast<float4*>(smem) + wq * 17 * 64 + lane;
    if (kh == 1) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
            xch[j * 64] = make_float4(o[j >> 2][4 * (j & 3)], o[j >> 2][4 * (j & 3) + 1], o[j >> 2][4 * (j & 3) + 2],
                                      o[j >> 2][4 * (j & 3) + 3]);
        xch[16 * 64] = make_float4(m_run, l, 0.f, 0.f);
    }
    __syncthreads();
    if (kh == 1) return;
    {
        const float4 ml = xch[16 * 64];
        const float M = fmaxf(m_run, ml.x);
        const float w0 = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - M);
        const float w1 = ml.x == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ml.x - M);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float4 x = xch[j * 64];
            f32x16& od = o[j >> 2];
            const int r = 4 * (j & 3);
            od[r] = od[r] * w0 + x.x * w1;
            od[r + 1] = od[r + 1] * w0 + x.y * w1;
            od[r + 2] = od[r + 2] * w0 + x.z * w1;
            od[r + 3] = od[r + 3] * w0 + x.w * w1;
        }
        l = l * w0 + ml.y * w1;
        m_run = M;
    }
    if (ks > 1) {
        if (qrow < a.nq) {
            const int64_t row = ((int64_t)split * a.B + b) * a.nq + qrow;
            float* po = a.part + row * (a.Hq * D) + head * D;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *(float4*)(po + 32 * dt + 8 * g4 + 4 * h) =
                        make_float4(o[dt][4 * g4 + 0], o[dt][4 * g4 + 1], o[dt][4 * g4 + 2], o[dt][4 * g4 + 3]);
            if (h == 0)
                *(float2*)(a.part + (int64_t)a.ksplit * a.B * a.nq * a.Hq * D + (row * a.Hq + head) * 2) =
                    make_float2(m_run, l);
        }
        return;
    }
    const float inv = 1.0f / l;
    if (a.out_f32) {
        if (qrow < a.nq) {
            float* of = a.out_f32 + ((int64_t)b * a.nq + qrow) * (a.Hq * D) + head * D;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *(float4*)(of + 32 * dt + 8 * g4 + 4 * h) =
                        make_float4(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv, o[dt][4 * g4 + 2] * inv,
                                    o[dt][4 * g4 + 3] * inv);
        }
        return;
    }
    if (qrow < a.nq) {
        uint16_t* op = a.out + ((int64_t)b * a.nq + qrow) * (a.Hq * D) + head * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 32 * dt + 8 * g4 + 4 * h;
                uint2 w;
                w.x = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 0] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 1] * inv) << 16);
                w.y = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 2] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 3] * inv) << 16);
                *(uint2*)(op + d) = w;
            }
        }
    }
}

// Combine the S key-range parts of one (item, query, head) row: M = max m_k, weights 2^(m_k - M) (0 for a
// part whose keys were all masked), out = sum w_k O_k / sum w_k l_k; a row with no unmasked key at all stays
// 0/0 = NaN as in ggml.  Half a wave per row, 16-byte partial reads, every load issued before the first use.
// TAIL (tail split, AttnArgs::split_from): only the rows of the split blocks F.., 128 (query, head) rows per block.
template <bool F16OUT, int S, bool TAIL = false, bool OUTF32 = false>
__global__ void __launch_bounds__(256) attn_merge_kernel(AttnArgs a) {
    const int64_t rows = (int64_t)a.B * a.nq * a.Hq;
    int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    if constexpr (TAIL) {
        const int rep = a.Hq / a.Hkv, qpb = 128 / rep, n_qt = (a.nq + qpb - 1) / qpb;
        const int64_t tb = r >> 7;
        if (tb >= (int64_t)a.B * a.Hkv * n_qt - a.split_from) return;
        const int blk = a.split_from + (int)tb, w = (int)(r & 127);
        const int qt = blk % n_qt, kvh = (blk / n_qt) % a.Hkv, b = blk / n_qt / a.Hkv;
        const int q = qt * qpb + w % qpb;
        if (q >= a.nq) return;
        r = ((int64_t)b * a.nq + q) * a.Hq + kvh * rep + w / qpb;
    }
    if (r >= rows) return;
    const int d = (threadIdx.x & 31) * 4;
    const float* ml = a.part + S * rows * D;
    float2 mlk[S];
    float4 ok[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        mlk[k] = *(const float2*)(ml + (k * rows + r) * 2);
        ok[k] = *(const float4*)(a.part + (k * rows + r) * D + d);
    }
    float M = mlk[0].x;
#pragma unroll
    for (int k = 1; k < S; ++k) M = fmaxf(M, mlk[k].x);
    float den = 0.f, v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const float w = mlk[k].x == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mlk[k].x - M);
        den += w * mlk[k].y;
        v[0] += w * ok[k].x;
        v[1] += w * ok[k].y;
        v[2] += w * ok[k].z;
        v[3] += w * ok[k].w;
    }
    const float inv = 1.0f / den;
    // row r = (b * nq + q) * Hq + head: out[b][q][head*128 + d] is contiguous in r * 128 + d
    if constexpr (OUTF32) {
        *(float4*)(a.out_f32 + r * D + d) = make_float4(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
        return;
    }
    *(uint2*)(a.out + r * D + d) =
        make_uint2((uint32_t)to_act<F16OUT>(v[0] * inv) | ((uint32_t)to_act<F16OUT>(v[1] * inv) << 16),
                   (uint32_t)to_act<F16OUT>(v[2] * inv) | ((uint32_t)to_act<F16OUT>(v[3] * inv) << 16));
}

int g_kh_mode = -1;

template <bool F16OUT, bool SPLIT, bool PVS>
void launch_t(const AttnArgs& a, dim3 grid, hipStream_t s, bool kh) {
    const size_t lds = Ring<SPLIT, PVS>::BYTES;
    // One workgroup per CU in every mode (round 6): each instance then runs one wave per SIMD, the only occupancy at
    // which attn2's hand-laid stream may reuse an MFMA's A / B register right after issuing it (tools/audit_mfma_war.py
    // classifies those pairs as single-wave).  Round 3's kernel (attn_kernel, ACE_MI_ATTN_V1) and the
    // two-per-CU fp16 instance are gone: the fp16 mode is a diagnostic precision, not a product one.
    if constexpr (PVS) {
        if constexpr (SPLIT) {
            if (a.f8 && kh) {  // f8c at two waves per SIMD (launch_attention's policy)
                if (a.kbias)
                    hipLaunchKernelGGL((attn_kh_kernel<F16OUT, true>), grid, dim3(512), lds, s, a);
                else
                    hipLaunchKernelGGL((attn_kh_kernel<F16OUT, false>), grid, dim3(512), lds, s, a);
                return;
            }
        }
        if (a.f8) {  // f8c (SPLIT) or pv8 (fp16 Q.K)
            if (a.kbias)
                hipLaunchKernelGGL((attn2_kernel<F16OUT, SPLIT, true, true, 1, true>), grid, dim3(256), lds, s, a);
            else
                hipLaunchKernelGGL((attn2_kernel<F16OUT, SPLIT, true, false, 1, true>), grid, dim3(256), lds, s, a);
            return;
        }
    }
    if constexpr (!SPLIT && PVS) {
        throw std::runtime_error("attention: hi/lo P.V with fp16 Q.K exists only with fp8 corrections (pv8)");
    } else {
        if (a.kbias)
            hipLaunchKernelGGL((attn2_kernel<F16OUT, SPLIT, PVS, true, 1>), grid, dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((attn2_kernel<F16OUT, SPLIT, PVS, false, 1>), grid, dim3(256), lds, s, a);
    }
}

}  // namespace

void launch_attention(ActType out_t, const AttnArgs& a, hipStream_t s) {
    ACEMI_CHECK(a.Hkv > 0 && a.Hq % a.Hkv == 0, "attention: Hq must be a multiple of Hkv");
    const int rep = a.Hq / a.Hkv;
    ACEMI_CHECK(rep == 1 || rep == 2 || rep == 4, "attention: n_rep must be 1, 2 or 4");
    ACEMI_CHECK(a.nk_pad % KT == 0 && a.nk_pad >= a.nk, "attention: nk_pad");
    const int qpb = 128 / rep;
    const int n_qt = (a.nq + qpb - 1) / qpb;
    ACEMI_CHECK(a.nq_pad >= n_qt * qpb, "attention: nq_pad too small");
    AttnArgs b = a;
    b.ksplit = 1;
    b.split_from = 0;
    {
        static int xcd = -1;  // ACE_MI_ATTN_XCD_ORDER=0: plain block order (A/B measurements)
        if (xcd < 0) {
            const char* e = std::getenv("ACE_MI_ATTN_XCD_ORDER");
            xcd = (e && e[0] == '0') ? 0 : 1;
        }
        b.xcd_order = xcd;
    }
    {
        // a grid of fewer than ~1.6 rounds over the CUs idles a third of the chip in its last
        // round: split each block's key range in two (B = 1 at 240 s: 376 blocks -> 752)
        static int n_cu = 0;
        if (n_cu == 0) {
            int dev = 0;
            ACEMI_HIP(hipGetDevice(&dev));
            ACEMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
        }
        const int64_t blocks = (int64_t)a.B * a.Hkv * n_qt;
        const int span = a.window > 0 ? std::min(a.nk, qpb + 2 * a.window) : a.nk;
        // (measured: full 240 s 317 -> 262 us incl. the merge; at 8 key tiles or fewer -- cross attention,
        // sliding windows -- the extra prologue and merge cost more than the round saves)
        // ACE_MI_ATTN_KSPLIT=1 never / 2 always (where a workspace exists) / 3 auto without the short-range split /
        // 4 see below / auto
        static int mode = -1;
        if (mode < 0) {
            const char* e = std::getenv("ACE_MI_ATTN_KSPLIT");
            mode = (e && (e[0] == '1' || e[0] == '2' || e[0] == '3' || e[0] == '4')) ? e[0] - '0' : 0;
        }
        // blocks resident per CU: one in every mode (launch_t)
        const int per_cu = 1;
        const int64_t slots = (int64_t)n_cu * per_cu;
        const int ntiles = (span + KT - 1) / KT;
        int S = 1;
        // tail split (default; ACE_MI_ATTN_TAIL_SPLIT=0: every block split): when the whole blocks overfill one
        // round by at most half a round, run one round of whole blocks and split only the rest -- the same
        // 1 + 1/2 rounds of key tiles per CU as splitting every block, one block prologue fewer per CU, a third of
        // the rows through the merge (240 s, B = 1: 256 whole blocks + 2 x 120 halves).  ACE_MI_ATTN_TAIL_MIN: the
        // fewest key tiles per block for which it is used where every-block splitting is not (default 16 = never)
        static int tail = -1, tail_min = 0;
        if (tail < 0) {
            const char* e = std::getenv("ACE_MI_ATTN_TAIL_SPLIT");
            tail = (e && e[0] == '0') ? 0 : 1;
            const char* m = std::getenv("ACE_MI_ATTN_TAIL_MIN");
            tail_min = m ? std::max(2, std::atoi(m)) : 16;
        }
        const int64_t F = slots & ~int64_t(7);
        const bool tail_fits = tail && (mode == 0 || mode == 3) && F > 0 && blocks > F && 2 * (blocks - F) <= slots;
        if (ntiles >= 16) {
            if (blocks * 10 < slots * 16) S = 2;
        } else if (mode == 4 || (mode == 0 && blocks * 2 <= slots)) {
            // short key ranges (cross attention, sliding windows, short sequences) split too when the grid fills at
            // most half a round (ACE_MI_ATTN_KSPLIT=4: whatever the grid), while it stays within one round and every
            // part keeps >= 2 key tiles.  Round 3 (the first kernel, profiles/r03_trace_60s_*.txt) lost: 698 us +
            // 48 merges 275 us per forward against ~950 us unsplit.  With attn2 it pays: 60 s (96 blocks on 256 CUs)
            // 165.1 against 163.1-163.4 steps/s (profiles/r05/attn_ksplit_short.txt)
            while (S < 4 && blocks * 2 * S <= slots && ntiles >= 4 * S) S *= 2;
        } else if (tail_fits && ntiles >= tail_min) {
            S = 2;
        }
        if (a.part && mode == 2) b.ksplit = 2;
        else if (a.part && (mode == 0 || mode == 3 || mode == 4)) b.ksplit = S;
        if (tail_fits && b.ksplit == 2) b.split_from = (int)F;
        // (round 5 also built an in-kernel merge -- the last part of a group merging through an sc1 partial round
        // trip and a ticket, no merge launch: neutral at 60 s, 4 % slower lines at 240 s, profiles/r05/attn_fused_merge.txt;
        // removed from the product library in round 6)
    }
    // (f32 output, AttnArgs::out_f32: the same split policy -- whole blocks write f32 rows themselves, the merges
    // below write f32 rows; until round 6 every block ran in two key-range parts with a full merge, 0.84 ms per 240 s
    // step of the quantized-activation mode)
    const int64_t n_blk = (int64_t)a.B * a.Hkv * n_qt;
    // XCD-aware order (attn_block): whole multiples of 8 launch indices per range
    const dim3 grid(b.split_from > 0 ? (unsigned)(b.split_from + 8 * ((2 * (n_blk - b.split_from) + 7) / 8))
                                     : (unsigned)(8 * ((n_blk * b.ksplit + 7) / 8)));
    const bool f16 = out_t == ActType::F16;
    ACEMI_CHECK(!a.f8 || a.pv_split, "attention: the fp8 correction modes need pv_split");
    // f8c kernel: attn_kh_kernel (two waves per SIMD) where a block streams >= 16 key tiles (full self-attention
    // layers; measured 240 s: full 173.3 vs 175.2 us, bs 8 1.340 vs 1.355 ms), attn2 on short ranges (cross 50.8 vs
    // 48.1 us, sliding 42.4 vs 41.4: the 8-wave prologue and the pair merge outweigh the gain), profiles/r06/attn_kh/
    bool kh;
    {
        static int env = -2;
        if (env == -2) {
            const char* e = std::getenv("ACE_MI_ATTN_KH");
            env = (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : -1;
        }
        const int mode = g_kh_mode >= 0 ? g_kh_mode : env;
        const int span = a.window > 0 ? std::min(a.nk, qpb + 2 * a.window) : a.nk;
        kh = mode == 1 || (mode < 0 && (span + KT - 1) / KT >= 16);
    }
    if (a.split) {
        ACEMI_CHECK(a.q_plane > 0 && a.k_plane > 0, "attention: split mode needs lo planes");
        if (a.pv_split) {
            ACEMI_CHECK(a.v_plane > 0, "attention: hi/lo P.V needs the V lo plane");
            f16 ? launch_t<true, true, true>(b, grid, s, kh) : launch_t<false, true, true>(b, grid, s, kh);
        } else {
            f16 ? launch_t<true, true, false>(b, grid, s, kh) : launch_t<false, true, false>(b, grid, s, kh);
        }
    } else if (a.pv_split) {
        ACEMI_CHECK(a.f8 && a.v_plane > 0, "attention: pv8 mode needs the fp8 V lo plane");
        f16 ? launch_t<true, false, true>(b, grid, s, kh) : launch_t<false, false, true>(b, grid, s, kh);
    } else {
        f16 ? launch_t<true, false, false>(b, grid, s, kh) : launch_t<false, false, false>(b, grid, s, kh);
    }
    ACEMI_HIP(hipGetLastError());
    if (b.ksplit > 1) {
        const int64_t rows = (int64_t)a.B * a.nq * a.Hq;
        ACEMI_CHECK(b.ksplit == 2 || b.ksplit == 4, "attention: the merge handles 2 or 4 key-split parts");
        const dim3 mgrid((unsigned)((rows + 7) / 8));
        if (a.out_f32) {
            if (b.split_from > 0)
                hipLaunchKernelGGL((attn_merge_kernel<false, 2, true, true>), dim3((unsigned)((n_blk - b.split_from) * 16)),
                                   dim3(256), 0, s, b);
            else if (b.ksplit == 2)
                hipLaunchKernelGGL((attn_merge_kernel<false, 2, false, true>), mgrid, dim3(256), 0, s, b);
            else
                hipLaunchKernelGGL((attn_merge_kernel<false, 4, false, true>), mgrid, dim3(256), 0, s, b);
        } else if (b.split_from > 0) {
            const dim3 tgrid((unsigned)((n_blk - b.split_from) * 16));  // 128 rows per split block, 8 per workgroup
            if (out_t == ActType::F16)
                hipLaunchKernelGGL((attn_merge_kernel<true, 2, true>), tgrid, dim3(256), 0, s, b);
            else
                hipLaunchKernelGGL((attn_merge_kernel<false, 2, true>), tgrid, dim3(256), 0, s, b);
        } else if (b.ksplit == 2) {
            if (out_t == ActType::F16)
                hipLaunchKernelGGL((attn_merge_kernel<true, 2>), mgrid, dim3(256), 0, s, b);
            else
                hipLaunchKernelGGL((attn_merge_kernel<false, 2>), mgrid, dim3(256), 0, s, b);
        } else {
            if (out_t == ActType::F16)
                hipLaunchKernelGGL((attn_merge_kernel<true, 4>), mgrid, dim3(256), 0, s, b);
            else
                hipLaunchKernelGGL((attn_merge_kernel<false, 4>), mgrid, dim3(256), 0, s, b);
        }
        ACEMI_HIP(hipGetLastError());
    }
}

void attn_kh_mode(int mode) { g_kh_mode = mode; }

size_t attn_part_floats(int B, int nq, int Hq) {
    const size_t rows = (size_t)B * nq * Hq;
    // up to four key-split parts: unnormalised O rows + (running max, sum) per row
    return 4 * rows * (D + 2);
}

}  // namespace acemi
