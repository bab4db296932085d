// Kernel self-test entries (include/acestep_mi355x.h, "test library"): run one gfx950 kernel on host buffers so
// the GPU parity tests can compare it with an fp64 / fp32 reference of the same op, and the kernel
// micro-benchmarks of tools/.  Built only into libacestep_mi355x_selftest.so (the product objects + this
// file, Makefile target `selftest`); the product library libacestep_mi355x.so does not contain them.
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "../../../include/acestep_mi355x_selftest.h"
#include "../kernels.h"
#include "quant.h"

namespace {

struct DevMem {
    void* p = nullptr;
    explicit DevMem(size_t bytes) { ACEMI_HIP(hipMalloc(&p, bytes ? bytes : 16)); }
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
    template <typename T>
    T* as() {
        return static_cast<T*>(p);
    }
};

}  // namespace

extern "C" {

ace_ggml_status ace_mi_kernel_gemm(int32_t act_type, int32_t epi, int32_t M, int32_t N, int32_t K, const uint16_t* A,
                                   const uint16_t* W, const float* bias, float* out_f32, uint16_t* out_u16) {
    using namespace acemi;
    if (!A || !W || M <= 0 || N % 128 != 0 || K % 64 != 0) return ACE_GGML_ERR_INVALID_ARG;
    const bool resid = epi == EPI_RESID || epi == EPI_RESID_GATED;
    if (epi != EPI_STORE_F32 && epi != EPI_SWIGLU && !resid) return ACE_GGML_ERR_UNSUPPORTED;
    if (((epi == EPI_STORE_F32 || resid) && !out_f32) || (epi == EPI_SWIGLU && !out_u16))
        return ACE_GGML_ERR_INVALID_ARG;
    if (epi == EPI_RESID_GATED && !bias) return ACE_GGML_ERR_INVALID_ARG;
    try {
        DevMem dA((size_t)M * K * 2), dW((size_t)N * K * 2), dB((size_t)N * 4), dC((size_t)M * N * 4);
        ACEMI_HIP(hipMemcpy(dA.p, A, (size_t)M * K * 2, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dW.p, W, (size_t)N * K * 2, hipMemcpyHostToDevice));
        if (bias) ACEMI_HIP(hipMemcpy(dB.p, bias, (size_t)N * 4, hipMemcpyHostToDevice));
        GemmEpilogue e;
        e.kind = epi;
        e.bias = bias && !resid ? dB.as<float>() : nullptr;
        if (resid) {  // out_f32 holds x on entry: x += acc (* gate[n], the gate passed as `bias`)
            ACEMI_HIP(hipMemcpy(dC.p, out_f32, (size_t)M * N * 4, hipMemcpyHostToDevice));
            e.c_f32 = dC.as<float>();
            e.ldc = N;
            e.gate = epi == EPI_RESID_GATED ? dB.as<float>() : nullptr;
            e.gate_stride = 0;
            e.rows_per_item = M;
        } else if (epi == EPI_STORE_F32) {
            e.c_f32 = dC.as<float>();
            e.ldc = N;
        } else {
            e.c_act = dC.as<uint16_t>();
            e.ldc = N / 2;
        }
        launch_gemm(act_type == 1 ? ActType::F16 : ActType::BF16, dA.as<uint16_t>(), K, dW.as<uint16_t>(), K, M, N,
                    K, e, nullptr);
        ACEMI_HIP(hipDeviceSynchronize());
        if (epi == EPI_STORE_F32 || resid)
            ACEMI_HIP(hipMemcpy(out_f32, dC.p, (size_t)M * N * 4, hipMemcpyDeviceToHost));
        else
            ACEMI_HIP(hipMemcpy(out_u16, dC.p, (size_t)M * (N / 2) * 2, hipMemcpyDeviceToHost));
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "ace_mi_kernel_gemm: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

}  // extern "C"

namespace {
// Device operands of one attention launch, prepared from host f32 q [B][nq][Hq*128] and kv
// [B][nk][2*Hkv*128] through the engine's own prep kernel (hi/lo planes, V^T, key bias).
struct AttnSetup {
    DevMem dq, dkv, dm, dqh, dkh, dvt, dkb, dout, dpart;
    acemi::AttnArgs a{};
    size_t nqf;
    AttnSetup(int B, int Hq, int Hkv, int nq, int nk, int window, float scale, int flags, const float* q,
              const float* kv, const int32_t* kmask)
        : dq((size_t)B * nq * Hq * 128 * 4), dkv((size_t)B * nk * 2 * Hkv * 128 * 4), dm((size_t)B * nk * 4),
          dqh((size_t)2 * B * Hq * acemi::round_up(nq, 128) * 128 * 2), dkh((size_t)2 * B * Hkv * acemi::round_up(nk, 128) * 128 * 2),
          dvt((size_t)2 * B * Hkv * 128 * acemi::round_up(nk, 128) * 2), dkb((size_t)B * acemi::round_up(nk, 128) * 4),
          dout((size_t)B * nq * Hq * 128 * 2), dpart(acemi::attn_part_floats(B, nq, Hq) * 4) {
        using namespace acemi;
        const int D = 128;
        const int nq_pad = (int)round_up(nq, 128), nk_pad = (int)round_up(nk, 128);
        ACEMI_HIP(hipMemset(dpart.p, 0, attn_part_floats(B, nq, Hq) * 4));  // the key-split tickets start at 0
        nqf = (size_t)B * nq * Hq * D;
        const size_t nkvf = (size_t)B * nk * 2 * Hkv * D;
        ACEMI_HIP(hipMemcpy(dq.p, q, nqf * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dkv.p, kv, nkvf * 4, hipMemcpyHostToDevice));
        if (kmask) ACEMI_HIP(hipMemcpy(dm.p, kmask, (size_t)B * nk * 4, hipMemcpyHostToDevice));
        const bool split = (flags & 1) != 0;
        PrepArgs pq{};
        pq.src = dq.as<float>();
        pq.ld = Hq * D;
        pq.q_col = 0;
        pq.k_col = -1;
        pq.v_col = -1;
        pq.hq = Hq;
        pq.hkv = Hkv;
        pq.n_tok = nq;
        pq.n_pad = nq_pad;
        pq.B = B;
        pq.qh = dqh.as<uint16_t>();
        const int64_t qpl = (int64_t)B * Hq * nq_pad * D, kpl = (int64_t)B * Hkv * nk_pad * D;
        pq.q_plane = split ? qpl : 0;
        const bool f8 = (flags & 8) && (flags & 16);  // f8c with split, pv8 without
        const bool pvs = (flags & 8) && (split || f8);
        pq.f8 = f8 ? 1 : 0;
        launch_attn_prep(pq, nullptr);
        PrepArgs pk{};
        pk.src = dkv.as<float>();
        pk.ld = 2 * Hkv * D;
        pk.q_col = -1;
        pk.k_col = 0;
        pk.v_col = Hkv * D;
        pk.hq = Hq;
        pk.hkv = Hkv;
        pk.n_tok = nk;
        pk.n_pad = nk_pad;
        pk.B = B;
        pk.kh = dkh.as<uint16_t>();
        pk.vt = dvt.as<uint16_t>();
        pk.k_plane = split ? kpl : 0;
        pk.v_plane = pvs || split ? kpl : 0;
        pk.f8 = f8 ? 1 : 0;
        launch_attn_prep(pk, nullptr);
        launch_key_bias(kmask ? dm.as<int32_t>() : nullptr, B, nk, 1, nk, nk_pad, dkb.as<float>(), nullptr);
        a.q = dqh.as<uint16_t>();
        a.k = dkh.as<uint16_t>();
        a.vt = dvt.as<uint16_t>();
        a.kbias = kmask ? dkb.as<float>() : nullptr;
        a.out = dout.as<uint16_t>();
        a.part = dpart.as<float>();
        a.B = B;
        a.Hq = Hq;
        a.Hkv = Hkv;
        a.nq = nq;
        a.nq_pad = nq_pad;
        a.nk = nk;
        a.nk_pad = nk_pad;
        a.window = window;
        a.scale = scale;
        a.split = split;
        a.causal = (flags & 2) != 0;
        a.pv_split = pvs;
        a.f8 = f8;
        a.q_plane = qpl;
        a.k_plane = kpl;
        a.v_plane = kpl;
        ACEMI_HIP(hipDeviceSynchronize());
    }
};
}  // namespace

extern "C" {

ace_ggml_status ace_mi_kernel_attention(int32_t B, int32_t Hq, int32_t Hkv, int32_t nq, int32_t nk, int32_t window,
                                        float scale, int32_t split, const float* q, const float* kv,
                                        const int32_t* kmask, float* out) {
    using namespace acemi;
    if (B <= 0 || Hq <= 0 || Hkv <= 0 || nq <= 0 || nk <= 0 || !q || !kv || !out) return ACE_GGML_ERR_INVALID_ARG;
    try {
        AttnSetup st(B, Hq, Hkv, nq, nk, window, scale, split, q, kv, kmask);
        launch_attention(ActType::BF16, st.a, nullptr);
        ACEMI_HIP(hipDeviceSynchronize());
        std::vector<uint16_t> h(st.nqf);
        ACEMI_HIP(hipMemcpy(h.data(), st.dout.p, st.nqf * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < st.nqf; ++i) {
            const uint32_t u = (uint32_t)h[i] << 16;
            std::memcpy(&out[i], &u, 4);
        }
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "ace_mi_kernel_attention: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

// Attention micro-benchmark: pseudo-random N(0,1)-like q / kv (fixed seed), average ms per launch over
// `iters` launches timed with hipEvents.  flags: bit 0 split (hi/lo) operands, bit 1 causal, bit 3 hi/lo P.V,
// bit 2 a key-padding mask (every 7th key masked), bit 4 the fp8 correction encoding (with bit 3: with bit 0 the f8c
// mode, without it pv8).
ace_ggml_status ace_mi_bench_attention(int32_t B, int32_t Hq, int32_t Hkv, int32_t nq, int32_t nk, int32_t window,
                                       int32_t flags, int32_t iters, float* avg_ms) {
    using namespace acemi;
    if (B <= 0 || Hq <= 0 || Hkv <= 0 || nq <= 0 || nk <= 0 || iters <= 0 || !avg_ms) return ACE_GGML_ERR_INVALID_ARG;
    try {
        std::vector<float> q((size_t)B * nq * Hq * 128), kv((size_t)B * nk * 2 * Hkv * 128);
        std::vector<int32_t> km((size_t)B * nk);
        uint32_t r = 2024u;
        auto rnd = [&]() {  // sum of 4 uniforms, centred: roughly N(0, 1/3)
            float acc = 0.f;
            for (int j = 0; j < 4; ++j) {
                r = r * 1664525u + 1013904223u;
                acc += (float)(r >> 8) * (1.0f / 16777216.0f);
            }
            return acc - 2.0f;
        };
        for (auto& v : q) v = 2.0f * rnd();
        for (auto& v : kv) v = rnd();
        for (size_t i = 0; i < km.size(); ++i) km[i] = (i % 7) != 6;
        AttnSetup st(B, Hq, Hkv, nq, nk, window, 1.0f / std::sqrt(128.0f), flags & 27, q.data(), kv.data(),
                     (flags & 4) ? km.data() : nullptr);
        hipEvent_t e0, e1;
        ACEMI_HIP(hipEventCreate(&e0));
        ACEMI_HIP(hipEventCreate(&e1));
        for (int i = 0; i < 2; ++i) launch_attention(ActType::BF16, st.a, nullptr);
        ACEMI_HIP(hipEventRecord(e0, nullptr));
        for (int i = 0; i < iters; ++i) launch_attention(ActType::BF16, st.a, nullptr);
        ACEMI_HIP(hipEventRecord(e1, nullptr));
        ACEMI_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        ACEMI_HIP(hipEventElapsedTime(&ms, e0, e1));
        *avg_ms = ms / (float)iters;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "ace_mi_bench_attention: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}



}  // extern "C"

extern "C" {

// GEMM micro-benchmark (random bf16/fp16 operands, device-resident): average ms per launch over
// `iters` launches timed with hipEvents.  variant -1 = the engine's automatic choice.
ace_ggml_status ace_mi_bench_gemm(int32_t act_type, int32_t epi, int32_t variant, int32_t M, int32_t N, int32_t K,
                                  int32_t iters, float* avg_ms) {
    using namespace acemi;
    if (M <= 0 || N % 128 != 0 || K % 64 != 0 || iters <= 0 || !avg_ms) return ACE_GGML_ERR_INVALID_ARG;
    try {
        std::vector<uint16_t> ha((size_t)M * K), hw((size_t)N * K);
        uint32_t st = 12345u;
        auto rnd = [&]() {  // uniform in [-1, 1) as bf16 / fp16 bits
            st = st * 1664525u + 1013904223u;
            const float f = (float)(st >> 8) * (2.0f / 16777216.0f) - 1.0f;
            if (act_type == 1) {
                _Float16 h = (_Float16)f;
                return __builtin_bit_cast(uint16_t, h);
            }
            uint32_t u;
            std::memcpy(&u, &f, 4);
            return (uint16_t)(u >> 16);
        };
        for (auto& v : ha) v = rnd();
        for (auto& v : hw) v = rnd();
        DevMem dA(ha.size() * 2), dW(hw.size() * 2), dC((size_t)M * N * 4), dG((size_t)N * 4);
        ACEMI_HIP(hipMemcpy(dA.p, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dW.p, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemset(dC.p, 0, (size_t)M * N * 4));
        ACEMI_HIP(hipMemset(dG.p, 0, (size_t)N * 4));
        GemmEpilogue e;
        e.kind = epi;
        e.ldc = (epi == EPI_SWIGLU) ? N / 2 : N;
        e.c_f32 = dC.as<float>();
        e.c_act = dC.as<uint16_t>();
        e.gate = dG.as<float>();
        e.rows_per_item = M;
        const ActType at = act_type == 1 ? ActType::F16 : ActType::BF16;
        // ACE_MI_BENCH_COLD=R: rotate over R device copies of W (R x |W| beyond the 256 MB MALL = weights cold in
        // every launch, as in a forward where each layer's weights were last read one step earlier)
        const char* ce = std::getenv("ACE_MI_BENCH_COLD");
        const int R = ce ? std::max(1, std::min(64, std::atoi(ce))) : 1;
        DevMem dWr((size_t)R * hw.size() * 2);
        for (int r = 0; r < R; ++r)
            ACEMI_HIP(hipMemcpy(dWr.as<uint16_t>() + (size_t)r * hw.size(), dW.p, hw.size() * 2, hipMemcpyDeviceToDevice));
        auto wptr = [&](int i) { return dWr.as<uint16_t>() + (size_t)(i % R) * hw.size(); };
        gemm_force_variant(variant);
        hipEvent_t e0, e1;
        ACEMI_HIP(hipEventCreate(&e0));
        ACEMI_HIP(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i) launch_gemm(at, dA.as<uint16_t>(), K, wptr(i), K, M, N, K, e, nullptr);
        ACEMI_HIP(hipEventRecord(e0, nullptr));
        for (int i = 0; i < iters; ++i)
            launch_gemm(at, dA.as<uint16_t>(), K, wptr(i + 3), K, M, N, K, e, nullptr);
        ACEMI_HIP(hipEventRecord(e1, nullptr));
        ACEMI_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        ACEMI_HIP(hipEventElapsedTime(&ms, e0, e1));
        *avg_ms = ms / iters;
        gemm_force_variant(-1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } catch (const std::exception& ex) {
        gemm_force_variant(-1);
        std::fprintf(stderr, "ace_mi_bench_gemm: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

}  // extern "C"

extern "C" {

// Staged dequant kernel on ggml block rows W [N][K]: out = bf16 bits of bf16(dequant(W)) [N][K].
ace_ggml_status ace_mi_kernel_dequant(int32_t qtype, int32_t N, int32_t K, const uint8_t* W_blocks, uint16_t* out) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (!W_blocks || !out || N <= 0 || K <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K) return ACE_GGML_ERR_INVALID_ARG;
    if (!quant::applies(t, K)) return ACE_GGML_ERR_INVALID_ARG;
    try {
        std::vector<uint8_t> qp(quant::q_plane_bytes(t, N, K));
        std::vector<float> sp(quant::s_plane_floats(t, N, K));
        quant::to_planes(t, W_blocks, N, K, qp.data(), sp.data());
        DevMem dq(qp.size()), ds(sp.size() * 4), dout((size_t)N * K * 2);
        ACEMI_HIP(hipMemcpy(dq.p, qp.data(), qp.size(), hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(ds.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice));
        WeightView w;
        w.fmt = t == quant::Q8_0 ? WF_Q8_0 : t == quant::Q4_K ? WF_Q4_K : WF_Q6_K;
        w.q = dq.p;
        w.s = ds.as<float>();
        launch_dequant_bf16(w, N, K, dout.as<uint16_t>(), nullptr);
        ACEMI_HIP(hipDeviceSynchronize());
        ACEMI_HIP(hipMemcpy(out, dout.p, (size_t)N * K * 2, hipMemcpyDeviceToHost));
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "ace_mi_kernel_dequant: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

// Dequant-fused GEMM on ggml block rows W [N][K]: out = A(bf16) . bf16(dequant(W))^T (+ bias).
ace_ggml_status ace_mi_kernel_gemm_q(int32_t qtype, int32_t epi, int32_t variant, int32_t M, int32_t N, int32_t K,
                                     const uint16_t* A, const uint8_t* W_blocks, const float* bias, float* out_f32,
                                     uint16_t* out_u16) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (!A || !W_blocks || M <= 0 || N % 128 != 0 || K % 64 != 0) return ACE_GGML_ERR_INVALID_ARG;
    if (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K) return ACE_GGML_ERR_INVALID_ARG;
    if (!quant::applies(t, K)) return ACE_GGML_ERR_INVALID_ARG;
    const bool resid = epi == EPI_RESID || epi == EPI_RESID_GATED;
    if (epi != EPI_STORE_F32 && epi != EPI_SWIGLU && !resid) return ACE_GGML_ERR_UNSUPPORTED;
    if (((epi == EPI_STORE_F32 || resid) && !out_f32) || (epi == EPI_SWIGLU && !out_u16))
        return ACE_GGML_ERR_INVALID_ARG;
    if (epi == EPI_RESID_GATED && !bias) return ACE_GGML_ERR_INVALID_ARG;
    const int vb = variant >= 0 ? (variant & 0xffff) : variant;  // (0x10000: forced past the picker's support check)
    if (variant < -1 || variant > 0x1ffff || vb % 100 > 25 || vb > 424) return ACE_GGML_ERR_INVALID_ARG;
    try {
        std::vector<uint8_t> qp(quant::q_plane_bytes(t, N, K));
        std::vector<float> sp(quant::s_plane_floats(t, N, K));
        quant::to_planes(t, W_blocks, N, K, qp.data(), sp.data());
        DevMem dA((size_t)M * K * 2), dQ(qp.size()), dS(sp.size() * 4), dB((size_t)N * 4), dC((size_t)M * N * 4);
        ACEMI_HIP(hipMemcpy(dA.p, A, (size_t)M * K * 2, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dQ.p, qp.data(), qp.size(), hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dS.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice));
        if (bias) ACEMI_HIP(hipMemcpy(dB.p, bias, (size_t)N * 4, hipMemcpyHostToDevice));
        GemmEpilogue e;
        e.kind = epi;
        e.bias = bias && !resid ? dB.as<float>() : nullptr;
        if (resid) {  // out_f32 holds x on entry: x += acc (* gate[n], the gate passed as `bias`)
            ACEMI_HIP(hipMemcpy(dC.p, out_f32, (size_t)M * N * 4, hipMemcpyHostToDevice));
            e.c_f32 = dC.as<float>();
            e.ldc = N;
            e.gate = epi == EPI_RESID_GATED ? dB.as<float>() : nullptr;
            e.gate_stride = 0;
            e.rows_per_item = M;
        } else if (epi == EPI_STORE_F32) {
            e.c_f32 = dC.as<float>();
            e.ldc = N;
        } else {
            e.c_act = dC.as<uint16_t>();
            e.ldc = N / 2;
        }
        WeightView w;
        w.fmt = t == quant::Q8_0 ? WF_Q8_0 : (t == quant::Q4_K ? WF_Q4_K : WF_Q6_K);
        w.q = dQ.p;
        w.s = dS.as<float>();
        gemm_force_variant(variant);
        launch_gemm(dA.as<uint16_t>(), K, w, M, N, K, e, nullptr);
        gemm_force_variant(-1);
        ACEMI_HIP(hipDeviceSynchronize());
        if (epi == EPI_STORE_F32 || resid)
            ACEMI_HIP(hipMemcpy(out_f32, dC.p, (size_t)M * N * 4, hipMemcpyDeviceToHost));
        else
            ACEMI_HIP(hipMemcpy(out_u16, dC.p, (size_t)M * (N / 2) * 2, hipMemcpyDeviceToHost));
    } catch (const std::exception& ex) {
        gemm_force_variant(-1);
        std::fprintf(stderr, "ace_mi_kernel_gemm_q: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

// ggml-faithful quantized-activation GEMM (kernels/gemm_a8.hip): x f32 [M][K] -> Q8_0 / Q8_K blocks on the device
// (returned in q_out [M][K], s_out [K/32][M], bsum_out [K/32][M] when non-null), then the integer-dot GEMM against
// ggml block rows W [N][K] with epilogue epi: 0 f32 store (+ bias), 3 residual (out_f32 holds x on entry; + bias),
// 7 SwiGLU f32 (out [M][N/2], gate|up interleaved in 16-column groups).
ace_ggml_status ace_mi_kernel_gemm_a8(int32_t qtype, int32_t epi, int32_t M, int32_t N, int32_t K, const float* x,
                                      const uint8_t* W_blocks, const float* bias, float* out_f32, int8_t* q_out,
                                      float* s_out, float* bsum_out) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (!x || !W_blocks || !out_f32 || M <= 0 || N % 128 != 0) return ACE_GGML_ERR_INVALID_ARG;
    if (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K) return ACE_GGML_ERR_INVALID_ARG;
    if (!quant::applies(t, K)) return ACE_GGML_ERR_INVALID_ARG;
    if (epi != EPI_STORE_F32 && epi != EPI_RESID && epi != EPI_SWIGLU_F32) return ACE_GGML_ERR_UNSUPPORTED;
    try {
        const int64_t ld_s = (M + 127) / 128 * 128;
        const int nb = K / 32;
        const int ncol = epi == EPI_SWIGLU_F32 ? N / 2 : N;
        std::vector<uint8_t> qp(quant::q_plane_bytes(t, N, K));
        std::vector<float> sp(quant::s_plane_floats(t, N, K));
        quant::to_planes(t, W_blocks, N, K, qp.data(), sp.data());
        DevMem dX((size_t)M * K * 4), dQ(qp.size()), dS(sp.size() * 4), dB((size_t)N * 4), dC((size_t)M * ncol * 4),
            dAq((size_t)M * K), dAs((size_t)nb * ld_s * 4), dAb((size_t)nb * ld_s * 4);
        ACEMI_HIP(hipMemcpy(dX.p, x, (size_t)M * K * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dQ.p, qp.data(), qp.size(), hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dS.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemset(dAs.p, 0, (size_t)nb * ld_s * 4));
        ACEMI_HIP(hipMemset(dAb.p, 0, (size_t)nb * ld_s * 4));
        if (bias) ACEMI_HIP(hipMemcpy(dB.p, bias, (size_t)N * 4, hipMemcpyHostToDevice));
        if (epi == EPI_RESID) ACEMI_HIP(hipMemcpy(dC.p, out_f32, (size_t)M * N * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipDeviceSynchronize());
        QAct a;
        a.kind = t == quant::Q8_0 ? QACT_Q8_0 : QACT_Q8_K;
        a.q = dAq.as<int8_t>();
        a.s = dAs.as<float>();
        a.bsum = dAb.as<float>();
        a.ld_s = ld_s;
        // Q8_0 with K % 64 == 0 runs the bf16-MFMA form unless ace_mi_kernel_gemm_a8_mode(0) (or ACE_MI_QACT_GEMM=0)
        // keeps it on the i8 kernel: the int8 blocks are returned either way
        const bool bf16_path = gemm_a8_bf16_path(t == quant::Q8_0 ? WF_Q8_0 : WF_Q4_K, K);
        DevMem dA16(bf16_path ? (size_t)M * K * 2 : 16), dW16(bf16_path ? (size_t)N * K * 2 : 16);
        launch_quantize_act(a.kind, dX.as<float>(), K, M, K, false, dAq.as<int8_t>(), dAs.as<float>(), dAb.as<float>(),
                            ld_s, nullptr, bf16_path ? dA16.as<uint16_t>() : nullptr);
        if (bf16_path) {
            a.q16 = dA16.as<uint16_t>();
            launch_q8_image(dQ.as<int8_t>(), (int64_t)N * K, dW16.as<uint16_t>(), nullptr);
        }
        GemmEpilogue e;
        e.kind = epi;
        e.bias = bias ? dB.as<float>() : nullptr;
        e.c_f32 = dC.as<float>();
        e.ldc = ncol;
        WeightView w;
        w.fmt = t == quant::Q8_0 ? WF_Q8_0 : (t == quant::Q4_K ? WF_Q4_K : WF_Q6_K);
        w.q = dQ.p;
        w.s = dS.as<float>();
        launch_gemm_a8(a, w, M, N, K, e, nullptr, bf16_path ? dW16.as<uint16_t>() : nullptr);
        ACEMI_HIP(hipDeviceSynchronize());
        ACEMI_HIP(hipMemcpy(out_f32, dC.p, (size_t)M * ncol * 4, hipMemcpyDeviceToHost));
        if (q_out) ACEMI_HIP(hipMemcpy(q_out, dAq.p, (size_t)M * K, hipMemcpyDeviceToHost));
        for (int b = 0; b < nb; ++b) {
            if (s_out)
                ACEMI_HIP(hipMemcpy(s_out + (size_t)b * M, dAs.as<float>() + (size_t)b * ld_s, (size_t)M * 4,
                                    hipMemcpyDeviceToHost));
            if (bsum_out)
                ACEMI_HIP(hipMemcpy(bsum_out + (size_t)b * M, dAb.as<float>() + (size_t)b * ld_s, (size_t)M * 4,
                                    hipMemcpyDeviceToHost));
        }
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "ace_mi_kernel_gemm_a8: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

// Which form ace_mi_kernel_gemm_a8 (and the q8 mode of this process) runs a Q8_0 GEMM in: -1 the environment / default
// (the bf16 MFMA), 0 the i8 kernel, 1 the bf16 MFMA.
ace_ggml_status ace_mi_kernel_gemm_a8_mode(int32_t mode) {
    if (mode < -1 || mode > 1) return ACE_GGML_ERR_INVALID_ARG;
    acemi::gemm_a8_mode(mode);
    return ACE_GGML_OK;
}

// Which kernel runs f8c attention in this process: -1 the environment / default policy, 0 attn2, 1 attn_kh_kernel.
ace_ggml_status ace_mi_kernel_attn_kh(int32_t mode) {
    if (mode < -1 || mode > 1) return ACE_GGML_ERR_INVALID_ARG;
    acemi::attn_kh_mode(mode);
    return ACE_GGML_OK;
}

// Dequant-fused GEMM micro-benchmark (random N(0, 0.02) weights quantized with the loader's encoder).
ace_ggml_status ace_mi_bench_gemm_q(int32_t qtype, int32_t epi, int32_t variant, int32_t M, int32_t N, int32_t K,
                                    int32_t iters, float* avg_ms) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (M <= 0 || N % 128 != 0 || K % 64 != 0 || iters <= 0 || !avg_ms) return ACE_GGML_ERR_INVALID_ARG;
    if (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K) return ACE_GGML_ERR_INVALID_ARG;
    if (!quant::applies(t, K)) return ACE_GGML_ERR_INVALID_ARG;
    try {
        uint32_t st = 777u;
        auto rnd = [&]() {
            st = st * 1664525u + 1013904223u;
            return ((float)(st >> 8) * (2.0f / 16777216.0f) - 1.0f);
        };
        std::vector<uint16_t> ha((size_t)M * K);
        for (auto& v : ha) {
            const float f = rnd();
            uint32_t u;
            std::memcpy(&u, &f, 4);
            v = (uint16_t)(u >> 16);
        }
        std::vector<float> hw((size_t)N * K);
        for (auto& v : hw) v = 0.02f * rnd();
        std::vector<uint8_t> blocks((size_t)N * quant::row_bytes(t, K));
        quant::quantize_rows(t, hw.data(), N, K, blocks.data());
        std::vector<uint8_t> qp(quant::q_plane_bytes(t, N, K));
        std::vector<float> sp(quant::s_plane_floats(t, N, K));
        quant::to_planes(t, blocks.data(), N, K, qp.data(), sp.data());
        DevMem dA(ha.size() * 2), dQ(qp.size()), dS(sp.size() * 4), dC((size_t)M * N * 4), dG((size_t)N * 4);
        ACEMI_HIP(hipMemcpy(dA.p, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dQ.p, qp.data(), qp.size(), hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(dS.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemset(dC.p, 0, (size_t)M * N * 4));
        ACEMI_HIP(hipMemset(dG.p, 0, (size_t)N * 4));
        GemmEpilogue e;
        e.kind = epi;
        e.ldc = (epi == EPI_SWIGLU) ? N / 2 : N;
        e.c_f32 = dC.as<float>();
        e.c_act = dC.as<uint16_t>();
        e.gate = dG.as<float>();
        e.rows_per_item = M;
        WeightView w;
        w.fmt = t == quant::Q8_0 ? WF_Q8_0 : (t == quant::Q4_K ? WF_Q4_K : WF_Q6_K);
        w.q = dQ.p;
        w.s = dS.as<float>();
        gemm_force_variant(variant);
        hipEvent_t e0, e1;
        ACEMI_HIP(hipEventCreate(&e0));
        ACEMI_HIP(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i) launch_gemm(dA.as<uint16_t>(), K, w, M, N, K, e, nullptr);
        ACEMI_HIP(hipEventRecord(e0, nullptr));
        for (int i = 0; i < iters; ++i) launch_gemm(dA.as<uint16_t>(), K, w, M, N, K, e, nullptr);
        ACEMI_HIP(hipEventRecord(e1, nullptr));
        ACEMI_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        ACEMI_HIP(hipEventElapsedTime(&ms, e0, e1));
        *avg_ms = ms / iters;
        gemm_force_variant(-1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } catch (const std::exception& ex) {
        gemm_force_variant(-1);
        std::fprintf(stderr, "ace_mi_bench_gemm_q: %s\n", ex.what());
        return ACE_GGML_ERR;
    }
    return ACE_GGML_OK;
}

}  // extern "C"
