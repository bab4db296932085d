// C++/OpenMP restatement of the acestep_ggml CPU DiT forward -- TEST / BENCH INFRASTRUCTURE ONLY
// (see oracle/__init__.py): the `cpu_baseline` of bench.py times it, tests/test_cpu_restatement.py checks
// it against the numpy oracle.  Never linked into or called by the product.
//
// It computes the graph of ace_dit::forward_dit (acestep_ggml/cpp/acestep_dit_model.cpp:1316-1560) with
// ggml-cpu's precision rules, the way ggml's CPU backend does it, because ggml itself cannot be built
// here (empty third_party/ggml submodule):
//   * ggml_mul_mat (:1194-1196, 1257, 1381, 1412, 1528-1531, 1551): the f32 activation is converted to
//     the weight's vec_dot_type (BF16 -> bf16 round-to-nearest-even, F16 -> fp16) and dotted with the
//     weight in f32; on CPUs with AVX512-BF16 the bf16 dot is vdpbf16ps (as ggml_vec_dot_bf16), F16
//     weights are widened with vcvtph2ps and FMA'd (as ggml_vec_dot_f16), else plain f32 loops;
//   * ggml_rms_norm (:1097-1106): sum of squares in double, scale = 1/sqrtf(mean + eps), then * w;
//   * attention (:1212-1256) in f32 with the GQA head map h -> h / n_rep, key-padding / sliding-window
//     masks, softmax with the row max -- streamed over key blocks (online softmax) instead of ggml's
//     materialised [16][N][N] f32 scores, which at 240 s would need ~70 GB of arena; the streamed form
//     does the same arithmetic work and no more, so its time is a lower bound on ggml's;
//   * everything else (AdaLN modulation, gates, residuals, SiLU, RoPE NEOX with ggml's f32 running
//     theta product, timestep sinusoids) in f32.
// Threads: OpenMP over output tiles / heads (OMP_NUM_THREADS, default every host core).
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

enum WType { WT_BF16 = 0, WT_F16 = 1 };

inline uint16_t bf16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
inline float bf16_f32(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
inline uint16_t f16_rne(float f) { return _cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT); }
inline float f16_f32(uint16_t h) { return _cvtsh_ss(h); }

// A weight matrix [N][K] (row-major, K contiguous) re-laid for the SIMD dot products:
//   bf16: per block of 16 rows, per k pair: 16 rows x {k, k+1}  (vdpbf16ps operand order)
//   f16:  per block of 16 rows, per k: 16 rows                  (vcvtph2ps operand order)
// plus the plain copy for the scalar path.  N % 16 == 0 and K % 2 == 0 for every DiT weight.
struct Mat {
    int N = 0, K = 0, type = WT_BF16;
    std::vector<uint16_t> plain, packed;
};

void pack(Mat& m) {
    const int nb = m.N / 16;
    m.packed.assign((size_t)m.N * m.K, 0);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nb; ++b)
        for (int k = 0; k < m.K; ++k)
            for (int r = 0; r < 16; ++r) {
                const uint16_t v = m.plain[(size_t)(b * 16 + r) * m.K + k];
                size_t dst;
                if (m.type == WT_BF16)
                    dst = (size_t)b * 16 * m.K + (size_t)(k / 2) * 32 + r * 2 + (k & 1);
                else
                    dst = (size_t)b * 16 * m.K + (size_t)k * 16 + r;
                m.packed[dst] = v;
            }
}

// ----------------------------------------------------------------- GEMM: y[M][N] (+)= act(x) . W^T
// x activations already converted to the weight's type (16-bit), [M][K].

// Register-blocked micro-kernel: MR = 6 rows x NB = 4 blocks of 16 columns = 24 zmm accumulators; per k
// step 4 weight loads + 6 broadcasts feed 24 dot instructions.  Tasks = (64-column panel, 96-row band):
// the panel's weights (64 x K x 2 B <= 768 KiB) stay in the core's L2 across the band.
__attribute__((target("avx512f,avx512bw,avx512vl,avx512bf16"))) void micro_bf16(const uint16_t* x, int K, const Mat& w,
                                                                               float* y, int N, int m0, int mr,
                                                                               int bb0, int nbb) {
    constexpr int MR = 6, NB = 4;
    __m512 acc[MR][NB];
    for (int i = 0; i < MR; ++i)
        for (int j = 0; j < NB; ++j) acc[i][j] = _mm512_setzero_ps();
    const uint16_t* wp[NB];
    for (int j = 0; j < NB; ++j) wp[j] = w.packed.data() + (size_t)(bb0 + std::min(j, nbb - 1)) * 16 * K;
    const uint16_t* xr[MR];
    for (int i = 0; i < MR; ++i) xr[i] = x + (size_t)(m0 + std::min(i, mr - 1)) * K;
    for (int k2 = 0; k2 < K / 2; ++k2) {
        __m512bh b[NB];
        for (int j = 0; j < NB; ++j) b[j] = (__m512bh)_mm512_loadu_si512((const void*)(wp[j] + (size_t)k2 * 32));
        for (int i = 0; i < MR; ++i) {
            // vbroadcastss from memory: a load-port op (a broadcast from a GPR would queue on port 5
            // beside the dot products)
            const __m512bh a = (__m512bh)_mm512_castps_si512(_mm512_set1_ps(*(const float*)(xr[i] + 2 * k2)));
            for (int j = 0; j < NB; ++j) acc[i][j] = _mm512_dpbf16_ps(acc[i][j], a, b[j]);
        }
    }
    for (int i = 0; i < mr; ++i)
        for (int j = 0; j < nbb; ++j) _mm512_storeu_ps(y + (size_t)(m0 + i) * N + (bb0 + j) * 16, acc[i][j]);
}

__attribute__((target("avx512f,avx512bw,avx512vl,f16c"))) void micro_f16(const uint16_t* x, int K, const Mat& w,
                                                                        float* y, int N, int m0, int mr, int bb0,
                                                                        int nbb) {
    constexpr int MR = 6, NB = 4;
    __m512 acc[MR][NB];
    for (int i = 0; i < MR; ++i)
        for (int j = 0; j < NB; ++j) acc[i][j] = _mm512_setzero_ps();
    const uint16_t* wp[NB];
    for (int j = 0; j < NB; ++j) wp[j] = w.packed.data() + (size_t)(bb0 + std::min(j, nbb - 1)) * 16 * K;
    const uint16_t* xr[MR];
    for (int i = 0; i < MR; ++i) xr[i] = x + (size_t)(m0 + std::min(i, mr - 1)) * K;
    for (int k = 0; k < K; ++k) {
        __m512 b[NB];
        for (int j = 0; j < NB; ++j) b[j] = _mm512_cvtph_ps(_mm256_loadu_si256((const __m256i*)(wp[j] + (size_t)k * 16)));
        for (int i = 0; i < MR; ++i) {
            const __m512 a = _mm512_set1_ps(_cvtsh_ss(xr[i][k]));
            for (int j = 0; j < NB; ++j) acc[i][j] = _mm512_fmadd_ps(a, b[j], acc[i][j]);
        }
    }
    for (int i = 0; i < mr; ++i)
        for (int j = 0; j < nbb; ++j) _mm512_storeu_ps(y + (size_t)(m0 + i) * N + (bb0 + j) * 16, acc[i][j]);
}

void gemm_avx512(const uint16_t* x, int M, const Mat& w, float* y, bool bf) {
    const int K = w.K, N = w.N, nb = N / 16;
    constexpr int MR = 6, NB = 4, BAND = 96;
    const int npanels = (nb + NB - 1) / NB, nbands = (M + BAND - 1) / BAND;
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int pn = 0; pn < npanels; ++pn)
        for (int band = 0; band < nbands; ++band) {
            const int bb0 = pn * NB, nbb = std::min(NB, nb - bb0);
            const int m_end = std::min(M, (band + 1) * BAND);
            for (int m0 = band * BAND; m0 < m_end; m0 += MR) {
                const int mr = std::min(MR, m_end - m0);
                if (bf)
                    micro_bf16(x, K, w, y, N, m0, mr, bb0, nbb);
                else
                    micro_f16(x, K, w, y, N, m0, mr, bb0, nbb);
            }
        }
}

void gemm_scalar(const uint16_t* x, int M, const Mat& w, float* y) {
    const int K = w.K, N = w.N;
    const bool bf = w.type == WT_BF16;
#pragma omp parallel
    {
        std::vector<float> xr((size_t)K), wr((size_t)K);
#pragma omp for schedule(static)
        for (int m = 0; m < M; ++m) {
            for (int k = 0; k < K; ++k) xr[k] = bf ? bf16_f32(x[(size_t)m * K + k]) : f16_f32(x[(size_t)m * K + k]);
            for (int n = 0; n < N; ++n) {
                const uint16_t* wrow = w.plain.data() + (size_t)n * K;
                float s = 0.f;
                for (int k = 0; k < K; ++k) s += xr[k] * (bf ? bf16_f32(wrow[k]) : f16_f32(wrow[k]));
                y[(size_t)m * N + n] = s;
            }
        }
    }
}

int g_isa = -1;  // 2 avx512 (+bf16), 1 avx512 without bf16, 0 scalar
int isa() {
    if (g_isa < 0) {
        __builtin_cpu_init();
        const bool f = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                       __builtin_cpu_supports("avx512vl");
        g_isa = f ? (__builtin_cpu_supports("avx512bf16") ? 2 : 1) : 0;
    }
    return g_isa;
}

// y[M][N] = mul_mat(W, x) (+ bias): x f32 [M][K] -> the weight's vec_dot_type -> dot in f32
void mul_mat(const Mat& w, const float* x, int M, const float* bias, float* y) {
    const int K = w.K;
    std::vector<uint16_t> xa((size_t)M * K);
    const bool bf = w.type == WT_BF16;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)M * K; ++i) xa[i] = bf ? bf16_rne(x[i]) : f16_rne(x[i]);
    if ((bf && isa() == 2) || (!bf && isa() >= 1))
        gemm_avx512(xa.data(), M, w, y, bf);
    else
        gemm_scalar(xa.data(), M, w, y);
    if (bias) {
#pragma omp parallel for schedule(static)
        for (int m = 0; m < M; ++m)
            for (int n = 0; n < w.N; ++n) y[(size_t)m * w.N + n] += bias[n];
    }
}

void rms_norm(const float* x, int M, int H, const float* w, float eps, float* y) {
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; ++m) {
        const float* r = x + (size_t)m * H;
        double ss = 0.0;
        for (int i = 0; i < H; ++i) ss += (double)(r[i] * r[i]);
        const float mean = (float)(ss / H);
        const float sc = 1.0f / sqrtf(mean + eps);
        for (int i = 0; i < H; ++i) {
            float v = r[i] * sc;
            y[(size_t)m * H + i] = w ? v * w[i] : v;
        }
    }
}

inline float silu(float v) { return v / (1.0f + expf(-v)); }

// ----------------------------------------------------------------- model
enum MatId { M_PROJ_IN = 0, M_COND, M_PROJ_OUT, M_TE_W1, M_TE_W2, M_TE_WP,  // TE: layer = 0 (t) / 1 (t - r)
             M_SQ, M_SK, M_SV, M_SO, M_CQ, M_CK, M_CV, M_CO, M_GATE, M_UP, M_DOWN, M_COUNT };
enum VecId { V_PROJ_IN_B = 0, V_COND_B, V_PROJ_OUT_B, V_NORM_OUT, V_OUT_TABLE, V_TE_B1, V_TE_B2, V_TE_BP,
             V_SA_NORM, V_CA_NORM, V_MLP_NORM, V_SQN, V_SKN, V_CQN, V_CKN, V_TABLE, V_COUNT };

struct Layer {
    Mat m[M_COUNT];
    std::vector<float> v[V_COUNT];
    bool sliding = false;
};

struct Model {
    int H, I, n_layers, hq, hkv, D, P, in_ch, audio, window;
    float eps, theta;
    Mat top[M_COUNT];
    std::vector<float> topv[V_COUNT];
    Mat te[2][3];
    std::vector<float> tev[2][3];
    std::vector<Layer> layers;
};

// f32 attention, streamed over key blocks: q [nq][hq*D], k/v [nk][hkv*D] -> out [nq][hq*D]
void attention_core(const Model& md, const float* q, const float* k, const float* v, int nq, int nk,
                    const int* key_ok, bool sliding, float* out) {
    const int D = md.D, hq = md.hq, rep = md.hq / md.hkv;
    const float scale = 1.0f / sqrtf((float)D);
    constexpr int QB = 16, KB = 64;
    const int nqb = (nq + QB - 1) / QB;
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int h = 0; h < hq; ++h)
        for (int qb = 0; qb < nqb; ++qb) {
            const int hk = h / rep;
            const int q0 = qb * QB, qn = std::min(QB, nq - q0);
            float o[QB][128], mrow[QB], lrow[QB], s[QB][KB];
            for (int i = 0; i < QB; ++i) {
                mrow[i] = -INFINITY;
                lrow[i] = 0.f;
                for (int d = 0; d < D; ++d) o[i][d] = 0.f;
            }
            int klo = 0, khi = nk;
            if (sliding) {
                klo = std::max(0, q0 - md.window);
                khi = std::min(nk, q0 + qn - 1 + md.window + 1);
            }
            for (int k0 = klo; k0 < khi; k0 += KB) {
                const int kn = std::min(KB, khi - k0);
                for (int i = 0; i < qn; ++i) {
                    const float* qr = q + (size_t)(q0 + i) * hq * D + h * D;
                    float mx = -INFINITY;
                    for (int j = 0; j < kn; ++j) {
                        const int kk = k0 + j;
                        const bool ok = (!key_ok || key_ok[kk]) && (!sliding || std::abs((q0 + i) - kk) <= md.window);
                        float dot = 0.f;
                        if (ok) {
                            const float* kr = k + (size_t)kk * md.hkv * D + hk * D;
#pragma omp simd reduction(+ : dot)
                            for (int d = 0; d < D; ++d) dot += qr[d] * kr[d];
                        }
                        s[i][j] = ok ? dot * scale : -INFINITY;
                        mx = std::max(mx, s[i][j]);
                    }
                    const float mnew = std::max(mrow[i], mx);
                    const float alpha = (mrow[i] == -INFINITY) ? 0.f : expf(mrow[i] - mnew);
                    float l = lrow[i] * alpha;
                    for (int d = 0; d < D; ++d) o[i][d] *= alpha;
                    for (int j = 0; j < kn; ++j) {
                        const float p = (mnew == -INFINITY) ? 0.f : expf(s[i][j] - mnew);
                        l += p;
                        if (p == 0.f) continue;
                        const float* vr = v + (size_t)(k0 + j) * md.hkv * D + hk * D;
#pragma omp simd
                        for (int d = 0; d < D; ++d) o[i][d] += p * vr[d];
                    }
                    mrow[i] = mnew;
                    lrow[i] = l;
                }
            }
            for (int i = 0; i < qn; ++i) {
                const float inv = 1.0f / lrow[i];  // an all-masked row: 0/0 = NaN, as ggml's soft_max
                float* orow = out + (size_t)(q0 + i) * hq * D + h * D;
                for (int d = 0; d < D; ++d) orow[d] = o[i][d] * inv;
            }
        }
}

void head_norm_rope(float* x, int n, int heads, int D, const float* w, float eps, const float* cs, const float* sn) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t < n; ++t)
        for (int h = 0; h < heads; ++h) {
            float* r = x + ((size_t)t * heads + h) * D;
            double ss = 0.0;
            for (int i = 0; i < D; ++i) ss += (double)(r[i] * r[i]);
            const float sc = 1.0f / sqrtf((float)(ss / D) + eps);
            for (int i = 0; i < D; ++i) r[i] = r[i] * sc * w[i];
            if (cs) {
                const int half = D / 2;
                for (int i = 0; i < half; ++i) {
                    const float c = cs[(size_t)t * half + i], s = sn[(size_t)t * half + i];
                    const float a = r[i], b = r[half + i];
                    r[i] = a * c - b * s;
                    r[half + i] = a * s + b * c;
                }
            }
        }
}

// attention() (:1175-1259): projections, QK-norm, RoPE (self only), core, o_proj
void attention_block(const Model& md, const Layer& ly, bool cross, const float* xq, int nq, const float* xkv, int nk,
                     const int* key_ok, const float* cs, const float* sn, float* out) {
    const int D = md.D;
    const Mat& Wq = ly.m[cross ? M_CQ : M_SQ];
    const Mat& Wk = ly.m[cross ? M_CK : M_SK];
    const Mat& Wv = ly.m[cross ? M_CV : M_SV];
    const Mat& Wo = ly.m[cross ? M_CO : M_SO];
    std::vector<float> q((size_t)nq * md.hq * D), k((size_t)nk * md.hkv * D), v((size_t)nk * md.hkv * D),
        a((size_t)nq * md.hq * D);
    mul_mat(Wq, xq, nq, nullptr, q.data());
    mul_mat(Wk, xkv, nk, nullptr, k.data());
    mul_mat(Wv, xkv, nk, nullptr, v.data());
    head_norm_rope(q.data(), nq, md.hq, D, ly.v[cross ? V_CQN : V_SQN].data(), md.eps, cs, sn);
    head_norm_rope(k.data(), nk, md.hkv, D, ly.v[cross ? V_CKN : V_SKN].data(), md.eps, cs, sn);
    attention_core(md, q.data(), k.data(), v.data(), nq, nk, key_ok, !cross && ly.sliding, a.data());
    mul_mat(Wo, a.data(), nq, nullptr, out);
}

void timestep_forward(const Model& md, int e, float t, float* temb, float* proj) {
    const int H = md.H;
    float f[256];
    const int half = 128;
    const float t_scaled = t * 1000.0f;
    const float log_max = logf(10000.0f);
    for (int i = 0; i < half; ++i) {
        const float ex = expf((-log_max) * (float)i / (float)half);
        const float arg = t_scaled * ex;
        f[i] = cosf(arg);
        f[half + i] = sinf(arg);
    }
    std::vector<float> h((size_t)H), st((size_t)H);
    mul_mat(md.te[e][0], f, 1, md.tev[e][0].data(), h.data());
    for (int i = 0; i < H; ++i) h[i] = silu(h[i]);
    mul_mat(md.te[e][1], h.data(), 1, md.tev[e][1].data(), temb);
    for (int i = 0; i < H; ++i) st[i] = silu(temb[i]);
    mul_mat(md.te[e][2], st.data(), 1, md.tev[e][2].data(), proj);
}

}  // namespace

extern "C" {

void* dcpu_create(int H, int I, int n_layers, int hq, int hkv, int D, int P, int in_ch, int audio, int window,
                  float eps, float theta, const int32_t* sliding) {
    auto* m = new Model();
    m->H = H, m->I = I, m->n_layers = n_layers, m->hq = hq, m->hkv = hkv, m->D = D, m->P = P, m->in_ch = in_ch;
    m->audio = audio, m->window = window, m->eps = eps, m->theta = theta;
    m->layers.resize(n_layers);
    for (int i = 0; i < n_layers; ++i) m->layers[i].sliding = sliding[i] != 0;
    return m;
}

void dcpu_destroy(void* h) { delete static_cast<Model*>(h); }

// 16-bit weight matrix [rows][cols] (bf16 or fp16 bits).  layer < 0: a top-level matrix; for the
// timestep MLPs (M_TE_*) `layer` selects time_embed (0) or time_embed_r (1).
int dcpu_matrix(void* h, int id, int layer, int type, const uint16_t* data, int rows, int cols) {
    auto* md = static_cast<Model*>(h);
    Mat* m;
    if (id >= M_TE_W1 && id <= M_TE_WP)
        m = &md->te[layer][id - M_TE_W1];
    else if (layer < 0)
        m = &md->top[id];
    else
        m = &md->layers[layer].m[id];
    if (rows % 16 || cols % 2) return -1;
    m->N = rows, m->K = cols, m->type = type;
    m->plain.assign(data, data + (size_t)rows * cols);
    pack(*m);
    return 0;
}

int dcpu_vector(void* h, int id, int layer, const float* data, int n) {
    auto* md = static_cast<Model*>(h);
    std::vector<float>* v;
    if (id >= V_TE_B1 && id <= V_TE_BP)
        v = &md->tev[layer][id - V_TE_B1];
    else if (layer < 0)
        v = &md->topv[id];
    else
        v = &md->layers[layer].v[id];
    v->assign(data, data + n);
    return 0;
}

int dcpu_isa() { return isa(); }

// diagnostics: seconds per y = mul_mat(W, x) of a random [M][K] x [N][K] problem (type 0 bf16, 1 f16)
double dcpu_bench_mul_mat(int M, int N, int K, int type, int iters) {
    Mat w;
    w.N = N, w.K = K, w.type = type;
    w.plain.resize((size_t)N * K);
    for (size_t i = 0; i < w.plain.size(); ++i) w.plain[i] = type == WT_BF16 ? bf16_rne(0.01f * (float)(i % 97)) : f16_rne(0.01f * (float)(i % 97));
    pack(w);
    std::vector<float> x((size_t)M * K, 0.5f), y((size_t)M * N);
    mul_mat(w, x.data(), M, nullptr, y.data());
    const double t0 = omp_get_wtime();
    for (int i = 0; i < iters; ++i) mul_mat(w, x.data(), M, nullptr, y.data());
    return (omp_get_wtime() - t0) / iters;
}

// forward_dit for one sample: hidden [T][audio], context [T][in_ch - audio], enc [L][H] (L may be 0),
// masks int32 or null -> out [T][audio]
int dcpu_forward(void* h, const float* hidden, const float* context, const float* enc, const int32_t* mask,
                 const int32_t* enc_mask, int T, int L, float t, float r, int max_layers, float* out) {
    const Model& md = *static_cast<Model*>(h);
    const int H = md.H, P = md.P, audio = md.audio, ctx_dim = md.in_ch - md.audio, D = md.D;
    const int Tp = T + (P - T % P) % P, Np = Tp / P;
    // input pack, context first (:1350-1382)
    std::vector<float> x0((size_t)Tp * md.in_ch, 0.f);
    for (int tt = 0; tt < T; ++tt) {
        if (context) std::memcpy(&x0[(size_t)tt * md.in_ch], context + (size_t)tt * ctx_dim, ctx_dim * 4);
        if (hidden) std::memcpy(&x0[(size_t)tt * md.in_ch + ctx_dim], hidden + (size_t)tt * audio, audio * 4);
    }
    std::vector<float> x((size_t)Np * H);
    mul_mat(md.top[M_PROJ_IN], x0.data(), Np, md.topv[V_PROJ_IN_B].data(), x.data());
    std::vector<float> encp;
    if (L > 0) {  // condition embedder (:1384-1414)
        encp.resize((size_t)L * H);
        mul_mat(md.top[M_COND], enc, L, md.topv[V_COND_B].data(), encp.data());
    }
    // timestep embeddings (:1416-1424)
    std::vector<float> temb_t(H), temb_r(H), proj_t((size_t)6 * H), proj_r((size_t)6 * H);
    timestep_forward(md, 0, t, temb_t.data(), proj_t.data());
    timestep_forward(md, 1, t - r, temb_r.data(), proj_r.data());
    std::vector<float> temb(H), proj((size_t)6 * H);
    for (int i = 0; i < H; ++i) temb[i] = temb_t[i] + temb_r[i];
    for (int i = 0; i < 6 * H; ++i) proj[i] = proj_t[i] + proj_r[i];
    // patch key mask (:1433-1449)
    std::vector<int> pm;
    if (mask) {
        pm.assign(Np, 0);
        for (int p = 0; p < Np; ++p)
            for (int k = 0; k < P; ++k) {
                const int idx = p * P + k;
                if (idx < T && mask[idx] != 0) {
                    pm[p] = 1;
                    break;
                }
            }
    }
    std::vector<int> em;
    if (enc_mask && L > 0) em.assign(enc_mask, enc_mask + L);
    // RoPE tables: theta_i = p * theta_scale^i as ggml's f32 running product
    const int half = D / 2;
    std::vector<float> cs((size_t)Np * half), sn((size_t)Np * half);
    const float theta_scale = powf(md.theta, -2.0f / (float)D);
    for (int p = 0; p < Np; ++p) {
        float th = (float)p;
        for (int i = 0; i < half; ++i) {
            cs[(size_t)p * half + i] = cosf(th);
            sn[(size_t)p * half + i] = sinf(th);
            th *= theta_scale;
        }
    }
    const int n_layers = max_layers > 0 ? std::min(md.n_layers, max_layers) : md.n_layers;
    std::vector<float> nrm((size_t)Np * H), a((size_t)Np * H), g((size_t)Np * md.I), u((size_t)Np * md.I);
    for (int li = 0; li < n_layers; ++li) {  // :1466-1535
        const Layer& ly = md.layers[li];
        std::vector<float> mod((size_t)6 * H);
        for (int i = 0; i < 6 * H; ++i) mod[i] = ly.v[V_TABLE][i] + proj[i];
        const float *shift_msa = &mod[0], *scale_msa = &mod[H], *gate_msa = &mod[2 * H];
        const float *c_shift = &mod[3 * H], *c_scale = &mod[4 * H], *c_gate = &mod[5 * H];
        rms_norm(x.data(), Np, H, ly.v[V_SA_NORM].data(), md.eps, nrm.data());
#pragma omp parallel for schedule(static)
        for (int m = 0; m < Np; ++m)
            for (int i = 0; i < H; ++i) nrm[(size_t)m * H + i] = nrm[(size_t)m * H + i] * (scale_msa[i] + 1.0f) + shift_msa[i];
        attention_block(md, ly, false, nrm.data(), Np, nrm.data(), Np, pm.empty() ? nullptr : pm.data(), cs.data(),
                        sn.data(), a.data());
#pragma omp parallel for schedule(static)
        for (int m = 0; m < Np; ++m)
            for (int i = 0; i < H; ++i) x[(size_t)m * H + i] += a[(size_t)m * H + i] * gate_msa[i];
        if (L > 0) {  // cross-attention: no AdaLN, gate or RoPE (:1502-1520)
            rms_norm(x.data(), Np, H, ly.v[V_CA_NORM].data(), md.eps, nrm.data());
            attention_block(md, ly, true, nrm.data(), Np, encp.data(), L, em.empty() ? nullptr : em.data(), nullptr,
                            nullptr, a.data());
#pragma omp parallel for schedule(static)
            for (int64_t i = 0; i < (int64_t)Np * H; ++i) x[i] += a[i];
        }
        rms_norm(x.data(), Np, H, ly.v[V_MLP_NORM].data(), md.eps, nrm.data());
#pragma omp parallel for schedule(static)
        for (int m = 0; m < Np; ++m)
            for (int i = 0; i < H; ++i) nrm[(size_t)m * H + i] = nrm[(size_t)m * H + i] * (c_scale[i] + 1.0f) + c_shift[i];
        mul_mat(ly.m[M_GATE], nrm.data(), Np, nullptr, g.data());
        mul_mat(ly.m[M_UP], nrm.data(), Np, nullptr, u.data());
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)Np * md.I; ++i) g[i] = silu(g[i]) * u[i];
        mul_mat(ly.m[M_DOWN], g.data(), Np, nullptr, a.data());
#pragma omp parallel for schedule(static)
        for (int m = 0; m < Np; ++m)
            for (int i = 0; i < H; ++i) x[(size_t)m * H + i] += a[(size_t)m * H + i] * c_gate[i];
    }
    // output head (:1537-1559)
    const float* ot = md.topv[V_OUT_TABLE].data();
    rms_norm(x.data(), Np, H, md.topv[V_NORM_OUT].data(), md.eps, nrm.data());
#pragma omp parallel for schedule(static)
    for (int m = 0; m < Np; ++m)
        for (int i = 0; i < H; ++i) {
            const float shift = ot[i] + temb[i], scale = ot[H + i] + temb[i];
            nrm[(size_t)m * H + i] = nrm[(size_t)m * H + i] * (scale + 1.0f) + shift;
        }
    std::vector<float> y((size_t)Np * P * audio);
    mul_mat(md.top[M_PROJ_OUT], nrm.data(), Np, nullptr, y.data());
    const float* pb = md.topv[V_PROJ_OUT_B].data();
    for (int tt = 0; tt < T; ++tt)
        for (int c = 0; c < audio; ++c) out[(size_t)tt * audio + c] = y[(size_t)tt * audio + c] + pb[c];
    return 0;
}

}  // extern "C"
