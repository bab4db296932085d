// ggml block quantizers for the DiT weights (see quant.h).  Compiled with
// -ffp-contract=off: every float expression rounds where ggml's scalar C does.
#include "quant.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

namespace acemi {
namespace quant {
namespace {

constexpr int QK8_0 = 32;
constexpr int QK_K = 256;
constexpr float GROUP_MAX_EPS = 1e-15f;

inline uint16_t fp32_to_fp16(float f) {  // GGML_FP32_TO_FP16 (F16C, round to nearest even)
    _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}
inline float fp16_to_fp32(uint16_t u) {
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (float)h;
}
inline int nearest_int(float fval) {  // ggml: magic-constant round-half-even
    float val = fval + 12582912.f;
    int i;
    std::memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

// ---------------------------------------------------------------- Q8_0
// quantize_row_q8_0_ref: d = amax/127, q = roundf(x * (1/d)) (half away from zero)
void q8_0_row(const float* x, int64_t k, uint8_t* y) {
    for (int64_t i = 0; i < k / QK8_0; ++i) {
        const float* xb = x + i * QK8_0;
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; ++j) amax = std::max(amax, std::fabs(xb[j]));
        const float d = amax / 127.0f;
        const float id = d ? 1.0f / d : 0.0f;
        uint8_t* blk = y + i * 34;
        const uint16_t dh = fp32_to_fp16(d);
        std::memcpy(blk, &dh, 2);
        for (int j = 0; j < QK8_0; ++j) {
            const float x0 = xb[j] * id;
            blk[2 + j] = (uint8_t)(int8_t)std::roundf(x0);
        }
    }
}

void q8_0_deq(const uint8_t* y, int64_t k, float* x) {
    for (int64_t i = 0; i < k / QK8_0; ++i) {
        const uint8_t* blk = y + i * 34;
        uint16_t dh;
        std::memcpy(&dh, blk, 2);
        const float d = fp16_to_fp32(dh);
        for (int j = 0; j < QK8_0; ++j) x[i * QK8_0 + j] = (float)(int8_t)blk[2 + j] * d;
    }
}

// ---------------------------------------------------------------- Q4_K
float make_qkx2_quants(int n, int nmax, const float* x, const float* weights, uint8_t* L, float* the_min,
                       uint8_t* Laux, float rmin, float rdelta, int nstep) {
    float min = x[0];
    float max = x[0];
    float sum_w = weights[0];
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < min) min = x[i];
        if (x[i] > max) max = x[i];
        const float w = weights[i];
        sum_w += w;
        sum_x += w * x[i];
    }
    if (min > 0) min = 0;
    if (max == min) {
        for (int i = 0; i < n; ++i) L[i] = 0;
        *the_min = -min;
        return 0.f;
    }
    float iscale = nmax / (max - min);
    float scale = 1 / iscale;
    float best_error = 0;
    for (int i = 0; i < n; ++i) {
        const int l = nearest_int(iscale * (x[i] - min));
        L[i] = (uint8_t)std::max(0, std::min(nmax, l));
        float diff = scale * L[i] + min - x[i];
        diff = diff * diff;
        best_error += weights[i] * diff;
    }
    for (int is = 0; is <= nstep; ++is) {
        iscale = (rmin + rdelta * is + nmax) / (max - min);
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < n; ++i) {
            int l = nearest_int(iscale * (x[i] - min));
            l = std::max(0, std::min(nmax, l));
            Laux[i] = (uint8_t)l;
            const float w = weights[i];
            sum_l += w * l;
            sum_l2 += w * l * l;
            sum_xl += w * l * x[i];
        }
        const float D = sum_w * sum_l2 - sum_l * sum_l;
        if (D > 0) {
            float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
            float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
            if (this_min > 0) {
                this_min = 0;
                this_scale = sum_xl / sum_l2;
            }
            float mad = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = diff * diff;
                mad += weights[i] * diff;
            }
            if (mad < best_error) {
                for (int i = 0; i < n; ++i) L[i] = Laux[i];
                best_error = mad;
                scale = this_scale;
                min = this_min;
            }
        }
    }
    *the_min = -min;
    return scale;
}

inline void get_scale_min_k4(int j, const uint8_t* q, uint8_t* d, uint8_t* m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

// block_q4_K = {fp16 d, fp16 dmin, u8 scales[12], u8 qs[128]}
void q4_k_row(const float* x, int64_t k, uint8_t* y) {
    uint8_t L[QK_K];
    uint8_t Laux[32];
    float weights[32];
    float mins[QK_K / 32];
    float scales[QK_K / 32];
    for (int64_t i = 0; i < k / QK_K; ++i) {
        uint8_t* blk = y + i * 144;
        uint8_t* sc = blk + 4;
        uint8_t* qs = blk + 16;
        std::memset(sc, 0, 12);
        float max_scale = 0;
        float max_min = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            float sum_x2 = 0;
            for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
            const float av_x = std::sqrt(sum_x2 / 32);
            for (int l = 0; l < 32; ++l) weights[l] = av_x + std::fabs(x[32 * j + l]);
            scales[j] = make_qkx2_quants(32, 15, x + 32 * j, weights, L + 32 * j, &mins[j], Laux, -1.f, 0.1f, 20);
            if (scales[j] > max_scale) max_scale = scales[j];
            if (mins[j] > max_min) max_min = mins[j];
        }
        const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
        const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
        for (int j = 0; j < QK_K / 32; ++j) {
            uint8_t ls = (uint8_t)nearest_int(inv_scale * scales[j]);
            uint8_t lm = (uint8_t)nearest_int(inv_min * mins[j]);
            ls = std::min<uint8_t>(63, ls);
            lm = std::min<uint8_t>(63, lm);
            if (j < 4) {
                sc[j] = ls;
                sc[j + 4] = lm;
            } else {
                sc[j + 4] = (ls & 0xF) | ((lm & 0xF) << 4);
                sc[j - 4] |= ((ls >> 4) << 6);
                sc[j - 0] |= ((lm >> 4) << 6);
            }
        }
        const uint16_t dh = fp32_to_fp16(max_scale / 63.f);
        const uint16_t mh = fp32_to_fp16(max_min / 63.f);
        std::memcpy(blk, &dh, 2);
        std::memcpy(blk + 2, &mh, 2);
        for (int j = 0; j < QK_K / 32; ++j) {
            uint8_t s, m;
            get_scale_min_k4(j, sc, &s, &m);
            const float d = fp16_to_fp32(dh) * s;
            if (!d) continue;
            const float dm = fp16_to_fp32(mh) * m;
            for (int ii = 0; ii < 32; ++ii) {
                int l = nearest_int((x[32 * j + ii] + dm) / d);
                L[32 * j + ii] = (uint8_t)std::max(0, std::min(15, l));
            }
        }
        uint8_t* q = qs;
        for (int j = 0; j < QK_K; j += 64) {
            for (int l = 0; l < 32; ++l) q[l] = L[j + l] | (L[j + l + 32] << 4);
            q += 32;
        }
        x += QK_K;
    }
}

void q4_k_deq(const uint8_t* y, int64_t k, float* x) {
    for (int64_t i = 0; i < k / QK_K; ++i) {
        const uint8_t* blk = y + i * 144;
        uint16_t dh, mh;
        std::memcpy(&dh, blk, 2);
        std::memcpy(&mh, blk + 2, 2);
        const float d = fp16_to_fp32(dh), min = fp16_to_fp32(mh);
        const uint8_t* q = blk + 16;
        int is = 0;
        for (int j = 0; j < QK_K; j += 64) {
            uint8_t sc, m;
            get_scale_min_k4(is + 0, blk + 4, &sc, &m);
            const float d1 = d * sc, m1 = min * m;
            get_scale_min_k4(is + 1, blk + 4, &sc, &m);
            const float d2 = d * sc, m2 = min * m;
            for (int l = 0; l < 32; ++l) *x++ = d1 * (q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *x++ = d2 * (q[l] >> 4) - m2;
            q += 32;
            is += 2;
        }
    }
}

// ---------------------------------------------------------------- Q6_K
float make_qx_quants_rmse1(int n, int nmax, const float* x, int8_t* L) {
    float max = 0;
    float amax = 0;
    for (int i = 0; i < n; ++i) {
        const float ax = std::fabs(x[i]);
        if (ax > amax) {
            amax = ax;
            max = x[i];
        }
    }
    if (amax < GROUP_MAX_EPS) {
        for (int i = 0; i < n; ++i) L[i] = 0;
        return 0.f;
    }
    float iscale = -nmax / max;
    float sumlx = 0;
    float suml2 = 0;
    for (int i = 0; i < n; ++i) {
        int l = nearest_int(iscale * x[i]);
        l = std::max(-nmax, std::min(nmax - 1, l));
        L[i] = (int8_t)(l + nmax);
        const float w = x[i] * x[i];
        sumlx += w * x[i] * l;
        suml2 += w * l * l;
    }
    float scale = suml2 ? sumlx / suml2 : 0.0f;
    float best = scale * sumlx;
    for (int is = -9; is <= 9; ++is) {
        if (is == 0) continue;
        iscale = -(nmax + 0.1f * is) / max;
        sumlx = suml2 = 0;
        for (int i = 0; i < n; ++i) {
            int l = nearest_int(iscale * x[i]);
            l = std::max(-nmax, std::min(nmax - 1, l));
            const float w = x[i] * x[i];
            sumlx += w * x[i] * l;
            suml2 += w * l * l;
        }
        if (suml2 > 0 && sumlx * sumlx > best * suml2) {
            for (int i = 0; i < n; ++i) {
                const int l = nearest_int(iscale * x[i]);
                L[i] = (int8_t)(nmax + std::max(-nmax, std::min(nmax - 1, l)));
            }
            scale = sumlx / suml2;
            best = scale * sumlx;
        }
    }
    return scale;
}

// block_q6_K = {u8 ql[128], u8 qh[64], int8 scales[16], fp16 d}
void q6_k_row(const float* x, int64_t k, uint8_t* y) {
    int8_t L[QK_K];
    float scales[QK_K / 16];
    for (int64_t i = 0; i < k / QK_K; ++i) {
        uint8_t* blk = y + i * 210;
        uint8_t* ql = blk;
        uint8_t* qh = blk + 128;
        int8_t* sc = (int8_t*)(blk + 192);
        float max_scale = 0;
        float max_abs_scale = 0;
        for (int ib = 0; ib < QK_K / 16; ++ib) {
            const float scale = make_qx_quants_rmse1(16, 32, x + 16 * ib, L + 16 * ib);
            scales[ib] = scale;
            const float abs_scale = std::fabs(scale);
            if (abs_scale > max_abs_scale) {
                max_abs_scale = abs_scale;
                max_scale = scale;
            }
        }
        if (max_abs_scale < GROUP_MAX_EPS) {
            std::memset(blk, 0, 210);
            x += QK_K;
            continue;
        }
        const float iscale = -128.f / max_scale;
        const uint16_t dh = fp32_to_fp16(1 / iscale);
        std::memcpy(blk + 208, &dh, 2);
        for (int ib = 0; ib < QK_K / 16; ++ib) sc[ib] = (int8_t)std::min(127, nearest_int(iscale * scales[ib]));
        for (int j = 0; j < QK_K / 16; ++j) {
            const float d = fp16_to_fp32(dh) * sc[j];
            if (!d) continue;
            for (int ii = 0; ii < 16; ++ii) {
                int l = nearest_int(x[16 * j + ii] / d);
                l = std::max(-32, std::min(31, l));
                L[16 * j + ii] = (int8_t)(l + 32);
            }
        }
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                const uint8_t q1 = L[j + l + 0] & 0xF;
                const uint8_t q2 = L[j + l + 32] & 0xF;
                const uint8_t q3 = L[j + l + 64] & 0xF;
                const uint8_t q4 = L[j + l + 96] & 0xF;
                ql[l + 0] = q1 | (q3 << 4);
                ql[l + 32] = q2 | (q4 << 4);
                qh[l] = (L[j + l] >> 4) | ((L[j + l + 32] >> 4) << 2) | ((L[j + l + 64] >> 4) << 4) |
                        ((L[j + l + 96] >> 4) << 6);
            }
            ql += 64;
            qh += 32;
        }
        x += QK_K;
    }
}

// q6 values (q - 32) of one block in natural order
void q6_k_values(const uint8_t* blk, int8_t* v) {
    const uint8_t* ql = blk;
    const uint8_t* qh = blk + 128;
    for (int h = 0; h < 2; ++h) {
        for (int l = 0; l < 32; ++l) {
            v[128 * h + l + 0] = (int8_t)((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
            v[128 * h + l + 32] = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
            v[128 * h + l + 64] = (int8_t)((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
            v[128 * h + l + 96] = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
        }
        ql += 64;
        qh += 32;
    }
}

void q6_k_deq(const uint8_t* y, int64_t k, float* x) {
    int8_t v[QK_K];
    for (int64_t i = 0; i < k / QK_K; ++i) {
        const uint8_t* blk = y + i * 210;
        const int8_t* sc = (const int8_t*)(blk + 192);
        uint16_t dh;
        std::memcpy(&dh, blk + 208, 2);
        const float d = fp16_to_fp32(dh);
        q6_k_values(blk, v);
        for (int l = 0; l < QK_K; ++l) x[i * QK_K + l] = d * sc[l / 16] * v[l];
    }
}

template <typename F>
void parallel_rows(int64_t rows, F&& f) {
    unsigned nt = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("OMP_NUM_THREADS")) nt = std::max(1, std::atoi(e));
    nt = std::max(1u, std::min<unsigned>(nt, 64u));
    if (rows < 64 || nt == 1) {
        f(0, rows);
        return;
    }
    const int64_t chunk = (rows + nt - 1) / nt;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) {
        const int64_t r0 = t * chunk, r1 = std::min(rows, r0 + chunk);
        if (r0 >= r1) break;
        th.emplace_back([&, r0, r1] { f(r0, r1); });
    }
    for (auto& t : th) t.join();
}

}  // namespace

QType parse(const char* value) {
    if (!value || !value[0]) return QNONE;
    std::string s(value);
    for (auto& ch : s) ch = (char)std::toupper((unsigned char)ch);
    if (s == "Q8" || s == "Q8_0") return Q8_0;
    if (s == "Q6" || s == "Q6_K") return Q6_K;
    if (s == "Q4" || s == "Q4_K" || s == "Q4_K_M") return Q4_K;
    return QNONE;
}

QType from_env(const char* primary_key) {
    const QType t = parse(std::getenv(primary_key));
    if (t != QNONE) return t;
    return parse(std::getenv("ACE_GGML_WEIGHT_QTYPE"));
}

QType from_env() { return from_env("ACE_GGML_DIT_WEIGHT_QTYPE"); }

const char* name(QType t) {
    switch (t) {
        case Q8_0: return "Q8_0";
        case Q4_K: return "Q4_K";
        case Q6_K: return "Q6_K";
        default: return "none";
    }
}

int block_values(QType t) { return t == Q8_0 ? QK8_0 : QK_K; }
size_t block_bytes(QType t) { return t == Q8_0 ? 34 : (t == Q4_K ? 144 : 210); }
size_t row_bytes(QType t, int64_t cols) { return (size_t)(cols / block_values(t)) * block_bytes(t); }
bool applies(QType t, int64_t cols) { return t != QNONE && cols % block_values(t) == 0; }

void quantize_rows(QType t, const float* src, int64_t rows, int64_t cols, uint8_t* dst) {
    if (!applies(t, cols)) throw std::runtime_error("quantize: bad row length");
    const size_t rb = row_bytes(t, cols);
    parallel_rows(rows, [&](int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; ++r) {
            const float* x = src + r * cols;
            uint8_t* y = dst + r * rb;
            if (t == Q8_0)
                q8_0_row(x, cols, y);
            else if (t == Q4_K)
                q4_k_row(x, cols, y);
            else
                q6_k_row(x, cols, y);
        }
    });
}

void dequantize_rows(QType t, const uint8_t* src, int64_t rows, int64_t cols, float* dst) {
    if (!applies(t, cols)) throw std::runtime_error("dequantize: bad row length");
    const size_t rb = row_bytes(t, cols);
    for (int64_t r = 0; r < rows; ++r) {
        const uint8_t* y = src + r * rb;
        float* x = dst + r * cols;
        if (t == Q8_0)
            q8_0_deq(y, cols, x);
        else if (t == Q4_K)
            q4_k_deq(y, cols, x);
        else
            q6_k_deq(y, cols, x);
    }
}

size_t q_plane_bytes(QType t, int64_t rows, int64_t cols) {
    return (size_t)(rows * (t == Q4_K ? cols / 2 : cols));
}
size_t s_plane_floats(QType t, int64_t rows, int64_t cols) {
    if (t == Q8_0) return (size_t)(rows * (cols / 32));
    if (t == Q4_K) return (size_t)(rows * (cols / 32) * 2);
    return (size_t)(rows * (cols / 16));
}

void to_planes(QType t, const uint8_t* blocks, int64_t rows, int64_t cols, uint8_t* qplane, float* splane) {
    const size_t rb = row_bytes(t, cols);
    parallel_rows(rows, [&](int64_t r0, int64_t r1) {
        int8_t v[QK_K];
        for (int64_t r = r0; r < r1; ++r) {
            const uint8_t* y = blocks + r * rb;
            if (t == Q8_0) {
                int8_t* q = (int8_t*)qplane + r * cols;
                float* s = splane + r * (cols / 32);
                for (int64_t b = 0; b < cols / 32; ++b) {
                    uint16_t dh;
                    std::memcpy(&dh, y + b * 34, 2);
                    s[b] = fp16_to_fp32(dh);
                    std::memcpy(q + b * 32, y + b * 34 + 2, 32);
                }
            } else if (t == Q4_K) {
                uint8_t* q = qplane + r * (cols / 2);
                float* s = splane + r * (cols / 32) * 2;
                for (int64_t b = 0; b < cols / QK_K; ++b) {
                    const uint8_t* blk = y + b * 144;
                    uint16_t dh, mh;
                    std::memcpy(&dh, blk, 2);
                    std::memcpy(&mh, blk + 2, 2);
                    const float d = fp16_to_fp32(dh), dmin = fp16_to_fp32(mh);
                    uint8_t vals[QK_K];
                    for (int j = 0; j < 4; ++j)
                        for (int l = 0; l < 32; ++l) {
                            vals[64 * j + l] = blk[16 + 32 * j + l] & 0xF;
                            vals[64 * j + 32 + l] = blk[16 + 32 * j + l] >> 4;
                        }
                    for (int j = 0; j < 8; ++j) {
                        uint8_t sc, m;
                        get_scale_min_k4(j, blk + 4, &sc, &m);
                        const int64_t g = b * 8 + j;  // 32-block index within the row
                        s[2 * g + 0] = d * sc;
                        s[2 * g + 1] = dmin * m;
                        uint8_t* dst = q + g * 16;
                        for (int i = 0; i < 16; ++i) {
                            const int kk = 8 * (i / 4) + (i % 4);
                            dst[i] = (uint8_t)(vals[32 * j + kk] | (vals[32 * j + kk + 4] << 4));
                        }
                    }
                }
            } else {
                int8_t* q = (int8_t*)qplane + r * cols;
                float* s = splane + r * (cols / 16);
                for (int64_t b = 0; b < cols / QK_K; ++b) {
                    const uint8_t* blk = y + b * 210;
                    const int8_t* sc = (const int8_t*)(blk + 192);
                    uint16_t dh;
                    std::memcpy(&dh, blk + 208, 2);
                    const float d = fp16_to_fp32(dh);
                    q6_k_values(blk, v);
                    std::memcpy(q + b * QK_K, v, QK_K);
                    for (int j = 0; j < 16; ++j) s[b * 16 + j] = d * sc[j];
                }
            }
        }
    });
}

}  // namespace quant
}  // namespace acemi
