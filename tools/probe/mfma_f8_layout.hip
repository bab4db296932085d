// Probe (GPU box): operand layout and block-scale semantics of v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands.
// For each candidate k-mapping of a lane's 32 bytes, packs random small-integer fp8 matrices A [32][64], B [64][32]
// by that mapping, runs one MFMA (scales 2^sa, 2^sb) and compares D (standard 32x32 f32 accumulator layout:
// lane l, reg r -> row 8 (r / 4) + 4 (l / 32) + r % 4, col l % 32) with the host product.  Prints one line per case.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) int v8i;
typedef __attribute__((ext_vector_type(16))) float v16f;

__global__ void k_mfma(const int* a, const int* b, float* d, int sa, int sb) {
    const int l = threadIdx.x;
    v8i A, B;
    for (int i = 0; i < 8; ++i) {
        A[i] = a[l * 8 + i];
        B[i] = b[l * 8 + i];
    }
    v16f C = {};
    C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C, 0, 0, 0, sa, 0, sb);
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = C[r];
}

static unsigned char to_e4m3(int v) {  // small integers -4..4
    if (v == 0) return 0;
    const int s = v < 0 ? 0x80 : 0;
    int a = v < 0 ? -v : v;
    int e = 0;
    while ((1 << (e + 1)) <= a) ++e;
    const int mant = (a - (1 << e)) * 8 / (1 << e);  // 3 mantissa bits
    return (unsigned char)(s | ((e + 7) << 3) | mant);
}

static int kmap(int hyp, int h, int i) {
    switch (hyp) {
        case 0: return 32 * h + i;
        case 1: return 8 * h + (i / 8) * 16 + i % 8;
        case 2: return 16 * h + (i / 16) * 32 + i % 16;
        case 3: return 4 * h + (i / 4) * 8 + i % 4;
        default: return 2 * h + (i / 2) * 4 + i % 2;
    }
}

int main() {
    srand(7);
    int Am[32][64], Bm[64][32];
    for (int m = 0; m < 32; ++m)
        for (int k = 0; k < 64; ++k) Am[m][k] = rand() % 9 - 4;
    for (int k = 0; k < 64; ++k)
        for (int n = 0; n < 32; ++n) Bm[k][n] = rand() % 9 - 4;
    int *da, *db;
    float* dd;
    hipMalloc(&da, 64 * 32);
    hipMalloc(&db, 64 * 32);
    hipMalloc(&dd, 64 * 16 * 4);
    const int scales[3][2] = {{127, 127}, {116, 127}, {127, 135}};
    for (int hyp = 0; hyp < 5; ++hyp) {
        unsigned char pa[64][32], pb[64][32];
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 32; ++i) {
                const int k = kmap(hyp, l / 32, i);
                pa[l][i] = to_e4m3(Am[l % 32][k]);
                pb[l][i] = to_e4m3(Bm[k][l % 32]);
            }
        hipMemcpy(da, pa, sizeof(pa), hipMemcpyHostToDevice);
        hipMemcpy(db, pb, sizeof(pb), hipMemcpyHostToDevice);
        for (int sc = 0; sc < 3; ++sc) {
            hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, da, db, dd, scales[sc][0], scales[sc][1]);
            float out[64 * 16];
            hipMemcpy(out, dd, sizeof(out), hipMemcpyDeviceToHost);
            const double f = std::ldexp(1.0, (scales[sc][0] - 127) + (scales[sc][1] - 127));
            int bad = 0;
            double maxd = 0;
            for (int l = 0; l < 64; ++l)
                for (int r = 0; r < 16; ++r) {
                    const int m = 8 * (r / 4) + 4 * (l / 32) + r % 4, n = l % 32;
                    double ref = 0;
                    for (int k = 0; k < 64; ++k) ref += (double)Am[m][k] * Bm[k][n];
                    ref *= f;
                    const double dlt = std::fabs(ref - out[l * 16 + r]);
                    if (dlt > 1e-6 * std::fabs(ref) + 1e-9) ++bad;
                    if (dlt > maxd) maxd = dlt;
                }
            printf("hyp %d scale_a %d scale_b %d: mismatches %d / 1024 (max |d| %.4g)\n", hyp, scales[sc][0], scales[sc][1],
                   bad, maxd);
        }
    }
    return 0;
}
