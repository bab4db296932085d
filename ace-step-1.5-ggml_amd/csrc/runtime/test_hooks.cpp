// Test-only hooks, read from the environment ONLY in the self-test library (built from this file with
// -DACEMI_TEST_HOOKS, Makefile SELFTEST): the product library is compiled without it and never reads them.
//   ACE_MI_TEST_FAULT="layer,row,col,amp"  adds amp to one 16 x 128 tile of the residual after that layer's
//                                          o-projection (the parity negative control, tests/test_gpu_parity_strict.py)
//   ACE_MI_TEST_VAE_FAULT="block,row,col,amp"  adds amp to one 16 x 128 tile of the VAE decoder's residual stream
//                                          after that block's first residual unit (tests/test_gpu_vae.py)
//   ACE_MI_GEMM_OVERRIDE="N:K:variant,..." dense-weight GEMM tile picks per shape (in-loop A/B runs,
//                                          tools/gpu_pick_inloop.sh)
#include <array>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "../kernels.h"

namespace acemi {

#ifdef ACEMI_TEST_HOOKS
bool test_fault_from_env(int& layer, int& row, int& col, float& amp) {
    const char* f = std::getenv("ACE_MI_TEST_FAULT");
    if (!f || !f[0]) return false;
    if (std::sscanf(f, "%d,%d,%d,%f", &layer, &row, &col, &amp) != 4)
        throw std::runtime_error("ACE_MI_TEST_FAULT must be layer,row,col,amp");
    return true;
}

bool test_vae_fault_from_env(int& block, int& row, int& col, float& amp) {
    const char* f = std::getenv("ACE_MI_TEST_VAE_FAULT");
    if (!f || !f[0]) return false;
    if (std::sscanf(f, "%d,%d,%d,%f", &block, &row, &col, &amp) != 4)
        throw std::runtime_error("ACE_MI_TEST_VAE_FAULT must be block,row,col,amp");
    return true;
}

int gemm_override_from_env(int N, int K) {
    static const std::vector<std::array<int, 3>> table = [] {
        std::vector<std::array<int, 3>> t;
        const char* e = std::getenv("ACE_MI_GEMM_OVERRIDE");
        while (e && *e) {
            int n = 0, k = 0, v = 0, used = 0;
            if (std::sscanf(e, "%d:%d:%d%n", &n, &k, &v, &used) != 3) break;
            t.push_back({n, k, v});
            e += used;
            if (*e == ',') ++e;
        }
        return t;
    }();
    for (const auto& x : table)
        if (x[0] == N && x[1] == K) return x[2];
    return -1;
}
#else
bool test_fault_from_env(int&, int&, int&, float&) { return false; }
bool test_vae_fault_from_env(int&, int&, int&, float&) { return false; }
int gemm_override_from_env(int, int) { return -1; }
#endif

}  // namespace acemi
