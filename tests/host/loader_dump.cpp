// Host-only check harness for the weight loaders (TEST INFRASTRUCTURE): compiles
// runtime/{json,gguf,quant,model,vae}.cpp with g++ against stub HIP memory functions (host malloc),
// loads a DiT and/or VAE checkpoint exactly as ace_ggml_load_dit / ace_ggml_load_vae do, and dumps
// every device buffer so tests/test_loader_cpu.py can check the layouts without a GPU.
//   usage: loader_dump dit|vae <model_dir> <out_dir>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

#include "runtime/model.h"
#include "runtime/vae.h"

// ---- stub HIP runtime: device memory is host memory
extern "C" {
hipError_t hipMalloc(void** p, size_t n) {
    *p = std::calloc(1, n ? n : 1);
    return hipSuccess;
}
hipError_t hipFree(void* p) {
    std::free(p);
    return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
    std::memcpy(d, s, n);
    return hipSuccess;
}
hipError_t hipMemset(void* d, int v, size_t n) {
    std::memset(d, v, n);
    return hipSuccess;
}
hipError_t hipDeviceSynchronize() { return hipSuccess; }
hipError_t hipMemcpy2DAsync(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind, hipStream_t) {
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t) { return "stub"; }
}
namespace acemi {  // kernels are not linked: the engines are never run here
void launch_conv_gemm(const ConvGemmArgs&, hipStream_t) {}
void launch_to_f16(const float*, int64_t, uint16_t*, hipStream_t) {}
void launch_pack_f16(const float*, int64_t, int, int, uint16_t*, hipStream_t) {}
void launch_conv_out(const uint16_t*, int, int, const uint16_t*, int, float*, hipStream_t, int) {}
void launch_fault_tile(float*, int, int, int, int, float, hipStream_t) {}
bool test_vae_fault_from_env(int&, int&, int&, float&) { return false; }
}  // namespace acemi

namespace {
std::ofstream g_index;
std::string g_out;

void dump(const std::string& name, const void* p, size_t bytes) {
    std::ofstream f(g_out + "/" + name + ".bin", std::ios::binary);
    f.write(static_cast<const char*>(p), (std::streamsize)bytes);
}

void weight(const std::string& name, const acemi::DevWeight& w) {
    using namespace acemi;
    const size_t rc = (size_t)w.rows * w.cols;
    size_t qb = 0, sb = 0;
    switch (w.fmt) {
        case WF_BF16: case WF_F16: qb = rc * 2; break;
        case WF_F32X3: qb = rc * 6; break;
        case WF_Q8_0: qb = rc; sb = rc / 32 * 4; break;
        case WF_Q4_K: qb = rc / 2; sb = rc / 32 * 8; break;
        case WF_Q6_K: qb = rc; sb = rc / 16 * 4; break;
    }
    dump(name + ".q", w.q, qb);
    if (sb) dump(name + ".s", w.s, sb);
    g_index << name << " W " << w.fmt << " " << w.rows << " " << w.cols << "\n";
}

void vec(const std::string& name, const float* p, size_t n) {
    dump(name, p, n * 4);
    g_index << name << " F " << n << "\n";
}
void u16(const std::string& name, const uint16_t* p, size_t n) {
    dump(name, p, n * 2);
    g_index << name << " H " << n << "\n";
}
}  // namespace

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: loader_dump dit|vae <model_dir> <out_dir>\n");
        return 2;
    }
    const std::string kind = argv[1];
    g_out = argv[3];
    g_index.open(g_out + "/index.txt");
    int hint = 0;
    try {
        if (kind == "dit") {
            acemi::DitModel m;
            acemi::load_dit_model(argv[2], m, hint);
            const auto& c = m.cfg;
            const int H = c.hidden;
            g_index << "act " << (int)m.act << " qtype " << m.qtype << "\n";
            weight("proj_in", m.proj_in_w);
            weight("proj_out", m.proj_out_w);
            weight("cond", m.cond_w);
            vec("out_table", m.out_table, 2 * (size_t)H);
            vec("tables", m.tables, (size_t)c.layers * 6 * H);
            for (int e = 0; e < 2; ++e) {
                const std::string p = "te" + std::to_string(e) + ".";
                g_index << p << "act " << (int)m.te[e].act << "\n";
                u16(p + "w1", m.te[e].w1, (size_t)H * 256);
                u16(p + "w2", m.te[e].w2, (size_t)H * H);
                u16(p + "wp", m.te[e].wp, (size_t)6 * H * H);
            }
            for (int i = 0; i < c.layers; ++i) {
                const auto& ly = m.layers[i];
                const std::string p = "l" + std::to_string(i) + ".";
                weight(p + "qkv", ly.w_qkv);
                weight(p + "o", ly.w_o);
                weight(p + "cq", ly.w_cq);
                weight(p + "ckv", ly.w_ckv);
                weight(p + "co", ly.w_co);
                weight(p + "gu", ly.w_gu);
                weight(p + "down", ly.w_down);
                vec(p + "self_norm", ly.self_norm, H);
            }
        } else {
            acemi::VaeModel m;
            acemi::load_vae_model(argv[2], m, hint);
            auto conv = [&](const std::string& n, const acemi::VaeConv& cv) {
                const size_t rows = cv.transposed ? (size_t)cv.stride * cv.cout : cv.cout;
                const size_t cols = (size_t)cv.taps * cv.cin;
                u16(n + ".w", cv.w, rows * cols);
                if (cv.b) vec(n + ".b", cv.b, cv.cout);
                g_index << n << " C " << cv.cin << " " << cv.cin_real << " " << cv.cout << " " << cv.taps << " "
                        << cv.dil << " " << cv.pad << " " << cv.stride << " " << (int)cv.transposed << "\n";
            };
            auto snake = [&](const std::string& n, const acemi::VaeSnake& s) {
                vec(n + ".ea", s.ea, s.C);
                vec(n + ".eb", s.eb, s.C);
            };
            conv("decoder.conv1", m.conv1);
            for (size_t i = 0; i < m.blocks.size(); ++i) {
                const std::string p = "decoder.block." + std::to_string(i);
                snake(p + ".snake1", m.blocks[i].s1);
                conv(p + ".conv_t1", m.blocks[i].ct);
                for (int j = 0; j < 3; ++j) {
                    const std::string q = p + ".res_unit" + std::to_string(j + 1);
                    conv(q + ".conv1", m.blocks[i].res[j].c1);
                    conv(q + ".conv2", m.blocks[i].res[j].c2);
                    snake(q + ".snake2", m.blocks[i].res[j].s2);
                }
            }
            conv("decoder.conv2", m.conv2);
            if (m.has_encoder) {
                conv("encoder.conv1", m.enc_conv1);
                for (size_t i = 0; i < m.enc_blocks.size(); ++i)
                    conv("encoder.block." + std::to_string(i) + ".conv1", m.enc_blocks[i].conv);
                conv("encoder.conv2", m.enc_conv2);
            }
            g_index << "hop " << m.cfg.hop_length << "\n";
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "load failed (hint %d): %s\n", hint, e.what());
        g_index << "error " << hint << " " << e.what() << "\n";
        return 1;
    }
    return 0;
}
