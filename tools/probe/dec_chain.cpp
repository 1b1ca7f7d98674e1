// Probe: the decode step's GEMM launches (the engine's own launchers, libwhisper_mi355x.so) as a chain of
// dependent launches in a replayed hipGraph, per shape, at M = 16 and 128 active clips (large-v3: d = 1280).
// Weights rotate over 32 copies (one per decoder layer, as in the step: cold) or stay fixed (hot).
// Build (from the repo root):
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -Inobs-whisper_amd/csrc -Iinclude tools/probe/dec_chain.cpp \
//     -Lnobs-whisper_amd/lib -lwhisper_mi355x -Wl,-rpath,'$ORIGIN/../../nobs-whisper_amd/lib' -o tools/probe/dec_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels.h"

using namespace wm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace wm { extern int g_dec_splits; }

static void* dalloc(size_t b) {
    void* p;
    CK(hipMalloc(&p, b));
    CK(hipMemset(p, 0, b));
    return p;
}

int main(int argc, char** argv) {
    const int d = 1280, NL = 32, REP = 10, CH = argc > 1 ? atoi(argv[1]) : 64;
    init_gelu_table();
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    // per-layer weights: qkv [3d][d], o [d][d], q [d][d], w1 [4d][d], w2 [d][4d]
    std::vector<void*> wqkv(NL), wo(NL), w1(NL), w2(NL);
    for (int l = 0; l < NL; l++) {
        wqkv[l] = dalloc((size_t)3 * d * d * 2);
        wo[l] = dalloc((size_t)d * d * 2);
        w1[l] = dalloc((size_t)4 * d * d * 2);
        w2[l] = dalloc((size_t)4 * d * d * 2);
    }
    float* bias = (float*)dalloc(4 * d * 4);
    float* lnw = (float*)dalloc(d * 4);
    float* x = (float*)dalloc((size_t)128 * d * 4);
    void* a_d = dalloc((size_t)128 * 4 * d * 2);
    void* o_d = dalloc((size_t)128 * 4 * d * 2);
    void* hln = dalloc((size_t)128 * d * 2);
    const long ws_elems = 64L << 20;
    float* ws = (float*)dalloc(ws_elems * 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto gp = [&](const void* A, int M, int K, const void* B, int N, void* out, long ldo) {
        GemmArgs g{};
        g.A = A; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = out; g.ldo = ldo; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.scale = 1.0f; g.sc_div = 1; g.sc_mod = 1; g.sc_lim = 0;
        g.splitk_ws = ws; g.splitk_ws_elems = ws_elems; g.slab_wt = 1;
        return g;
    };
    auto time_chain = [&](const char* name, int M, bool hot, const std::function<void(int)>& body) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < CH; i++) body(hot ? 0 : i % NL);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < REP; r++) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("M=%3d %-34s %s %7.2f us per call\n", M, name, hot ? "hot " : "cold", ms * 1e3 / REP / CH);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    };
    const DType dt = DType::BF16;
    for (int M : {16, 128}) {
        for (int hot = 0; hot < 2; hot++) {
            time_chain("qkv partials (N 3840)", M, hot, [&](int l) { launch_gemm_partials(dt, gp(hln, M, d, wqkv[l], 3 * d, nullptr, 3 * d), st); });
            time_chain("d x d partials", M, hot, [&](int l) { launch_gemm_partials(dt, gp(hln, M, d, wo[l], d, nullptr, d), st); });
            time_chain("d x d store (gemm + reduce)", M, hot, [&](int l) { launch_gemm(dt, EPI_STORE, gp(hln, M, d, wo[l], d, o_d, d), st); });
            time_chain("d x d resid+LN (gemm + reduce_ln)", M, hot, [&](int l) {
                GemmArgs g = gp(a_d, M, d, wo[l], d, x, d);
                g.ln_w = lnw; g.ln_b = bias; g.ln_out = hln;
                launch_gemm(dt, EPI_RESID, g, st);
            });
            time_chain("fc1 gelu (N 5120)", M, hot, [&](int l) { launch_gemm(dt, EPI_GELU, gp(hln, M, d, w1[l], 4 * d, o_d, 4 * d), st); });
            time_chain("fc1 partials (N 5120)", M, hot, [&](int l) { launch_gemm_partials(dt, gp(hln, M, d, w1[l], 4 * d, nullptr, 4 * d), st); });
            time_chain("fc2 resid+LN (K 5120)", M, hot, [&](int l) {
                GemmArgs g = gp(o_d, M, 4 * d, w2[l], d, x, d);
                g.ln_w = lnw; g.ln_b = bias; g.ln_out = hln;
                launch_gemm(dt, EPI_RESID, g, st);
            });
            time_chain("fc2 partials (K 5120)", M, hot, [&](int l) { launch_gemm_partials(dt, gp(o_d, M, 4 * d, w2[l], d, nullptr, d), st); });
            time_chain("layer set: qkv,o+ln,q,o2+ln,fc1,fc2+ln", M, hot, [&](int l) {
                launch_gemm_partials(dt, gp(hln, M, d, wqkv[l], 3 * d, nullptr, 3 * d), st);
                GemmArgs g = gp(a_d, M, d, wo[l], d, x, d);
                g.ln_w = lnw; g.ln_b = bias; g.ln_out = hln;
                launch_gemm(dt, EPI_RESID, g, st);
                launch_gemm(dt, EPI_STORE, gp(hln, M, d, wo[(l + 1) % NL], d, o_d, d), st);
                launch_gemm(dt, EPI_RESID, g, st);
                launch_gemm(dt, EPI_GELU, gp(hln, M, d, w1[l], 4 * d, o_d, 4 * d), st);
                GemmArgs g2 = gp(o_d, M, 4 * d, w2[l], d, x, d);
                g2.ln_w = lnw; g2.ln_b = bias; g2.ln_out = hln;
                launch_gemm(dt, EPI_RESID, g2, st);
            });
            if (M <= 32) {
                time_chain("small d x d resid", M, hot, [&](int l) { launch_gemm_small(dt, EPI_RESID, gp(a_d, M, d, wo[l], d, x, d), false, st); });
                time_chain("small d x d store + LN prologue", M, hot, [&](int l) {
                    GemmArgs g = gp(x, M, d, wo[l], d, o_d, d);
                    g.a_ln_w = lnw; g.a_ln_b = bias;
                    launch_gemm_small(dt, EPI_STORE, g, true, st);
                });
                time_chain("small fc2 resid (K 5120)", M, hot, [&](int l) { launch_gemm_small(dt, EPI_RESID, gp(o_d, M, 4 * d, w2[l], d, x, d), false, st); });
            }
        }
    }
    return 0;
}
