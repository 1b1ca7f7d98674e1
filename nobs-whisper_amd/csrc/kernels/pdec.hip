// Persistent decode step: host side (block layout, split counts, the launch). The kernel and its design
// notes: pdec_body.h.
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace wm {

void pdec_launch_f16_1(const PdecArgs& a, size_t lds, hipStream_t st);
void pdec_launch_bf16_1(const PdecArgs& a, size_t lds, hipStream_t st);
void pdec_launch_q_1(const PdecArgs& a, size_t lds, hipStream_t st);
void pdec_launch_f16_4(const PdecArgs& a, size_t lds, hipStream_t st);
void pdec_launch_bf16_4(const PdecArgs& a, size_t lds, hipStream_t st);
void pdec_launch_q_4(const PdecArgs& a, size_t lds, hipStream_t st);

namespace {
constexpr int kG = 256, kNT = 256;
}

long g_pdec_spin_ticks = 5000000;
unsigned long long* g_pdec_stamps = nullptr;
int g_pdec_blocks = 0;
std::atomic<int> g_pdec_gen{0};
std::atomic<long> g_pdec_give_ups_total{0};

bool pdec_supported(int d, int H, bool quant) {
    if (H * 64 != d) return false;
    return d == 768 || d == 1024 || d == 1280 || (!quant && (d == 384 || d == 512));
}

PdecGranules pdec_granules(int d, int L, int H) {
    const long R = kPdecMaxRows;
    PdecGranules g{};
    long o = 0;
    g.x0 = o; o += R * d;
    g.x1 = o; o += R * d;
    g.x2 = o; o += R * d;
    g.qkv = o; o += R * 3 * d / 2;
    g.so = o; o += R * d / 2;
    g.qx = o; o += R * d / 2;
    g.xo = o; o += R * d / 2;
    g.ff = o; o += R * 2 * d;
    g.part = o; o += (long)std::max(kG, (int)R * H * pdec_cross_splits(H, 1 << 20)) * 66;  // every task's partial
    g.err_bytes = o * 8;
    g.zero_bytes = g.err_bytes + 16;
    g.bytes = g.zero_bytes + 256;
    return g;
}

// at most 8 key splits per (row, head): the split-0 merge reads fewer partials and fewer workgroups poll
// (measured at 1 clip, caps 6 / 8 / 16 / none: base 191.5 / 188.5 / 192.0 / 195.8 us per step, large-v3
// unchanged within noise). A function of the model shape only, not of the clip count (round 5, ADVICE r4:
// a clip's result must not change with the number of clips still decoding): above 256 tasks (large-v3 at
// 2-4 clips) workgroups take several.
int pdec_cross_splits(int H, int rows) { return std::max(1, std::min({kG / H, rows / 16, 8})); }

void launch_pdec(DType dt, const PdecArgs& a, hipStream_t st) {
    if (a.M < 1 || a.M > kPdecMaxRows) WM_FAIL("pdec: %d rows", a.M);
    if ((long)a.M * (a.d / 64) * a.s_cross * 66 > a.gr.err_bytes / 8 - a.gr.part) WM_FAIL("pdec: split count");
    // self attention in one chunk (16 rows per lane group); cross-attention tasks of at most 1536 rows (the
    // scores buffer)
    if (a.n_text_ctx > 16 * kNT / 8 || (a.n_audio_ctx + a.s_cross - 1) / a.s_cross > 1536) WM_FAIL("pdec: context sizes");
    const PdecLds ll = pdec_lds(a.d, a.M, a.s_cross);
    if (ll.bytes > 160 * 1024) WM_FAIL("pdec: %d bytes of LDS", ll.bytes);
    const size_t lds = ll.bytes;
    WM_CHECK(hipMemsetAsync(a.sync, 0, a.gr.bytes, st));
    const bool one = a.M == 1;  // the one-row build (the app's one clip per call)
    if (a.quant) {
        if (dt != DType::F16) WM_FAIL("pdec: GGML blocks with a bf16 context");
        one ? pdec_launch_q_1(a, lds, st) : pdec_launch_q_4(a, lds, st);
    } else if (dt == DType::F16) {
        one ? pdec_launch_f16_1(a, lds, st) : pdec_launch_f16_4(a, lds, st);
    } else {
        one ? pdec_launch_bf16_1(a, lds, st) : pdec_launch_bf16_4(a, lds, st);
    }
}

}  // namespace wm
