// Persistent decode step for few clips (the kernel; instantiated by pdec_f16.hip, pdec_bf16.hip, pdec_q.hip and
// their one-row *_1.hip builds): the whole decoder (every layer) of one decode step of <= kPdecMaxRows clips in
// ONE launch, its phases handing off through data-tagged granules instead of kernel boundaries (SURVEY.md §8a
// row a10, the hot loop of whisper_full: whisper.rs:127-129 -> state.rs:147; the app transcribes one clip per
// call, so this is the latency its user feels).
//
// Why: at one clip a large-v3 decoder layer streams 46 MB of weights +
// 7.7 MB of cross K/V (~8 us at HBM speed) but took ~78 us as 8 dependent launches of 5-15 us each:
// launch boundaries, ramp-up and dependent-load latency, not bytes. Here the grid is one 256-thread
// workgroup per CU (G = 256), resident for the whole step:
//   per layer, 8 phases:  A  LN1 + QKV projection (+ q/k scale, rounding to T)        all WGs, column slices
//                         B  self attention over the cache + this position             one (clip, head) task per WG
//                         C  out projection + residual                                 all WGs
//                         D  LN + cross-Q projection (+ scale)                         all WGs
//                         E  cross attention over the cached K/V, split over keys;     (clip, head, split) tasks,
//                            split 0 of each (clip, head) merges the splits             dealt round-robin
//                         F  cross-out projection + residual                           all WGs
//                         G  LN + FC1 + GELU (ggml's f16 table)                       all WGs
//                         H  FC2 + residual                                            all WGs
//   then the final LayerNorm of every row (the logits GEMM is the next launch).
// A projection phase: each WG owns a contiguous slice of output columns (N / G of them), so its weights
// are ONE contiguous range of the [N][K] matrix; it issues their loads into registers a phase ahead, after
// its previous publish (the loader-runs-ahead idea of MI355X_MICROARCH.md "prefetch-credit", in registers
// instead of an LDS ring). Every WG gathers the whole (small) input: M rows of d, computes the LayerNorm
// itself (ggml_norm: double sums in one canonical order for every M) and stages the rows in LDS as T; one
// wave per output column, lanes split K, f32 accumulation, wave sums by DPP.
//
// Hand-offs (cdna_hip_programming.md Guideline 16 R2; MI355X_MICROARCH.md rows handoff-1to1 / allgather):
// every handed-off value travels as ONE naturally aligned 8-byte granule {tag, 32 data bits} written by one
// sc1 store; the data is the flag. A producer neither drains nor signals; a consumer re-reads the granules it
// needs with sc1 loads (16 in flight per thread in the wide sweeps) until every tag equals the phase's tag
// (layer * 8 + phase + 1), then uses the data bits. x rows travel as f32 granules, everything rounded to T
// (q/k/v, attention outputs, cross-Q, GELU rows) as packed T pairs; a cross-attention split publishes its
// partial {o[64], max, sum} as 66 granules that split 0's workgroup gathers. The block is zeroed by a memset
// node before every launch, and a buffer is reused by the next layer (safe: every layer's phase A reads all
// of x0, i.e. waits for every workgroup's last phase of the layer before).
// Bounded waits: a wait gives up after spin_ticks of s_memrealtime (100 MHz; 50 ms by default), sets the
// error word and the workgroup exits; every other wait sees the error word and exits too, so the grid always
// drains (e.g. when another kernel holds CUs and not all 256 workgroups can be resident). The host then
// re-runs the step on the launch-per-kernel path (engine.cpp decode_step; counted as a give-up in the
// state's kernel stats), so a failed launch costs time, never results.
//
// Numerics (vs oracle/oracle_whisper.cpp, ggml's): LayerNorm as layernorm_kernel (double sums, separately
// rounded ops, output rounded to T = ggml's f16 src1); projections f32-accumulated products of T
// operands; q, k scaled by d_head^-0.25 then rounded to T, v rounded to T (the self cache holds T);
// attention scores f32, softmax in f32 over each split with the split's own max, the unnormalised
// weights rounded to T before P.V (ggml rounds the normalised P to f16: another rounding point, the
// same precision), splits merged with exp(m_s - m) in f32 and the result rounded to T (the out
// projection's src1). A row's results do not depend on the other rows (round 5): the key-split count is a
// function of the model shape (pdec_cross_splits), the LayerNorm sums run in one order for every M, and the
// one-row and four-row builds share every reduction, so a clip decodes the same bits whether 1 or 4 clips
// share the step (tests/test_gpu_pdec.py::test_pdec_batch_equals_single).
#pragma once
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace wm {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kG = 256;         // workgroups = CUs (one per CU)
constexpr int kNT = 256;        // threads per workgroup
constexpr int kPhases = 8;
constexpr int kPartG = 66;      // granules per cross-attention partial: o[64], max, sum
enum { P_X0 = 0, P_QKV, P_SELF, P_X1, P_XQ, P_XATT, P_X2, P_FF };

// global (not flat) address space for the plain loads: flat loads also count in lgkmcnt
template <typename P>
__device__ __forceinline__ const __attribute__((address_space(1))) P* gp(const P* p) {
    return (const __attribute__((address_space(1))) P*)p;
}

// The thread index as a value the compiler cannot treat as loop-invariant: per-lane addresses are then
// recomputed where they are used instead of being hoisted out of the layer loop and held in registers
// for the whole kernel (which cost ~250 registers of this one-wave-per-SIMD kernel)
__device__ __forceinline__ int ptid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// sum over the 8 lanes of a key row (quad xor 1, quad xor 2, half-row mirror)
__device__ __forceinline__ float sum8(float a) {
    a += dppf<0xB1>(a);
    a += dppf<0x4E>(a);
    return a + dppf<0x141>(a);
}
// Whole-wave reductions without LDS round trips: DPP inside each 16-lane row (xor 1, xor 2, half-row
// mirror, row mirror: every lane ends with its row's sum), then the four row sums read as scalars and
// added in row order, so every lane gets the same bits. (tools/probe/wave_reduce.hip checks the DPP
// lane maps on the device.)
__device__ __forceinline__ float lane_f(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float dppf_rows(float x) {  // rows outside the ROWS mask read 0
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float x) {
    x += dppf<0xB1>(x);
    x += dppf<0x4E>(x);
    x += dppf<0x141>(x);
    x += dppf<0x140>(x);  // every lane: its row's sum r_i
    x += dppf_rows<0x142, 0xA>(x);  // row_bcast:15 into rows 1, 3: r0 + r1, r2 + r3
    x += dppf_rows<0x143, 0xC>(x);  // row_bcast:31 into rows 2, 3: lane 63 = (r2 + r3) + (r0 + r1)
    return lane_f(x, 63);
}
__device__ __forceinline__ float wave_max(float x) {
    x = fmaxf(x, dppf<0xB1>(x));
    x = fmaxf(x, dppf<0x4E>(x));
    x = fmaxf(x, dppf<0x141>(x));
    x = fmaxf(x, dppf<0x140>(x));
    return fmaxf(fmaxf(lane_f(x, 0), lane_f(x, 16)), fmaxf(lane_f(x, 32), lane_f(x, 48)));
}
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)b, CTRL, 0xF, 0xF, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double lane_d(double x, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wave_sum_d(double x) {
    x += dppd<0xB1>(x);
    x += dppd<0x4E>(x);
    x += dppd<0x141>(x);
    x += dppd<0x140>(x);
    return (lane_d(x, 0) + lane_d(x, 16)) + (lane_d(x, 32) + lane_d(x, 48));
}


}  // namespace

// ---- the kernel -----------------------------------------------------------------------------------------
// Projection over the WG's column slice [c0, c1) of an [N][K] matrix: wave w takes columns c0 + w + 4 j
// (j < NCW), lane l the 16-byte vectors l + 64 v (v < NV) of each column. Weights are loaded into
// registers by `load` (before the phase's wait) and multiplied by `run` with the M rows staged in LDS.
// 8 weights of a GGML block (weights 8g .. 8g+7; r = {qs bytes 8(g&1) .. +7 (q4/q5) or 8g .. +7 (q8),
// q5 high bits, d | m << 16}) -> T, ggml's dequantize_row_* arithmetic (exact in f32, one rounding):
// gemm.hip qraw_deq with the type at run time
template <typename T>
__device__ __forceinline__ void deq8(int qt, uint32_t b0, uint32_t b1, uint32_t qh, uint32_t dm, int g, float (&wf)[8]) {
    const float dd = (float)__builtin_bit_cast(half_t, (uint16_t)(dm & 0xFFFF));
    const float mm = (float)__builtin_bit_cast(half_t, (uint16_t)(dm >> 16));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t byte = ((i < 4 ? b0 : b1) >> (8 * (i & 3))) & 0xFF;
        float v;
        if (qt == 8) {
            v = (float)(int8_t)byte * dd;
        } else {
            int x = (g >> 1) ? (int)(byte >> 4) : (int)(byte & 15);
            if (qt == 6 || qt == 7) x |= (int)((qh >> (8 * g + i)) & 1) << 4;
            if (qt == 3 || qt == 7) v = (float)x * dd + mm;
            else v = (float)(x - (qt == 6 ? 16 : 8)) * dd;
        }
        wf[i] = (float)(T)v;
    }
}

// Projection over the WG's column slice [c0, c1) of an [N][K] matrix: wave w takes columns c0 + w + 4 j
// (j < NCW). Plain weights: lane l the 16-byte vectors l + 64 v (v < NV) of each column. GGML blocks
// (PdecMat.qt != 0): lane l the 32-weight blocks l + 64 v (v < NB = NV / 3) of each column, their quant
// bytes in slots 2v (and 2v + 1 for q8_0) and {q5 high bits, d | m << 16} in slot 2 NB + v. Weights are
// loaded into registers by `load` (before the phase's wait) and multiplied by `run` with the M rows
// staged in LDS.
template <typename T, int NCW, int NV, bool Q>
struct ColSlice {
    static constexpr int NB = NV / 3;
    u32x4 w[NCW][NV];
    float bias[NCW];  // the bias of each of the lane's columns (loaded with the weights: no dependent load later)
    int c0, nc, K, qt;
    // pairs: slices of whole column pairs (2i, 2i + 1), for outputs handed off as packed T pairs
    // (every load is issued, lanes without data reading the zero page zp: a "cond ? load : 0" would
    // make the register's zero write wait for the load last in flight into it)
    __device__ __forceinline__ void load(const PdecMat& W, const float* b, int N, int K_, bool pairs, const void* zp) {
        K = K_;
        qt = Q ? W.qt : 0;
        const int w0 = blockIdx.x, u = pairs ? 2 : 1, nu = N / u;
        c0 = u * (int)((long)w0 * nu / kG);
        nc = u * (int)((long)(w0 + 1) * nu / kG) - c0;
        const int wave = ptid() >> 6, lane = ptid() & 63;
#pragma unroll
        for (int j = 0; j < NCW; j++) bias[j] = *gp(wave + 4 * j < nc ? b + c0 + wave + 4 * j : (const float*)zp);
        if (!Q) {
            const int nvec = K >> 3;
#pragma unroll
            for (int j = 0; j < NCW; j++) {
                const int cl = wave + 4 * j;
                const T* row = (const T*)W.w + (long)(c0 + (cl < nc ? cl : 0)) * K;
#pragma unroll
                for (int v = 0; v < NV; v++) {
                    const int vi = lane + 64 * v;
                    const T* src = (cl < nc && vi < nvec) ? row + vi * 8 : (const T*)zp;
                    w[j][v] = __builtin_nontemporal_load(gp((const u32x4*)src));
                }
            }
            return;
        }
        const int nblk = K >> 5;
        const uint8_t* qs = (const uint8_t*)W.w;
#pragma unroll
        for (int j = 0; j < NCW; j++) {
            const int cl = wave + 4 * j;
            const long n = c0 + (cl < nc ? cl : 0);
#pragma unroll
            for (int v = 0; v < NB; v++) {
                const int bi = lane + 64 * v;
                const bool in = cl < nc && bi < nblk;
                const long blk = n * nblk + (in ? bi : 0);
                const uint8_t* pa = !in ? (const uint8_t*)zp : (qt == 8 ? qs + n * K + 32L * bi : qs + n * (K / 2) + 16L * bi);
                const uint8_t* pb = (in && qt == 8) ? pa + 16 : (const uint8_t*)zp;
                const bool q5 = qt == 6 || qt == 7, wide = qt == 3 || qt == 7;  // (uniform)
                const u32x4 a = __builtin_nontemporal_load(gp((const u32x4*)pa));
                const u32x4 b = __builtin_nontemporal_load(gp((const u32x4*)pb));
                u32x4 meta;
                meta.x = *gp((in && q5) ? W.qh + blk : (const uint32_t*)zp);
                meta.y = wide ? *gp(in ? (const uint32_t*)W.dm + blk : (const uint32_t*)zp)
                              : (uint32_t)*gp(in ? W.dm + blk : (const uint16_t*)zp);
                meta.z = meta.w = 0;
                w[j][2 * v] = a;
                w[j][2 * v + 1] = b;
                w[j][2 * NB + v] = meta;
            }
        }
    }
    // acc[j][m] (all lanes) = sum_k xs[m][k] * W[c0 + wave + 4j][k]. The rows' LDS vectors of a step are
    // read unconditionally first (rows >= M and lanes past K read row 0 / vector 0: their weights are 0 or
    // their sums unused), so the reads are not serialised behind per-row branches.
    template <int MAXM>
    __device__ __forceinline__ void run(const T* xs, int ldx, int M, float (&acc)[NCW][MAXM]) const {
        const int lane = ptid() & 63;
#pragma unroll
        for (int j = 0; j < NCW; j++)
#pragma unroll
            for (int m = 0; m < MAXM; m++) acc[j][m] = 0.0f;
        auto fma8 = [&](const float (&wf)[8], int j, const u32x4 (&xv)[MAXM]) {
#pragma unroll
            for (int m = 0; m < MAXM; m++) {
                if (m < M) {  // (uniform)
                    const T* xe = (const T*)&xv[m];
                    float acc_ = acc[j][m];
#pragma unroll
                    for (int e = 0; e < 8; e++) acc_ = __builtin_fmaf((float)xe[e], wf[e], acc_);
                    acc[j][m] = acc_;
                }
            }
        };
        auto rows = [&](int koff, u32x4 (&xv)[MAXM]) {
#pragma unroll
            for (int m = 0; m < MAXM; m++) xv[m] = *(const u32x4*)(xs + (long)(m < M ? m : 0) * ldx + koff);
        };
        if (!Q) {
            const int nvec = K >> 3;
#pragma unroll
            for (int v = 0; v < NV; v++) {
                const int vi = lane + 64 * v;
                u32x4 xv[MAXM];
                rows(vi < nvec ? vi * 8 : 0, xv);  // (lanes past K hold zero weights)
#pragma unroll
                for (int j = 0; j < NCW; j++) {
                    // one weight vector widened at a time (the prefetched weights stay packed in registers)
                    float wf[8];
                    const T* we = (const T*)&w[j][v];
#pragma unroll
                    for (int e = 0; e < 8; e++) wf[e] = (float)we[e];
                    fma8(wf, j, xv);
                }
            }
        } else {
            const int nblk = K >> 5;
#pragma unroll
            for (int v = 0; v < NB; v++) {
                const int bi = lane + 64 * v;
                const int kb = bi < nblk ? bi * 32 : 0;  // (blocks past K: zero scales)
                u32x4 xv[4][MAXM];
#pragma unroll
                for (int g = 0; g < 4; g++) rows(kb + g * 8, xv[g]);
#pragma unroll
                for (int j = 0; j < NCW; j++) {
                    const u32x4 a = w[j][2 * v], b = w[j][2 * v + 1], meta = w[j][2 * NB + v];
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        float wf[8];
                        const uint32_t b0 = qt == 8 ? (g < 2 ? a[2 * g] : b[2 * g - 4]) : a[2 * (g & 1)];
                        const uint32_t b1 = qt == 8 ? (g < 2 ? a[2 * g + 1] : b[2 * g - 3]) : a[2 * (g & 1) + 1];
                        deq8<T>(qt, b0, b1, meta.x, meta.y, g, wf);
                        fma8(wf, j, xv[g]);
                    }
                }
            }
        }
#pragma unroll
        for (int m = 0; m < MAXM; m++)
            if (m < M) {  // (uniform; the column chains of a row interleave)
#pragma unroll
                for (int j = 0; j < NCW; j++) acc[j][m] = wave_sum(acc[j][m]);
            }
    }
};

// LayerNorm of rows [0, M <= 4) of xf (f32 [M][D], LDS) into out (T, row stride D; LDS or global),
// layernorm_kernel's arithmetic (double sums, separately rounded ops). The sums run in ONE canonical order
// whatever M is (a row's result must not depend on how many rows share the launch): a row's
// elements form 4 partitions q (k = l + 64 (q + 4 e), lane l), each summed sequentially over e and reduced
// over the wave's lanes by the same DPP tree, then the 4 partition sums added in q order. The WPR = 4 / M
// waves of a row (M <= 2; one wave per row for M > 2) take QW = 4 / WPR partitions each; all element reads
// are issued into registers at once (no branch per element). gamma / beta (gam, bet) are LDS copies staged a
// phase ahead (ln_issue / ln_commit in the kernel). lred: LDS doubles [2][kPdecMaxRows][4].
template <typename T, int D, int WPR>
__device__ __forceinline__ void ln_rows_w(const float* xf, int M, const float* gam, const float* bet, T* out, double* lred) {
#pragma clang fp contract(off)
    constexpr int QW = 4 / WPR;
    constexpr int NE = ((D + 63) / 64 + 3) / 4;
    const int tid = ptid(), wave = tid >> 6, lane = tid & 63;
    const int r = wave % WPR, m = wave / WPR;
    const bool on = m < M;
    const float* x = xf + (long)(on ? m : 0) * D;
    float v[QW][NE];
#pragma unroll
    for (int j = 0; j < QW; j++)
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const int k = lane + 64 * (r * QW + j + 4 * e);
            const float xv = x[k < D ? k : 0];
            v[j][e] = k < D ? xv : 0.0f;
        }
#pragma unroll
    for (int j = 0; j < QW; j++) {
        double s = 0.0;
#pragma unroll
        for (int e = 0; e < NE; e++) s += (double)v[j][e];
        s = wave_sum_d(s);
        if (lane == 0 && on) lred[m * 4 + r * QW + j] = s;
    }
    __syncthreads();
    const double st = (((0.0 + lred[m * 4]) + lred[m * 4 + 1]) + lred[m * 4 + 2]) + lred[m * 4 + 3];
    const float mean = (float)(st / D);
#pragma unroll
    for (int j = 0; j < QW; j++) {
        double s2 = 0.0;
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const int k = lane + 64 * (r * QW + j + 4 * e);
            v[j][e] = v[j][e] - mean;
            if (k < D) s2 += (double)(v[j][e] * v[j][e]);
        }
        s2 = wave_sum_d(s2);
        if (lane == 0 && on) lred[16 + m * 4 + r * QW + j] = s2;
    }
    __syncthreads();
    const double st2 = (((0.0 + lred[16 + m * 4]) + lred[16 + m * 4 + 1]) + lred[16 + m * 4 + 2]) + lred[16 + m * 4 + 3];
    const float variance = (float)(st2 / D);
    const float scale = 1.0f / sqrtf(variance + 1e-5f);
    if (on) {
#pragma unroll
        for (int j = 0; j < QW; j++)
#pragma unroll
            for (int e = 0; e < NE; e++) {
                const int k = lane + 64 * (r * QW + j + 4 * e);
                if (k < D) {
                    float t = v[j][e] * scale;
                    t = t * gam[k];
                    out[(long)m * D + k] = (T)(t + bet[k]);
                }
            }
    }
    __syncthreads();  // lred is rewritten by the next call
}
template <typename T, int D>
__device__ __forceinline__ void ln_rows(const float* xf, int M, const float* gam, const float* bet, T* out, double* lred) {
    if (M == 1) ln_rows_w<T, D, 4>(xf, M, gam, bet, out, lred);
    else if (M == 2) ln_rows_w<T, D, 2>(xf, M, gam, bet, out, lred);
    else ln_rows_w<T, D, 1>(xf, M, gam, bet, out, lred);
}

// ---- hand-offs: data-tagged granules ----------------------------------------------------------------------
// (MI355X_MICROARCH.md price table rows handoff-1to1 / allgather; cdna_hip_programming.md Guideline 16 R2)
// Every handed-off value travels as ONE naturally aligned 8-byte granule {tag, 32 bits of data} written by
// ONE sc1 store: the data is the flag, so a producer neither drains nor signals, and a consumer re-reads
// the granules it needs (sc1 loads) until every tag equals the phase's tag = layer * 8 + phase + 1 (never 0).
// The block is zeroed by a memset node before every launch. A buffer is reused by the next layer: safe
// because every layer's phase A reads all of x0, i.e. waits for every workgroup's last phase of the layer
// before, and every buffer of layer l + 1 is written after some workgroup's phase A of layer l + 1.
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ void put_g(unsigned long long* g, long i, unsigned tag, uint32_t bits) {
    __hip_atomic_store((gu64*)(g + i), ((unsigned long long)tag << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long get_g(const unsigned long long* g, long i) {
    return __hip_atomic_load((gu64*)(g + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (T)lo) | ((uint32_t)__builtin_bit_cast(uint16_t, (T)hi) << 16);
}
template <typename T>
__device__ __forceinline__ T lo_t(uint32_t v) { return __builtin_bit_cast(T, (uint16_t)(v & 0xFFFF)); }
template <typename T>
__device__ __forceinline__ T hi_t(uint32_t v) { return __builtin_bit_cast(T, (uint16_t)(v >> 16)); }

// The workgroup waits for granules addr(0 .. n-1) of g to carry `tag` (every thread its own i = tid + kNT u,
// U loads in flight per pass) and hands each granule's data to put(i, bits). A thread gives up after
// spin_ticks (100 MHz) or when another workgroup set the error word; false = give up (the caller returns,
// so every workgroup drains).
template <int U = 8, typename A, typename P>
__device__ __forceinline__ bool sweep(const unsigned long long* g, int n, unsigned tag, A addr, P put, unsigned* err,
                                      int* lflag, long spin_ticks) {
    bool ok = true;
    for (int b = 0; b < n && ok; b += kNT * U) {
        unsigned long long v[U];
        long t0 = 0;
        for (int it = 0;; it++) {
            bool done = true;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int i = b + ptid() + kNT * u;
                v[u] = i < n ? get_g(g, addr(i)) : (unsigned long long)tag << 32;
                done &= (unsigned)(v[u] >> 32) == tag;
            }
            if (done) break;
            const long now = (long)__builtin_amdgcn_s_memrealtime();
            if (it == 0) t0 = now;
            if (now - t0 > spin_ticks) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
            if ((it & 15) == 15 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (ok) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int i = b + ptid() + kNT * u;
                if (i < n) put(i, (uint32_t)v[u]);
            }
        }
    }
    if (!ok) *lflag = 0;  // set to 1 at the start; a workgroup that gave up exits, so it never goes back
    __syncthreads();
    const bool r = *lflag != 0;
    __syncthreads();
    return r;
}

// Attention over keys/values rows [r0, r1) of (K, V) [rows][64] T (at most 1536 rows): 32 lane groups of
// 8 lanes, a key row per group, chunks of 32 U rows. attn_load issues every K and V row load of the first
// chunk into registers (rows from earlier launches: before the wait for this step's query); row `fresh`
// (this position's k, v, handed off in this launch) is not loaded: attn_task takes it from fk / fv (LDS
// f32). Later chunks (ranges over 32 U rows) are loaded by attn_task into the K registers once the first
// chunk's keys are scored (MULTI; a task of one chunk compiles without the loops). Leaves in res (LDS): o[64] = sum_t p_t v_t, res[64] = max score, res[65] =
// sum_t p_t, with p_t = e^(s_t - max) (rounded to T as the P.V operand).
template <typename T, int U>
__device__ __forceinline__ void attn_rows(const T* __restrict__ X, int t0, int r1, int fresh, u32x4 (&r)[U], const void* zp) {
    const int lane8 = ptid() & 7, grp = ptid() >> 3;
    constexpr int NG = kNT / 8;
#pragma unroll
    for (int u = 0; u < U; u++) {  // (rows out of range read the zero page: every load is issued)
        const int t = t0 + grp + NG * u;
        r[u] = *gp((const u32x4*)((t < r1 && t != fresh) ? X + (long)t * 64 + lane8 * 8 : (const T*)zp));
    }
}
template <typename T, int U>
__device__ __forceinline__ void attn_load(const T* __restrict__ K, const T* __restrict__ V, int r0, int r1, int fresh,
                                          u32x4 (&rk)[U], u32x4 (&rv)[U], const void* zp) {
    attn_rows<T, U>(K, r0, r1, fresh, rk, zp);
    attn_rows<T, U>(V, r0, r1, fresh, rv, zp);
}
template <typename T, int U, bool MULTI>
__device__ __forceinline__ void attn_task(const float* qs, const T* __restrict__ K, const T* __restrict__ V, u32x4 (&rk)[U],
                                          const u32x4 (&rv)[U], int r0, int r1, int fresh, const float* fk, const float* fv,
                                          float* sc, float* red, float* res, const void* zp) {
    const int tid = ptid(), lane8 = tid & 7, grp = tid >> 3, wave = tid >> 6, lane = tid & 63;
    constexpr int NG = kNT / 8, CH = NG * U;
    // (branch-free per row: every LDS value is read up front, rows are selected, not branched on)
    float qv[8], fkv[8], fvv[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
        qv[e] = qs[lane8 * 8 + e];
        fkv[e] = fresh >= 0 ? fk[lane8 * 8 + e] : 0.0f;
        fvv[e] = fresh >= 0 ? fv[lane8 * 8 + e] : 0.0f;
    }
    float lmax = -INFINITY;
    for (int c0 = r0; c0 < (MULTI ? r1 : r0 + 1); c0 += CH) {
        if (c0 != r0) attn_rows<T, U>(K, c0, r1, fresh, rk, zp);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (c0 + NG * u >= r1) break;  // (uniform: a register row of no key is not computed)
            const int t = c0 + grp + NG * u;
            const T* ke = (const T*)&rk[u];
            const bool fr = t == fresh;
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e++) a += qv[e] * (fr ? fkv[e] : (float)ke[e]);
            a = sum8(a);
            if (t < r1 && lane8 == 0) sc[t - r0] = a;
            lmax = t < r1 ? fmaxf(lmax, a) : lmax;
        }
    }
    lmax = wave_max(lmax);
    if (lane == 0) red[wave] = lmax;
    __syncthreads();
    const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float lsum = 0.0f;
    for (int t = tid; t < r1 - r0; t += kNT) {
        const float e = __expf(sc[t] - mx);
        lsum += e;
        sc[t] = (float)(T)e;  // unnormalised weight rounded to T (the P.V operand)
    }
    lsum = wave_sum(lsum);
    __syncthreads();  // red[] read above by every wave, sc[] complete
    if (lane == 0) red[wave] = lsum;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] = 0.0f;
    auto pv = [&](int c0, const u32x4 (&r)[U]) {
        float p[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = c0 + grp + NG * u;
            p[u] = sc[t < r1 ? t - r0 : 0];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (c0 + NG * u >= r1) break;
            const int t = c0 + grp + NG * u;
            if (t < r1) {  // (rows past the range: their V registers are zero, skipped all the same)
                const bool fr = t == fresh;
                const T* ve = (const T*)&r[u];
#pragma unroll
                for (int e = 0; e < 8; e++) acc[e] += p[u] * (fr ? fvv[e] : (float)ve[e]);
            }
        }
    };
    pv(r0, rv);
    for (int c0 = r0 + CH; MULTI && c0 < r1; c0 += CH) {
        attn_rows<T, U>(V, c0, r1, fresh, rk, zp);
        pv(c0, rk);
    }
    // reduce over the 8 groups of a wave (lanes lane8 + 8 g): DPP for xor 8, permutes for 16 and 32; then over the 4 waves in LDS
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] += dppf<0x128>(acc[e]);  // xor 8 (row rotate by 8)
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] += __shfl_xor(acc[e], 16);  // (8 independent permutes per round)
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] += __shfl_xor(acc[e], 32);
    __syncthreads();
    float* ow = red + 8;  // [4 waves][64]
    if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; e++) ow[wave * 64 + lane * 8 + e] = acc[e];
    }
    __syncthreads();
    if (tid < 64) {
        res[tid] = (ow[tid] + ow[64 + tid]) + (ow[128 + tid] + ow[192 + tid]);
        if (tid == 0) {
            res[64] = mx;
            res[65] = (red[0] + red[1]) + (red[2] + red[3]);
        }
    }
    __syncthreads();
}

// The layer descriptors and the rows' token / position / slot are constant for the launch: read through
// the constant address space they are scalar loads (lgkmcnt), which never wait behind the vector-memory
// weight stream the way a vector load of a descriptor would (vmcnt retires in order).
typedef __attribute__((address_space(4))) const PdecLayer CLayer;
typedef __attribute__((address_space(4))) const PdecMat CMat;
typedef __attribute__((address_space(4))) const int CInt;
__device__ __forceinline__ PdecMat cmat(CMat& m) {
    PdecMat r;
    r.w = m.w;
    r.qh = m.qh;
    r.dm = m.dm;
    r.qt = m.qt;
    return r;
}

template <typename T, int D, int MAXM, bool Q>
__global__ void __launch_bounds__(kNT, 1) pdec_kernel(const PdecArgs a) {
    constexpr int H = D / 64;
    // register slots per lane per column: 16-byte vectors of plain weights, or 3 per 32-weight block
    constexpr int NV1 = Q ? 3 * ((D / 32 + 63) / 64) : (D / 8 + 63) / 64;          // K = d
    constexpr int NV4 = Q ? 3 * ((4 * D / 32 + 63) / 64) : (4 * D / 8 + 63) / 64;  // K = 4d
    // columns per workgroup: single columns (x rows, f32 granules) or pairs (packed T granules)
    constexpr int C1 = (D + kG - 1) / kG;
    constexpr int CQ = 2 * ((3 * D / 2 + kG - 1) / kG), CX = 2 * ((D / 2 + kG - 1) / kG), C4 = 2 * ((2 * D + kG - 1) / kG);
    constexpr int NC1 = (C1 + 3) / 4, NCQ = (CQ + 3) / 4, NCX = (CX + 3) / 4, NC4 = (C4 + 3) / 4;
    constexpr int CMAX = std::max(CQ, C4);  // (== PdecLds::cmax)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const PdecLds LL = pdec_lds(D, a.M, a.s_cross);
    T* xs = (T*)(smem + LL.xs);              // [rows][4d] T: the projections' rows
    float* xf = (float*)(smem + LL.xf);      // [rows][d] f32: a handed-off x row
    float* sc = (float*)(smem + LL.sc);      // scores [1536]
    float* red = (float*)(smem + LL.red);    // [8 + 256]
    float* qf = (float*)(smem + LL.qf);      // q, fresh k, fresh v [3][64]
    float* res = (float*)(smem + LL.res);    // attention result [64 + 2]
    float* ost = (float*)(smem + LL.ost);    // packed outputs [rows][CMAX]
    double* lred = (double*)(smem + LL.lred);  // LayerNorm partial sums [8]
    float* lnp = (float*)(smem + LL.lnp);    // LayerNorm gamma, beta [6][d]
    float* part = (float*)(smem + LL.part);  // the cross partials a merging workgroup gathers [S][66]
    int* lflag = (int*)(smem + LL.lflag);
    uint16_t* gtab = (uint16_t*)(smem + LL.gtab);  // GELU table, |x| < 10 (1-2 clips only)
    const bool ltab = MAXM == 1 || a.M <= 2;  // (the one-row build never reads the global table)

    const int M = a.M, L = a.L, w0 = blockIdx.x, tid = ptid(), wave = tid >> 6, lane = tid & 63;
    const PdecGranules& G = a.gr;
    unsigned long long* gb = (unsigned long long*)a.sync;
    unsigned long long *g_x0 = gb + G.x0, *g_x1 = gb + G.x1, *g_x2 = gb + G.x2, *g_qkv = gb + G.qkv;
    unsigned long long *g_so = gb + G.so, *g_qx = gb + G.qx, *g_xo = gb + G.xo, *g_ff = gb + G.ff;
    unsigned long long* g_part = gb + G.part;
    unsigned* err = (unsigned*)((char*)a.sync + G.err_bytes);
    const void* zp = (const char*)a.sync + G.zero_bytes;  // 256 zero bytes (zeroed per launch, never written)
    const T* te = (const T*)a.tok_emb;
    const float* te32 = a.te_f32 ? (const float*)a.tok_emb : nullptr;
    const T* self = (const T*)a.self_cache;
    const T* cross = (const T*)a.cross_cache;
    const long spin = a.spin_ticks;
    if (tid == 0) *lflag = 1;

    auto tag = [&](int l, int p) { return (unsigned)(l * 8 + p + 1); };
    // debug: per (WG, layer, phase) the 100 MHz clock when the phase's input arrived and when it published
    auto stamp = [&](int l, int p, int k) {
        if (a.stamps && tid == 0) a.stamps[(((long)w0 * a.L + l) * 8 + p) * 2 + k] = __builtin_amdgcn_s_memrealtime();
    };
    auto f32_of = [](uint32_t b) { return __builtin_bit_cast(float, b); };
    // sweeps of a whole buffer into LDS: x rows (f32) -> xf, packed T rows of width 2 * nw -> xs (row stride 2 * nw)
    auto sweep_xf = [&](unsigned long long* g, unsigned tg) {
        return sweep(g, M * D, tg, [](int i) { return (long)i; }, [&](int i, uint32_t b) { xf[i] = f32_of(b); }, err, lflag, spin);
    };
    auto sweep_xs = [&](unsigned long long* g, int nw, unsigned tg) {  // (the GELU rows: 2d granules per row)
        return sweep<16>(g, M * nw, tg, [](int i) { return (long)i; },
                     [&](int i, uint32_t b) { xs[2 * i] = lo_t<T>(b); xs[2 * i + 1] = hi_t<T>(b); }, err, lflag, spin);
    };
    // packed outputs: lane m of wave w holds column c0 + w + 4 j of row m; staged in LDS, then one granule per pair
    auto publish_pairs = [&](unsigned long long* g, int nw, int c0, int nc, unsigned tg) {
        __syncthreads();
        const int np = nc >> 1;
        for (int q = tid; q < M * np; q += kNT) {
            const int m = q / np, pi = q % np;
            put_g(g, (long)m * nw + (c0 >> 1) + pi, tg, pack2<T>(ost[m * CMAX + 2 * pi], ost[m * CMAX + 2 * pi + 1]));
        }
    };

    // the residual stream of the workgroup's own columns (c1_0 + wave + 4 j), lane m holding row m
    const int c1_0 = (int)((long)w0 * D / kG), c1_n = (int)((long)(w0 + 1) * D / kG) - c1_0;
    float xcur[NC1][MAXM];

    ColSlice<T, NCQ, NV1, Q> wq;
    ColSlice<T, NC1, NV1, Q> wo, wxo;
    ColSlice<T, NCX, NV1, Q> wxq;
    ColSlice<T, NC4, NV1, Q> wf1;
    ColSlice<T, NC1, NV4, Q> wf2;
    CLayer* LT = (CLayer*)a.layers;
    CInt* TOK = (CInt*)a.tok;
    CInt* POS = (CInt*)a.pos;
    CInt* SLOT = (CInt*)a.slot;
    wq.load(cmat(LT[0].qkv), LT[0].bqkv, 3 * D, D, true, zp);

    // LayerNorm gamma / beta into lnp slots (LN1 at 0, 1; cross LN at 2, 3; LN2 at 4, 5): issued into
    // registers ahead of the LayerNorm's phase (B for the cross LN, E for LN2, H for the next layer's LN1
    // or the final LN), stored after the next phase's wait (C, F) or before A's wait (LN1)
    constexpr int NGL = (2 * D + kNT - 1) / kNT;
    float lv[NGL];
    auto ln_issue = [&](const float* gw, const float* gb) {
#pragma unroll
        for (int u = 0; u < NGL; u++) {
            const int i = tid + kNT * u;
            const int ii = i < 2 * D ? i : 2 * D - 1;  // (2d is a multiple of 256 for every d built)
            lv[u] = *gp(ii < D ? gw + ii : gb + (ii - D));
        }
    };
    auto ln_commit = [&](int slot) {
#pragma unroll
        for (int u = 0; u < NGL; u++) {
            const int i = tid + kNT * u;
            if (i < 2 * D) lnp[slot * D + i] = lv[u];
        }
    };
    ln_issue(LT[0].ln1_w, LT[0].ln1_b);
    ln_commit(0);
    if (ltab) {  // ggml's f16 GELU table, the |x| < 10 bit patterns of each sign, into LDS
        constexpr int NV = 2 * kPdecGeluHalf * 2 / 16;  // 16-byte vectors
        u32x4 t[(NV + kNT - 1) / kNT];
#pragma unroll
        for (int u = 0; u < (NV + kNT - 1) / kNT; u++) {
            const int i = tid + kNT * u, half = i >= NV / 2, j = i - half * (NV / 2);
            t[u] = *gp((const u32x4*)(a.gelu_tab + (half ? 0x8000 : 0)) + (i < NV ? j : 0));
        }
#pragma unroll
        for (int u = 0; u < (NV + kNT - 1) / kNT; u++) {
            const int i = tid + kNT * u;
            if (i < NV) ((u32x4*)gtab)[i] = t[u];
        }
    }

    for (int l = 0; l < L; l++) {
        CLayer& W = LT[l];
        // ---- A: LN1 + QKV (q, k scaled; rounded to T) ----------------------------------------------------------
        {
            if (l == 0) {  // token + position embedding (embed_kernel's arithmetic)
                for (int i = tid; i < M * D; i += kNT) {
                    const int m = i / D, k = i % D;
                    const long t = TOK[m], p = POS[m];
                    xf[i] = (te32 ? te32[t * D + k] : (float)te[t * D + k]) + a.pos_d[p * D + k];
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < NC1; j++)
#pragma unroll
                    for (int m = 0; m < MAXM; m++) {
                        const int cl = wave + 4 * j;
                        xcur[j][m] = (m < M && cl < c1_n) ? xf[m * D + c1_0 + cl] : 0.0f;
                    }
            } else {
                ln_commit(0);  // (issued after the previous H's publish; the sweep's barriers order the reads)
                if (!sweep_xf(g_x0, tag(l, 0))) return;
            }
            stamp(l, 0, 0);
            ln_rows<T, D>(xf, M, lnp, lnp + D, xs, lred);
            __syncthreads();
            float acc[NCQ][MAXM];
            wq.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NCQ; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < wq.nc && lane == m) {
                        const int n = wq.c0 + cl;
                        float v = acc[j][m] + wq.bias[j];
                        if (n < 2 * D) v = v * a.k_scale;
                        ost[m * CMAX + cl] = (float)(T)v;
                    }
                }
            publish_pairs(g_qkv, 3 * D / 2, wq.c0, wq.nc, tag(l, 1));
            stamp(l, 0, 1);
        }
        // ---- B: self attention of (row, head) over the cache + this position (one task each) ----------------
        {
            // phase C's and D's weights and D's LayerNorm parameters land under this phase: an attention
            // workgroup (whose output everyone waits for) issues D's after its query arrived, so its wait
            // is not behind them, and starts C with all of them in registers
            wo.load(cmat(W.o), W.bo, D, D, false, zp);
            auto ahead = [&] {
                wxq.load(cmat(W.xq), W.bxq, D, D, true, zp);
                ln_issue(W.lnx_w, W.lnx_b);
            };
            if (w0 >= M * H) ahead();
            if (w0 < M * H) {
                const int m = w0 / H, h = w0 % H;
                const int pos = POS[m], nkv = pos + 1;
                const long sl = SLOT[m];
                T* Kc = (T*)self + (((sl * L + l) * 2 + 0) * H + h) * (long)a.n_text_ctx * 64;
                T* Vc = (T*)self + (((sl * L + l) * 2 + 1) * H + h) * (long)a.n_text_ctx * 64;
                u32x4 rk[16], rv[16];
                attn_load<T, 16>(Kc, Vc, 0, nkv, pos, rk, rv, zp);  // the cached rows land while the query is awaited
                // q, k, v of head h: granules h * 32 + i of each third of the row
                if (!sweep<1>(g_qkv, 96, tag(l, 1), [&](int i) { return (long)m * (3 * D / 2) + (i >> 5) * (D / 2) + h * 32 + (i & 31); },
                           [&](int i, uint32_t b) {
                               qf[2 * i] = (float)lo_t<T>(b);
                               qf[2 * i + 1] = (float)hi_t<T>(b);
                           }, err, lflag, spin))
                    return;
                stamp(l, 1, 0);
                ahead();
                if (tid < 64) {  // append this position's k, v to the cache (read by the next steps' launches)
                    Kc[(long)pos * 64 + tid] = (T)qf[64 + tid];
                    Vc[(long)pos * 64 + tid] = (T)qf[128 + tid];
                }
                attn_task<T, 16, false>(qf, Kc, Vc, rk, rv, 0, nkv, pos, qf + 64, qf + 128, sc, red, res, zp);
                if (tid < 32) {
                    const float inv = 1.0f / res[65];
                    put_g(g_so, (long)m * (D / 2) + h * 32 + tid, tag(l, 2), pack2<T>(res[2 * tid] * inv, res[2 * tid + 1] * inv));
                }
                stamp(l, 1, 1);
            }
        }
        // ---- C: out projection + residual -----------------------------------------------------------------------
        {
            if (!sweep_xs(g_so, D / 2, tag(l, 2))) return;
            ln_commit(2);  // (read after phase D's sweep barriers)
            stamp(l, 2, 0);
            float acc[NC1][MAXM];
            wo.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < wo.nc && lane == m) {
                        const int n = wo.c0 + cl;
                        xcur[j][m] = (acc[j][m] + wo.bias[j]) + xcur[j][m];
                        put_g(g_x1, (long)m * D + n, tag(l, 3), __builtin_bit_cast(uint32_t, xcur[j][m]));
                    }
                }
            stamp(l, 2, 1);
        }
        // ---- D: LN + cross-Q projection (scaled; rounded to T) --------------------------------------------------
        {
            if (!sweep_xf(g_x1, tag(l, 3))) return;
            stamp(l, 3, 0);
            ln_rows<T, D>(xf, M, lnp + 2 * D, lnp + 3 * D, xs, lred);
            __syncthreads();
            float acc[NCX][MAXM];
            wxq.template run<MAXM>(xs, D, M, acc);
            wxo.load(cmat(W.xo), W.bxo, D, D, false, zp);  // (after the GEMV: its operand waits are not behind it)
#pragma unroll
            for (int j = 0; j < NCX; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < wxq.nc && lane == m) {
                        const int n = wxq.c0 + cl;
                        ost[m * CMAX + cl] = (float)(T)((acc[j][m] + wxq.bias[j]) * a.k_scale);
                    }
                }
            publish_pairs(g_qx, D / 2, wxq.c0, wxq.nc, tag(l, 4));
            stamp(l, 3, 1);
        }
        // ---- E: cross attention over the cached K/V, split over keys; split 0 of a (row, head) merges -----------
        // The split count is a function of the model shape only (pdec_cross_splits): M * H * S tasks, dealt to
        // the workgroups round-robin (task t by workgroup t % 256). Every task's attention and publish comes
        // before any merge waits, so no wait can stand behind another workgroup's unfinished task.
        {
            // phase G's weights and LayerNorm parameters: a task workgroup issues them once its outputs are
            // out (issuing 4d x d of weights stalls the wave while the memory pipeline is full)
            auto ahead = [&] {
                ln_issue(W.ln2_w, W.ln2_b);
                wf1.load(cmat(W.f1), W.b1, 4 * D, D, true, zp);
            };
            const int S = a.s_cross, NT = M * H * S;
            const bool multi = NT > kG;  // (uniform) some workgroups take two or more tasks
            const int T_ = a.n_audio_ctx;
            if (w0 >= NT) ahead();
            for (int t = w0; t < NT; t += kG) {
                const int m = t / (H * S), h = (t / S) % H, s = t % S;
                const int r0 = (int)((long)s * T_ / S), r1 = (int)((long)(s + 1) * T_ / S);
                const long sl = SLOT[m];
                const T* Kc = cross + (((sl * L + l) * 2 + 0) * H + h) * (long)T_ * 64;
                const T* Vc = cross + (((sl * L + l) * 2 + 1) * H + h) * (long)T_ * 64;
                u32x4 rk[8], rv[8];
                attn_load<T, 8>(Kc, Vc, r0, r1, -1, rk, rv, zp);  // constant for the window: issued before the wait
                if (!sweep<1>(g_qx, 32, tag(l, 4), [&](int i) { return (long)m * (D / 2) + h * 32 + i; },
                           [&](int i, uint32_t b) {
                               qf[2 * i] = (float)lo_t<T>(b);
                               qf[2 * i + 1] = (float)hi_t<T>(b);
                           }, err, lflag, spin))
                    return;
                if (t == w0) stamp(l, 4, 0);
                attn_task<T, 8, true>(qf, Kc, Vc, rk, rv, r0, r1, -1, qf, qf, sc, red, res, zp);  // (no fresh row)
                // the partial {o[64], max, sum} as 66 granules (split 0 of a one-task workgroup keeps its own in LDS)
                unsigned long long* gp0 = g_part + (long)(t - s) * kPartG;
                if (s > 0 || multi) {
                    if (tid < kPartG) put_g(gp0 + (long)s * kPartG, tid, tag(l, 4), __builtin_bit_cast(uint32_t, res[tid]));
                } else if (tid < kPartG) {
                    part[tid] = res[tid];
                }
                if (t + kG >= NT) ahead();  // (after the workgroup's last task: lands while the other splits finish)
            }
            // merges: o = sum_s e^(m_s - m) o_s / sum_s e^(m_s - m) l_s, by split 0's workgroup
            for (int t = w0; t < NT; t += kG) {
                if (t % S != 0) continue;  // (uniform)
                const int m = t / (H * S), h = (t / S) % H;
                unsigned long long* gp0 = g_part + (long)t * kPartG;
                const int g0 = multi ? 0 : kPartG;  // one-task workgroups hold split 0's partial already
                if (!sweep<16>(gp0 + g0, S * kPartG - g0, tag(l, 4), [](int i) { return (long)i; },
                               [&](int i, uint32_t b) { part[g0 + i] = f32_of(b); }, err, lflag, spin))
                    return;
                if (tid < 64) {
                    float mx = -INFINITY;
                    for (int u = 0; u < S; u++) mx = fmaxf(mx, part[u * kPartG + 64]);
                    float Lsum = 0.0f, o = 0.0f;
                    for (int u = 0; u < S; u++) {
                        const float ms = part[u * kPartG + 64];
                        const float wgt = ms != -INFINITY ? __expf(ms - mx) : 0.0f;
                        Lsum += wgt * part[u * kPartG + 65];
                        o += wgt * part[u * kPartG + tid];
                    }
                    res[tid] = o * (1.0f / Lsum);
                }
                __syncthreads();
                if (tid < 32) put_g(g_xo, (long)m * (D / 2) + h * 32 + tid, tag(l, 5), pack2<T>(res[2 * tid], res[2 * tid + 1]));
                __syncthreads();  // part and res read before the next merge / layer rewrites them
            }
            if (w0 < NT) stamp(l, 4, 1);
        }
        // ---- F: cross-out projection + residual -------------------------------------------------------------------
        {
            if (!sweep_xs(g_xo, D / 2, tag(l, 5))) return;
            ln_commit(4);
            stamp(l, 5, 0);
            float acc[NC1][MAXM];
            wxo.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < wxo.nc && lane == m) {
                        const int n = wxo.c0 + cl;
                        xcur[j][m] = (acc[j][m] + wxo.bias[j]) + xcur[j][m];
                        put_g(g_x2, (long)m * D + n, tag(l, 6), __builtin_bit_cast(uint32_t, xcur[j][m]));
                    }
                }
            stamp(l, 5, 1);
        }
        // ---- G: LN + FC1 + GELU (ggml's f16 table; rounded to T) ----------------------------------------------
        {
            if (!sweep_xf(g_x2, tag(l, 6))) return;
            stamp(l, 6, 0);
            ln_rows<T, D>(xf, M, lnp + 4 * D, lnp + 5 * D, xs, lred);
            __syncthreads();
            float acc[NC4][MAXM];
            wf1.template run<MAXM>(xs, D, M, acc);
            // GELU by ggml's f16 table (LDS up to 2 clips, the global table past that); phase H's weights
            // are issued after the publish
            float gx[NC4];
            uint16_t gt[NC4];
#pragma unroll
            for (int j = 0; j < NC4; j++) {
                const int cl = wave + 4 * j;
                gx[j] = 0.0f;
#pragma unroll
                for (int m = 0; m < MAXM; m++)
                    if (lane == m) gx[j] = acc[j][m] + wf1.bias[j];
                const unsigned hb = (lane < M && cl < wf1.nc) ? __builtin_bit_cast(uint16_t, (half_t)gx[j]) : 0u;
                const unsigned hq = hb & 0x7FFF;
                if (ltab) {
                    // |h| < 10 from LDS; past it the table holds h itself (tanhf rounds to 1), -0 for the
                    // negatives (1 + tanhf = 0) and the NaNs: no global lookup, so using the result never
                    // waits on the weight stream issued below
                    const uint16_t tv = gtab[(hq < kPdecGeluHalf ? hq : 0u) + (hb >> 15) * kPdecGeluHalf];
                    gt[j] = hq < kPdecGeluHalf ? tv : (uint16_t)((hq > 0x7C00u || !(hb & 0x8000u)) ? hb : 0x8000u);
                } else {
                    gt[j] = *gp(a.gelu_tab + hb);
                }
            }
#pragma unroll
            for (int j = 0; j < NC4; j++) {
                const int cl = wave + 4 * j;
                if (lane < M && cl < wf1.nc) {
                    const float x = gx[j];
                    const float g = x <= -10.0f ? 0.0f : (x >= 10.0f ? x : (float)__builtin_bit_cast(half_t, gt[j]));
                    ost[lane * CMAX + cl] = (float)(T)g;
                }
            }
            publish_pairs(g_ff, 2 * D, wf1.c0, wf1.nc, tag(l, 7));
            stamp(l, 6, 1);
            asm volatile("" ::: "memory");
            wf2.load(cmat(W.f2), W.b2, D, 4 * D, false, zp);
        }
        // ---- H: FC2 + residual -> the next layer's x0 ------------------------------------------------------------
        {
            if (!sweep_xs(g_ff, 2 * D, tag(l, 7))) return;
            stamp(l, 7, 0);
            float acc[NC1][MAXM];
            wf2.template run<MAXM>(xs, 4 * D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < wf2.nc && lane == m) {
                        const int n = wf2.c0 + cl;
                        xcur[j][m] = (acc[j][m] + wf2.bias[j]) + xcur[j][m];
                        put_g(g_x0, (long)m * D + n, tag(l + 1, 0), __builtin_bit_cast(uint32_t, xcur[j][m]));
                    }
                }
            stamp(l, 7, 1);
            asm volatile("" ::: "memory");
            if (l + 1 < L) {  // the next layer's QKV weights and LN1 (its sweep is behind them: A needs both)
                wq.load(cmat(LT[l + 1].qkv), LT[l + 1].bqkv, 3 * D, D, true, zp);
                ln_issue(LT[l + 1].ln1_w, LT[l + 1].ln1_b);
            } else {
                ln_issue(a.lnd_w, a.lnd_b);  // the final LayerNorm (workgroup 0)
            }
        }
    }
    // ---- final LayerNorm of every row -> the logits GEMM's input ----------------------------------------------
    if (w0 == 0) {
        ln_commit(0);
        if (!sweep_xf(g_x0, tag(L, 0))) return;
        ln_rows<T, D>(xf, M, lnp, lnp + D, (T*)a.out_dh, lred);
    }
}

// one launcher per (compute type, weight form); the GGML-block form is built for the catalog's quantized
// shapes (small 768, medium 1024, large-v3 1280)
// MAXM: the rows the kernel's register arrays and unrolled loops are built for (1 for the app's one clip
// per call: a much smaller loop body, 4 otherwise)
template <typename T, bool Q, int MAXM>
void pdec_launch_t(const PdecArgs& a, size_t lds, hipStream_t st) {
#define WM_PD(DD)                                                        \
    case DD:                                                            \
        pdec_kernel<T, DD, MAXM, Q><<<kG, kNT, lds, st>>>(a);           \
        return;
    if constexpr (!Q) {
        switch (a.d) { WM_PD(384) WM_PD(512) default: break; }
    }
    switch (a.d) { WM_PD(768) WM_PD(1024) WM_PD(1280) default: break; }
#undef WM_PD
    WM_FAIL("pdec: d %d%s", a.d, Q ? " (GGML blocks)" : "");
}

}  // namespace wm
