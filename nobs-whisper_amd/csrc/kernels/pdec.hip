// Persistent decode step for few clips: the whole decoder (every layer) of one decode step in ONE
// launch, its phases handing off through the L2 with counters instead of kernel boundaries
// (the hot loop of whisper_full: whisper.rs:127-129 -> state.rs:147; the app
// transcribes one clip per call, so this is the latency its user feels).
//
// Why: at one clip a large-v3 decoder layer streams 46 MB of weights +
// 7.7 MB of cross K/V (~8 us at HBM speed) but took ~78 us as 8 dependent launches of 5-15 us each:
// launch boundaries, ramp-up and dependent-load latency, not bytes. Here the grid is one 256-thread
// workgroup per CU (G = 256), resident for the whole step:
//   per layer, 8 phases:  A  LN1 + QKV projection (+ q/k scale, rounding to T)        all WGs, column slices
//                         B  self attention over the cache, split over keys            (clip, head, split) tasks
//                         C  split merge + out projection + residual                   all WGs
//                         D  LN + cross-Q projection (+ scale)                         all WGs
//                         E  cross attention over the cached K/V, split over keys      (clip, head, split) tasks
//                         F  split merge + cross-out projection + residual             all WGs
//                         G  LN + FC1 + GELU (ggml's f16 table)                       all WGs
//                         H  FC2 + residual                                            all WGs
//   then the final LayerNorm of every row (the logits GEMM is the next launch).
// A projection phase: each WG owns a contiguous slice of output columns (N / G of them), so its weights
// are ONE contiguous range of the [N][K] matrix; it issues their loads into registers BEFORE waiting for
// the phase's input, so the weight stream of phase p overlaps the hand-off of phase p-1 (the loader-runs-
// ahead idea of MI355X_MICROARCH.md "prefetch-credit", in registers instead of an LDS ring). Every WG
// gathers the whole (small) input vector: M rows of d, computes the LayerNorm itself (ggml_norm: double
// sums) and stages the rows in LDS as T; one wave per output column, lanes split K, f32 accumulation.
//
// Hand-offs (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", Valid forms, table
// row 1): every payload word is stored write-through (sc1) and drained (s_waitcnt vmcnt(0) in every
// storing wave), the workgroup barrier, then ONE lane adds 1 to the phase's counter (agent-scope atomic),
// sharded per XCD (8 words, blockIdx % 8) so 256 arrivals spread over 8 lines; the consumer's wave 0
// polls the 8 shards with sc1 loads (+ s_sleep) until all G workgroups arrived, the workgroup barrier,
// then EVERY load of a handed-off byte is an sc1 load (no acquire fence needed: the row's conditions
// hold). Counters are per (layer, phase), zeroed by a memset node before every launch.
// Bounded spins: a wait gives up after ~50 ms (s_memrealtime, 100 MHz), sets the error word and the
// workgroup exits; every other wait sees the error word and exits too, so the grid always drains (e.g.
// when another kernel holds CUs and not all 256 workgroups can be resident). The host then re-runs the
// step on the launch-per-kernel path (engine.cpp), so a failed launch costs time, never results.
//
// Numerics (vs oracle/oracle_whisper.cpp, ggml's): LayerNorm as layernorm_kernel (double sums, separately
// rounded ops, output rounded to T = ggml's f16 src1); projections f32-accumulated products of T
// operands; q, k scaled by d_head^-0.25 then rounded to T, v rounded to T (the self cache holds T);
// attention scores f32, softmax in f32 over each split with the split's own max, the unnormalised
// weights rounded to T before P.V (ggml rounds the normalised P to f16: another rounding point, the
// same precision), splits merged with exp(m_s - m) in f32 and the result rounded to T (the out
// projection's src1). Results per row do not depend on the other rows' presence for a fixed (M, H):
// the split count is a function of M (batch == single holds within the path at equal M only).
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace wm {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kG = 256;         // workgroups = CUs (one per CU)
constexpr int kNT = 256;        // threads per workgroup
constexpr int kPhases = 8;
constexpr int kPartStride = 68; // floats per attention partial: m, l, pad x2, o[64]
enum { P_X0 = 0, P_QKV, P_SELF, P_X1, P_XQ, P_XATT, P_X2, P_FF };

// global (not flat) address space for the plain loads: flat loads also count in lgkmcnt
template <typename P>
__device__ __forceinline__ const __attribute__((address_space(1))) P* gp(const P* p) {
    return (const __attribute__((address_space(1))) P*)p;
}

__device__ __forceinline__ float ld_sc1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fffffff, 0x00020000);
}
// 16-byte sc1 load / store of a buffer written inside this launch (aux 16 = sc1)
__device__ __forceinline__ float4 ld4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
    return __builtin_bit_cast(float4, v);
}
__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 16);
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
__device__ __forceinline__ float wave_sum(float x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ float wave_max(float x) {
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    return x;
}

__device__ __forceinline__ float gelu_t(float x, const uint16_t* tab) {  // == gelu_ggml (gemm.hip gelu_tab)
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return (float)__builtin_bit_cast(half_t, tab[__builtin_bit_cast(uint16_t, (half_t)x)]);
}

}  // namespace

// ---- synchronisation ---------------------------------------------------------------------------------
__device__ __forceinline__ void pd_signal(unsigned* sync, int idx) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 payload stores have landed
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(sync + idx * 8 + (blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0 polls the 8 shards of counter idx until every workgroup arrived; false = give up (error word set)
__device__ __forceinline__ bool pd_wait(unsigned* sync, unsigned* err, int idx, int* lflag, long spin_ticks) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const unsigned need = lane < 8 ? (unsigned)((kG - lane + 7) / 8) : 0u;
        const unsigned* c = sync + idx * 8 + (lane & 7);
        const long t0 = (long)__builtin_amdgcn_s_memrealtime();
        int ok = 1;
        for (;;) {
            const unsigned v = lane < 8 ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            if (__all(v >= need)) break;
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
            if ((long)__builtin_amdgcn_s_memrealtime() - t0 > spin_ticks) {
                if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) *lflag = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the payload loads below the poll
    __syncthreads();
    const int ok = *lflag;
    __syncthreads();  // lflag is rewritten by the next wait
    return ok != 0;
}

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
template <typename T, int NCW, int NV>
struct ColSlice {
    static constexpr int NB = NV / 3;
    u32x4 w[NCW][NV];
    int c0, nc, K, qt;
    __device__ __forceinline__ void load(const PdecMat& W, int N, int K_) {
        K = K_;
        qt = W.qt;
        const int w0 = blockIdx.x;
        c0 = (int)((long)w0 * N / kG);
        nc = (int)((long)(w0 + 1) * N / kG) - c0;
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (qt == 0) {
            const int nvec = K >> 3;
#pragma unroll
            for (int j = 0; j < NCW; j++) {
                const int cl = wave + 4 * j;
                const T* row = (const T*)W.w + (long)(c0 + (cl < nc ? cl : 0)) * K;
#pragma unroll
                for (int v = 0; v < NV; v++) {
                    const int vi = lane + 64 * v;
                    w[j][v] = (cl < nc && vi < nvec) ? __builtin_nontemporal_load(gp((const u32x4*)(row + vi * 8)))
                                                     : (u32x4){0, 0, 0, 0};
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
                u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0}, meta = {0, 0, 0, 0};
                if (cl < nc && bi < nblk) {
                    const long blk = n * nblk + bi;
                    if (qt == 8) {
                        a = __builtin_nontemporal_load(gp((const u32x4*)(qs + n * K + 32L * bi)));
                        b = __builtin_nontemporal_load(gp((const u32x4*)(qs + n * K + 32L * bi + 16)));
                    } else {
                        a = __builtin_nontemporal_load(gp((const u32x4*)(qs + n * (K / 2) + 16L * bi)));
                    }
                    meta.x = (qt == 6 || qt == 7) ? *gp(W.qh + blk) : 0u;
                    meta.y = (qt == 3 || qt == 7) ? *gp((const uint32_t*)W.dm + blk) : (uint32_t)*gp(W.dm + blk);
                }
                w[j][2 * v] = a;
                w[j][2 * v + 1] = b;
                w[j][2 * NB + v] = meta;
            }
        }
    }
    // acc[j][m] (all lanes) = sum_k xs[m][k] * W[c0 + wave + 4j][k]
    template <int MAXM>
    __device__ __forceinline__ void run(const T* xs, int ldx, int M, float (&acc)[NCW][MAXM]) const {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < NCW; j++)
#pragma unroll
            for (int m = 0; m < MAXM; m++) acc[j][m] = 0.0f;
        auto fma8 = [&](const float (&wf)[8], int j, int koff) {
#pragma unroll
            for (int m = 0; m < MAXM; m++) {
                if (m >= M) break;
                const u32x4 xv = *(const u32x4*)(xs + (long)m * ldx + koff);
                const T* xe = (const T*)&xv;
                float acc_ = acc[j][m];
#pragma unroll
                for (int e = 0; e < 8; e++) acc_ = __builtin_fmaf((float)xe[e], wf[e], acc_);
                acc[j][m] = acc_;
            }
        };
        if (qt == 0) {
            const int nvec = K >> 3;
#pragma unroll
            for (int v = 0; v < NV; v++) {
                const int vi = lane + 64 * v;
                if (vi >= nvec) break;
#pragma unroll
                for (int j = 0; j < NCW; j++) {
                    // one weight vector widened at a time (the prefetched weights stay packed in registers)
                    float wf[8];
                    const T* we = (const T*)&w[j][v];
#pragma unroll
                    for (int e = 0; e < 8; e++) wf[e] = (float)we[e];
                    fma8(wf, j, vi * 8);
                }
            }
        } else {
            const int nblk = K >> 5;
#pragma unroll
            for (int v = 0; v < NB; v++) {
                const int bi = lane + 64 * v;
                if (bi >= nblk) break;
#pragma unroll
                for (int j = 0; j < NCW; j++) {
                    const u32x4 a = w[j][2 * v], b = w[j][2 * v + 1], meta = w[j][2 * NB + v];
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        float wf[8];
                        const uint32_t b0 = qt == 8 ? (g < 2 ? a[2 * g] : b[2 * g - 4]) : a[2 * (g & 1)];
                        const uint32_t b1 = qt == 8 ? (g < 2 ? a[2 * g + 1] : b[2 * g - 3]) : a[2 * (g & 1) + 1];
                        deq8<T>(qt, b0, b1, meta.x, meta.y, g, wf);
                        fma8(wf, j, bi * 32 + g * 8);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NCW; j++)
#pragma unroll
            for (int m = 0; m < MAXM; m++)
                if (m < M && wave + 4 * j < nc) acc[j][m] = wave_sum(acc[j][m]);
    }
};

// LayerNorm of rows [0, M) of x (f32 [M][D], written inside this launch: sc1 loads) into xs (T, LDS,
// row stride D): one wave per row, layernorm_kernel's arithmetic (double sums, separately rounded ops)
template <typename T, int D>
__device__ __forceinline__ void ln_rows(const float* x, int M, const float* __restrict__ w, const float* __restrict__ b,
                                        T* xs, bool from_emb, const T* te, const float* te32, const float* pe,
                                        const int* tok, const int* pos) {
#pragma clang fp contract(off)
    constexpr int NPL = (D + 63) / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int m = wave; m < M; m += 4) {
        float v[NPL];
        if (from_emb) {  // layer 0: token + position embedding (embed_kernel's arithmetic)
            const long t = tok[m], p = pos[m];
#pragma unroll
            for (int e = 0; e < NPL; e++) {
                const int k = lane + 64 * e;
                v[e] = k < D ? (te32 ? te32[t * D + k] : (float)te[t * D + k]) + pe[p * D + k] : 0.0f;
            }
        } else {
#pragma unroll
            for (int e = 0; e < NPL; e++) {
                const int k = lane + 64 * e;
                v[e] = k < D ? ld_sc1(x + (long)m * D + k) : 0.0f;
            }
        }
        double s = 0.0;
#pragma unroll
        for (int e = 0; e < NPL; e++) s += (double)v[e];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        const float mean = (float)(s / D);
        double s2 = 0.0;
#pragma unroll
        for (int e = 0; e < NPL; e++) {
            const int k = lane + 64 * e;
            v[e] = v[e] - mean;
            if (k < D) s2 += (double)(v[e] * v[e]);
        }
        for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
        const float variance = (float)(s2 / D);
        const float scale = 1.0f / sqrtf(variance + 1e-5f);
#pragma unroll
        for (int e = 0; e < NPL; e++) {
            const int k = lane + 64 * e;
            if (k < D) {
                float t = v[e] * scale;
                t = t * w[k];
                xs[(long)m * D + k] = (T)(t + b[k]);
            }
        }
    }
}

// Merge the attention partials of every (row, head) (S splits each) into xs (T [M][D], LDS): thread
// per (row, head, 4 dims); o = sum_s e^(m_s - m) o_s / sum_s e^(m_s - m) l_s. Branch-free, the loads of
// 8 splits issued together (an empty split holds m = -inf, l = 0, o = 0 and gets weight 0).
template <typename T, int D>
__device__ __forceinline__ void merge_parts(const float* part, int M, int S, T* xs) {
    constexpr int H = D / 64;
    const __amdgpu_buffer_rsrc_t r = rsrc(part);
    for (int q = threadIdx.x; q < M * H * 16; q += kNT) {
        const int mh = q >> 4, j4 = (q & 15) * 4;
        const int base = mh * S * kPartStride;
        float mx = -INFINITY;
        for (int s0 = 0; s0 < S; s0 += 8) {
            float ms[8];
#pragma unroll
            for (int u = 0; u < 8; u++) ms[u] = s0 + u < S ? ld_sc1(part + base + (s0 + u) * kPartStride) : -INFINITY;
#pragma unroll
            for (int u = 0; u < 8; u++) mx = fmaxf(mx, ms[u]);
        }
        float L = 0.0f;
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s0 = 0; s0 < S; s0 += 8) {
            float2 ml[8];
            float4 os[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int sb = base + min(s0 + u, S - 1) * kPartStride;
                const float4 h = ld4_sc1(r, sb * 4);  // m, l, pad, pad
                ml[u] = make_float2(h.x, h.y);
                os[u] = ld4_sc1(r, (sb + 4 + j4) * 4);
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const float wgt = (s0 + u < S && ml[u].x != -INFINITY) ? __expf(ml[u].x - mx) : 0.0f;
                L += wgt * ml[u].y;
                o.x += wgt * os[u].x; o.y += wgt * os[u].y; o.z += wgt * os[u].z; o.w += wgt * os[u].w;
            }
        }
        const float inv = 1.0f / L;
        const int m = mh / H, h = mh % H;
        T* dst = xs + (long)m * D + h * 64 + j4;
        dst[0] = (T)(o.x * inv); dst[1] = (T)(o.y * inv); dst[2] = (T)(o.z * inv); dst[3] = (T)(o.w * inv);
    }
}

// One attention task: query q (64 f32 in LDS), keys/values rows [r0, r1) of (K, V) [rows][64] T, plus,
// if fresh >= 0 and in range, row `fresh` taken from fk / fv (LDS f32) instead of the cache. Writes the
// partial {max, sum, 0, 0, o[64]} (f32) to out with sc1 stores. 32 lane groups of 8 lanes, a key row
// per group and U rows in flight per group (every load of a chunk issued before its first use; the
// first V chunk is issued under the softmax).
template <typename T>
__device__ __forceinline__ void attn_task(const float* qs, const T* __restrict__ K, const T* __restrict__ V, int r0, int r1,
                                          int fresh, const float* fk, const float* fv, float* sc, float* red, float* out) {
    const int tid = threadIdx.x, lane8 = tid & 7, grp = tid >> 3, wave = tid >> 6, lane = tid & 63;
    constexpr int NG = kNT / 8, U = 8, CH = NG * U;
    const u32x4 zero = {0, 0, 0, 0};
    float qv[8];
#pragma unroll
    for (int e = 0; e < 8; e++) qv[e] = qs[lane8 * 8 + e];
    auto load_rows = [&](const T* base, int t0, u32x4 (&raw)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            raw[u] = (t < r1 && t != fresh) ? *gp((const u32x4*)(base + (long)t * 64 + lane8 * 8)) : zero;
        }
    };
    float lmax = -INFINITY;
    u32x4 raw[U];
    for (int t0 = r0 + grp; t0 < r1; t0 += CH) {
        load_rows(K, t0, raw);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            const T* ke = (const T*)&raw[u];
            float a = 0.0f;
            if (t == fresh) {
#pragma unroll
                for (int e = 0; e < 8; e++) a += qv[e] * fk[lane8 * 8 + e];
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) a += qv[e] * (float)ke[e];
            }
            a = sum8(a);
            if (t < r1) {
                if (lane8 == 0) sc[t - r0] = a;
                lmax = fmaxf(lmax, a);
            }
        }
    }
    load_rows(V, r0 + grp, raw);  // the first V chunk lands under the softmax
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
    for (int t0 = r0 + grp; t0 < r1; t0 += CH) {
        if (t0 != r0 + grp) load_rows(V, t0, raw);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            if (t >= r1) break;
            const float p = sc[t - r0];
            if (t == fresh) {
#pragma unroll
                for (int e = 0; e < 8; e++) acc[e] += p * fv[lane8 * 8 + e];
            } else {
                const T* ve = (const T*)&raw[u];
#pragma unroll
                for (int e = 0; e < 8; e++) acc[e] += p * (float)ve[e];
            }
        }
    }
    // reduce over the 8 groups of a wave (lanes lane8 + 8 g) by shuffles, then over the 4 waves in LDS
#pragma unroll
    for (int e = 0; e < 8; e++) {
        acc[e] += __shfl_xor(acc[e], 8);
        acc[e] += __shfl_xor(acc[e], 16);
        acc[e] += __shfl_xor(acc[e], 32);
    }
    __syncthreads();
    float* ow = red + 8;  // [4 waves][64]
    if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; e++) ow[wave * 64 + lane * 8 + e] = acc[e];
    }
    __syncthreads();
    if (tid < 64) {
        const float o = (ow[tid] + ow[64 + tid]) + (ow[128 + tid] + ow[192 + tid]);
        st_sc1(out + 4 + tid, o);
        if (tid == 0) {
            st_sc1(out, mx);
            st_sc1(out + 1, (red[0] + red[1]) + (red[2] + red[3]));
        }
    }
}

template <typename T, int D, int MAXM>
__global__ void __launch_bounds__(kNT, 1) pdec_kernel(const PdecArgs a) {
    constexpr int H = D / 64;
    // register slots per lane per column: 16-byte vectors of plain weights, or 3 per 32-weight block
    constexpr int NV1 = std::max((D / 8 + 63) / 64, 3 * ((D / 32 + 63) / 64));          // K = d
    constexpr int NV4 = std::max((4 * D / 8 + 63) / 64, 3 * ((4 * D / 32 + 63) / 64));  // K = 4d
    constexpr int CQ = (3 * D + kG - 1) / kG, C1 = (D + kG - 1) / kG, C4 = (4 * D + kG - 1) / kG;
    constexpr int NCQ = (CQ + 3) / 4, NC1 = (C1 + 3) / 4, NC4 = (C4 + 3) / 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* xs = (T*)smem;                                                 // [M][4d] T
    float* sc = (float*)(smem + (size_t)MAXM * 4 * D * sizeof(T));    // scores [1536]
    float* red = sc + 1536;                                          // [8 + 256]
    float* qf = red + 8 + 256;                                       // q, fresh k, fresh v [3][64]
    int* lflag = (int*)(qf + 192);

    const int M = a.M, L = a.L, w0 = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    unsigned* sync = a.sync;
    unsigned* err = a.sync + (L + 1) * kPhases * 8;
    const T* te = (const T*)a.tok_emb;
    const float* te32 = a.te_f32 ? (const float*)a.tok_emb : nullptr;
    const T* self = (const T*)a.self_cache;
    const T* cross = (const T*)a.cross_cache;
    const __amdgpu_buffer_rsrc_t rff = rsrc(a.ff);

    auto idx = [&](int l, int p) { return l * kPhases + p; };
    // debug: per (WG, layer, phase) the 100 MHz clock when the phase's input arrived and when it signalled
    auto stamp = [&](int l, int p, int k) {
        if (a.stamps && tid == 0) a.stamps[(((long)w0 * a.L + l) * kPhases + p) * 2 + k] = __builtin_amdgcn_s_memrealtime();
    };
    // residual of the WG's own columns: x_old (sc1, or the embedding at layer 0) + v
    auto x_old = [&](const float* x, int l, int m, int n) -> float {
        if (l == 0 && x == a.x0) {
            const long t = a.tok[m], p = a.pos[m];
            return (te32 ? te32[t * D + n] : (float)te[t * D + n]) + a.pos_d[p * D + n];
        }
        return ld_sc1(x + (long)m * D + n);
    };

    for (int l = 0; l < L; l++) {
        const PdecLayer& W = a.layers[l];
        // ---- A: LN1 + QKV ------------------------------------------------------------------------------
        {
            ColSlice<T, NCQ, NV1> cs;
            cs.load(W.qkv, 3 * D, D);
            if (l > 0 && !pd_wait(sync, err, idx(l, P_X0), lflag, a.spin_ticks)) return;
            stamp(l, 0, 0);
            ln_rows<T, D>(a.x0, M, W.ln1_w, W.ln1_b, xs, l == 0, te, te32, a.pos_d, a.tok, a.pos);
            __syncthreads();
            float acc[NCQ][MAXM];
            cs.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NCQ; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        float v = acc[j][m] + W.bqkv[n];
                        if (n < 2 * D) v = v * a.k_scale;
                        st_sc1(a.qkv + (long)m * 3 * D + n, (float)(T)v);
                    }
                }
            pd_signal(sync, idx(l, P_QKV));
            stamp(l, 0, 1);
        }
        // ---- B: self attention -----------------------------------------------------------------------------
        {
            if (!pd_wait(sync, err, idx(l, P_QKV), lflag, a.spin_ticks)) return;
            stamp(l, 1, 0);
            const int S = a.s_self;
            if (w0 < M * H * S) {
                const int m = w0 / (H * S), h = (w0 / S) % H, s = w0 % S;
                const int pos = a.pos[m], nkv = pos + 1;
                const int r0 = (int)((long)s * nkv / S), r1 = (int)((long)(s + 1) * nkv / S);
                if (tid < 192) qf[tid] = ld_sc1(a.qkv + (long)m * 3 * D + (tid >> 6) * D + h * 64 + (tid & 63));
                __syncthreads();
                const long sl = a.slot[m];
                T* Kc = (T*)self + (((sl * L + l) * 2 + 0) * H + h) * (long)a.n_text_ctx * 64;
                T* Vc = (T*)self + (((sl * L + l) * 2 + 1) * H + h) * (long)a.n_text_ctx * 64;
                if (r0 <= pos && pos < r1 && tid < 64) {  // append this position's k, v to the cache
                    Kc[(long)pos * 64 + tid] = (T)qf[64 + tid];
                    Vc[(long)pos * 64 + tid] = (T)qf[128 + tid];
                }
                attn_task<T>(qf, Kc, Vc, r0, r1, pos, qf + 64, qf + 128, sc, red,
                             a.spart + (long)w0 * kPartStride);
            }
            pd_signal(sync, idx(l, P_SELF));
            stamp(l, 1, 1);
        }
        // ---- C: merge + out projection + residual ------------------------------------------------------------
        {
            ColSlice<T, NC1, NV1> cs;
            cs.load(W.o, D, D);
            if (!pd_wait(sync, err, idx(l, P_SELF), lflag, a.spin_ticks)) return;
            stamp(l, 2, 0);
            merge_parts<T, D>(a.spart, M, a.s_self, xs);
            __syncthreads();
            float acc[NC1][MAXM];
            cs.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        const float v = acc[j][m] + W.bo[n];
                        st_sc1(a.x1 + (long)m * D + n, v + x_old(a.x0, l, m, n));
                    }
                }
            pd_signal(sync, idx(l, P_X1));
            stamp(l, 2, 1);
        }
        // ---- D: LN + cross-Q projection --------------------------------------------------------------------
        {
            ColSlice<T, NC1, NV1> cs;
            cs.load(W.xq, D, D);
            if (!pd_wait(sync, err, idx(l, P_X1), lflag, a.spin_ticks)) return;
            stamp(l, 3, 0);
            ln_rows<T, D>(a.x1, M, W.lnx_w, W.lnx_b, xs, false, te, te32, a.pos_d, a.tok, a.pos);
            __syncthreads();
            float acc[NC1][MAXM];
            cs.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        st_sc1(a.qx + (long)m * D + n, (float)(T)((acc[j][m] + W.bxq[n]) * a.k_scale));
                    }
                }
            pd_signal(sync, idx(l, P_XQ));
            stamp(l, 3, 1);
        }
        // ---- E: cross attention over the cached K/V --------------------------------------------------------
        {
            if (!pd_wait(sync, err, idx(l, P_XQ), lflag, a.spin_ticks)) return;
            stamp(l, 4, 0);
            const int S = a.s_cross;
            if (w0 < M * H * S) {
                const int m = w0 / (H * S), h = (w0 / S) % H, s = w0 % S;
                const int T_ = a.n_audio_ctx;
                const int r0 = (int)((long)s * T_ / S), r1 = (int)((long)(s + 1) * T_ / S);
                if (tid < 64) qf[tid] = ld_sc1(a.qx + (long)m * D + h * 64 + tid);
                __syncthreads();
                const long sl = a.slot[m];
                const T* Kc = cross + (((sl * L + l) * 2 + 0) * H + h) * (long)T_ * 64;
                const T* Vc = cross + (((sl * L + l) * 2 + 1) * H + h) * (long)T_ * 64;
                attn_task<T>(qf, Kc, Vc, r0, r1, -1, nullptr, nullptr, sc, red, a.xpart + (long)w0 * kPartStride);
            }
            pd_signal(sync, idx(l, P_XATT));
            stamp(l, 4, 1);
        }
        // ---- F: merge + cross-out projection + residual ---------------------------------------------------------
        {
            ColSlice<T, NC1, NV1> cs;
            cs.load(W.xo, D, D);
            if (!pd_wait(sync, err, idx(l, P_XATT), lflag, a.spin_ticks)) return;
            stamp(l, 5, 0);
            merge_parts<T, D>(a.xpart, M, a.s_cross, xs);
            __syncthreads();
            float acc[NC1][MAXM];
            cs.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        const float v = acc[j][m] + W.bxo[n];
                        st_sc1(a.x2 + (long)m * D + n, v + ld_sc1(a.x1 + (long)m * D + n));
                    }
                }
            pd_signal(sync, idx(l, P_X2));
            stamp(l, 5, 1);
        }
        // ---- G: LN + FC1 + GELU ------------------------------------------------------------------------------
        {
            ColSlice<T, NC4, NV1> cs;
            cs.load(W.f1, 4 * D, D);
            if (!pd_wait(sync, err, idx(l, P_X2), lflag, a.spin_ticks)) return;
            stamp(l, 6, 0);
            ln_rows<T, D>(a.x2, M, W.ln2_w, W.ln2_b, xs, false, te, te32, a.pos_d, a.tok, a.pos);
            __syncthreads();
            float acc[NC4][MAXM];
            cs.template run<MAXM>(xs, D, M, acc);
#pragma unroll
            for (int j = 0; j < NC4; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        st_sc1(a.ff + (long)m * 4 * D + n, (float)(T)gelu_t(acc[j][m] + W.b1[n], a.gelu_tab));
                    }
                }
            pd_signal(sync, idx(l, P_FF));
            stamp(l, 6, 1);
        }
        // ---- H: FC2 + residual ----------------------------------------------------------------------------------
        {
            ColSlice<T, NC1, NV4> cs;
            cs.load(W.f2, D, 4 * D);
            if (!pd_wait(sync, err, idx(l, P_FF), lflag, a.spin_ticks)) return;
            stamp(l, 7, 0);
            for (int q = tid; q < M * D; q += kNT) {  // the GELU rows (f32 values of T) -> LDS as T
                const float4 v = ld4_sc1(rff, q * 16);
                T* dst = xs + (long)q * 4;
                dst[0] = (T)v.x; dst[1] = (T)v.y; dst[2] = (T)v.z; dst[3] = (T)v.w;
            }
            __syncthreads();
            float acc[NC1][MAXM];
            cs.template run<MAXM>(xs, 4 * D, M, acc);
#pragma unroll
            for (int j = 0; j < NC1; j++)
#pragma unroll
                for (int m = 0; m < MAXM; m++) {
                    const int cl = wave + 4 * j;
                    if (m < M && cl < cs.nc && lane == m) {
                        const int n = cs.c0 + cl;
                        const float v = acc[j][m] + W.b2[n];
                        st_sc1(a.x0 + (long)m * D + n, v + ld_sc1(a.x2 + (long)m * D + n));
                    }
                }
            pd_signal(sync, idx(l + 1, P_X0));
            stamp(l, 7, 1);
        }
    }
    // ---- final LayerNorm of every row -> the logits GEMM's input ----------------------------------------------
    if (w0 == 0) {
        if (!pd_wait(sync, err, idx(L, P_X0), lflag, a.spin_ticks)) return;
        ln_rows<T, D>(a.x0, M, a.lnd_w, a.lnd_b, (T*)a.out_dh, false, te, te32, a.pos_d, a.tok, a.pos);
    }
}

long g_pdec_spin_ticks = 5000000;
unsigned long long* g_pdec_stamps = nullptr;

bool pdec_supported(int d, int H) { return H * 64 == d && (d == 384 || d == 512 || d == 768 || d == 1024 || d == 1280); }

size_t pdec_sync_bytes(int L) { return ((size_t)(L + 1) * kPhases * 8 + 4) * sizeof(unsigned); }

int pdec_splits(int M, int H, int rows) { return std::max(1, std::min(kG / (M * H), rows / 16)); }

void launch_pdec(DType dt, const PdecArgs& a, hipStream_t st) {
    if (a.M < 1 || a.M > kPdecMaxRows) WM_FAIL("pdec: %d rows", a.M);
    if (a.M * (a.d / 64) * a.s_self > kG || a.M * (a.d / 64) * a.s_cross > kG) WM_FAIL("pdec: split counts");
    const size_t lds = (size_t)kPdecMaxRows * 4 * a.d * 2 + (1536 + 8 + 256 + 192 + 4) * sizeof(float);
    WM_CHECK(hipMemsetAsync(a.sync, 0, pdec_sync_bytes(a.L), st));
#define WM_PD(TT, DD) pdec_kernel<TT, DD, kPdecMaxRows><<<kG, kNT, lds, st>>>(a)
#define WM_PD_D(TT)                                     \
    switch (a.d) {                                      \
        case 384: WM_PD(TT, 384); break;                \
        case 512: WM_PD(TT, 512); break;                \
        case 768: WM_PD(TT, 768); break;                \
        case 1024: WM_PD(TT, 1024); break;              \
        case 1280: WM_PD(TT, 1280); break;              \
        default: WM_FAIL("pdec: d %d", a.d);            \
    }
    if (dt == DType::F16) { WM_PD_D(half_t) } else { WM_PD_D(bf16_t) }
#undef WM_PD_D
#undef WM_PD
}

}  // namespace wm
