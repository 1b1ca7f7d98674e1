// MFMA GEMM for every projection of the Whisper graph: C[M][N] = A[M][K] . B[N][K]^T (+bias),
// f16 or bf16 operands, f32 accumulation (v_mfma_f32_16x16x32_{f16,bf16}), with the graph's
// elementwise tails fused into the epilogue (bias, GELU, residual add, positional embedding,
// q/k scaling, KV-cache scatter). SURVEY.md §8a rows a7-a10.
//
// Both operands are K-contiguous ("NT"), the natural layout of GGML/PyTorch linear weights, so
// A and B fragments come from the same LDS image shape: [rows][64 halves] = 8 x 16-byte chunks
// per row, chunk index XOR-swizzled with (row>>1)&7 so that the 16 lanes of a ds_read_b128 group
// that read one chunk column of 16 consecutive rows hit 16 distinct 16-byte bank slots.
// Staging: 16-byte global loads to registers issued one K-tile ahead, written to the other LDS
// buffer after the MFMAs of the current tile (one barrier per K-tile).
//
// A's row addressing is affine per batch (row m -> base + (m/rpb)*bstride + (m%rpb)*rstride) so
// the conv stem is a plain GEMM over a sliding window of the time-major, zero-padded input:
// conv1 (stride 1) uses rstride = n_mels, conv2 (stride 2) rstride = 2d, with the weights
// reordered to [out][tap][in] at load time (implicit im2col, no im2col buffer).
//
// Roofline: MFMA-bound for the encoder/cross-KV/prefill shapes (M = B*1500), HBM-bound on the
// weights for decode steps (M = number of active sequences).
#include <mutex>
#include "../common.h"
#include "../kernels.h"

#include <algorithm>
#include <cmath>
#include <vector>

namespace wm {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ggml's GELU is a table over f16 inputs (GGML_GELU_FP16, built with the host's tanhf at ggml
// init): the same table, built the same way on the host once per context and uploaded, then one
// L2-resident 2-byte gather per output in the epilogues (bit-exact to the oracle's
// oracle/oracle_whisper.cpp:253 gelu_ggml; a device tanhf formula is not, and costs ~30 % of the
// FC1 GEMM).
__device__ uint16_t g_gelu_tab[65536];

void init_gelu_table() {
    static std::vector<uint16_t> tab;
    static std::mutex mu;  // contexts may be created from several threads
    std::lock_guard<std::mutex> lk(mu);
    if (tab.empty()) {
        tab.resize(65536);
        const float GELU_COEF_A = 0.044715f;
        const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
        for (int i = 0; i < 65536; i++) {
            const uint16_t u = (uint16_t)i;
            const float x = (float)__builtin_bit_cast(_Float16, u);
            const float g = 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
            tab[i] = __builtin_bit_cast(uint16_t, (_Float16)g);
        }
    }
    WM_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_gelu_tab), tab.data(), tab.size() * sizeof(uint16_t)));
}

const uint16_t* gelu_table_device() {
    static const uint16_t* p = [] {
        void* q = nullptr;
        WM_CHECK(hipGetSymbolAddress(&q, HIP_SYMBOL(g_gelu_tab)));
        return (const uint16_t*)q;
    }();
    return p;
}

// == gelu_ggml(x), bit for bit
__device__ __forceinline__ float gelu_tab(float x) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return (float)__builtin_bit_cast(half_t, g_gelu_tab[__builtin_bit_cast(uint16_t, (half_t)x)]);
}

// The same table in LDS for the big GEMMs' epilogues (LDS is free after their main loop): the
// entries of |h| < 12 only, [0, 0x4A00) positive and [0x4A00, 0x9400) negative f16 bit patterns
// (inputs in (-10, 10) round to |h| <= 10), 75.8 KB loaded by LDS-DMA per tile. A random 2-byte
// gather from LDS costs a few LDS cycles per wave; from the global table it is one TA pass per lane.
typedef __attribute__((address_space(3))) const uint16_t* lds_u16_t;
constexpr int kGeluLdsEntries = 2 * 0x4A00;
__device__ __forceinline__ float gelu_ltab(float x, lds_u16_t t) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const uint16_t u = __builtin_bit_cast(uint16_t, (half_t)x);
    return (float)__builtin_bit_cast(half_t, t[(u & 0x7FFF) + (u >> 15) * 0x4A00]);
}
// stage the LDS table at `dst` (16-byte aligned): 512 threads, 16-byte LDS-DMA pieces
__device__ __forceinline__ void gelu_ltab_stage(char* dst, int tid) {
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int NCH = kGeluLdsEntries / 8;  // 4736 = 74 x 64
    static_assert(NCH % 64 == 0, "whole wave pieces");
    const int wave = tid >> 6, lane = tid & 63;
    for (int c0 = wave * 64; c0 < NCH; c0 += 512) {
        const int c = c0 + lane, e = c * 8;
        const uint16_t* src = g_gelu_tab + (e < 0x4A00 ? e : 0x8000 + (e - 0x4A00));
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(dst + c0 * 16), 16, 0, 0);
    }
}

// tanh-GELU by formula, x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)), for the fp8 mode and bf16
// encoders (neither is a bit-exact whisper.cpp path, so they skip the table and its 75.8 KB LDS copy
// per tile). The quotient is x * rcp(1 + e) (v_rcp_f32, ~1 ulp of f32) instead of IEEE division's
// scale / fma / fixup sequence: the result is rounded to bf16 (2^-9) right after.
__device__ __forceinline__ float gelu_formula(float x) {
    const float u = 1.5957691216057308f * (x + 0.044715f * x * x * x);
    return x * __builtin_amdgcn_rcpf(1.0f + __expf(-u));
}

template <int EPI, typename T, bool NOB = false>
__device__ __forceinline__ void epilogue(const GemmArgs& g, int m, int n, float v) {
    if (!NOB && g.bias) v = v + g.bias[n];
    if constexpr (EPI == EPI_STORE) {
        if (g.sc_div > 0 && ((n / g.sc_div) % g.sc_mod) < g.sc_lim) v = v * g.scale;
        const long orow = (m / g.o_rpb) * g.o_bstride + (m % g.o_rpb) + g.o_off;
        ((T*)g.out)[orow * g.ldo + n] = (T)v;
    } else if constexpr (EPI == EPI_GELU) {
        const long orow = (m / g.o_rpb) * g.o_bstride + (m % g.o_rpb) + g.o_off;
        ((T*)g.out)[orow * g.ldo + n] = (T)gelu_tab(v);
    } else if constexpr (EPI == EPI_GELU_F) {
        const long orow = (m / g.o_rpb) * g.o_bstride + (m % g.o_rpb) + g.o_off;
        ((T*)g.out)[orow * g.ldo + n] = (T)gelu_formula(v);
    } else if constexpr (EPI == EPI_RESID) {
        float* o = (float*)g.out + (long)m * g.ldo + n;
        *o = v + *o;
    } else if constexpr (EPI == EPI_GELU_POS) {
        ((float*)g.out)[(long)m * g.ldo + n] = gelu_tab(v) + g.pos[(long)(m % g.pos_rows) * g.N + n];
    } else if constexpr (EPI == EPI_F32) {
        ((float*)g.out)[(long)m * g.ldo + n] = v;
    } else if constexpr (EPI == EPI_CROSSKV) {
        const int b = m / g.ctx, t = m % g.ctx;
        const int l = n / (2 * g.d), kv = (n / g.d) & 1, h = (n % g.d) >> 6, dh = n & 63;
        if (kv == 0) v = v * g.scale;
        const long slot = g.row_slot[b];
        ((T*)g.cache)[((((slot * g.L + l) * 2 + kv) * g.H + h) * g.ctx + t) * 64 + dh] = (T)v;
    } else if constexpr (EPI == EPI_QKV_DEC) {
        const int part = n / g.d;
        if (part == 0) {
            ((T*)g.out)[(long)m * g.ldo + n] = (T)(v * g.scale);
        } else {
            const int kv = part - 1, nn = n - part * g.d, h = nn >> 6, dh = nn & 63;
            if (kv == 0) v = v * g.scale;
            const long slot = g.row_slot[m], pos = g.row_pos[m];
            ((T*)g.cache)[((((slot * g.L + g.layer) * 2 + kv) * g.H + h) * g.ctx + pos) * 64 + dh] = (T)v;
        }
    }
}

// 16 consecutive outputs of row m starting at column n (n % 16 == 0): the same math as
// `epilogue`, with 16-byte loads/stores whenever the row segment is in bounds and aligned.
// NOB: the caller has added the bias already (gemm8p_kernel loads its lane's 16 bias values once per tile)
template <int EPI, typename T, bool LTAB = false, bool NOB = false>
__device__ __forceinline__ void epilogue16(const GemmArgs& g, int m, int n, float (&v)[16], lds_u16_t ltab = nullptr) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    bool vec = n + 16 <= g.N && EPI != EPI_QKV_DEC;
    long base = 0;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_GELU_F) {
        const long orow = (m / g.o_rpb) * g.o_bstride + (m % g.o_rpb) + g.o_off;
        base = orow * g.ldo + n;
        vec = vec && (((uintptr_t)((T*)g.out + base)) & 15) == 0;
    } else if constexpr (EPI == EPI_RESID || EPI == EPI_F32 || EPI == EPI_GELU_POS) {
        base = (long)m * g.ldo + n;
        vec = vec && (((uintptr_t)((float*)g.out + base)) & 15) == 0;
    }
    if (!vec) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (n + k < g.N) epilogue<EPI, T, NOB>(g, m, n + k, v[k]);
        return;
    }
    if (!NOB && g.bias) {
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 b = *(const float4*)(g.bias + n + k);
            v[k] = v[k] + b.x; v[k + 1] = v[k + 1] + b.y; v[k + 2] = v[k + 2] + b.z; v[k + 3] = v[k + 3] + b.w;
        }
    }
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_GELU_F || EPI == EPI_CROSSKV) {
        float sc = 1.0f;
        T* dst;
        if constexpr (EPI == EPI_CROSSKV) {
            const int b = m / g.ctx, t = m % g.ctx;
            const int l = n / (2 * g.d), kv = (n / g.d) & 1, h = (n % g.d) >> 6, dh = n & 63;
            if (kv == 0) sc = g.scale;
            const long slot = g.row_slot[b];
            dst = (T*)g.cache + ((((slot * g.L + l) * 2 + kv) * g.H + h) * g.ctx + t) * 64 + dh;
        } else {
            if constexpr (EPI == EPI_STORE)
                if (g.sc_div > 0 && ((n / g.sc_div) % g.sc_mod) < g.sc_lim) sc = g.scale;
            dst = (T*)g.out + base;
        }
        T o[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            float x = v[k];
            if constexpr (EPI == EPI_GELU) x = LTAB ? gelu_ltab(x, ltab) : gelu_tab(x);
            else if constexpr (EPI == EPI_GELU_F) x = gelu_formula(x);
            else if (sc != 1.0f) x = x * sc;
            o[k] = (T)x;
        }
        *(u4*)dst = *(const u4*)&o[0];
        *(u4*)(dst + 8) = *(const u4*)&o[8];
    } else if constexpr (EPI == EPI_RESID) {
        float* o = (float*)g.out + base;
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            float4 x = *(const float4*)(o + k);
            x.x = v[k] + x.x; x.y = v[k + 1] + x.y; x.z = v[k + 2] + x.z; x.w = v[k + 3] + x.w;
            *(float4*)(o + k) = x;
        }
    } else if constexpr (EPI == EPI_GELU_POS) {
        float* o = (float*)g.out + base;
        const float* p = g.pos + (long)(m % g.pos_rows) * g.N + n;
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 pp = *(const float4*)(p + k);
            float4 x;
            if constexpr (LTAB) {
                x.x = gelu_ltab(v[k], ltab) + pp.x; x.y = gelu_ltab(v[k + 1], ltab) + pp.y;
                x.z = gelu_ltab(v[k + 2], ltab) + pp.z; x.w = gelu_ltab(v[k + 3], ltab) + pp.w;
            } else {
                x.x = gelu_tab(v[k]) + pp.x; x.y = gelu_tab(v[k + 1]) + pp.y;
                x.z = gelu_tab(v[k + 2]) + pp.z; x.w = gelu_tab(v[k + 3]) + pp.w;
            }
            *(float4*)(o + k) = x;
        }
    } else if constexpr (EPI == EPI_F32) {
        float* o = (float*)g.out + base;
#pragma unroll
        for (int k = 0; k < 16; k += 4) *(float4*)(o + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
    }
}

// SPLIT: blockIdx.z owns K range [z*kc, min(K, (z+1)*kc)) and writes its partial f32 tile to
// g.splitk_ws[z][M][N]; splitk_reduce_kernel sums the slabs and runs the epilogue.
template <typename T, int BM, int BN, int WM, int WN, int EPI, bool SPLIT>
__global__ void __launch_bounds__(256) gemm_kernel(const GemmArgs g, const int kc) {
    typedef typename Frag<T>::type FT;
    constexpr int BK = 64;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int A_PER_T = BM * 8 / 256, B_PER_T = BN * 8 / 256;
    static_assert(WM * WN == 4, "4 waves");
    __shared__ u32x4 lds[2][(BM + BN) * 8];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const T* A = (const T*)g.A;
    const T* B = (const T*)g.B;

    const T* a_ptr[A_PER_T];
    int a_lds[A_PER_T], a_k[A_PER_T];
    bool a_ok[A_PER_T];
#pragma unroll
    for (int i = 0; i < A_PER_T; i++) {
        const int c = tid + i * 256, row = c >> 3, kc = c & 7;
        const int m = m0 + row;
        a_ok[i] = m < g.M;
        const int mm = a_ok[i] ? m : 0;
        a_ptr[i] = A + (mm / g.a_rpb) * g.a_bstride + (mm % g.a_rpb) * g.a_rstride + kc * 8;
        a_k[i] = kc * 8;
        a_lds[i] = row * 8 + (kc ^ ((row >> 1) & 7));
    }
    const T* b_ptr[B_PER_T];
    int b_lds[B_PER_T], b_k[B_PER_T];
    bool b_ok[B_PER_T];
#pragma unroll
    for (int i = 0; i < B_PER_T; i++) {
        const int c = tid + i * 256, row = c >> 3, kc = c & 7;
        const int n = n0 + row;
        b_ok[i] = n < g.N;
        b_ptr[i] = B + (long)(b_ok[i] ? n : 0) * g.K + kc * 8;
        b_k[i] = kc * 8;
        b_lds[i] = BM * 8 + row * 8 + (kc ^ ((row >> 1) & 7));
    }

    const int kend = SPLIT ? min(g.K, (int)blockIdx.z * kc + kc) : g.K;
    u32x4 ra[A_PER_T], rb[B_PER_T];
    const u32x4 zero = {0, 0, 0, 0};
    auto gload = [&](int kt) {
        const int kb = kt * BK;
#pragma unroll
        for (int i = 0; i < A_PER_T; i++)
            ra[i] = (a_ok[i] && kb + a_k[i] < kend) ? *(const u32x4*)(a_ptr[i] + kb) : zero;
#pragma unroll
        for (int i = 0; i < B_PER_T; i++)
            rb[i] = (b_ok[i] && kb + b_k[i] < kend) ? *(const u32x4*)(b_ptr[i] + kb) : zero;
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_PER_T; i++) lds[buf][a_lds[i]] = ra[i];
#pragma unroll
        for (int i = 0; i < B_PER_T; i++) lds[buf][b_lds[i]] = rb[i];
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int k0 = SPLIT ? blockIdx.z * kc : 0;
    const int nk = (kend - k0 + BK - 1) / BK;
    const int kt0 = k0 / BK;
    gload(kt0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload(kt0 + kt + 1);
#pragma unroll
        for (int s = 0; s < 2; s++) {
            FT af[TM], bfr[TN];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < TM; i++) {
                const int row = wm * WTM + i * 16 + (lane & 15);
                af[i] = __builtin_bit_cast(FT, lds[cur][row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int j = 0; j < TN; j++) {
                const int row = wn * WTN + j * 16 + (lane & 15);
                bfr[j] = __builtin_bit_cast(FT, lds[cur][BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int i = 0; i < TM; i++)
#pragma unroll
                for (int j = 0; j < TN; j++) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int n = n0 + wn * WTN + j * 16 + (lane & 15);
            if (n >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
                if (m >= g.M) continue;
                if constexpr (SPLIT) g.splitk_ws[((long)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][r];
                else epilogue<EPI, T>(g, m, n, acc[i][j][r]);
            }
        }
}

// Large-M (encoder / cross-KV / prefill) GEMM: 128x128x64 tiles staged global->LDS by
// global_load_lds_dwordx4 (no register staging), two LDS stages, 4 waves x (64x64) of
// v_mfma_f32_16x16x32. The LDS image is the same XOR-swizzled [row][8 x 16 B] image as above: the
// DMA writes lane-linearly (wave base + lane*16), so the swizzle is applied to the per-lane
// SOURCE address (lane l of an 8-row piece loads logical chunk (l&7)^((row>>1)&7)), and the
// fragment reads apply the same involution. Rows past M/N are clamped to the last valid row
// (their outputs are never stored); K must be a multiple of 64. Blocks are remapped so that the
// tiles sharing an A row-panel run on the same XCD (bijective remap, guide T1).
template <typename T, int EPI>
__global__ void __launch_bounds__(256) gemm_glds_kernel(const GemmArgs g, const int tiles_n) {
    typedef typename Frag<T>::type FT;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int BM = 128, BN = 128, BK = 64;
    __shared__ u32x4 lds[2][(BM + BN) * 8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int m0 = (wgid / tiles_n) * BM, n0 = (wgid % tiles_n) * BN;
    const T* A = (const T*)g.A;
    const T* B = (const T*)g.B;
    const T* a_src[4];
    const T* b_src[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = (wave * 4 + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int m = min(m0 + r, g.M - 1);
        a_src[i] = A + (m / g.a_rpb) * g.a_bstride + (m % g.a_rpb) * g.a_rstride + c * 8;
        const int n = min(n0 + r, g.N - 1);
        b_src[i] = B + (long)n * g.K + c * 8;
    }
    auto issue = [&](int stage, int kt) {
        const int kb = kt * BK;
#pragma unroll
        for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + kb), (lds_ptr_t)&lds[stage][(wave * 4 + i) * 64], 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + kb), (lds_ptr_t)&lds[stage][BM * 8 + (wave * 4 + i) * 64],
                                             16, 0, 0);
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = g.K / BK;
    issue(0, 0);
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            issue(cur ^ 1, kt + 1);
            asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
#pragma unroll
        for (int s = 0; s < 2; s++) {
            FT af[4], bfr[4];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = wm * 64 + i * 16 + (lane & 15);
                af[i] = __builtin_bit_cast(FT, lds[cur][row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int row = wn * 64 + j * 16 + (lane & 15);
                bfr[j] = __builtin_bit_cast(FT, lds[cur][BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int n = n0 + wn * 64 + j * 16 + (lane & 15);
            if (n >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
                if (m < g.M) epilogue<EPI, T>(g, m, n, acc[i][j][r]);
            }
        }
}

// 256x256x64 tiles, 8 waves (2 x 4), each wave 128x64 (8 x 4 MFMA 16x16x32 tiles, 128 accumulator
// registers): twice the MFMA work per barrier of the 128x128 kernel and 0.375 LDS fragment reads
// per MFMA. Same LDS-DMA staging, swizzle and XCD remap; 2 stages x 64 KiB LDS, one block per CU.
// PIPE: fragment reads of the next k-step are issued under the current k-step's MFMAs (two
// register sets), one barrier per K-tile placed between the two k-steps; the DMA of tile t+2 is
// issued right after that barrier into the buffer tile t has just released.
template <typename T, int EPI, bool PIPE>
__global__ void __launch_bounds__(512) gemm256_kernel(const GemmArgs g, const int tiles_n) {
    typedef typename Frag<T>::type FT;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int BM = 256, BN = 256, BK = 64;
    __shared__ u32x4 lds[2][(BM + BN) * 8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int m0 = (wgid / tiles_n) * BM, n0 = (wgid % tiles_n) * BN;
    const T* A = (const T*)g.A;
    const T* B = (const T*)g.B;
    // A tile = 32 pieces of 8 rows x 128 B; 8 waves x 4 pieces. Same for B.
    const T* a_src[4];
    const T* b_src[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = (wave * 4 + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int m = min(m0 + r, g.M - 1);
        a_src[i] = A + (m / g.a_rpb) * g.a_bstride + (m % g.a_rpb) * g.a_rstride + c * 8;
        const int n = min(n0 + r, g.N - 1);
        b_src[i] = B + (long)n * g.K + c * 8;
    }
    auto issue = [&](int stage, int kt) {
        const int kb = kt * BK;
#pragma unroll
        for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + kb), (lds_ptr_t)&lds[stage][(wave * 4 + i) * 64], 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + kb), (lds_ptr_t)&lds[stage][BM * 8 + (wave * 4 + i) * 64],
                                             16, 0, 0);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = g.K / BK;
    if constexpr (PIPE) {
        auto read_frags = [&](int buf, int s, FT (&af)[8], FT (&bfr)[4]) {
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int row = wn * 64 + j * 16 + (lane & 15);
                bfr[j] = __builtin_bit_cast(FT, lds[buf][BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int row = wm * 128 + i * 16 + (lane & 15);
                af[i] = __builtin_bit_cast(FT, lds[buf][row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
        };
        auto mfmas = [&](const FT (&af)[8], const FT (&bfr)[4]) {
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
            __builtin_amdgcn_s_setprio(0);
        };
        FT a0[8], b0[4], a1[8], b1[4];
        issue(0, 0);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (nk > 1) issue(1, 1);
        read_frags(0, 0, a0, b0);
        for (int kt = 0; kt < nk; kt++) {
            const int cur = kt & 1;
            read_frags(cur, 1, a1, b1);  // k-step 1 of this tile, under k-step 0's MFMAs
            mfmas(a0, b0);
            // tile kt+1 landed (this wave's DMA), every wave done reading tile kt
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (kt + 2 < nk) issue(cur, kt + 2);
            if (kt + 1 < nk) read_frags(cur ^ 1, 0, a0, b0);  // next tile's k-step 0, under k-step 1
            mfmas(a1, b1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
    issue(0, 0);
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            issue(cur ^ 1, kt + 1);
            asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
#pragma unroll
        for (int s = 0; s < 2; s++) {
            FT af[8], bfr[4];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int row = wn * 64 + j * 16 + (lane & 15);
                bfr[j] = __builtin_bit_cast(FT, lds[cur][BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int row = wm * 128 + i * 16 + (lane & 15);
                af[i] = __builtin_bit_cast(FT, lds[cur][row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
            __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    }
    // epilogue: each wave transposes its 128x64 tile through LDS 16 rows at a time so every lane
    // owns 16 consecutive columns of one row (16-byte stores instead of 4-byte column stores)
    constexpr int LDW = 68;  // padded f32 row stride of the staging image
    float* stg = (float*)&lds[0][0] + wave * 16 * LDW;
#pragma unroll
    for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) stg[((lane >> 4) * 4 + r) * LDW + j * 16 + (lane & 15)] = acc[i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int row = lane >> 2, c0 = (lane & 3) * 16;
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 x = *(const float4*)(stg + row * LDW + c0 + k);
            v[k] = x.x; v[k + 1] = x.y; v[k + 2] = x.z; v[k + 3] = x.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int m = m0 + wm * 128 + i * 16 + row, n = n0 + wn * 64 + c0;
        if (m < g.M && n < g.N) epilogue16<EPI, T>(g, m, n, v);
    }
}

// 256x256x64 tiles, 8 waves (2 x 4), each wave 128x64 — the phase-interleaved schedule of the
// guide's 256^2 8-phase template, restated for this engine's operand layout. A K-tile is four
// phases, one per C quadrant of the wave (64 rows x 32 columns x K 64 = 16 MFMAs): each phase reads
// the register subtile it needs (P1: B cols 0-31 + A rows 0-63; P2: B cols 32-63; P3: A rows
// 64-127; P4: none — A rows 64-127 and B cols 0-31 are still in registers), then a barrier, the
// LDS wait, the 16 MFMAs, and a second barrier. The two M-halves of the workgroup (wave groups
// wr = 0, 1; a SIMD holds one wave of each) run one barrier apart, so on every SIMD one wave
// issues LDS reads and DMA while the other keeps the MFMA pipe busy.
// Staging (LDS-DMA, 2 buffers x 64 KiB, one K-tile each; buffer = K-tile & 1): the B half-tiles of
// K-tile kt+2 are issued in P4(kt) (B of buffer kt&1 was last read in P2(kt)), the A half-tiles of
// K-tile kt+1 in P1(kt) (A of that buffer was last read in P3(kt-1)); both at least two barriers
// after the last read of the bytes they replace, for either wave group. P4(kt) retires everything
// of K-tile kt+1 with a counted vmcnt (only the 4 B loads just issued may stay in flight), and the
// first read of K-tile kt+1 comes one phase later, after a barrier every issuing wave has passed
// after its wait. (Issuing all of K-tile kt+2 in P4(kt), a full K-tile ahead, measured 10 %
// slower: the burst of 8 LDS-DMA per thread in one phase costs more than the extra distance.)

template <typename T, int EPI>
__global__ void __launch_bounds__(512) gemm8p_kernel(const GemmArgs g, const int tiles_n, const int gm) {
    typedef typename Frag<T>::type FT;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int BM = 256, BK = 64;
    __shared__ u32x4 lds[2][(BM + 256) * 8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, qx = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qx + 1) : rr * (qx + 1) + (xcd - rr) * qx) + (orig >> 3);
    // grouped tile order (gm > 0): each group of gm m-tiles walks its m-tiles fastest, so the
    // workgroups an XCD runs at once share B (weight) tiles and a few A tiles in its L2
    int mt = wgid / tiles_n, nt = wgid % tiles_n;
    if (gm > 0) {
        const int tiles_m = (g.M + BM - 1) / BM, per = gm * tiles_n, grp = wgid / per, f0 = grp * gm;
        const int gsz = min(gm, tiles_m - f0), r = wgid - grp * per;
        mt = f0 + r % gsz;
        nt = r / gsz;
    }
    const int m0 = mt * BM, n0 = nt * 256;
    // debug stamps (g.stamps): entry, main loop start, main loop end, epilogue end (shader clock), per workgroup
    auto stamp = [&](int k) {
        if (g.stamps && tid == 0) g.stamps[(long)blockIdx.x * 4 + k] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    const T* A = (const T*)g.A;
    const T* B = (const T*)g.B;
    // DMA sources: half-tile h (rows h*128 .. +127) = 2 pieces of 8 rows x 128 B per wave
    const T* a_src[2][2];
    const T* b_src[2][2];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int r = h * 128 + (wave * 2 + i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const int m = min(m0 + r, g.M - 1);
            a_src[h][i] = A + (m / g.a_rpb) * g.a_bstride + (m % g.a_rpb) * g.a_rstride + c * 8;
            const int n = min(n0 + r, g.N - 1);
            b_src[h][i] = B + (long)n * g.K + c * 8;
        }
    auto stage_a = [&](int kt) {
        u32x4* st = &lds[kt & 1][0];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int i = 0; i < 2; i++)
                __builtin_amdgcn_global_load_lds((const void*)(a_src[h][i] + kt * BK),
                                                 (lds_ptr_t)&st[(h * 16 + wave * 2 + i) * 64], 16, 0, 0);
    };
    auto stage_b = [&](int kt) {
        u32x4* st = &lds[kt & 1][BM * 8];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int i = 0; i < 2; i++)
                __builtin_amdgcn_global_load_lds((const void*)(b_src[h][i] + kt * BK),
                                                 (lds_ptr_t)&st[(h * 16 + wave * 2 + i) * 64], 16, 0, 0);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    FT a0[4][2], a1[4][2], b0[2][2], b1[2][2];  // [frag][k-step]
    auto read_a = [&](int buf, int mq, FT (&af)[4][2]) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int row = wm * 128 + (mq * 4 + i) * 16 + (lane & 15), ch = s * 4 + (lane >> 4);
                af[i][s] = __builtin_bit_cast(FT, lds[buf][row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
    };
    auto read_b = [&](int buf, int nq, FT (&bf)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int row = wn * 64 + (nq * 2 + j) * 16 + (lane & 15), ch = s * 4 + (lane >> 4);
                bf[j][s] = __builtin_bit_cast(FT, lds[buf][BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
    };
    auto mfma_q = [&](int mq, int nq, const FT (&af)[4][2], const FT (&bf)[2][2]) {
        asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
                for (int s = 0; s < 2; s++) acc[mq * 4 + i][nq * 2 + j] = mfma16x16x32(af[i][s], bf[j][s], acc[mq * 4 + i][nq * 2 + j]);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_barrier" ::: "memory");
    };
    const int nk = g.K / BK;
    // prologue: K-tile 0 (A, B), then B of K-tile 1 and A of K-tile 1
    stage_a(0);
    stage_b(0);
    if (nk > 1) { stage_b(1); stage_a(1); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (wm == 1) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind
    stamp(1);
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        // P1 (issuing the A pieces in P2, or split over P1-P3, measured the same in the engine's encode
        // phase, profiles/r06_gemm_dv_ab.txt)
        read_b(buf, 0, b0);
        read_a(buf, 0, a0);
        if (kt >= 1 && kt + 1 < nk) stage_a(kt + 1);
        mfma_q(0, 0, a0, b0);
        // P2
        read_b(buf, 1, b1);
        mfma_q(0, 1, a0, b1);
        // P3
        read_a(buf, 1, a1);
        mfma_q(1, 1, a1, b1);
        // P4: B of K-tile kt+2, then K-tile kt+1 complete (this wave's part)
        if (kt + 2 < nk) {
            stage_b(kt + 2);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        mfma_q(1, 0, a1, b0);
    }
    if (wm == 0) asm volatile("s_barrier" ::: "memory");  // the barrier counts of both groups match
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stamp(2);
    constexpr int LDW = 68;  // padded f32 row stride of the staging image
    float* stg = (float*)&lds[0][0] + wave * 16 * LDW;
    constexpr bool LT = EPI == EPI_GELU || EPI == EPI_GELU_POS;
    char* ltab_g = (char*)&lds[0][0] + 8 * 16 * LDW * 4;  // after the 8 staging images (34816 B)
    static_assert(8 * 16 * LDW * 4 + kGeluLdsEntries * 2 <= (BM + 256) * 8 * 16 * 2, "GELU table fits");
    if constexpr (LT) {
        gelu_ltab_stage(ltab_g, tid);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const lds_u16_t ltab = (lds_u16_t)(const void*)ltab_g;
    // Coalesced epilogue (round 6). Lane (row = lane >> 2, q = lane & 3) of a wave's 16-row x 64-column sub-tile
    // handles 16 of the row's columns, chosen so that each of its store instructions covers a contiguous 64-byte
    // run of the row with its 3 neighbours: f32 outputs the columns 16 k + 4 q + (0..3), k = 0..3 (four 16-byte
    // stores), compute-type outputs 32 h + 8 q + (0..7), h = 0..1 (two). (Sixteen consecutive columns per lane
    // made every store instruction 64 scattered 16-byte pieces.) Arithmetic and bits are unchanged.
    const int row = lane >> 2, q = lane & 3;
    const int nb = n0 + wn * 64;  // the wave's 64 columns
    constexpr bool F32O = EPI == EPI_RESID || EPI == EPI_F32 || EPI == EPI_GELU_POS;
    auto colk = [&](int k) { return F32O ? nb + 16 * (k >> 2) + 4 * q + (k & 3) : nb + 32 * (k >> 3) + 8 * q + (k & 7); };
    const bool full = nb + 64 <= g.N;  // (EPI_GELU_POS / EPI_RESID / EPI_F32 outputs are f32 rows of g.ldo floats)
    // the bias of those columns, loaded once per tile (it was 4 dependent 16-byte loads per sub-tile)
    float bia[16];
#pragma unroll
    for (int k = 0; k < 16; k++) bia[k] = 0.0f;
    if (g.bias) {
        if (full && (((uintptr_t)g.bias) & 15) == 0) {
#pragma unroll
            for (int k = 0; k < 16; k += 4) {
                const float4 b = *(const float4*)(g.bias + colk(k));
                bia[k] = b.x; bia[k + 1] = b.y; bia[k + 2] = b.z; bia[k + 3] = b.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) bia[k] = colk(k) < g.N ? g.bias[colk(k)] : 0.0f;
        }
    }
    // EPI_RESID: the residual row segments are read PF sub-tiles ahead (a register ring of PF x 64 bytes per
    // lane): with one sub-tile in flight the read-modify-write of the f32 residual (512 KB per tile) ran at the
    // latency-bound ~16 GB/s per CU and took longer than the main loop (round-6 clock stamps,
    // tools/gemm_stamps.py: 64k cycles against 55k)
    constexpr int PF = EPI == EPI_RESID ? 4 : 1;
    auto resid_ptr = [&](int i) -> float* {
        const int m = m0 + wm * 128 + i * 16 + row;
        float* p = (float*)g.out + (long)m * g.ldo + nb + 4 * q;
        return (m < g.M && full && (((uintptr_t)p) & 15) == 0 && (g.ldo & 3) == 0) ? p : nullptr;
    };
    float4 rx[PF][4];
    if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int pq = 0; pq < PF; pq++) {
            const float* p = resid_ptr(pq);
#pragma unroll
            for (int k = 0; k < 4; k++) rx[pq][k] = p ? *(const float4*)(p + 16 * k) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    // EPI_CROSSKV (round 6): the wave's 64 columns are one head of one layer's K or V, and a row of its cache plane
    // [slot][L][2][H][ctx][64] is 128 contiguous bytes. Lane (r8 = lane >> 3, c8 = 8 (lane & 7)) writes 8 columns of
    // rows r8 and r8 + 8 of a sub-tile, so every store instruction writes 8 whole consecutive rows, 1 KiB
    // contiguous. (The generic lane map below writes 16 half rows per instruction: the K/V GEMM of a large-v3
    // layer at 128 clips took 2.84 ms against 1.49 ms for the same shape with a row-major store,
    // tools/debug/xkv_shape.py.) Same arithmetic: (acc + bias) * scale for K, rounded once.
    // EPI_QKV_DEC (the prefill's QKV projection: q rows to out, k / v rows into the self cache at each row's
    // position, consecutive positions for a clip's prompt) takes the same map; it went per element before.
    bool xdone = false;
    if constexpr (EPI == EPI_CROSSKV || EPI == EPI_QKV_DEC) {
        if (full && (EPI == EPI_CROSSKV || ((((uintptr_t)g.out) & 15) == 0 && (g.ldo & 7) == 0 && g.d % 64 == 0))) {
            const int r8 = lane >> 3, c8 = (lane & 7) * 8, n = nb + c8;
            float b8[8];
#pragma unroll
            for (int k = 0; k < 8; k++) b8[k] = g.bias ? g.bias[n + k] : 0.0f;
            float sc;
            long colpart, sstride;
            int part = 0;
            if constexpr (EPI == EPI_CROSSKV) {
                const int l = g.layer + n / (2 * g.d), kv = (n / g.d) & 1, hh = (n % g.d) >> 6, dh = n & 63;
                sc = kv == 0 ? g.scale : 1.0f;
                colpart = (((long)l * 2 + kv) * g.H + hh) * g.ctx * 64 + dh;
                sstride = (long)g.L * 2 * g.H * g.ctx * 64;
            } else {
                part = n / g.d;  // 0 q, 1 k, 2 v
                const int nn = n - part * g.d, hh = nn >> 6, dh = nn & 63;
                sc = part <= 1 ? g.scale : 1.0f;
                colpart = (((long)g.layer * 2 + (part == 2)) * g.H + hh) * g.ctx * 64 + dh;
                sstride = (long)g.L * 2 * g.H * g.ctx * 64;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int r = 0; r < 4; r++) stg[((lane >> 4) * 4 + r) * LDW + j * 16 + (lane & 15)] = acc[i][j][r];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                float x[2][8];
#pragma unroll
                for (int h2 = 0; h2 < 2; h2++) {
                    const float4 a = *(const float4*)(stg + (r8 + 8 * h2) * LDW + c8);
                    const float4 b = *(const float4*)(stg + (r8 + 8 * h2) * LDW + c8 + 4);
                    x[h2][0] = a.x; x[h2][1] = a.y; x[h2][2] = a.z; x[h2][3] = a.w;
                    x[h2][4] = b.x; x[h2][5] = b.y; x[h2][6] = b.z; x[h2][7] = b.w;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int h2 = 0; h2 < 2; h2++) {
                    const int m = m0 + wm * 128 + i * 16 + r8 + 8 * h2;
                    if (m >= g.M) continue;
                    T o[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        float v = x[h2][k];
                        if (g.bias) v = v + b8[k];
                        if (EPI == EPI_QKV_DEC && part == 0) v = v * sc;  // (q: always scaled, as the element form)
                        else if (sc != 1.0f) v = v * sc;
                        o[k] = (T)v;
                    }
                    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                    T* dst;
                    if constexpr (EPI == EPI_CROSSKV) {
                        const int bb = m / g.ctx, t = m - bb * g.ctx;
                        dst = (T*)g.cache + (long)g.row_slot[bb] * sstride + colpart + (long)t * 64;
                    } else if (part == 0) {
                        dst = (T*)g.out + (long)m * g.ldo + n;
                    } else {
                        dst = (T*)g.cache + (long)g.row_slot[m] * sstride + colpart + (long)g.row_pos[m] * 64;
                    }
                    *(u4*)dst = *(const u4*)&o[0];
                }
            }
            xdone = true;
        }
    }
    if (!xdone) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        float4 cur[4];
        if constexpr (EPI == EPI_RESID) {
#pragma unroll
            for (int k = 0; k < 4; k++) cur[k] = rx[i % PF][k];
            if (i + PF < 8) {
                const float* p = resid_ptr(i + PF);
#pragma unroll
                for (int k = 0; k < 4; k++) rx[i % PF][k] = p ? *(const float4*)(p + 16 * k) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) stg[((lane >> 4) * 4 + r) * LDW + j * 16 + (lane & 15)] = acc[i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 x = *(const float4*)(stg + row * LDW + (colk(k) - nb));
            v[k] = x.x; v[k + 1] = x.y; v[k + 2] = x.z; v[k + 3] = x.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (g.bias) {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = v[k] + bia[k];
        }
        const int m = m0 + wm * 128 + i * 16 + row;
        if (m >= g.M) continue;
        if constexpr (EPI == EPI_RESID) {
            float* p = resid_ptr(i);
            if (p) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int c = 4 * k;
                    *(float4*)(p + 16 * k) = make_float4(v[c] + cur[k].x, v[c + 1] + cur[k].y, v[c + 2] + cur[k].z,
                                                         v[c + 3] + cur[k].w);
                }
                continue;
            }
        } else if constexpr (EPI == EPI_F32 || EPI == EPI_GELU_POS) {
            float* p = (float*)g.out + (long)m * g.ldo + nb + 4 * q;
            if (full && (((uintptr_t)p) & 15) == 0 && (g.ldo & 3) == 0) {
                const float* pp = EPI == EPI_GELU_POS ? g.pos + (long)(m % g.pos_rows) * g.N + nb + 4 * q : nullptr;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float4 x = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
                    if constexpr (EPI == EPI_GELU_POS) {
                        const float4 ps = *(const float4*)(pp + 16 * k);
                        if constexpr (LT) {
                            x.x = gelu_ltab(x.x, ltab) + ps.x; x.y = gelu_ltab(x.y, ltab) + ps.y;
                            x.z = gelu_ltab(x.z, ltab) + ps.z; x.w = gelu_ltab(x.w, ltab) + ps.w;
                        } else {
                            x.x = gelu_tab(x.x) + ps.x; x.y = gelu_tab(x.y) + ps.y;
                            x.z = gelu_tab(x.z) + ps.z; x.w = gelu_tab(x.w) + ps.w;
                        }
                    }
                    *(float4*)(p + 16 * k) = x;
                }
                continue;
            }
        } else if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_GELU_F || EPI == EPI_CROSSKV) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            if (full) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int n = nb + 32 * h + 8 * q;  // 8 columns of one head (64-aligned blocks)
                    float sc = 1.0f;
                    T* dst;
                    if constexpr (EPI == EPI_CROSSKV) {
                        const int bb = m / g.ctx, t = m % g.ctx;
                        const int l = n / (2 * g.d), kv = (n / g.d) & 1, hh = (n % g.d) >> 6, dh = n & 63;
                        if (kv == 0) sc = g.scale;
                        dst = (T*)g.cache + ((((long)g.row_slot[bb] * g.L + l) * 2 + kv) * g.H + hh) * g.ctx * 64 + (long)t * 64 + dh;
                    } else {
                        if constexpr (EPI == EPI_STORE)
                            if (g.sc_div > 0 && ((n / g.sc_div) % g.sc_mod) < g.sc_lim) sc = g.scale;
                        const long orow = (m / g.o_rpb) * g.o_bstride + (m % g.o_rpb) + g.o_off;
                        dst = (T*)g.out + orow * g.ldo + n;
                    }
                    if ((((uintptr_t)dst) & 15) == 0) {
                        T o[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            float x = v[8 * h + k];
                            if constexpr (EPI == EPI_GELU) x = LT ? gelu_ltab(x, ltab) : gelu_tab(x);
                            else if constexpr (EPI == EPI_GELU_F) x = gelu_formula(x);
                            else if (sc != 1.0f) x = x * sc;
                            o[k] = (T)x;
                        }
                        *(u4*)dst = *(const u4*)&o[0];
                    } else {
#pragma unroll
                        for (int k = 0; k < 8; k++) epilogue<EPI, T, true>(g, m, n + k, v[8 * h + k]);
                    }
                }
                continue;
            }
        }
        // edge tiles (columns past N, unaligned rows): per element, the bias already added
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (colk(k) < g.N) epilogue<EPI, T, true>(g, m, colk(k), v[k]);
    }
    }  // !xdone
    if (g.stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stamp(3);
    }
}

// fp8 variant of gemm8p_kernel (large-v3-turbo's fp8 weights, BASELINE configs[4]): A and B are
// OCP e4m3 bytes with one f32 scale per row (A: per token row, from the quantizing LayerNorm;
// B: per output channel, quantized once at load), C = (A8 . B8^T) * sa[m] * sb[n] then the same
// epilogues. The MFMA is the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with every E8M0
// block scale 127 (= 1.0): the 2x-bf16-rate fp8 path (the non-scaled fp8 MFMA runs at the bf16
// rate). A K-tile is 128 elements = the same 128 bytes per row as the bf16 kernel's 64, so the
// LDS image, swizzle, DMA schedule, barriers and counted waits are unchanged; one MFMA per
// (fragment, K-tile) instead of two, i.e. half the K-tiles for the same MFMA cycles per tile.
// A lane's 32 operand bytes are the 16-byte chunks (l>>4) and (l>>4)+4 of its row, read identically
// for A and B, which is the instruction's own k order (see frag below).
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma_mx8(i32x8 a, i32x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
template <typename T, int EPI>
__global__ void __launch_bounds__(512) gemm8p_mx_kernel(const GemmArgs g, const int tiles_n, const float* __restrict__ sa,
                                                        const float* __restrict__ sb) {
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int BM = 256, BK = 128;  // BK in fp8 elements = bytes
    // one __shared__ object only: a second one beside the LDS-DMA staging array makes hipcc wait
    // vmcnt(0) before the first LDS read of every K-step (guide §5 "Projection GEMM" item 4(a))
    __shared__ u32x4 lds[2][(BM + 256) * 8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int m0 = (wgid / tiles_n) * BM, n0 = (wgid % tiles_n) * 256;
    const uint8_t* A = (const uint8_t*)g.A;
    const uint8_t* B = (const uint8_t*)g.B;
    const uint8_t* a_src[2][2];
    const uint8_t* b_src[2][2];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int r = h * 128 + (wave * 2 + i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const int m = min(m0 + r, g.M - 1);
            a_src[h][i] = A + (m / g.a_rpb) * g.a_bstride + (m % g.a_rpb) * g.a_rstride + c * 16;
            const int n = min(n0 + r, g.N - 1);
            b_src[h][i] = B + (long)n * g.K + c * 16;
        }
    auto stage_a = [&](int kt) {
        u32x4* st = &lds[kt & 1][0];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int i = 0; i < 2; i++)
                __builtin_amdgcn_global_load_lds((const void*)(a_src[h][i] + kt * BK),
                                                 (lds_ptr_t)&st[(h * 16 + wave * 2 + i) * 64], 16, 0, 0);
    };
    auto stage_b = [&](int kt) {
        u32x4* st = &lds[kt & 1][BM * 8];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int i = 0; i < 2; i++)
                __builtin_amdgcn_global_load_lds((const void*)(b_src[h][i] + kt * BK),
                                                 (lds_ptr_t)&st[(h * 16 + wave * 2 + i) * 64], 16, 0, 0);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    i32x8 a0[4], a1[4], b0[2], b1[2];
    // lane l's operand registers 0-3 / 4-7 hold k = 16(l>>4) + [0, 16) / 64 + 16(l>>4) + [0, 16) of the
    // K-tile (probed on gfx950: tools/probe/mx_layout.hip), so the 16-byte chunks (l>>4) and
    // (l>>4) + 4 of the row are loaded: instruction k == memory k, and a 32-k MX block (scale lane
    // row + 16 * block) is 32 consecutive bytes of the row
    auto frag = [&](const u32x4* img, int row) -> i32x8 {
        const int c0 = lane >> 4, sw = (row >> 1) & 7;
        const u32x4 x = img[row * 8 + (c0 ^ sw)], y = img[row * 8 + ((c0 + 4) ^ sw)];
        return (i32x8){(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)y[0], (int)y[1], (int)y[2], (int)y[3]};
    };
    auto read_a = [&](int buf, int mq, i32x8 (&af)[4]) {
#pragma unroll
        for (int i = 0; i < 4; i++) af[i] = frag(&lds[buf][0], wm * 128 + (mq * 4 + i) * 16 + (lane & 15));
    };
    auto read_b = [&](int buf, int nq, i32x8 (&bf)[2]) {
#pragma unroll
        for (int j = 0; j < 2; j++) bf[j] = frag(&lds[buf][BM * 8], wn * 64 + (nq * 2 + j) * 16 + (lane & 15));
    };
    auto mfma_q = [&](int mq, int nq, const i32x8 (&af)[4], const i32x8 (&bf)[2]) {
        asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[mq * 4 + i][nq * 2 + j] = mfma_mx8(af[i], bf[j], acc[mq * 4 + i][nq * 2 + j]);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_barrier" ::: "memory");
    };
    const int nk = g.K / BK;
    stage_a(0);
    stage_b(0);
    if (nk > 1) { stage_b(1); stage_a(1); asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (wm == 1) asm volatile("s_barrier" ::: "memory");
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        read_b(buf, 0, b0);
        read_a(buf, 0, a0);
        if (kt >= 1 && kt + 1 < nk) stage_a(kt + 1);
        mfma_q(0, 0, a0, b0);
        read_b(buf, 1, b1);
        mfma_q(0, 1, a0, b1);
        read_a(buf, 1, a1);
        mfma_q(1, 1, a1, b1);
        if (kt + 2 < nk) {
            stage_b(kt + 2);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        mfma_q(1, 0, a1, b0);
    }
    if (wm == 0) asm volatile("s_barrier" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    constexpr int LDW = 68;
    float* stg = (float*)&lds[0][0] + wave * 16 * LDW;
    constexpr bool LT = EPI == EPI_GELU || EPI == EPI_GELU_POS;
    char* ltab_g = (char*)&lds[0][0] + 8 * 16 * LDW * 4;
    if constexpr (LT) {
        gelu_ltab_stage(ltab_g, tid);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const lds_u16_t ltab = (lds_u16_t)(const void*)ltab_g;
    const int row = lane >> 2, c0 = (lane & 3) * 16;
    const int nb = min(n0 + wn * 64 + c0, g.N - 16);
    float bs[16];
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
        const float4 x = *(const float4*)(sb + nb + k);
        bs[k] = x.x; bs[k + 1] = x.y; bs[k + 2] = x.z; bs[k + 3] = x.w;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) stg[((lane >> 4) * 4 + r) * LDW + j * 16 + (lane & 15)] = acc[i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 x = *(const float4*)(stg + row * LDW + c0 + k);
            v[k] = x.x; v[k + 1] = x.y; v[k + 2] = x.z; v[k + 3] = x.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int m = m0 + wm * 128 + i * 16 + row, n = n0 + wn * 64 + c0;
        if (m < g.M && n < g.N) {
            const float am = sa[m];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = (v[k] * am) * bs[k];
            epilogue16<EPI, T, LT>(g, m, n, v, ltab);
        }
    }
}

// fp8 e4m3 (OCP) row quantization: q[r][k] = sat(x[r][k] / s[r]), s[r] = max|x[r][:]| / 448
// (1 for an all-zero row). One wave per row, K % 8 == 0; used for the weights at load time.
template <typename T>
__global__ void __launch_bounds__(256) quant_rows_fp8_kernel(const T* __restrict__ x, long rows, int K,
                                                             uint8_t* __restrict__ q, float* __restrict__ s) {
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const T* xr = x + r * K;
    float amax = 0.f;
    for (int k = lane * 8; k < K; k += 512) {
        const u32x4 w = *(const u32x4*)(xr + k);
        const T* t = (const T*)&w;
#pragma unroll
        for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf((float)t[j]));
    }
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float sc = amax > 0.f ? amax / 448.f : 1.f, inv = 1.f / sc;
    if (lane == 0) s[r] = sc;
    uint8_t* qr = q + r * K;
    for (int k = lane * 8; k < K; k += 512) {
        const u32x4 w = *(const u32x4*)(xr + k);
        const T* t = (const T*)&w;
        uint32_t lo = 0, hi = 0;
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf((float)t[0] * inv, -448.f), 448.f),
                                             fminf(fmaxf((float)t[1] * inv, -448.f), 448.f), lo, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf((float)t[2] * inv, -448.f), 448.f),
                                             fminf(fmaxf((float)t[3] * inv, -448.f), 448.f), lo, true);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf((float)t[4] * inv, -448.f), 448.f),
                                             fminf(fmaxf((float)t[5] * inv, -448.f), 448.f), hi, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf((float)t[6] * inv, -448.f), 448.f),
                                             fminf(fmaxf((float)t[7] * inv, -448.f), 448.f), hi, true);
        *(uint2*)(qr + k) = make_uint2(lo, hi);
    }
}

// Decode-step GEMM (M <= 128 active clips): one workgroup = all M rows x 64 columns x one K chunk.
// The chunk's K-tiles stream through a 4-deep LDS ring filled by LDS-DMA (96 KiB): four tiles are
// in flight from the start and each consumed slot is refilled at once, so a workgroup pays about
// one memory latency per four K-tiles. The grid is (N/64) x splits with the partial tile written
// to the split-K slab (or through the epilogue when the chunk is the whole K). Rows past M are
// clamped (their outputs are never stored).
// W8 (fp8 mode, g.w8_scale != null): the weights are OCP e4m3 bytes [N][K] with one f32 scale per
// output column; a B tile is 64 rows x 64 bytes (4 chunks of 16 bytes per row, chunk index XOR
// (row>>2)&3), each lane's 8 bytes are widened to the MFMA type in registers (exact: e4m3 values are
// representable in f16 and bf16) and the column scale multiplies the f32 sum before the store. Half
// the weight bytes of the decode step; the activations stay in the compute type.
// BM (round 6): rows per workgroup, 128, 64 or 32. Steps of <= 32 clips (the 8-GPU shard of configs[3]: 16 per
// rank) staged 128 A rows per K-tile of which 96+ repeated the last row (clamped); BM = 32 / 64 stage only about
// the rows that exist (M = 16: 8.2 -> 7.1 us per xq GEMM, the 16-clip line 1106 -> 1172 audio-s/s). Every output's k order (K-tiles, then the two 32-deep MFMA steps) is the same for both, so the bits are.
template <typename T, int EPI, bool SPLIT, int AUXB = 0, bool W8 = false, int BM = 128>
__global__ void __launch_bounds__(256) gemm_dec_kernel(const GemmArgs g, const int kc) {
    typedef typename Frag<T>::type FT;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int BN = 64, BK = 64, MAXT = 4;
    constexpr int MI = BM / 32;  // row fragments per wave (2 x 2 waves, BM / 2 rows each)
    constexpr int AP = BM / 32;  // A pieces (8 rows x 128 B) per wave and stage
    static_assert(BM == 128 || BM == 64 || BM == 32, "BM");
    constexpr int BCH = W8 ? 4 : 8;             // 16-byte chunks per B row
    constexpr int STAGE = BM * 8 + BN * BCH;    // u32x4 per stage
    __shared__ u32x4 lds[MAXT * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;  // 2 x 2 waves, each BM / 2 rows x 32 columns
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * BM;  // row chunk (prefill: M > 128 as chunks of 128 rows, same math per row)
    const int k0 = SPLIT ? blockIdx.z * kc : 0;
    const int nkt = min(kc, g.K - k0) / BK;
    const T* A = (const T*)g.A;
    const T* B = (const T*)g.B;
    // per stage: A = BM / 8 pieces of 8 rows (AP per wave), B = 8 pieces (2 per wave)
    const T* a_src[AP];
    const T* b_src[2];
    const uint8_t* b8_src = nullptr;
#pragma unroll
    for (int i = 0; i < AP; i++) {
        const int r = (wave * AP + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int m = min(m0 + r, g.M - 1);
        a_src[i] = A + (long)m * g.a_rstride + k0 + c * 8;
    }
    if constexpr (W8) {  // one piece per wave: 16 rows x 4 chunks; LDS slot p = row*4 + phys chunk
        const int r = wave * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 2) & 3);
        const int n = min(n0 + r, g.N - 1);
        b8_src = (const uint8_t*)g.B + (long)n * g.K + k0 + c * 16;
    } else {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int r = (wave * 2 + i) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const int n = min(n0 + r, g.N - 1);
            b_src[i] = B + (long)n * g.K + k0 + c * 8;
        }
    }
    auto issue = [&](int t) {
        u32x4* st = &lds[(t & (MAXT - 1)) * STAGE];
#pragma unroll
        for (int i = 0; i < AP; i++)
            __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + t * BK), (lds_ptr_t)&st[(wave * AP + i) * 64], 16, 0, 0);
        if constexpr (W8) {
            __builtin_amdgcn_global_load_lds((const void*)(b8_src + t * BK), (lds_ptr_t)&st[BM * 8 + wave * 64], 16, 0, AUXB);
        } else {
#pragma unroll
            for (int i = 0; i < 2; i++)
                __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + t * BK), (lds_ptr_t)&st[BM * 8 + (wave * 2 + i) * 64], 16, 0, AUXB);
        }
    };
    constexpr int PER_STAGE = AP + (W8 ? 1 : 2);  // DMA instructions per wave and stage
    for (int t = 0; t < min(nkt, MAXT); t++) issue(t);
    f32x4 acc[MI][2];
#pragma unroll
    for (int i = 0; i < MI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < nkt; t++) {
        // this wave's DMAs of stage t have landed when at most PER_STAGE per later issued stage are outstanding
        const int ahead = min(nkt - 1, t + MAXT - 1) - t;
        if constexpr (PER_STAGE == 6) {
            if (ahead >= 3) asm volatile("s_waitcnt vmcnt(18)\n\ts_barrier" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else if constexpr (PER_STAGE == 4) {
            if (ahead >= 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else if constexpr (PER_STAGE == 3) {
            if (ahead >= 3) asm volatile("s_waitcnt vmcnt(9)\n\ts_barrier" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else if constexpr (PER_STAGE == 2) {
            if (ahead >= 3) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else {
            static_assert(PER_STAGE == 5, "vmcnt table");
            if (ahead >= 3) asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        const u32x4* st = &lds[(t & (MAXT - 1)) * STAGE];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            FT af[MI], bfr[2];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < MI; i++) {
                const int row = wm * (BM / 2) + i * 16 + (lane & 15);
                af[i] = __builtin_bit_cast(FT, st[row * 8 + (ch ^ ((row >> 1) & 7))]);
            }
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int row = wn * 32 + j * 16 + (lane & 15);
                if constexpr (W8) {
                    // 8 e4m3 bytes: 16-byte chunk ch>>1 (swizzled), half ch&1
                    const uint2 w8 = ((const uint2*)&st[BM * 8 + row * 4 + ((ch >> 1) ^ ((row >> 2) & 3))])[ch & 1];
                    // v_cvt_scalef32_pk_{bf16,f16}_fp8: two bytes -> two values per instruction (scale 1)
                    uint32_t e[4];
                    if constexpr (std::is_same<T, half_t>::value) {
                        typedef _Float16 v2h __attribute__((ext_vector_type(2)));
                        e[0] = __builtin_bit_cast(uint32_t, (v2h)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w8.x, 1.0f, false));
                        e[1] = __builtin_bit_cast(uint32_t, (v2h)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w8.x, 1.0f, true));
                        e[2] = __builtin_bit_cast(uint32_t, (v2h)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w8.y, 1.0f, false));
                        e[3] = __builtin_bit_cast(uint32_t, (v2h)__builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w8.y, 1.0f, true));
                    } else {
                        typedef __bf16 v2b __attribute__((ext_vector_type(2)));
                        e[0] = __builtin_bit_cast(uint32_t, (v2b)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w8.x, 1.0f, false));
                        e[1] = __builtin_bit_cast(uint32_t, (v2b)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w8.x, 1.0f, true));
                        e[2] = __builtin_bit_cast(uint32_t, (v2b)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w8.y, 1.0f, false));
                        e[3] = __builtin_bit_cast(uint32_t, (v2b)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w8.y, 1.0f, true));
                    }
                    bfr[j] = __builtin_bit_cast(FT, e);
                } else {
                    bfr[j] = __builtin_bit_cast(FT, st[BM * 8 + row * 8 + (ch ^ ((row >> 1) & 7))]);
                }
            }
#pragma unroll
            for (int i = 0; i < MI; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
        }
        if (t + MAXT < nkt) {
            __syncthreads();  // every wave is done with this slot
            issue(t + MAXT);
        }
    }
#pragma unroll
    for (int i = 0; i < MI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int n = n0 + wn * 32 + j * 16 + (lane & 15);
            if (n >= g.N) continue;
            const float wsc = W8 ? g.w8_scale[n] : 1.0f;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
                if (m >= g.M) continue;
                const float v = W8 ? acc[i][j][r] * wsc : acc[i][j][r];
                if constexpr (SPLIT) {
                    float* p = &g.splitk_ws[((long)blockIdx.z * g.M + m) * g.N + n];
                    // slab_wt: write-through (sc1) slab stores, so the lines leave the XCD's L2 while the
                    // kernel runs instead of at its end (the kernel boundary writes dirty L2 lines back)
                    if (g.slab_wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else *p = v;
                }
                else epilogue<EPI, T>(g, m, n, v);
            }
        }
}

// debug/tuning override: -1 auto, 0 register-staged, 1 LDS-DMA 128^2, 2 LDS-DMA 256^2, 3 same,
// pipelined, 4 256^2 phase-interleaved (the auto choice for big GEMMs)
int g_gemm_variant = -1;
unsigned long long* g_gemm_stamps = nullptr;

// gemm_dec_kernel row tile: the smallest of 32 / 64 / 128 rows that holds the step (the grid's row chunks
// stay cdiv(M, 128): a smaller tile is only taken when one tile holds every row). WHISPER_MI355X_DEC_BM (or
// whisper_mi355x_set_dec_bm, a test hook) caps the tile from below for the A/B (128: always 128 rows, the
// round-5 kernel). Every value gives the same bits.
int g_dec_bm = 0;  // 0: the environment's value (default 32)
static int dec_bm_min() {
    static const int v = getenv("WHISPER_MI355X_DEC_BM") ? atoi(getenv("WHISPER_MI355X_DEC_BM")) : 32;
    return g_dec_bm > 0 ? g_dec_bm : v;
}
template <typename T, int EPI, bool SPLIT, bool W8>
static void launch_dec(const GemmArgs& g, int tiles, int splits, int kc, hipStream_t st) {
    if (g.M <= 32 && dec_bm_min() <= 32) {
        gemm_dec_kernel<T, EPI, SPLIT, 2, W8, 32><<<dim3(tiles, 1, splits), 256, 0, st>>>(g, kc);
    } else if (g.M <= 64 && dec_bm_min() <= 64) {
        gemm_dec_kernel<T, EPI, SPLIT, 2, W8, 64><<<dim3(tiles, 1, splits), 256, 0, st>>>(g, kc);
    } else {
        // 65..128 rows stay one 128-row tile: two 64-row chunks (on gridDim.y, or 8 ids apart so both land on one
        // XCD's L2) read each weight tile twice and measured slower in the 128-clip step (decode 809 -> 832-840 ms,
        // profiles/r06_bm_m64_ab_*.json) though some isolated shapes gained (xq 11.9 -> 10.7 us)
        gemm_dec_kernel<T, EPI, SPLIT, 2, W8, 128><<<dim3(tiles, cdiv(g.M, 128), splits), 256, 0, st>>>(g, kc);
    }
}

template <typename T, int EPI>
__global__ void splitk_reduce_kernel(const GemmArgs g, int splits) {
    const long total = (long)g.M * g.N;
    if ((g.N & 3) == 0) {  // 16-byte slab reads, 4 columns per thread (same per-element z order)
        const long total4 = total >> 2;
        for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
            for (int z = 0; z < splits; z++) {
                const float4 w = ((const float4*)(g.splitk_ws + z * total))[i];
                v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
            }
            const int m = (int)((i * 4) / g.N), n = (int)((i * 4) % g.N);
            epilogue<EPI, T>(g, m, n, v.x);
            epilogue<EPI, T>(g, m, n + 1, v.y);
            epilogue<EPI, T>(g, m, n + 2, v.z);
            epilogue<EPI, T>(g, m, n + 3, v.w);
        }
        return;
    }
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        float v = 0.0f;
#pragma unroll 4
        for (int z = 0; z < splits; z++) v += g.splitk_ws[z * total + i];
        epilogue<EPI, T>(g, (int)(i / g.N), (int)(i % g.N), v);
    }
}

// split-K reduce of a residual GEMM fused with the next LayerNorm: one block per row m; the
// updated residual row stays in registers for the LN (decode steps: saves a launch per LN).
template <typename T, int NPT>
__global__ void __launch_bounds__(256) splitk_reduce_resid_ln_kernel(const GemmArgs g, int splits) {
    __shared__ double sh[4];
    const int m = blockIdx.x, tid = threadIdx.x;
    const long total = (long)g.M * g.N;
    float* xrow = (float*)g.out + (long)m * g.ldo;
    float a[NPT], v[NPT];
#pragma unroll
    for (int k = 0; k < NPT; k++) a[k] = 0.0f;
    // z outer so each iteration has NPT independent loads in flight (same per-element z order)
#pragma unroll 4
    for (int z = 0; z < splits; z++) {
        const float* w = g.splitk_ws + z * total + (long)m * g.N;
#pragma unroll
        for (int k = 0; k < NPT; k++) {
            const int n = tid + 256 * k;
            if (n < g.N) a[k] += w[n];
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int n = tid + 256 * k;
        v[k] = 0.0f;
        if (n < g.N) {
            float x = a[k];
            if (g.bias) x = x + g.bias[n];
            x = x + xrow[n];
            xrow[n] = x;
            v[k] = x;
        }
    }
    block256_layernorm<T, NPT>(v, g.N, g.ln_w, g.ln_b, (T*)g.ln_out + (long)m * g.N, sh);
}

// Same contract as splitk_reduce_resid_ln_kernel for N % 4 == 0, N <= 4096: one thread per 4
// consecutive columns (16-byte slab reads, all splits in flight at once), ceil(N/256) waves per row.
template <typename T>
__global__ void __launch_bounds__(1024) splitk_reduce_resid_ln4_kernel(const GemmArgs g, int splits) {
#pragma clang fp contract(off)  // ggml_norm's separately rounded ops (the __f*_rn forms alone are contracted)
    __shared__ double sh[16];
    const int m = blockIdx.x, tid = threadIdx.x, nw = blockDim.x >> 6;
    const long total = (long)g.M * g.N;
    const int n = tid * 4;
    const bool on = n < g.N;
    float x[4] = {0.f, 0.f, 0.f, 0.f};
    float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), b4 = w4;
    if (on) {
        // every load of the row goes out at once (splits <= 16, the residual, bias and LN parameters):
        // one memory round trip; the sums keep the split order
        const float* w = g.splitk_ws + (long)m * g.N + n;
        float4 p[16];
#pragma unroll
        for (int z = 0; z < 16; z++)
            if (z < splits) p[z] = *(const float4*)(w + z * total);
        float4* xr = (float4*)((float*)g.out + (long)m * g.ldo + n);
        const float4 r = *xr;
        const float4 b = g.bias ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        w4 = *(const float4*)(g.ln_w + n);
        b4 = *(const float4*)(g.ln_b + n);
#pragma unroll
        for (int z = 0; z < 16; z++)
            if (z < splits) {
                x[0] += p[z].x; x[1] += p[z].y; x[2] += p[z].z; x[3] += p[z].w;
            }
        if (g.bias) {
            x[0] = x[0] + b.x; x[1] = x[1] + b.y; x[2] = x[2] + b.z; x[3] = x[3] + b.w;
        }
        x[0] = x[0] + r.x; x[1] = x[1] + r.y; x[2] = x[2] + r.z; x[3] = x[3] + r.w;
        *xr = make_float4(x[0], x[1], x[2], x[3]);
    }
    // ggml_norm: double sums, float mean / variance, (v*scale)*w + b separately rounded
    auto block_sum = [&](double v) {
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((tid & 63) == 0) sh[tid >> 6] = v;
        __syncthreads();
        double r = 0.0;
        for (int i = 0; i < nw; i++) r += sh[i];
        __syncthreads();
        return r;
    };
    double s = on ? (((double)x[0] + (double)x[1]) + (double)x[2]) + (double)x[3] : 0.0;
    s = block_sum(s);
    const float mean = (float)(s / g.N);
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        x[k] = __fsub_rn(x[k], mean);
        s2 += (double)__fmul_rn(x[k], x[k]);
    }
    s2 = block_sum(on ? s2 : 0.0);
    const float variance = (float)(s2 / g.N);
    const float scale = 1.0f / sqrtf(variance + 1e-5f);
    if (!on) return;
    const float wv[4] = {w4.x, w4.y, w4.z, w4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
    T y[4];
#pragma unroll
    for (int k = 0; k < 4; k++) y[k] = (T)((x[k] * scale) * wv[k] + bv[k]);  // plain ops: the pragma applies
    *(uint2*)((T*)g.ln_out + (long)m * g.N + n) = *(const uint2*)y;
}

// ---- GGML block-quantized weights (QMat) -------------------------------------------------------
// One lane's share of a 32-weight block for an MFMA 16x16x32 B fragment: weights 8g .. 8g + 7 of
// block b of row n (g = lane >> 4, the fragment's k order). raw = {qs bytes (2 dwords), q5 high bits,
// d | m << 16 (m = 0 for the *_0 types, which store d only)}; dequantized exactly as ggml's dequantize_row_* (oracle/oracle_whisper.cpp, the
// engine's load-time dequantizer in model.cpp), w = (q - off) * d or q * d + m in f32, then rounded
// once to the compute type.
template <int QT>
__device__ __forceinline__ u32x4 qraw_load(const QMat& q, long n, int K, int b, int g) {
    u32x4 r;
    const long bi = n * (K / 32) + b;
    const uint2 qs = QT == 8 ? *(const uint2*)(q.qs + n * K + 32L * b + 8 * g)
                             : *(const uint2*)(q.qs + n * (K / 2) + 16L * b + 8 * (g & 1));
    r.x = qs.x;
    r.y = qs.y;
    r.z = (QT == 6 || QT == 7) ? q.qh[bi] : 0u;
    r.w = (QT == 3 || QT == 7) ? ((const uint32_t*)q.dm)[bi] : (uint32_t)q.dm[bi];  // d | m << 16, or d
    return r;
}
template <int QT, typename T>
__device__ __forceinline__ u32x4 qraw_deq(u32x4 r, int g) {
    const float dd = (float)__builtin_bit_cast(half_t, (uint16_t)(r.w & 0xFFFF));
    const float mm = (float)__builtin_bit_cast(half_t, (uint16_t)(r.w >> 16));
    T o[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t byte = ((i < 4 ? r.x : r.y) >> (8 * (i & 3))) & 0xFF;
        float v;
        if constexpr (QT == 8) {
            v = (float)(int8_t)byte * dd;
        } else {
            int x = (g >> 1) ? (int)(byte >> 4) : (int)(byte & 15);
            if constexpr (QT == 6 || QT == 7) x |= (int)((r.z >> (8 * g + i)) & 1) << 4;
            if constexpr (QT == 3 || QT == 7) v = (float)x * dd + mm;
            else v = (float)(x - (QT == 6 ? 16 : 8)) * dd;
        }
        o[i] = (T)v;
    }
    return *(const u32x4*)o;
}

// rows [0, rows) of a QMat -> compute type [rows][K] (the encoder's and the prefill's per-layer
// scratch copy): one thread per 8 weights
template <typename T, int QT>
__global__ void __launch_bounds__(256) dequant_kernel(const QMat q, long rows, int K, T* __restrict__ out) {
    const long i = blockIdx.x * 256L + threadIdx.x, per_row = K / 8;
    if (i >= rows * per_row) return;
    const long n = i / per_row;
    const int e = (int)(i - n * per_row) * 8, b = e / 32, g = (e & 31) / 8;
    *(u32x4*)(out + n * K + e) = qraw_deq<QT, T>(qraw_load<QT>(q, n, K, b, g), g);
}

template <typename T>
static void launch_dequant_t(const QMat& q, long rows, int K, T* out, hipStream_t st) {
    const unsigned grid = (unsigned)((rows * (K / 8) + 255) / 256);
    switch (q.type) {
        case 2: dequant_kernel<T, 2><<<grid, 256, 0, st>>>(q, rows, K, out); break;
        case 3: dequant_kernel<T, 3><<<grid, 256, 0, st>>>(q, rows, K, out); break;
        case 6: dequant_kernel<T, 6><<<grid, 256, 0, st>>>(q, rows, K, out); break;
        case 7: dequant_kernel<T, 7><<<grid, 256, 0, st>>>(q, rows, K, out); break;
        case 8: dequant_kernel<T, 8><<<grid, 256, 0, st>>>(q, rows, K, out); break;
        default: WM_FAIL("dequant: ggml type %d not supported", q.type);
    }
}

// several matrices of one GGML type in one launch (a decoder layer's six projections: the decode
// steps of > 32 clips dequantize each layer once per step into the scratch their split-K GEMMs read)
template <typename T, int QT>
__global__ void __launch_bounds__(256) dequant_multi_kernel(const DequantJobs J) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= J.start[J.n]) return;
    int j = 0;
    while (j + 1 < J.n && i >= J.start[j + 1]) j++;
    const long li = i - J.start[j], per_row = J.K[j] / 8;
    const long n = li / per_row;
    const int e = (int)(li - n * per_row) * 8, b = e / 32, g = (e & 31) / 8;
    *(u32x4*)((T*)J.out[j] + n * J.K[j] + e) = qraw_deq<QT, T>(qraw_load<QT>(J.q[j], n, J.K[j], b, g), g);
}

template <typename T>
static void launch_dequant_multi_t(const DequantJobs& J, hipStream_t st) {
    const unsigned grid = (unsigned)((J.start[J.n] + 255) / 256);
    switch (J.q[0].type) {
        case 2: dequant_multi_kernel<T, 2><<<grid, 256, 0, st>>>(J); break;
        case 3: dequant_multi_kernel<T, 3><<<grid, 256, 0, st>>>(J); break;
        case 6: dequant_multi_kernel<T, 6><<<grid, 256, 0, st>>>(J); break;
        case 7: dequant_multi_kernel<T, 7><<<grid, 256, 0, st>>>(J); break;
        case 8: dequant_multi_kernel<T, 8><<<grid, 256, 0, st>>>(J); break;
        default: WM_FAIL("dequant: ggml type %d not supported", J.q[0].type);
    }
}

void launch_dequant_multi(DType dt, DequantJobs J, hipStream_t st) {
    if (J.n <= 0) return;
    J.start[0] = 0;
    for (int j = 0; j < J.n; j++) {
        if (J.q[j].type != J.q[0].type || J.K[j] % 32) WM_FAIL("dequant_multi: mixed types or K %% 32");
        J.start[j + 1] = J.start[j] + J.rows[j] * (J.K[j] / 8);
    }
    if (dt == DType::F16) launch_dequant_multi_t<half_t>(J, st);
    else launch_dequant_multi_t<bf16_t>(J, st);
}

void launch_dequant(DType dt, const QMat& q, long rows, int K, void* out, hipStream_t st) {
    if (rows <= 0) return;
    if (K % 32) WM_FAIL("dequant: K %% 32 != 0 (K=%d)", K);
    if (dt == DType::F16) launch_dequant_t<half_t>(q, rows, K, (half_t*)out, st);
    else launch_dequant_t<bf16_t>(q, rows, K, (bf16_t*)out, st);
}

// sum of a double over TPR consecutive lanes (TPR = 16 or 32, aligned groups), the same value in each:
// within 16 lanes by DPP (quad xor 1, quad xor 2, half-row mirror, row mirror: VALU, no LDS), then for
// TPR = 32 one xor-16 exchange. Used by the LayerNorm prologue of gemm_small_kernel (double sums, as
// ggml_norm), where six dependent ds_bpermute rounds per sum were most of the prologue.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int TPR>
__device__ __forceinline__ double row_sum_f64(double v) {
    static_assert(TPR == 16 || TPR == 32, "16- or 32-lane rows");
    v += dpp_f64<0xB1>(v);
    v += dpp_f64<0x4E>(v);
    v += dpp_f64<0x141>(v);
    v += dpp_f64<0x140>(v);
    if constexpr (TPR == 32) v += __shfl_xor(v, 16);
    return v;
}

// Decode steps of <= 32 active clips (the app's one clip per call, whisper.rs:83-85; one rank's shard
// of configs[3] at 8 GPUs): one workgroup = 16 output columns x all M rows x the whole K. Its 8 waves
// split K (wave w: the 32-wide K-steps w, w + 8, ...) and add their partial sums in LDS in wave order, so no
// split-K slab leaves the chip and no reduce launch follows. Weights are read once, by 16-byte loads
// straight into the B fragments (a chunk of K-steps in flight before its MFMAs, the next chunk issued
// before the current one is consumed); the <= 32 activation rows are re-read from L2 by every
// workgroup. LNA: A is the f32 residual stream; the workgroup applies ggml_norm (double sums, f32
// mean / variance, (v*scale)*w + b separately rounded, as block256_layernorm) to its rows in the
// prologue, into an LDS image, so the LayerNorm launch of the split-K path disappears too.
template <typename T, int EPI, bool LNA, int NR, int QT = 0>
__global__ void __launch_bounds__(512) gemm_small_kernel(const GemmArgs g) {
#pragma clang fp contract(off)
    typedef typename Frag<T>::type FT;
    constexpr int NW = 8, CH = 5;  // waves; K-steps (32 each) per load chunk
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n0 = blockIdx.x * 16, K = g.K;
    const int lda = K + 8;  // LDS row stride of the LNA image (16-byte pad: conflict-free b128 reads)
    T* aimg = (T*)smem;
    float* red = (float*)(smem + (LNA ? (size_t)NR * 16 * lda * sizeof(T) : 0));
    const u32x4 zero = {0, 0, 0, 0};
    // this wave's K-steps of 32: wave, wave + NW, wave + 2 NW, ... (K % 32 == 0)
    const int nst = (K / 32 - wave + NW - 1) / NW;
    const int k0 = wave * 32 + 8 * (lane >> 4);
    const long nrow = min(n0 + (lane & 15), g.N - 1);
    const T* bp = (const T*)g.B + nrow * K + k0;
    const int gq = lane >> 4;  // quantized B: this lane's 8 weights of a block
    u32x4 bq[2][CH], aq[2][NR][CH];
    auto load_b = [&](int c, u32x4 (&b)[CH]) {
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int st = c * CH + u;
            if constexpr (QT == 0) b[u] = st < nst ? __builtin_nontemporal_load((const u32x4*)(bp + 32 * NW * st)) : zero;
            else b[u] = st < nst ? qraw_load<QT>(g.q, nrow, K, wave + NW * st, gq) : zero;
        }
    };
    // the first chunk of weights is in flight while the prologue runs (it does not depend on A), and so
    // are the epilogue's bias and residual operands (thread tid < NR*256 owns output (m, n) below)
    load_b(0, bq[0]);
    const int em = (tid >> 8) * 16 + ((tid >> 4) & 15), en = n0 + (tid & 15);
    const bool eon = tid < NR * 256 && em < g.M && en < g.N;
    float e_bias = 0.0f, e_res = 0.0f;
    if (eon && g.bias) e_bias = g.bias[en];
    if constexpr (EPI == EPI_RESID)
        if (eon) e_res = ((const float*)g.out)[(long)em * g.ldo + en];
    if constexpr (LNA) {
        // all 512 threads at once: TPR threads per row, thread `part` of row r holds the float4 columns
        // part*4 + j*TPR*4 (every load instruction reads whole 512-byte row segments), sums in double
        // in j order, then a shuffle tree over the row's lanes (one wave holds 64 / TPR rows)
        constexpr int ROWS = NR * 16, TPR = 512 / ROWS, NJ = 1280 / (TPR * 4);
        const int r = tid / TPR, part = tid % TPR, nj = K / (TPR * 4);
        const bool live = r < g.M;
        const float* xr = (const float*)g.A + (long)min(r, g.M - 1) * g.a_rstride;
        float4 v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; j++) v[j] = j < nj ? *(const float4*)(xr + (part + j * TPR) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; j++) s += (((double)v[j].x + (double)v[j].y) + (double)v[j].z) + (double)v[j].w;
        s = row_sum_f64<TPR>(s);
        const float mean = (float)(s / K);
        double s2 = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            if (j < nj) {
                v[j].x = v[j].x - mean; v[j].y = v[j].y - mean; v[j].z = v[j].z - mean; v[j].w = v[j].w - mean;
                s2 += (((double)(v[j].x * v[j].x) + (double)(v[j].y * v[j].y)) + (double)(v[j].z * v[j].z)) +
                      (double)(v[j].w * v[j].w);
            }
        }
        s2 = row_sum_f64<TPR>(s2);
        const float scale = 1.0f / sqrtf((float)(s2 / K) + 1e-5f);
        T* ar = aimg + (long)r * lda;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            if (j >= nj) continue;
            const int c = (part + j * TPR) * 4;
            const float4 w4 = *(const float4*)(g.a_ln_w + c), b4 = *(const float4*)(g.a_ln_b + c);
            T o[4];
            o[0] = live ? (T)((v[j].x * scale) * w4.x + b4.x) : (T)0.0f;
            o[1] = live ? (T)((v[j].y * scale) * w4.y + b4.y) : (T)0.0f;
            o[2] = live ? (T)((v[j].z * scale) * w4.z + b4.z) : (T)0.0f;
            o[3] = live ? (T)((v[j].w * scale) * w4.w + b4.w) : (T)0.0f;
            *(uint2*)(ar + c) = *(const uint2*)o;
        }
        __syncthreads();
    }
    const T* ap[NR];
    bool arow[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {
        const int r = i * 16 + (lane & 15);
        arow[i] = r < g.M;
        ap[i] = LNA ? aimg + (long)r * lda + k0 : (const T*)g.A + (long)min(r, g.M - 1) * g.a_rstride + k0;
    }
    f32x4 acc[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto load_a = [&](int c, u32x4 (&a)[NR][CH]) {
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int st = c * CH + u;
#pragma unroll
            for (int i = 0; i < NR; i++) a[i][u] = st < nst && arow[i] ? *(const u32x4*)(ap[i] + 32 * NW * st) : zero;
        }
    };
    auto mma = [&](const u32x4 (&b)[CH], const u32x4 (&a)[NR][CH]) {
#pragma unroll
        for (int u = 0; u < CH; u++) {
            u32x4 bu = b[u];
            if constexpr (QT != 0) bu = qraw_deq<QT, T>(bu, gq);
#pragma unroll
            for (int i = 0; i < NR; i++)
                acc[i] = mfma16x16x32(__builtin_bit_cast(FT, a[i][u]), __builtin_bit_cast(FT, bu), acc[i]);
        }
    };
    const int nch = (nst + CH - 1) / CH;  // <= 4 (K <= 5120)
    load_a(0, aq[0]);
    for (int c = 0; c < nch; c += 2) {
        if (c + 1 < nch) { load_b(c + 1, bq[1]); load_a(c + 1, aq[1]); }
        mma(bq[0], aq[0]);
        if (c + 1 < nch) {
            if (c + 2 < nch) { load_b(c + 2, bq[0]); load_a(c + 2, aq[0]); }
            mma(bq[1], aq[1]);
        }
    }
    // partial sums of the 8 waves -> LDS, summed in wave order
#pragma unroll
    for (int i = 0; i < NR; i++)
#pragma unroll
        for (int r = 0; r < 4; r++) red[((wave * NR + i) * 16 + 4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[i][r];
    __syncthreads();
    if (eon) {
        const int i = tid >> 8, row = (tid >> 4) & 15, col = tid & 15;
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; w++) v += red[((w * NR + i) * 16 + row) * 16 + col];
        if (g.bias) v = v + e_bias;  // epilogue<>'s arithmetic with the operands loaded up front
        if constexpr (EPI == EPI_RESID) {
            ((float*)g.out)[(long)em * g.ldo + en] = v + e_res;
        } else {
            GemmArgs ge = g;
            ge.bias = nullptr;
            epilogue<EPI, T>(ge, em, en, v);
        }
    }
}

bool gemm_small_ok(int M, int K, bool lna) { return M >= 1 && K % 32 == 0 && K <= 5120 && (!lna || (K <= 1280 && K % 128 == 0)); }

template <typename T, int EPI, int QT>
static void launch_small_q(const GemmArgs& g, bool lna, hipStream_t st) {
    const int nr = g.M <= 16 ? 1 : 2;
    const size_t red = (size_t)8 * nr * 256 * sizeof(float);
    const size_t img = lna ? (size_t)nr * 16 * (g.K + 8) * sizeof(T) : 0;
    const unsigned grid = cdiv(g.N, 16);
    if (lna) {
        if (nr == 1) gemm_small_kernel<T, EPI, true, 1, QT><<<grid, 512, img + red, st>>>(g);
        else gemm_small_kernel<T, EPI, true, 2, QT><<<grid, 512, img + red, st>>>(g);
    } else {
        if (nr == 1) gemm_small_kernel<T, EPI, false, 1, QT><<<grid, 512, red, st>>>(g);
        else gemm_small_kernel<T, EPI, false, 2, QT><<<grid, 512, red, st>>>(g);
    }
}

// one launch per chunk of <= 32 rows (more rows only with block-quantized weights: every chunk reads
// the blocks, L2/MALL-hot after the first)
template <typename T, int EPI>
static void launch_small_t(const GemmArgs& g0, bool lna, hipStream_t st) {
    const size_t a_es = lna ? sizeof(float) : sizeof(T);
    const size_t o_es = (EPI == EPI_RESID || EPI == EPI_F32) ? sizeof(float) : sizeof(T);
    for (int m0 = 0; m0 < g0.M; m0 += 32) {
        GemmArgs g = g0;
        g.M = std::min(32, g0.M - m0);
        g.A = (const char*)g0.A + (size_t)m0 * g0.a_rstride * a_es;
        g.out = (char*)g0.out + (size_t)m0 * g0.ldo * o_es;
        g.a_rpb = g.o_rpb = g.M;
        switch (g.q.type) {
            case 0: launch_small_q<T, EPI, 0>(g, lna, st); break;
            case 2: launch_small_q<T, EPI, 2>(g, lna, st); break;
            case 3: launch_small_q<T, EPI, 3>(g, lna, st); break;
            case 6: launch_small_q<T, EPI, 6>(g, lna, st); break;
            case 7: launch_small_q<T, EPI, 7>(g, lna, st); break;
            case 8: launch_small_q<T, EPI, 8>(g, lna, st); break;
            default: WM_FAIL("small-M GEMM: ggml type %d not supported", g.q.type);
        }
    }
}

template <typename T>
static void launch_small_dt(int epi, const GemmArgs& g, bool lna, hipStream_t st) {
    switch (epi) {
        case EPI_STORE: launch_small_t<T, EPI_STORE>(g, lna, st); break;
        case EPI_GELU: launch_small_t<T, EPI_GELU>(g, lna, st); break;
        case EPI_RESID: launch_small_t<T, EPI_RESID>(g, lna, st); break;
        case EPI_F32: launch_small_t<T, EPI_F32>(g, lna, st); break;
        default: WM_FAIL("small-M GEMM epilogue %d not supported", epi);
    }
}

void launch_gemm_small(DType dt, int epi, const GemmArgs& g, bool lna, hipStream_t st) {
    if (g.M <= 0 || g.N <= 0) return;
    if (!gemm_small_ok(g.M, g.K, lna) || g.o_rpb != g.M || g.a_rpb != g.M || g.o_off || (epi == EPI_STORE && g.o_bstride))
        WM_FAIL("small-M GEMM shape not supported (M=%d K=%d)", g.M, g.K);
    if (dt == DType::F16) launch_small_dt<half_t>(epi, g, lna, st);
    else launch_small_dt<bf16_t>(epi, g, lna, st);
}

int g_dec_splits = 0;  // debug/tuning override of the decode-step split count (0 = heuristic)
static int dec_splits_override() { return g_dec_splits; }
// decode-step split count: the largest keeping the grid <= 256 workgroups (one per CU), with chunks
// of >= 2 K-tiles and at most 12 splits. Independent of M, so a row's sums never depend on the batch.
// Large-v3: FC1 3 splits, QKV 4, N = d GEMMs 10, FC2 12; against the round-2 rule (the smallest count
// reaching >= 160 workgroups, <= 8 splits) decode 844 -> 838 ms per step at 128 clips, 659 -> 654 at 64,
// 433 -> 413 at 16 (profiles/r02_dec_fill_ab.txt). Decode-step weights are read once per step by one
// workgroup each: non-temporal LDS-DMA (aux = 2).
static int dec_splits_for(int tiles, int nk) {
    int splits = 1;
    while (tiles * (splits + 1) <= 256 && splits < 12 && (splits + 1) * 2 <= nk) splits++;
    return splits;
}

template <typename T>
static void launch_reduce_resid_ln(const GemmArgs& g, int splits, hipStream_t st) {
    if (g.N % 4 == 0 && g.N <= 4096 && splits <= 16) {
        const int threads = cdiv(g.N / 4, 64) * 64;
        splitk_reduce_resid_ln4_kernel<T><<<g.M, threads, 0, st>>>(g, splits);
        return;
    }
    const int npt = cdiv(g.N, 256);
    if (npt <= 4) splitk_reduce_resid_ln_kernel<T, 4><<<g.M, 256, 0, st>>>(g, splits);
    else if (npt <= 8) splitk_reduce_resid_ln_kernel<T, 8><<<g.M, 256, 0, st>>>(g, splits);
    else WM_FAIL("fused LN width %d > 2048", g.N);
}

// the plain split-K reduce of a decode step: one thread per 4 columns (N % 4 == 0), 64-thread
// workgroups when that is under 64K threads so the work spreads over every CU (at 128 clips a d-wide
// reduce is 41K threads: 160 busy 256-thread workgroups before, 640 of 64 now); the same bits
template <typename T, int EPI>
static void launch_splitk_reduce(const GemmArgs& g, int splits, hipStream_t st) {
    const long total = (long)g.M * g.N, work = (g.N & 3) == 0 ? total / 4 : total;
    const int thr = work < 65536 ? 64 : 256;
    splitk_reduce_kernel<T, EPI><<<std::min<long>(4096, cdiv(work, thr)), thr, 0, st>>>(g, splits);
}

// The encoder GEMMs' tile order (gemm8p_kernel gm). Row-major (n fastest) lets the 32 workgroups an XCD
// runs at once cover ~1.6 m-tiles x 20 n-tiles of FC1, so every B tile is fetched by every XCD for every
// m-tile; groups of 4 m-tiles make them a 4 x 8 block. Measured (large-v3, 128 x 30 s, rocprofv3
// FETCH_SIZE x2, profiles/r05_gemm_gm_pmc.txt): FC1 2068 -> 1111 MB per launch, QKV 1243 -> 848 MB; the
// d-wide GEMMs (5 n-tiles) fetched more (857 -> 987 MB), and stay row-major. The encode phase time does not
// move (321.3 / 320.1 / 324.0 / 331.8 ms at gm 0 / 4 / 8 / 16): the kernel is bound by its MFMA / LDS
// schedule, not by L2 misses.
static int gemm_group_m(int tiles_n) {
    static const int env = getenv("WHISPER_MI355X_GEMM_GM") ? atoi(getenv("WHISPER_MI355X_GEMM_GM")) : -1;
    if (env >= 0) return env;
    return tiles_n >= 8 ? 4 : 0;
}

template <typename T, int EPI>
static void launch_t(const GemmArgs& g, hipStream_t st) {
    if (g.w8_scale) {  // e4m3 weights: the decode-step split-K kernel only
        const bool fused_ln = EPI == EPI_RESID && g.ln_out != nullptr;
        if (!(g.splitk_ws && g.M <= 128 && g.K % 64 == 0 && g_gemm_variant != 0 && (EPI != EPI_RESID || fused_ln))) WM_FAIL("e4m3 weights need the decode-step GEMM path (M %d <= 128, K %% 64 == 0)", g.M);
    }
    const bool big256 = g_gemm_variant >= 2 ||
                        (g_gemm_variant < 0 && (g.N % 256 == 0 || g.N >= 1024) && g.M >= 1024);
    if ((long)g.M * g.N >= 256L * 128 * 128 && g.K % 64 == 0 && big256) {
        const int tn = cdiv(g.N, 256);
        if (g_gemm_variant == 2) gemm256_kernel<T, EPI, false><<<tn * cdiv(g.M, 256), 512, 0, st>>>(g, tn);
        else if (g_gemm_variant == 3) gemm256_kernel<T, EPI, true><<<tn * cdiv(g.M, 256), 512, 0, st>>>(g, tn);
        else {
            GemmArgs ga = g;
            ga.stamps = g_gemm_stamps;
            gemm8p_kernel<T, EPI><<<tn * cdiv(g.M, 256), 512, 0, st>>>(ga, tn, gemm_group_m(tn));
        }
        return;
    }
    if ((long)g.M * g.N >= 256L * 128 * 128 && g.K % 64 == 0 && g_gemm_variant != 0) {
        const int tn = cdiv(g.N, 128);
        gemm_glds_kernel<T, EPI><<<tn * cdiv(g.M, 128), 256, 0, st>>>(g, tn);
        return;
    }
    if ((long)g.M * g.N >= 256L * 128 * 128) {
        dim3 grid(cdiv(g.N, 128), cdiv(g.M, 128));
        gemm_kernel<T, 128, 128, 2, 2, EPI, false><<<grid, 256, 0, st>>>(g, g.K);
        return;
    }
    const bool fused_ln = EPI == EPI_RESID && g.ln_out != nullptr;
    const int nk = cdiv(g.K, 64);
    if (g.splitk_ws && (g.M <= 128 || !fused_ln) && g.K % 64 == 0 && g_gemm_variant != 0) {
        // decode step and small prefill (gemm_dec_kernel; M > 128 as 128-row chunks, gridDim.y): the
        // split count depends on N and K only (dec_splits_for), so a row's sums, and the bits of every
        // result, do not depend on how many clips share the launch (batch == single). (Chunks of >= 5
        // K-tiles measured faster in isolation, 9.6 vs 10.4 us at N = K = 1280, but not in the decode
        // step: 82.0 vs 81.6 us of GEMM + reduce per layer.)
        const int tiles = cdiv(g.N, 64);
        int splits = dec_splits_for(tiles, nk);
        if (dec_splits_override() > 0) splits = std::min(dec_splits_override(), nk);
        // unsplit at M <= 64 (the logits GEMM of a small batch): the 64-row register-staged kernel
        // below wastes less of its tile (measured 23 vs 51 us at M = 16, N = 51866)
        const bool small_unsplit = splits == 1 && !fused_ln && g.M <= 64 && !g.w8_scale;
        if (g.w8_scale && (long)splits * g.M * g.N > g.splitk_ws_elems) WM_FAIL("e4m3 decode GEMM: split-K workspace too small");
        if ((long)splits * g.M * g.N <= g.splitk_ws_elems && !small_unsplit) {
            const int kc = cdiv(nk, splits) * 64;
            splits = cdiv(g.K, kc);
            if (splits == 1 && !fused_ln) {
                if (g.w8_scale) launch_dec<T, EPI, false, true>(g, tiles, 1, kc, st);
                else launch_dec<T, EPI, false, false>(g, tiles, 1, kc, st);
                return;
            }
            if (g.w8_scale) launch_dec<T, EPI, true, true>(g, tiles, splits, kc, st);
            else launch_dec<T, EPI, true, false>(g, tiles, splits, kc, st);
            if (fused_ln) {
                launch_reduce_resid_ln<T>(g, splits, st);
            } else {
                launch_splitk_reduce<T, EPI>(g, splits, st);
            }
            return;
        }
    }
    if (g.splitk_ws && g.M <= 128) {
        // decode step (M = active clips <= 128): one M tile, the weight stream read exactly once;
        // K split to ~128 workgroups with >= 4 K-tiles each (partial slabs: M*N*splits*8 bytes)
        const int BM = g.M <= 64 ? 64 : 128;
        const int tiles = cdiv(g.N, 64);
        int splits = std::min(std::max(1, 128 / tiles), std::max(1, nk / 4));
        while (splits > 1 && (long)splits * g.M * g.N > g.splitk_ws_elems) splits--;
        if (splits > 1 || fused_ln) {
            const int kc = cdiv(cdiv(g.K, splits), 64) * 64;
            splits = cdiv(g.K, kc);
            dim3 grid(tiles, 1, splits);
            if (BM == 64) gemm_kernel<T, 64, 64, 2, 2, EPI, true><<<grid, 256, 0, st>>>(g, kc);
            else gemm_kernel<T, 128, 64, 2, 2, EPI, true><<<grid, 256, 0, st>>>(g, kc);
            if (fused_ln) {
                const int npt = cdiv(g.N, 256);
                if (npt <= 4) splitk_reduce_resid_ln_kernel<T, 4><<<g.M, 256, 0, st>>>(g, splits);
                else if (npt <= 8) splitk_reduce_resid_ln_kernel<T, 8><<<g.M, 256, 0, st>>>(g, splits);
                else WM_FAIL("fused LN width %d > 2048", g.N);
            } else {
                launch_splitk_reduce<T, EPI>(g, splits, st);
            }
        } else {
            dim3 grid(tiles, 1);
            if (BM == 64) gemm_kernel<T, 64, 64, 2, 2, EPI, false><<<grid, 256, 0, st>>>(g, g.K);
            else gemm_kernel<T, 128, 64, 2, 2, EPI, false><<<grid, 256, 0, st>>>(g, g.K);
        }
        return;
    }
    if (fused_ln) WM_FAIL("fused LN requires the decode split-K path");
    const int tiles = cdiv(g.N, 64) * cdiv(g.M, 64);
    int splits = std::min(16, std::max(1, 512 / tiles));
    splits = std::min(splits, std::max(1, nk / 2));
    while (splits > 1 && (long)splits * g.M * g.N > g.splitk_ws_elems) splits--;
    if (!g.splitk_ws || splits <= 1) {
        dim3 grid(cdiv(g.N, 64), cdiv(g.M, 64));
        gemm_kernel<T, 64, 64, 2, 2, EPI, false><<<grid, 256, 0, st>>>(g, g.K);
        return;
    }
    const int kc = cdiv(cdiv(g.K, splits), 64) * 64;
    splits = cdiv(g.K, kc);
    dim3 grid(cdiv(g.N, 64), cdiv(g.M, 64), splits);
    gemm_kernel<T, 64, 64, 2, 2, EPI, true><<<grid, 256, 0, st>>>(g, kc);
    const long total = (long)g.M * g.N;
    splitk_reduce_kernel<T, EPI><<<std::min<long>(1024, cdiv(total, 256)), 256, 0, st>>>(g, splits);
}

template <typename T>
static void launch_dt(int epi, const GemmArgs& g, hipStream_t st) {
    switch (epi) {
        case EPI_STORE: launch_t<T, EPI_STORE>(g, st); break;
        case EPI_GELU: launch_t<T, EPI_GELU>(g, st); break;
        case EPI_GELU_F: launch_t<T, EPI_GELU_F>(g, st); break;
        case EPI_RESID: launch_t<T, EPI_RESID>(g, st); break;
        case EPI_GELU_POS: launch_t<T, EPI_GELU_POS>(g, st); break;
        case EPI_F32: launch_t<T, EPI_F32>(g, st); break;
        case EPI_CROSSKV: launch_t<T, EPI_CROSSKV>(g, st); break;
        case EPI_QKV_DEC: launch_t<T, EPI_QKV_DEC>(g, st); break;
        default: WM_FAIL("bad epilogue %d", epi);
    }
}

template <typename T>
static int launch_partials_t(const GemmArgs& g, hipStream_t st) {
    if (!g.splitk_ws || g.M > 128 || g.K % 64 != 0) return 0;
    const int nk = g.K / 64, tiles = cdiv(g.N, 64);
    int splits = dec_splits_for(tiles, nk);
    if (dec_splits_override() > 0) splits = std::min(dec_splits_override(), nk);
    const int kc = cdiv(nk, splits) * 64;
    splits = cdiv(g.K, kc);
    if ((long)splits * g.M * g.N > g.splitk_ws_elems) return 0;
    if (g.w8_scale) launch_dec<T, EPI_STORE, true, true>(g, tiles, splits, kc, st);
    else launch_dec<T, EPI_STORE, true, false>(g, tiles, splits, kc, st);
    return splits;
}


int launch_gemm_partials(DType dt, const GemmArgs& g, hipStream_t st) {
    return dt == DType::F16 ? launch_partials_t<half_t>(g, st) : launch_partials_t<bf16_t>(g, st);
}

template <typename T>
static void launch_mx_t(int epi, const GemmArgs& g, const float* sa, const float* sb, hipStream_t st) {
    const int tn = cdiv(g.N, 256), grid = tn * cdiv(g.M, 256);
    switch (epi) {
        case EPI_STORE: gemm8p_mx_kernel<T, EPI_STORE><<<grid, 512, 0, st>>>(g, tn, sa, sb); break;
        case EPI_GELU: gemm8p_mx_kernel<T, EPI_GELU><<<grid, 512, 0, st>>>(g, tn, sa, sb); break;
        case EPI_GELU_F: gemm8p_mx_kernel<T, EPI_GELU_F><<<grid, 512, 0, st>>>(g, tn, sa, sb); break;
        case EPI_RESID: gemm8p_mx_kernel<T, EPI_RESID><<<grid, 512, 0, st>>>(g, tn, sa, sb); break;
        default: WM_FAIL("fp8 GEMM epilogue %d not supported", epi);
    }
}

void launch_gemm_fp8(DType dt, int epi, const GemmArgs& g, const float* a_scale, const float* b_scale, hipStream_t st) {
    if (g.M <= 0 || g.N <= 0) return;
    if (g.K % 128 != 0 || g.N % 16 != 0 || g.a_rpb <= 0 || g.o_rpb <= 0 || !a_scale || !b_scale)
        WM_FAIL("fp8 gemm shape not supported (N=%d K=%d)", g.N, g.K);
    if (dt == DType::F16) launch_mx_t<half_t>(epi, g, a_scale, b_scale, st);
    else launch_mx_t<bf16_t>(epi, g, a_scale, b_scale, st);
}

void launch_quant_rows_fp8(DType dt, const void* x, long rows, int K, void* q, float* s, hipStream_t st) {
    if (rows <= 0) return;
    if (K % 8 != 0) WM_FAIL("fp8 quantization needs K %% 8 == 0");
    const unsigned grid = (unsigned)((rows + 3) / 4);
    if (dt == DType::F16) quant_rows_fp8_kernel<half_t><<<grid, 256, 0, st>>>((const half_t*)x, rows, K, (uint8_t*)q, s);
    else quant_rows_fp8_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)x, rows, K, (uint8_t*)q, s);
}

void launch_gemm(DType dt, int epi, const GemmArgs& g, hipStream_t st) {
    if (g.M <= 0 || g.N <= 0) return;
    if (g.K % 8 != 0 || g.a_rpb <= 0 || g.o_rpb <= 0) WM_FAIL("gemm shape not supported (K=%d)", g.K);
    if (dt == DType::F16) launch_dt<half_t>(epi, g, st);
    else launch_dt<bf16_t>(epi, g, st);
}

}  // namespace wm
