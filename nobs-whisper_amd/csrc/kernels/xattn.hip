// Decode-step cross attention computed straight from the encoder output (SURVEY.md §8a row a10,
// the roofline kernel of the headline benchmark).
//
// whisper.cpp caches K = s*(E.Wk^T) and V = E.Wv^T + bv for every decoder layer ([ext] kv_cross)
// and each decode step reads both: 2 x 1500 x d values per clip and layer. Both products are linear
// in the encoder output E [1500][d], so per head h the same scores and outputs are
//   score_t  = q_h . K_h[t]            = E[t] . Q'_h,   Q'_h = s * Wk_h^T q_h        (d values)
//   o_h      = sum_t p_t V_h[t] / l    = (sum_t p_t E[t] / l) . Wv_h^T + bv_h
// so a step needs ONE pass over E per clip and layer instead of a pass over K and one over V:
// half the HBM bytes of the cached form, and no 31 GB cross cache at batch 128. The extra work is
// MFMA work (E [16 rows][d] x Q' [d][2H] and P [H][16] x E [16][d] per tile), which this
// HBM-bound step has to spare.
//
//   xattn_qproj_kernel    Q'_h = s * Wk_h^T q_h for every head, split into hi + lo parts of the
//                         MFMA type so the scores keep ~16 mantissa bits (Q' rows 0..H-1 = hi,
//                         H..2H-1 = lo); a batched [n x 64] . [64 x d] GEMM per head.
//   xattn_step_kernel     one workgroup = one clip x one split of the 1500 rows; E tiles of 16
//                         rows stream HBM -> LDS by LDS-DMA (3 stages, two tiles in flight across
//                         raw barriers); each wave owns CT x 32 columns: partial scores
//                         S^T[16][2H] (v_mfma_16x16x32, A = E rows), a cross-wave reduce in LDS,
//                         online softmax per head (lazy rescale: the running max moves only when
//                         a tile exceeds it by more than `thr` in log2 units), then
//                         O^T[cols][heads] += E^T . P^T (v_mfma_32x32x16, A = E^T by
//                         ds_read_b64_tr_b16 from the same LDS image). Writes the unnormalised
//                         partial O, m and l of its split.
//   xattn_combine_kernel  merges the splits, E~ = sum_s w_s O_s / L (hi + lo parts again), and
//                         applies Wv_h + bv: o[i][h*64+j] in the MFMA type, the input of the
//                         cross-attention output projection.
//
// Roofline: HBM-bound on E: 1500 x d x 2 bytes per clip and layer (3.84 MB for large-v3).
// Numerics vs whisper.cpp: no rounding of K and V to the cache type (the products are formed in
// f32 from the same rounded E and weights), P rounded to the MFMA type as ggml rounds it to f16
// (here before the final 1/l instead of after it).
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace wm {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));

// 16-byte chunk swizzle inside each 256-byte group of an LDS row: conflict-free for ds_read_b128
// of 16 rows x one chunk and for ds_read_b64_tr_b16 of 4 rows x 2 chunks (guide T10 image (b)).
__device__ __forceinline__ int xsw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int xphys(int row, int ch) { return (ch & ~15) | ((ch & 15) ^ xsw(row)); }

template <int N>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ v4s ds_read_tr(unsigned lds_addr) {
    v4s r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr));
    return r;
}
// Reductions over the 16 lanes of a row by DPP (quad xor 1, quad xor 2, half-row mirror, row
// mirror): no LDS round trips, unlike __shfl_xor (ds_bpermute). Every lane gets the same bits (each
// step adds two values commutatively).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max16(float x) {
    x = fmaxf(x, dpp_f<0xB1>(x));
    x = fmaxf(x, dpp_f<0x4E>(x));
    x = fmaxf(x, dpp_f<0x141>(x));
    return fmaxf(x, dpp_f<0x140>(x));
}
__device__ __forceinline__ float sum16(float x) {
    x = x + dpp_f<0xB1>(x);
    x = x + dpp_f<0x4E>(x);
    x = x + dpp_f<0x141>(x);
    return x + dpp_f<0x140>(x);
}

// LDS writes of this wave done, then the workgroup barrier. A raw s_barrier, not __syncthreads():
// the latter waits vmcnt(0) and would drain the LDS-DMA tiles kept in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---- Q' projection -----------------------------------------------------------------------------
// grid (cdiv(d, 64 MT), H, cdiv(n, 16 NT)), 256 threads: wave w = columns [64 MT x + 16 MT w, +16 MT) x
// 16 NT tokens, K = 64. Swapped product C^T[c][tok] = Wk_h^T[c][:] . q_h[tok][:]: a lane holds 4
// consecutive columns of one token, stored as one 8-byte hi and one 8-byte lo write. Every (MT, NT)
// gives the same bits (one MFMA pair per 16 x 16 tile whatever the tiling).
template <typename T, int MT, int NT, bool STG = false>
__global__ void __launch_bounds__(256) xattn_qproj_kernel(const T* __restrict__ q, const T* __restrict__ wkt, int n, int d,
                                                          int H, float scale, T* __restrict__ qx) {
    typedef typename Frag<T>::type FT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = blockIdx.x * 64 * MT + wave * 16 * MT, h = blockIdx.y, i0 = blockIdx.z * 16 * NT;
    // STG: the hi / lo tiles of the workgroup (16 NT tokens x 64 MT columns) staged in LDS, then written as
    // whole 16-byte chunks of each token's row (the MFMA layout gives a lane 8 bytes of 4 columns)
    constexpr int SW = 64 * MT + 8;  // padded row of the staging image (T elements)
    __shared__ __attribute__((aligned(16))) T simg[STG ? 2 * 16 * NT * SW : 1];
    if (!STG && c0 >= d) return;  // wave-uniform (the launch keeps d % (64 MT) == 0 for STG)
    const u32x4 zero = {0, 0, 0, 0};
    FT af[MT][2], bq[NT][2];
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
        const int c = c0 + mt * 16 + (lane & 15);
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
            af[mt][ks] = __builtin_bit_cast(FT, *(const u32x4*)(wkt + ((long)h * d + c) * 64 + ks * 32 + 8 * (lane >> 4)));
    }
#pragma unroll
    for (int nt = 0; nt < NT; nt++) {
        const int i = i0 + nt * 16 + (lane & 15);
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
            bq[nt][ks] = __builtin_bit_cast(FT, i < n ? *(const u32x4*)(q + (long)i * d + h * 64 + ks * 32 + 8 * (lane >> 4)) : zero);
    }
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ks++) acc = mfma16x16x32(af[mt][ks], bq[nt][ks], acc);
            const int i = i0 + nt * 16 + (lane & 15);
            T hi[4], lo[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float v = acc[r] * scale;
                hi[r] = (T)v;
                lo[r] = (T)(v - (float)hi[r]);
            }
            if constexpr (STG) {
                const int tl = nt * 16 + (lane & 15), cl = wave * 16 * MT + mt * 16 + 4 * (lane >> 4);
                *(uint2*)(simg + tl * SW + cl) = *(const uint2*)hi;
                *(uint2*)(simg + (16 * NT + tl) * SW + cl) = *(const uint2*)lo;
                continue;
            }
            if (i >= n) continue;
            const int c = c0 + mt * 16 + 4 * (lane >> 4);
            *(uint2*)(qx + ((long)i * 2 * H + h) * d + c) = *(const uint2*)hi;
            *(uint2*)(qx + ((long)i * 2 * H + H + h) * d + c) = *(const uint2*)lo;
        }
    if constexpr (STG) {
        __syncthreads();
        constexpr int CH = 64 * MT / 8, ROWS = 2 * 16 * NT;  // 16-byte chunks per row, hi + lo rows
        const int cb = blockIdx.x * 64 * MT;
        for (int e = threadIdx.x; e < ROWS * CH; e += 256) {
            const int row = e / CH, ch = e - row * CH;
            const int part = row / (16 * NT), tl = row - part * 16 * NT, i = i0 + tl;
            if (i < n)
                *(u32x4*)(qx + ((long)i * 2 * H + part * H + h) * d + cb + ch * 8) = *(const u32x4*)(simg + row * SW + ch * 8);
        }
    }
}

// ---- one pass over E per (clip, split) ------------------------------------------------------------
// NW waves x CT column tiles of 32: d = NW*CT*32, H = d/64, NQ = ceil(2H/16) score column tiles.
// AUX: cache-policy bits of the E loads (2 = non-temporal).
template <typename T, int NW, int CT, int AUX>
__global__ void __launch_bounds__(NW * 64) xattn_step_kernel(const T* __restrict__ enc, const int* __restrict__ slot,
                                                             const T* __restrict__ qx, int Tn, int splits, float thr,
                                                             float* __restrict__ opart, float* __restrict__ ml, int ostg = 0) {
    typedef typename Frag<T>::type FT;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int D = NW * CT * 32, H = D / 64, NQ = (2 * H + 15) / 16;
    constexpr int RC = D / 8;            // 16-byte chunks per E row
    constexpr int NS = 3;                // LDS stages
    constexpr int TILE = 16 * RC;        // u32x4 per 16-row tile
    constexpr int NH = (H + 15) / 16;    // score column tiles holding the hi columns (0..H-1)
    constexpr int RSR = 16 * NH + 4;     // f32 row stride of the score partials (bank spread)
    // P image [32 heads][PS] T, rows 0..15 of a head contiguous; PS = 20 (not 16): the P.V operand reads of 32
    // lanes (one head each, 8 bytes at rows 4 hh and 8 + 4 hh) then hit 32 distinct bank pairs (head stride 10
    // dwords) instead of 4-way conflicting at a stride of 8 dwords
    constexpr int PS = 20;
    constexpr int STG_B = NS * TILE * 16, RED_B = NW * 16 * RSR * 4, P_B = 32 * PS * (int)sizeof(T);
    static_assert(RC % 16 == 0, "d must be a multiple of 128");
    static_assert(H * 16 <= NW * 64, "one softmax lane per (head, row)");
    static_assert(H <= 32, "heads are the N = 32 side of the P.V MFMA");
    // ONE LDS object (a second __shared__ object can make hipcc wait vmcnt(0) before LDS reads)
    __shared__ __attribute__((aligned(16))) char lds[STG_B + RED_B + P_B + 32 * 4 + 16];
    u32x4* stg = (u32x4*)lds;
    float* red = (float*)(lds + STG_B);
    T* pimg = (T*)(lds + STG_B + RED_B);              // P [head][PS] (rows 0..15 used)
    float* alph = (float*)(lds + STG_B + RED_B + P_B);  // per-head rescale of the tile
    int* flag = (int*)(alph + 32);                      // [2]: some head rescaled at tile t (parity t&1)

    const int sp = blockIdx.x, i = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nt_all = (Tn + 15) >> 4;
    const int tb = sp * nt_all / splits, ntile = (sp + 1) * nt_all / splits - tb;
    const T* E = enc + (long)slot[i] * Tn * D;
    const int cw = wave * CT * 32;  // this wave's first column

    for (int e = tid; e < 32 * PS; e += NW * 64) pimg[e] = (T)0.0f;
    if (tid < 32) alph[tid] = 1.0f;
    if (tid < 2) flag[tid] = 0;

    // Q' fragments (B operand of the scores): head' = j*16 + (lane&15), 8 columns per lane
    const u32x4 zero = {0, 0, 0, 0};
    FT qf[CT][NQ];
    {
        const T* Q = qx + (long)i * 2 * H * D;
#pragma unroll
        for (int kk = 0; kk < CT; kk++)
#pragma unroll
            for (int j = 0; j < NQ; j++) {
                const int hp = j * 16 + (lane & 15);
                qf[kk][j] = __builtin_bit_cast(
                    FT, hp < 2 * H ? *(const u32x4*)(Q + (long)hp * D + cw + kk * 32 + 8 * (lane >> 4)) : zero);
            }
        // consume the loads here, before any LDS-DMA is issued, so hipcc's wait for them sits outside the loop
#pragma unroll
        for (int kk = 0; kk < CT; kk++)
#pragma unroll
            for (int j = 0; j < NQ; j++) asm volatile("" ::"v"(qf[kk][j]));
    }
    // LDS-DMA sources: piece p = wave + k*NW (64 chunks), lane -> physical chunk -> (row, logical chunk)
    int prow[CT], poff[CT];
#pragma unroll
    for (int k = 0; k < CT; k++) {
        const int qq = (wave + k * NW) * 64 + lane;
        const int row = qq / RC, pc = qq - row * RC;
        prow[k] = row;
        poff[k] = xphys(row, pc) * 8;
    }
    auto issue = [&](int t) {
        const int row0 = (tb + t) * 16;
        u32x4* st = stg + (t % NS) * TILE;
#pragma unroll
        for (int k = 0; k < CT; k++) {
            const int gr = min(row0 + prow[k], Tn - 1);
            __builtin_amdgcn_global_load_lds((const void*)(E + (long)gr * D + poff[k]),
                                             (lds_ptr_t)(st + (wave + k * NW) * 64), 16, 0, AUX);
        }
    };

    f32x16 oacc[CT];
#pragma unroll
    for (int k = 0; k < CT; k++)
#pragma unroll
        for (int r = 0; r < 16; r++) oacc[k][r] = 0.0f;
    float m_run = -INFINITY, l_run = 0.0f;  // softmax lanes (tid < 16H): head tid>>4
    const float LOG2E = 1.44269504088896340736f;
    const int hh = lane >> 5;

    issue(0);
    if (ntile > 1) issue(1);
    for (int t = 0; t < ntile; t++) {
        // B1: tile t landed (this wave's pieces), every wave left tile t-1 (stage (t+2)%3 is free)
        if (t + 1 < ntile) wait_vm<CT>();
        else wait_vm<0>();
        lds_barrier();
        if (t + 2 < ntile) issue(t + 2);
        const u32x4* st = stg + (t % NS) * TILE;

        // scores: S^T[row][head'] over this wave's columns
        f32x4 sacc[NQ];
#pragma unroll
        for (int j = 0; j < NQ; j++) sacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        {
            const int row = lane & 15;
            FT ef[CT];  // all reads in flight before the first MFMA
#pragma unroll
            for (int kk = 0; kk < CT; kk++)
                ef[kk] = __builtin_bit_cast(FT, st[row * RC + xphys(row, (cw >> 3) + kk * 4 + (lane >> 4))]);
#pragma unroll
            for (int kk = 0; kk < CT; kk++)
#pragma unroll
                for (int j = 0; j < NQ; j++) sacc[j] = mfma16x16x32(ef[kk], qf[kk][j], sacc[j]);
        }
        {
            // hi + lo of every head inside the wave before the cross-wave exchange: the lo column
            // H+h sits in tile jh + H/16 at lane offset H%16 (or one tile further, 16 lanes back),
            // constant per tile, so a DPP row shift brings it under its hi column
            constexpr int J0 = H / 16, D0 = H % 16;
            float* rw = red + wave * 16 * RSR;
#pragma unroll
            for (int jh = 0; jh < NH; jh++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float lo;
                    if constexpr (D0 == 0) {
                        lo = sacc[jh + J0][r];
                    } else {
                        const float a = dpp_f<0x100 + D0>(sacc[jh + J0][r]);  // lane L <- L + D0
                        // lane L <- L - (16 - D0); no such tile: those lanes are past the last head
                        const float b = jh + J0 + 1 < NQ ? dpp_f<0x110 + 16 - D0>(sacc[min(jh + J0 + 1, NQ - 1)][r]) : 0.0f;
                        lo = (lane & 15) < 16 - D0 ? a : b;
                    }
                    rw[(4 * (lane >> 4) + r) * RSR + jh * 16 + (lane & 15)] = sacc[jh][r] + lo;
                }
        }
        lds_barrier();  // B2: partial scores of every wave in LDS

        // online softmax, one lane per (head, row); hi + lo partials summed in a fixed order
        if (tid < 16 * H) {
            const int h = tid >> 4, r = tid & 15;
            float sv = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                sv += red[(w * 16 + r) * RSR + h];
            }
            const float s2 = (tb + t) * 16 + r < Tn ? sv * LOG2E : -INFINITY;
            const float mx = max16(s2);
            float alpha = 1.0f;
            if (mx > m_run + thr) {  // first tile (m_run = -inf) or the max moved by more than thr
                alpha = __builtin_amdgcn_exp2f(m_run - mx);
                m_run = mx;
                flag[t & 1] = 1;
            }
            const T pt = (T)__builtin_amdgcn_exp2f(s2 - m_run);
            l_run = l_run * alpha + sum16((float)pt);
            pimg[h * PS + r] = pt;
            if (r == 0) alph[h] = alpha;
        }
        if (tid == 0) flag[(t + 1) & 1] = 0;  // last read in tile t-1's P.V, before B1
        lds_barrier();  // B3: P, alpha and the flag in LDS

        // O^T[cols][heads] += E^T . P^T  (every lane active: the transposed reads need EXEC = all ones).
        // E^T fragments by inline-asm ds_read_b64_tr_b16: with an LDS-DMA in flight hipcc puts
        // vmcnt(0) in front of the builtin form (it cannot rule out the DMA writing the bytes it
        // reads), which would drain the prefetch of tile t+2; the DMA/read ordering here is the
        // explicit vmcnt + barrier of B1. P, the E^T fragments and the rescale flag are all read
        // before the one wait.
        FT pf;
        {
            const T* pr = pimg + (lane & 31) * PS + 4 * hh;
            const v4s lo = *(const v4s*)pr;
            const v4s hi = *(const v4s*)(pr + 8);
            pf = __builtin_bit_cast(FT, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
        const int tg = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
        const int rlo = 4 * hh + tq, rhi = rlo + 8;
        const unsigned img = (unsigned)(unsigned long)(lds_ptr_t)(const void*)st;
        v4s elo[CT], ehi[CT];
#pragma unroll
        for (int k = 0; k < CT; k++) {
            const int ch = ((cw + k * 32) >> 3) + tg * 2 + (tp >> 1);
            elo[k] = ds_read_tr(img + rlo * RC * 16 + 16 * xphys(rlo, ch) + 8 * (tp & 1));
            ehi[k] = ds_read_tr(img + rhi * RC * 16 + 16 * xphys(rhi, ch) + 8 * (tp & 1));
        }
        const int fl = flag[t & 1];
        const float al = alph[lane & 31];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs behind the wait (guide §5.4 rule 18)
        if (fl) {
#pragma unroll
            for (int k = 0; k < CT; k++)
#pragma unroll
                for (int r = 0; r < 16; r++) oacc[k][r] *= al;
        }
#pragma unroll
        for (int k = 0; k < CT; k++) {
            const FT ef = __builtin_bit_cast(FT, __builtin_shufflevector(elo[k], ehi[k], 0, 1, 2, 3, 4, 5, 6, 7));
            oacc[k] = mfma32x32x16(ef, pf, oacc[k]);
        }
    }

    // partial O (unnormalised) [i][sp][h][c], m and l [i][sp][h][2] (write-through stores of the
    // partials measured no faster, not kept)
    const int h = lane & 31;
    if (ostg) {
        // (round 6) the wave's O^T tile [H][CT x 32 columns] staged in the free E stages (rows padded by 4 floats),
        // then written as 16-byte chunks of consecutive columns per lane: every store instruction covers whole
        // 128-byte lines of the head rows (the direct form below writes 32 bytes of each of 32 rows). Same values.
        constexpr int OW = CT * 32 + 4;
        static_assert(NW * H * OW * 4 <= STG_B, "O staging fits the E stages");
        __syncthreads();  // every wave is done with the last E stage
        float* so = (float*)lds + wave * H * OW;
        if (h < H) {
#pragma unroll
            for (int k = 0; k < CT; k++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int c = k * 32 + 8 * g + 4 * hh;
                    *(f32x4*)(so + h * OW + c) = (f32x4){oacc[k][4 * g], oacc[k][4 * g + 1], oacc[k][4 * g + 2], oacc[k][4 * g + 3]};
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        float* ob = opart + ((long)i * splits + sp) * H * D + cw;
        for (int e = lane; e < H * CT * 8; e += 64) {
            const int hr = e / (CT * 8), ch = e - hr * (CT * 8);
            *(f32x4*)(ob + (long)hr * D + ch * 4) = *(const f32x4*)(so + hr * OW + ch * 4);
        }
    } else if (h < H) {
        float* o = opart + (((long)i * splits + sp) * H + h) * D;
#pragma unroll
        for (int k = 0; k < CT; k++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int c = cw + k * 32 + 8 * g + 4 * hh;
                const f32x4 v = {oacc[k][4 * g], oacc[k][4 * g + 1], oacc[k][4 * g + 2], oacc[k][4 * g + 3]};
                *(f32x4*)(o + c) = v;
            }
    }
    if (tid < 16 * H && (tid & 15) == 0) {
        float* p = ml + (((long)i * splits + sp) * H + (tid >> 4)) * 2;
        p[0] = m_run;
        p[1] = l_run;
    }
}

// ---- merge the splits and apply Wv ---------------------------------------------------------------
// grid (H, cdiv(n, TOK)), 512 threads. Phase A (every thread, coalesced 16-byte partial reads): the
// merged E~ = sum_s w_s O_s / L of TOK tokens x d columns, split into hi / lo rows of an LDS image
// [2 TOK][d] (16-byte chunks XOR-swizzled by row). Phase B: wave w takes the 32-column k-steps
// w, w+8, ...: M = 2 TOK (hi, lo rows), N = 64 outputs, Wv rows straight from global (L2-shared by the
// head's token blocks); the 8 waves' partial products are summed through LDS.
// TOK = 8 (the default): one 16-row MFMA tile holds the hi and lo rows, and twice the workgroups fill
// the chip (160 -> 320 at 128 clips); every output is bit-identical to TOK = 16 (each MFMA output row
// is its own dot product; the final sum keeps the wave order, hi before lo).
// m is in log2 units (the step kernel scales scores by log2 e).
template <typename T, int TOK, int PF, bool EARLYW>
__global__ void __launch_bounds__(512) xattn_combine_kernel(const float* __restrict__ opart, const float* __restrict__ ml,
                                                            int splits, const T* __restrict__ wv, const float* __restrict__ bv,
                                                            int n, int d, int H, T* __restrict__ out) {
    typedef typename Frag<T>::type FT;
    constexpr int DMAX = 1280;
    // 16-row A tiles: (hi 0-15, lo 16-31) for TOK = 16, (hi 0-7, lo 8-15) for 8, (hi 0-3, lo 4-7, rows
    // 8-15 unused: MFMA output rows are independent) for 4
    constexpr int NA = TOK >= 8 ? TOK / 8 : 1, RT = 16 * NA;
    const int h = blockIdx.x, i0 = blockIdx.y * TOK;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    __shared__ __attribute__((aligned(16))) char lds[RT * DMAX * 2 + TOK * 16 * 4];
    T* aimg = (T*)lds;                           // [RT][d]: rows 0..TOK-1 hi, TOK..2 TOK-1 lo
    float* red = (float*)lds;                    // after phase B: [8 waves][RT][64] (reuses aimg)
    float* wgt = (float*)(lds + RT * DMAX * 2);  // [TOK tokens][16 splits]
    static_assert(8 * RT * 64 * 4 <= RT * DMAX * 2, "reduce image fits the A image");
    auto slot_of = [&](int row, int ch) { return row * d + ((ch & ~15) | ((ch & 15) ^ (row & 15))) * 8; };
    // the split weights: every split's (m, l) loaded at once (one memory round trip), then the
    // reductions in split order
    if (tid < TOK) {
        const int i = i0 + tid;
        if (i < n) {
            const float* p = ml + ((long)i * splits * H + h) * 2;
            float2 q[16];
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s < splits) q[s] = *(const float2*)(p + (long)s * H * 2);
            float M = -INFINITY;
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s < splits) M = fmaxf(M, q[s].x);
            float L = 0.0f;
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s < splits) L += __builtin_amdgcn_exp2f(q[s].x - M) * q[s].y;
            const float inv = 1.0f / L;
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s < splits) wgt[tid * 16 + s] = __builtin_amdgcn_exp2f(q[s].x - M) * inv;
        } else {
            for (int s = 0; s < splits; s++) wgt[tid * 16 + s] = 0.0f;
        }
    }
    // Wv fragments of this wave's k-steps (w, w+8, ...; d <= 1280 gives at most 5), loaded before
    // phase A so their L2 latency overlaps the partial-O reads (loading them after phase A fits two
    // workgroups per CU but spills: 19.4 vs 18.2 us at 128 clips)
    constexpr int KMAX = DMAX / 256;
    const int r16 = lane & 15, kq = lane >> 4;
    FT bfp[KMAX][4];
    auto load_wv = [&]() {
#pragma unroll
        for (int k = 0; k < KMAX; k++) {
            const int ks = wave + 8 * k;
            if (ks < d / 32) {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    bfp[k][j] = __builtin_bit_cast(FT, *(const u32x4*)(wv + ((long)h * 64 + j * 16 + r16) * d + ks * 32 + 8 * kq));
            }
        }
    };
    if constexpr (EARLYW) load_wv();
    // the partial sums: NE chunks per split, PF splits in flight (the first PF go out with the weight
    // and Wv loads, before the barrier; a slot is reloaded with split s + PF once split s is summed);
    // split order per element kept
    const int q4 = d / 4;
    constexpr int NE = (TOK * (DMAX / 4) + 511) / 512;
    float4 a[NE], x[PF][NE];
    const float* src[NE];
#pragma unroll
    for (int j = 0; j < NE; j++) {
        a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int e = min(tid + 512 * j, TOK * q4 - 1);
        const int t = e / q4, c = (e - t * q4) * 4;
        src[j] = opart + ((long)min(i0 + t, n - 1) * splits * H + h) * d + c;
    }
#pragma unroll
    for (int u = 0; u < PF; u++)
        if (u < splits) {
#pragma unroll
            for (int j = 0; j < NE; j++) x[u][j] = *(const float4*)(src[j] + (long)u * H * d);
        }
    __syncthreads();
    for (int s0 = 0; s0 < splits; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int s = s0 + u;
            if (s >= splits) break;
#pragma unroll
            for (int j = 0; j < NE; j++) {
                const int t = min(tid + 512 * j, TOK * q4 - 1) / q4;
                const float w = wgt[t * 16 + s];
                a[j].x += w * x[u][j].x; a[j].y += w * x[u][j].y; a[j].z += w * x[u][j].z; a[j].w += w * x[u][j].w;
            }
            if (s + PF < splits) {
#pragma unroll
                for (int j = 0; j < NE; j++) x[u][j] = *(const float4*)(src[j] + (long)(s + PF) * H * d);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NE; j++) {
        const int e = tid + 512 * j;
        if (e >= TOK * q4) break;
        const int t = e / q4, c = (e - t * q4) * 4;
        const float v[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
        T hi[4], lo[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hi[k] = (T)v[k];
            lo[k] = (T)(v[k] - (float)hi[k]);
        }
        const int ch = c >> 3, half = ((c >> 2) & 1) * 4;
        *(uint2*)(aimg + slot_of(t, ch) + half) = *(const uint2*)hi;
        *(uint2*)(aimg + slot_of(TOK + t, ch) + half) = *(const uint2*)lo;
    }
    if constexpr (!EARLYW) load_wv();
    __syncthreads();
    f32x4 acc[NA][4];
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[a][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
        const int ks = wave + 8 * k;
        if (ks >= d / 32) break;  // wave-uniform
#pragma unroll
        for (int a = 0; a < NA; a++) {
            const FT af = *(const FT*)(aimg + slot_of(a * 16 + r16, ks * 4 + kq));
#pragma unroll
            for (int j = 0; j < 4; j++) acc[a][j] = mfma16x16x32(af, bfp[k][j], acc[a][j]);
        }
    }
    __syncthreads();  // every wave is done with aimg
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) red[(wave * RT + a * 16 + 4 * kq + r) * 64 + j * 16 + r16] = acc[a][j][r];
    __syncthreads();
    for (int e = tid; e < TOK * 64; e += 512) {
        const int ti = e >> 6, j = e & 63;
        if (i0 + ti >= n) continue;
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < 8; w++) v += red[(w * RT + ti) * 64 + j] + red[(w * RT + TOK + ti) * 64 + j];
        out[(long)(i0 + ti) * d + h * 64 + j] = (T)(v + bv[h * 64 + j]);
    }
}

int xattn_splits(int n, int Tn) {
    const int nn = std::max(1, n);
    const int s = std::max(1, std::min(16, (256 + nn - 1) / nn));
    return std::min(s, (Tn + 15) / 16);
}

bool xattn_supported(int d) { return d == 384 || d == 512 || d == 768 || d == 1024 || d == 1280; }

void launch_xattn_qproj(DType dt, const void* q, const void* wkt, int n, int d, int H, float scale, void* qx,
                        hipStream_t st) {
    if (n <= 0) return;
    // tile per wave: 32 columns x 64 tokens (MT 2, NT 4): twice the workgroups of the round-2 shape
    // (64 x 64; the same bits), 64-clip shard 2340-2352 vs 2314-2330 audio-s/s, 128 clips neutral
    // (profiles/r03_xcomb_tok_ab.txt)
    dim3 grid(cdiv(d, 64 * 2), H, cdiv(n, 16 * 4));
    // staged row stores (d % 128 == 0: every model): 9.90 -> 7.81 us per large-v3 launch at 128 clips in the
    // decode step, the same bits (profiles/r05_qproj_stg_ab.txt); WHISPER_MI355X_QPROJ_STG=0 for the 8-byte
    // stores straight from the MFMA layout
    static const int stg = getenv("WHISPER_MI355X_QPROJ_STG") ? atoi(getenv("WHISPER_MI355X_QPROJ_STG")) : 1;
    if (stg && d % 128 == 0) {
        if (dt == DType::F16)
            xattn_qproj_kernel<half_t, 2, 4, true><<<grid, 256, 0, st>>>((const half_t*)q, (const half_t*)wkt, n, d, H, scale, (half_t*)qx);
        else
            xattn_qproj_kernel<bf16_t, 2, 4, true><<<grid, 256, 0, st>>>((const bf16_t*)q, (const bf16_t*)wkt, n, d, H, scale, (bf16_t*)qx);
        return;
    }
    if (dt == DType::F16)
        xattn_qproj_kernel<half_t, 2, 4><<<grid, 256, 0, st>>>((const half_t*)q, (const half_t*)wkt, n, d, H, scale, (half_t*)qx);
    else
        xattn_qproj_kernel<bf16_t, 2, 4><<<grid, 256, 0, st>>>((const bf16_t*)q, (const bf16_t*)wkt, n, d, H, scale, (bf16_t*)qx);
}

template <typename T>
static void launch_step_t(const void* enc, const int* slot, const void* qx, int n, int Tn, int d, int splits, float thr,
                          float* opart, float* ml, hipStream_t st) {
    dim3 grid(splits, n);
    // E is streamed once per launch (491 MB at batch 128: more than the MALL holds), so its LDS-DMA
    // loads are non-temporal (aux = 2): 86.6 vs 102.4 us per decode launch, 3075 vs 2921 audio-s/s.
    // partial-O stores staged through LDS (whole 128-byte lines per instruction): 87.4 -> 85.7 us per 128-clip launch,
    // the same bits (profiles/r06_xstep_ostg_ab.txt); WHISPER_MI355X_XSTEP_OSTG=0 for the direct stores
    static const int ostg = getenv("WHISPER_MI355X_XSTEP_OSTG") ? atoi(getenv("WHISPER_MI355X_XSTEP_OSTG")) : 1;
#define WM_XSTEP(NW_, CT_) \
    xattn_step_kernel<T, NW_, CT_, 2><<<grid, NW_ * 64, 0, st>>>((const T*)enc, slot, (const T*)qx, Tn, splits, thr, opart, ml, ostg)
    switch (d) {
        case 384: WM_XSTEP(4, 3); break;
        case 512: WM_XSTEP(8, 2); break;
        case 768: WM_XSTEP(8, 3); break;
        case 1024: WM_XSTEP(8, 4); break;
        case 1280: WM_XSTEP(8, 5); break;
        default: WM_FAIL("direct cross attention needs d in {384,512,768,1024,1280}");
    }
#undef WM_XSTEP
}

void launch_xattn_step(DType dt, const void* enc, const int* slot, const void* qx, int n, int Tn, int d, int splits,
                       float thr, float* opart, float* ml, hipStream_t st) {
    if (n <= 0) return;
    if (splits < 1 || splits > 16 || splits > (Tn + 15) / 16) WM_FAIL("bad split count %d", splits);
    if (dt == DType::F16) launch_step_t<half_t>(enc, slot, qx, n, Tn, d, splits, thr, opart, ml, st);
    else launch_step_t<bf16_t>(enc, slot, qx, n, Tn, d, splits, thr, opart, ml, st);
}

void launch_xattn_combine(DType dt, const float* opart, const float* ml, int splits, const void* wv, const float* bv, int n,
                          int d, int H, void* out, hipStream_t st) {
    if (n <= 0) return;
    if (splits > 16 || d % 128 || d > 1280) WM_FAIL("combine shape not supported");
    // Tokens per workgroup: the largest of 16 / 8 / 4 that still gives >= 160 workgroups, else 4. Every
    // choice gives the same bits (each MFMA output row is its own dot product; the final sum keeps the wave
    // order). The Wv fragments are fetched once per workgroup, so fewer tokens per workgroup re-read Wv
    // more: large-v3 (tools/xattn_tune.py, rocprofv3 trace, profiles/r05_xcomb_tok.txt) 128 clips 18.7 us
    // at 8 tokens (320 workgroups, one per CU: two rounds) -> 13.0 at 16; 64 clips 11.0 at 8 (13.5 at 16);
    // 16 clips 12.1 at 4 (15.2 at 8). At 16 tokens the Wv fragments are loaded after the partial sums
    // (171 VGPRs; before them, 256 and spills: 15.1 us). Two splits' loads in flight at 4 and 8 tokens.
    static const int tok_env = getenv("WHISPER_MI355X_XCOMB_TOK") ? atoi(getenv("WHISPER_MI355X_XCOMB_TOK")) : 0;
    int tok = 4;
    for (int t : {16, 8})
        if (H * cdiv(n, t) >= 160) { tok = t; break; }
    if (tok_env == 4 || tok_env == 8 || tok_env == 16) tok = tok_env;
    const dim3 grid(H, cdiv(n, tok));
#define WM_XCOMB(T_, TOK_, PF_, E_) xattn_combine_kernel<T_, TOK_, PF_, E_><<<grid, 512, 0, st>>>(opart, ml, splits, (const T_*)wv, bv, n, d, H, (T_*)out)
#define WM_XCOMB_T(T_)                              \
    if (tok == 4) WM_XCOMB(T_, 4, 2, true);         \
    else if (tok == 16) WM_XCOMB(T_, 16, 1, false); \
    else WM_XCOMB(T_, 8, 2, true);
    if (dt == DType::F16) {
        WM_XCOMB_T(half_t)
    } else {
        WM_XCOMB_T(bf16_t)
    }
#undef WM_XCOMB_T
#undef WM_XCOMB
}

}  // namespace wm
