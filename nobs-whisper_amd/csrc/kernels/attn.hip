// Attention kernels.
//
// Encoder: flash-style self-attention over the 1500 audio positions, d_head = 64, one workgroup =
// 64 queries of one (chunk, head), 4 waves x 16 query rows. K tiles are staged in LDS row-major
// (XOR-swizzled 16-byte chunks) and V tiles transposed, so S = Q.K^T and O += P.V are both
// v_mfma_f32_16x16x32 with ds_read_b128 operand fetches. Softmax runs online per row (16 lanes
// per row, xor-shuffle reductions), P is rounded to the MFMA input type before P.V as ggml does.
// Roofline: MFMA-bound (4*T^2*64 FLOP per head).
//
// Decoder: one query per (token, head) over a KV cache [slot][L][2][H][ctx][64] — the self cache
// (ctx 448, n_kv = pos+1) or the cross cache (ctx 1500). Three phases in one workgroup: scores
// (8 lanes x 16 B per key row, coalesced 1 KiB per wave-instruction), block softmax in LDS,
// P.V with 8 lanes per value row. Roofline: HBM-bound, 2 x n_kv x 128 B per (token, head).
#include "../common.h"
#include "../kernels.h"

namespace wm {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <typename T>
__global__ void __launch_bounds__(256) attn_enc_kernel(const T* __restrict__ qkv, T* __restrict__ out, int Tn, int d) {
    typedef typename Frag<T>::type FT;
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long base = (long)b * Tn;
    const int ld = 3 * d;
    __shared__ u32x4 Ks[64 * 8];
    __shared__ u32x4 Vts[64 * 8];
    __shared__ u32x4 Ps[4][16 * 8];

    const u32x4 zero = {0, 0, 0, 0};
    FT qf[2];
    {
        const int qrow = qb * 64 + wave * 16 + (lane & 15);
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int ch = s * 4 + (lane >> 4);
            u32x4 v = qrow < Tn ? *(const u32x4*)(qkv + (base + qrow) * ld + h * 64 + ch * 8) : zero;
            qf[s] = __builtin_bit_cast(FT, v);
        }
    }
    float m_i[4], l_i[4];
    f32x4 o[4];
#pragma unroll
    for (int r = 0; r < 4; r++) { m_i[r] = -INFINITY; l_i[r] = 0.0f; o[r] = (f32x4){0.f, 0.f, 0.f, 0.f}; }

    const int n_kt = (Tn + 63) / 64;
    T* Vt_el = (T*)Vts;
    T* P_el = (T*)Ps[wave];
    for (int kt = 0; kt < n_kt; kt++) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int c = tid + i * 256, key = c >> 3, kc = c & 7;
            const int kg = kt * 64 + key;
            u32x4 kv = zero, vv = zero;
            if (kg < Tn) {
                kv = *(const u32x4*)(qkv + (base + kg) * ld + d + h * 64 + kc * 8);
                vv = *(const u32x4*)(qkv + (base + kg) * ld + 2 * d + h * 64 + kc * 8);
            }
            Ks[key * 8 + swz(key, kc)] = kv;
            const T* ve = (const T*)&vv;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int dim = kc * 8 + e;
                Vt_el[(dim * 8 + swz(dim, key >> 3)) * 8 + (key & 7)] = ve[e];
            }
        }
        __syncthreads();
        f32x4 sacc[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            sacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int row = j * 16 + (lane & 15);
                const FT kf = __builtin_bit_cast(FT, Ks[row * 8 + swz(row, s * 4 + (lane >> 4))]);
                sacc[j] = mfma16x16x32(qf[s], kf, sacc[j]);
            }
        }
        float mx[4];
#pragma unroll
        for (int r = 0; r < 4; r++) mx[r] = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int key = kt * 64 + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float v = key < Tn ? sacc[j][r] * 0.125f : -INFINITY;
                sacc[j][r] = v;
                mx[r] = fmaxf(mx[r], v);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int o2 = 1; o2 < 16; o2 <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o2));
        }
        float alpha[4], rs[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const float mn = fmaxf(m_i[r], mx[r]);
            alpha[r] = __expf(m_i[r] - mn);
            m_i[r] = mn;
            rs[r] = 0.0f;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const T pt = (T)__expf(sacc[j][r] - m_i[r]);
                rs[r] += (float)pt;
                const int row = (lane >> 4) * 4 + r, key = j * 16 + (lane & 15);
                P_el[(row * 8 + swz(row, key >> 3)) * 8 + (key & 7)] = pt;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int o2 = 1; o2 < 16; o2 <<= 1) rs[r] += __shfl_xor(rs[r], o2);
            l_i[r] = l_i[r] * alpha[r] + rs[r];
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) o[j][r] *= alpha[r];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P stores landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int prow = lane & 15;
            const FT pf = __builtin_bit_cast(FT, Ps[wave][prow * 8 + swz(prow, s * 4 + (lane >> 4))]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int vrow = j * 16 + (lane & 15);
                const FT vf = __builtin_bit_cast(FT, Vts[vrow * 8 + swz(vrow, s * 4 + (lane >> 4))]);
                o[j] = mfma16x16x32(pf, vf, o[j]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = qb * 64 + wave * 16 + (lane >> 4) * 4 + r;
        if (row >= Tn) continue;
        const float inv = 1.0f / l_i[r];
#pragma unroll
        for (int j = 0; j < 4; j++) out[(base + row) * d + h * 64 + j * 16 + (lane & 15)] = (T)(o[j][r] * inv);
    }
}

// ------------------------------------------------------------------------------------------------
// Encoder self-attention, swapped-product form. One workgroup = 256 queries of one (window, head):
// 8 waves x 32 queries; K/V tiles of 64 keys double-buffered in LDS (one barrier per tile, the next
// tile's global loads in flight under the current tile's MFMAs).
//   S^T[key][q] = K . Q^T     v_mfma_f32_32x32x16: A = K rows (ds_read_b128, XOR-swizzled image),
//                             B = this wave's Q (registers, loaded once)
//   softmax over keys         a lane holds 32 of the 64 keys of its query (lane^32 the other 32):
//                             31 in-lane fmax + 1 exchange; row sums stay per lane until the end
//   O^T[dim][q] += V^T . P^T  B = the S^T accumulator itself (registers 8s..8s+7 -> k-step s, in
//                             the permuted key order of that layout), A = V^T via
//                             ds_read_b64_tr_b16 from a row-major V image (no transposing store)
// Exponentials in base 2 with the 1/8 scale and log2(e) folded into one FMA.
// MINW = 4 (variant 5; with PK = false variant 6, the default): the register allocation held to 128 VGPRs so that two workgroups
// share a CU (4 waves per SIMD); they drift apart between their barriers, so one workgroup's softmax
// runs beside the other's MFMAs: 578 vs 694 us per 32-window large-v3 launch (random bf16 operands,
// profiles/r03_attn_encoder_variants.txt). MINW = 1 (variant 2): 138 VGPRs, one workgroup per CU.
// PK = false (variant 6): the exponent arguments and row sums as scalar v_fma_f32 / v_add_f32 (inline asm,
// so the compiler cannot re-pack them) instead of v_pk_fma_f32 / v_pk_add_f32, which the guide prices
// above two scalar ops beside MFMAs; the same per-element operations, so the same bits. No VGPR spill at
// 128 (variant 5: 2); encode 325.9 -> 324.6 ms per step at 128 clips (profiles/r03_attn_encoder_variants.txt).
// XCD (round 6): a 1-D grid of nqb x H x B workgroups whose id L runs on XCD L % 8; workgroup L takes the
// (query block, head, window) of index (L % 8) * (G / 8) + L / 8, so the query blocks of one (window, head)
// share an XCD and its L2 fetches their K / V once (id order: they were consecutive ids, i.e. up to 6
// XCDs, each fetching the same 384 KB). Same work per workgroup, same bits.
template <typename T, int MINW = 1, bool PK = true>
__global__ void __launch_bounds__(512, MINW) attn_enc2_kernel(const T* __restrict__ qkv, T* __restrict__ out, int Tn, int d,
                                                             int nqb = 0, int H = 0) {
    typedef typename Frag<T>::type FT;
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s* lds_v4s_t;
    int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    if (nqb > 0) {
        const int L = blockIdx.x, G = gridDim.x;
        const int p = (L & 7) * (G >> 3) + (L >> 3);
        qb = p % nqb;
        h = (p / nqb) % H;
        b = p / (nqb * H);
    }
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int hh = lane >> 5, ql = lane & 31;
    const long base = (long)b * Tn;
    const int ld = 3 * d;
    __shared__ u32x4 Ks[2][64 * 8];
    __shared__ u32x4 Vs[2][64 * 8];
    const u32x4 zero = {0, 0, 0, 0};

    const int q = qb * 256 + wave * 32 + ql;
    FT qf[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const u32x4 v = q < Tn ? *(const u32x4*)(qkv + (base + q) * ld + h * 64 + s * 16 + hh * 8) : zero;
        qf[s] = __builtin_bit_cast(FT, v);
    }
    // staging: thread -> (key, 16-byte chunk) of the K and V tiles
    const int skey = tid >> 3, sch = tid & 7;
    const int k_slot = skey * 8 + (sch ^ ((skey >> 1) & 7));
    const int v_slot = skey * 8 + (sch ^ (((skey >> 1) & 1) << 2));
    auto load_kv = [&](int kt, u32x4& kv, u32x4& vv) {
        const int kg = kt * 64 + skey;
        kv = zero;
        vv = zero;
        if (kg < Tn) {
            const T* src = qkv + (base + kg) * ld + h * 64 + sch * 8;
            kv = *(const u32x4*)(src + d);
            vv = *(const u32x4*)(src + 2 * d);
        }
    };
    // transposed-read address (bytes within a V image) for rows r0..r0+3, this lane's dims. Every
    // r0 used is 4*hh + a multiple of 8, so the swizzle bit ((row >> 1) & 1) is (tq >> 1) & 1 for
    // all of them: one lane base per dim block, the rest a compile-time offset (ds_read offset field)
    const int tg = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
    int vbase[2];
#pragma unroll
    for (int db = 0; db < 2; db++) {
        const int ch = db * 4 + tg * 2 + (tp >> 1);
        vbase[db] = (4 * hh + tq) * 128 + 16 * (ch ^ (((tq >> 1) & 1) << 2)) + 8 * (tp & 1);
    }

    f32x16 oacc[2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int r = 0; r < 16; r++) oacc[i][r] = 0.0f;
    float m_run = -INFINITY, l_run = 0.0f;
    const float c = 0.125f * 1.44269504088896340736f;

    const int n_kt = (Tn + 63) / 64;
    {
        u32x4 kv, vv;
        load_kv(0, kv, vv);
        Ks[0][k_slot] = kv;
        Vs[0][v_slot] = vv;
    }
    __syncthreads();
    for (int kt = 0; kt < n_kt; kt++) {
        const int cur = kt & 1;
        const bool more = kt + 1 < n_kt;
        u32x4 nk = zero, nv = zero;
        if (more) load_kv(kt + 1, nk, nv);
        f32x16 sacc[2];
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
#pragma unroll
            for (int r = 0; r < 16; r++) sacc[kb][r] = 0.0f;
            const int key = kb * 32 + ql;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const FT kf = __builtin_bit_cast(FT, Ks[cur][key * 8 + ((s * 2 + hh) ^ ((key >> 1) & 7))]);
                sacc[kb] = mfma32x32x16(kf, qf[s], sacc[kb]);
            }
        }
        if (kt * 64 + 64 > Tn) {
#pragma unroll
            for (int kb = 0; kb < 2; kb++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int key = kt * 64 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    if (key >= Tn) sacc[kb][r] = -INFINITY;
                }
        }
        float mx = sacc[0][0];
#pragma unroll
        for (int kb = 0; kb < 2; kb++)
#pragma unroll
            for (int r = 0; r < 16; r++) mx = fmaxf(mx, sacc[kb][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float m_new = fmaxf(m_run, mx * c);
        // the running max of no query in the wave moved: alpha = 1 for every lane, skip the rescale
        const bool moved = __builtin_amdgcn_ballot_w64(m_new != m_run) != 0;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        // exponent arguments and row sums two at a time (v_pk_fma_f32 / v_pk_add_f32); the two
        // partial sums of a lane are added at the end of the tile
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 c2 = {c, c}, nm2 = {-m_new, -m_new};
        FT pf[4];
        f2 ls2 = {0.0f, 0.0f};
        if constexpr (PK) {
#pragma unroll
            for (int kb = 0; kb < 2; kb++)
#pragma unroll
                for (int sp = 0; sp < 2; sp++)
#pragma unroll
                    for (int j = 0; j < 8; j += 2) {
                        const f2 x = {sacc[kb][sp * 8 + j], sacc[kb][sp * 8 + j + 1]};
                        const f2 e = __builtin_elementwise_fma(x, c2, nm2);
                        const f2 p = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
                        ls2 += p;
                        pf[kb * 2 + sp][j] = (T)p.x;
                        pf[kb * 2 + sp][j + 1] = (T)p.y;
                    }
        } else {
            const float nm = -m_new;
            float lx = 0.0f, ly = 0.0f;
#pragma unroll
            for (int kb = 0; kb < 2; kb++)
#pragma unroll
                for (int sp = 0; sp < 2; sp++)
#pragma unroll
                    for (int j = 0; j < 8; j += 2) {
                        float ex, ey;
                        asm("v_fma_f32 %0, %1, %2, %3" : "=v"(ex) : "v"(sacc[kb][sp * 8 + j]), "v"(c), "v"(nm));
                        asm("v_fma_f32 %0, %1, %2, %3" : "=v"(ey) : "v"(sacc[kb][sp * 8 + j + 1]), "v"(c), "v"(nm));
                        const float px = __builtin_amdgcn_exp2f(ex), py = __builtin_amdgcn_exp2f(ey);
                        asm("v_add_f32 %0, %1, %2" : "=v"(lx) : "v"(lx), "v"(px));
                        asm("v_add_f32 %0, %1, %2" : "=v"(ly) : "v"(ly), "v"(py));
                        pf[kb * 2 + sp][j] = (T)px;
                        pf[kb * 2 + sp][j + 1] = (T)py;
                    }
            ls2 = f2{lx, ly};
        }
        l_run = l_run * alpha + (ls2.x + ls2.y);
        if (moved) {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int r = 0; r < 16; r++) oacc[i][r] *= alpha;
        }
        const char* vimg = (const char*)Vs[cur];
#pragma unroll
        for (int db = 0; db < 2; db++)
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int r0 = (s >> 1) * 32 + (s & 1) * 16;  // + 4 hh, in vbase
                const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(vimg + vbase[db] + r0 * 128));
                const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(vimg + vbase[db] + (r0 + 8) * 128));
                const FT vf = __builtin_bit_cast(FT, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                oacc[db] = mfma32x32x16(vf, pf[s], oacc[db]);
            }
        if (more) {
            Ks[cur ^ 1][k_slot] = nk;
            Vs[cur ^ 1][v_slot] = nv;
        }
        __syncthreads();
    }
    if (q >= Tn) return;
    const float inv = 1.0f / (l_run + __shfl_xor(l_run, 32));
    T* orow = out + (base + q) * d + h * 64;
#pragma unroll
    for (int db = 0; db < 2; db++)
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            T v4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v4[j] = (T)(oacc[db][rr * 4 + j] * inv);
            *(uint2*)(orow + db * 32 + rr * 8 + 4 * hh) = *(const uint2*)v4;
        }
}

// ------------------------------------------------------------------------------------------------
// attn_enc2_kernel software-pipelined across key tiles (variant 3 of whisper_mi355x_bench_attn_encoder;
// measured slower, kept bit-identical under test): iteration t issues the
// score MFMAs of tile t+1 first, then runs the softmax of tile t and its P.V MFMAs, so a wave has
// independent MFMA work in flight under its exponentials instead of alternating MFMA-only and
// VALU-only phases in lockstep with its SIMD partner. K runs one tile ahead of V in the same two LDS
// slots each: iteration t reads K(t+1) and V(t) and fills K(t+2), V(t+1). Every per-element operation
// and its order is attn_enc2_kernel's, so the outputs are bit-identical.
template <typename T>
__global__ void __launch_bounds__(512) attn_enc3_kernel(const T* __restrict__ qkv, T* __restrict__ out, int Tn, int d) {
    typedef typename Frag<T>::type FT;
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s* lds_v4s_t;
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int hh = lane >> 5, ql = lane & 31;
    const long base = (long)b * Tn;
    const int ld = 3 * d;
    __shared__ u32x4 Ks[2][64 * 8];
    __shared__ u32x4 Vs[2][64 * 8];
    const u32x4 zero = {0, 0, 0, 0};

    const int q = qb * 256 + wave * 32 + ql;
    FT qf[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const u32x4 v = q < Tn ? *(const u32x4*)(qkv + (base + q) * ld + h * 64 + s * 16 + hh * 8) : zero;
        qf[s] = __builtin_bit_cast(FT, v);
    }
    const int skey = tid >> 3, sch = tid & 7;
    const int k_slot = skey * 8 + (sch ^ ((skey >> 1) & 7));
    const int v_slot = skey * 8 + (sch ^ (((skey >> 1) & 1) << 2));
    auto load_k = [&](int kt) -> u32x4 {
        const int kg = kt * 64 + skey;
        return kg < Tn ? *(const u32x4*)(qkv + (base + kg) * ld + d + h * 64 + sch * 8) : zero;
    };
    auto load_v = [&](int kt) -> u32x4 {
        const int kg = kt * 64 + skey;
        return kg < Tn ? *(const u32x4*)(qkv + (base + kg) * ld + 2 * d + h * 64 + sch * 8) : zero;
    };
    const int tg = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
    int vbase[2];
#pragma unroll
    for (int db = 0; db < 2; db++) {
        const int ch = db * 4 + tg * 2 + (tp >> 1);
        vbase[db] = (4 * hh + tq) * 128 + 16 * (ch ^ (((tq >> 1) & 1) << 2)) + 8 * (tp & 1);
    }
    const int n_kt = (Tn + 63) / 64;
    // S^T of tile kt from K slot ks, masked past Tn
    auto scores = [&](int kt, int ks, f32x16* sacc) {
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
#pragma unroll
            for (int r = 0; r < 16; r++) sacc[kb][r] = 0.0f;
            const int key = kb * 32 + ql;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const FT kf = __builtin_bit_cast(FT, Ks[ks][key * 8 + ((s * 2 + hh) ^ ((key >> 1) & 7))]);
                sacc[kb] = mfma32x32x16(kf, qf[s], sacc[kb]);
            }
        }
        if (kt * 64 + 64 > Tn) {
#pragma unroll
            for (int kb = 0; kb < 2; kb++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int key = kt * 64 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    if (key >= Tn) sacc[kb][r] = -INFINITY;
                }
        }
    };

    f32x16 oacc[2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int r = 0; r < 16; r++) oacc[i][r] = 0.0f;
    float m_run = -INFINITY, l_run = 0.0f;
    const float c = 0.125f * 1.44269504088896340736f;

    // prologue: K(0), V(0) -> slot 0, K(1) -> K slot 1; S(0)
    Ks[0][k_slot] = load_k(0);
    Vs[0][v_slot] = load_v(0);
    if (n_kt > 1) Ks[1][k_slot] = load_k(1);
    __syncthreads();
    f32x16 scur[2];
    scores(0, 0, scur);
    __syncthreads();  // every wave has read K slot 0 before iteration 0 refills it with K(2)
    for (int t = 0; t < n_kt; t++) {
        const int cur = t & 1;
        const bool more1 = t + 1 < n_kt, more2 = t + 2 < n_kt;
        u32x4 nk = zero, nv = zero;
        if (more2) nk = load_k(t + 2);
        if (more1) nv = load_v(t + 1);
        f32x16 snext[2];
        if (more1) scores(t + 1, cur ^ 1, snext);
        // softmax of tile t (attn_enc2_kernel's operations, same order)
        float mx = scur[0][0];
#pragma unroll
        for (int kb = 0; kb < 2; kb++)
#pragma unroll
            for (int r = 0; r < 16; r++) mx = fmaxf(mx, scur[kb][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float m_new = fmaxf(m_run, mx * c);
        const bool moved = __builtin_amdgcn_ballot_w64(m_new != m_run) != 0;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        const f2 c2 = {c, c}, nm2 = {-m_new, -m_new};
        FT pf[4];
        f2 ls2 = {0.0f, 0.0f};
#pragma unroll
        for (int kb = 0; kb < 2; kb++)
#pragma unroll
            for (int sp = 0; sp < 2; sp++)
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const f2 x = {scur[kb][sp * 8 + j], scur[kb][sp * 8 + j + 1]};
                    const f2 e = __builtin_elementwise_fma(x, c2, nm2);
                    const f2 p = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
                    ls2 += p;
                    pf[kb * 2 + sp][j] = (T)p.x;
                    pf[kb * 2 + sp][j + 1] = (T)p.y;
                }
        l_run = l_run * alpha + (ls2.x + ls2.y);
        if (moved) {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int r = 0; r < 16; r++) oacc[i][r] *= alpha;
        }
        const char* vimg = (const char*)Vs[cur];
#pragma unroll
        for (int db = 0; db < 2; db++)
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int r0 = (s >> 1) * 32 + (s & 1) * 16;
                const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(vimg + vbase[db] + r0 * 128));
                const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(vimg + vbase[db] + (r0 + 8) * 128));
                const FT vf = __builtin_bit_cast(FT, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                oacc[db] = mfma32x32x16(vf, pf[s], oacc[db]);
            }
        if (more2) Ks[cur][k_slot] = nk;
        if (more1) Vs[cur ^ 1][v_slot] = nv;
        __syncthreads();
        if (more1) {
            scur[0] = snext[0];
            scur[1] = snext[1];
        }
    }
    if (q >= Tn) return;
    const float inv = 1.0f / (l_run + __shfl_xor(l_run, 32));
    T* orow = out + (base + q) * d + h * 64;
#pragma unroll
    for (int db = 0; db < 2; db++)
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            T v4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v4[j] = (T)(oacc[db][rr * 4 + j] * inv);
            *(uint2*)(orow + db * 32 + rr * 8 + 4 * hh) = *(const uint2*)v4;
        }
}

// Sums over the 8 lanes of a key row by DPP (quad xor 1, quad xor 2, half-row mirror): the same bits as
// the xor butterfly (after two steps every lane of a quad holds the quad sum), without LDS round trips.
template <int CTRL>
__device__ __forceinline__ float dpp8_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8(float a) {
    a += dpp8_f<0xB1>(a);
    a += dpp8_f<0x4E>(a);
    return a + dpp8_f<0x141>(a);
}

// ------------------------------------------------------------------------------------------------
// FQ: q is not read from a buffer but reduced from the cross-Q projection's split-K slabs
// (DecSlabs; q = (T)((sum_z + bias) * scale), the EPI_STORE epilogue of that GEMM).
template <typename T, bool FQ, int NTH = 256, int U = 8>
__device__ __forceinline__ void attn_dec_body(const T* __restrict__ q, int q_stride, const DecSlabs sl,
                                              const T* __restrict__ cache, const int* __restrict__ slot,
                                              const int* __restrict__ n_kv_arr, int L, int layer, int H, int ctx, int d,
                                              T* __restrict__ out) {
    const int i = blockIdx.x, h = blockIdx.y;
    constexpr int NG = NTH / 8, NW = NTH / 64;
    const int tid = threadIdx.x, lane8 = tid & 7, grp = tid >> 3;  // NG groups of 8 lanes
    const int n_kv = n_kv_arr[i];
    const long s = slot[i];
    const T* K = cache + (((s * L + layer) * 2 + 0) * H + h) * (long)ctx * 64;
    const T* V = cache + (((s * L + layer) * 2 + 1) * H + h) * (long)ctx * 64;
    __shared__ float sc[1536];
    __shared__ float red[NTH];
    __shared__ float acc_s[NG][65];

    // Loads: U key rows per lane group per chunk, the next chunk issued before the current one is
    // consumed (two chunks in flight); the first K chunk is issued before q is formed (it does not
    // depend on q) and the first V chunk before the softmax (it does not depend on P). The arithmetic
    // (per-key sums, the block max, the sum tree, P rounded to T, the P.V order per lane group) is
    // the round-2 kernel's: the sum keeps its tree association (lanes t, t+64, t+128, t+192 first,
    // then halving inside one wave), with 2 barriers instead of 9.
    constexpr int CHR = NG * U;
    const u32x4 zero = {0, 0, 0, 0};
    auto load_rows = [&](const T* base, int t0, u32x4 (&raw)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            raw[u] = t < n_kv ? *(const u32x4*)(base + (long)t * 64 + lane8 * 8) : zero;
        }
    };
    u32x4 ra[U], rb[U];
    load_rows(K, grp, ra);
    float qv[8];
    if constexpr (FQ) {
        if (tid < 64) {
            const float* p = sl.ws + (long)i * sl.ld + h * 64 + tid;
            float pz[16], v = 0.0f;  // every split's load at once (one round trip), summed in split order
#pragma unroll
            for (int z = 0; z < 16; z++)
                if (z < sl.splits) pz[z] = p[z * sl.zstride];
#pragma unroll
            for (int z = 0; z < 16; z++)
                if (z < sl.splits) v += pz[z];
            if (sl.bias) v = v + sl.bias[h * 64 + tid];
            red[tid] = (float)(T)(v * sl.scale);
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8; e++) qv[e] = red[lane8 * 8 + e];
        __syncthreads();
    } else {
        const u32x4 raw = *(const u32x4*)(q + (long)i * q_stride + h * 64 + lane8 * 8);
        const T* qe = (const T*)&raw;
#pragma unroll
        for (int e = 0; e < 8; e++) qv[e] = (float)qe[e];
    }
    // phase 1: scores
    float lmax = -INFINITY;
    auto scores = [&](int t0, const u32x4 (&raw)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            const T* ke = (const T*)&raw[u];
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e++) a += qv[e] * (float)ke[e];
            a = sum8(a);  // DPP, no ds_bpermute round trips (same bits as the xor butterfly)
            if (t < n_kv) {
                if (lane8 == 0) sc[t] = a;
                lmax = fmaxf(lmax, a);
            }
        }
    };
    {
        int t0 = grp;
        for (; t0 + CHR < n_kv; t0 += 2 * CHR) {
            load_rows(K, t0 + CHR, rb);
            scores(t0, ra);
            if (t0 + 2 * CHR < n_kv) load_rows(K, t0 + 2 * CHR, ra);
            scores(t0 + CHR, rb);
        }
        if (t0 < n_kv) scores(t0, ra);
    }
    load_rows(V, grp, ra);  // lands under the softmax
    // block max (order-free), then the sum in the round-2 tree's association
    const int wave = tid >> 6, lane = tid & 63;
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    if (lane == 0) red[wave] = lmax;
    __syncthreads();
    float mx = red[0];
#pragma unroll
    for (int w = 1; w < NW; w++) mx = fmaxf(mx, red[w]);
    float lsum = 0.0f;
    for (int t = tid; t < n_kv; t += NTH) {
        const float e = expf(sc[t] - mx);
        sc[t] = e;
        lsum += e;
    }
    __syncthreads();  // every wave has read red[0..NW)
    red[tid] = lsum;
    __syncthreads();
    if (wave == 0) {
        float r;
        if constexpr (NTH == 256) {
            r = (red[lane] + red[lane + 128]) + (red[lane + 64] + red[lane + 192]);
        } else {  // wider workgroups (few clips): the waves' partials in wave order
            r = red[lane];
#pragma unroll
            for (int w = 1; w < NW; w++) r = r + red[lane + 64 * w];
        }
        for (int o = 32; o > 0; o >>= 1) r = r + __shfl_down(r, o);
        if (lane == 0) red[0] = r;
    }
    __syncthreads();
    const float inv = 1.0f / red[0];
    for (int t = tid; t < n_kv; t += NTH) sc[t] = (float)(T)(sc[t] * inv);  // P rounded as ggml's f16 src1
    __syncthreads();
    // phase 3: O = P.V
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] = 0.0f;
    auto pv = [&](int t0, const u32x4 (&raw)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + NG * u;
            const T* ve = (const T*)&raw[u];
            const float p = t < n_kv ? sc[t] : 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e++) acc[e] += p * (float)ve[e];
        }
    };
    {
        int t0 = grp;
        for (; t0 + CHR < n_kv; t0 += 2 * CHR) {
            load_rows(V, t0 + CHR, rb);
            pv(t0, ra);
            if (t0 + 2 * CHR < n_kv) load_rows(V, t0 + 2 * CHR, ra);
            pv(t0 + CHR, rb);
        }
        if (t0 < n_kv) pv(t0, ra);
    }
#pragma unroll
    for (int e = 0; e < 8; e++) acc_s[grp][lane8 * 8 + e] = acc[e];
    __syncthreads();
    if (tid < 64) {
        float a = 0.0f;
        for (int g2 = 0; g2 < NG; g2++) a += acc_s[g2][tid];
        out[(long)i * d + h * 64 + tid] = (T)a;
    }
}

// One body, three kernel names so profiles separate the uses: the self cache (prefill), the cross
// cache in a decode step (one token per clip, q reduced from slabs: the roofline kernel) and the
// cross cache in a prefill.
template <typename T>
__global__ void __launch_bounds__(256) attn_self_kernel(const T* __restrict__ q, int q_stride, const T* __restrict__ cache,
                                                        const int* __restrict__ slot, const int* __restrict__ n_kv_arr,
                                                        int L, int layer, int H, int ctx, int d, T* __restrict__ out) {
    attn_dec_body<T, false>(q, q_stride, DecSlabs{}, cache, slot, n_kv_arr, L, layer, H, ctx, d, out);
}
template <typename T>
__global__ void __launch_bounds__(256) attn_cross_prefill_kernel(const T* __restrict__ q, int q_stride,
                                                                 const T* __restrict__ cache, const int* __restrict__ slot,
                                                                 const int* __restrict__ n_kv_arr, int L, int layer, int H,
                                                                 int ctx, int d, T* __restrict__ out) {
    attn_dec_body<T, false>(q, q_stride, DecSlabs{}, cache, slot, n_kv_arr, L, layer, H, ctx, d, out);
}
template <typename T>
__global__ void __launch_bounds__(256) attn_cross_step_kernel(const DecSlabs sl, const T* __restrict__ cache,
                                                              const int* __restrict__ slot, const int* __restrict__ n_kv_arr,
                                                              int L, int layer, int H, int ctx, int d, T* __restrict__ out) {
    attn_dec_body<T, true>(nullptr, 0, sl, cache, slot, n_kv_arr, L, layer, H, ctx, d, out);
}
// decode steps of few clips (<= 4: the app's one clip per call; n x H workgroups leave most CUs idle):
// 1024 threads (128 lane groups) per (clip, head), so each pass over the 1500 cached keys is 2-3 memory
// round trips instead of 6; the sum of the softmax adds the waves' partials in wave order (another
// association than the 256-thread tree: results can differ in the last bits between the two widths)
template <typename T>
__global__ void __launch_bounds__(1024) attn_cross_step_wide_kernel(const DecSlabs sl, const T* __restrict__ cache,
                                                                    const int* __restrict__ slot, const int* __restrict__ n_kv_arr,
                                                                    int L, int layer, int H, int ctx, int d, T* __restrict__ out) {
    attn_dec_body<T, true, 1024, 4>(nullptr, 0, sl, cache, slot, n_kv_arr, L, layer, H, ctx, d, out);
}

// Decode-step self attention, one wave per (token, head), HPB heads per workgroup. The prologue
// reduces this token's q, k, v from the QKV projection's split-K slabs (EPI_QKV_DEC arithmetic: q
// and k scaled, rounded to T), appends k, v to the self cache at pos[i] and attends keys
// [0, pos) from the cache plus the fresh key from registers. Scores: 8 lanes per key row (16 B
// each), U rows in flight per lane group; softmax and P.V reductions are wave shuffles.
// Sums over the 8 lanes of a key row by DPP (quad xor 1, quad xor 2, half-row mirror): the same
// bits as the xor butterfly, without LDS round trips. NT: the cached K and V rows (read once per
// step) by non-temporal loads.
template <typename T, int HPB, bool NT>
__global__ void __launch_bounds__(64 * HPB) attn_self_step_kernel(const DecSlabs sl, T* __restrict__ cache,
                                                                  const int* __restrict__ slot,
                                                                  const int* __restrict__ pos_arr, int L, int layer,
                                                                  int H, int ctx, int d, T* __restrict__ out) {
    const int i = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = blockIdx.y * HPB + w;
    const int lane8 = lane & 7, grp = lane >> 3;  // 8 groups of 8 lanes
    __shared__ float qs[HPB][64], ks[HPB][64], vs[HPB][64];
    __shared__ float sc[HPB][448];
    const int pos = pos_arr[i];
    const long s = slot[i];
    T* K = cache + (((s * L + layer) * 2 + 0) * H + h) * (long)ctx * 64;
    T* V = cache + (((s * L + layer) * 2 + 1) * H + h) * (long)ctx * 64;
    // the first U cached key rows of each lane group are issued before the prologue's slab loads (round 6): they
    // do not depend on this step's q / k / v, so both land in one memory round trip (as in attn_dec_body)
    constexpr int U = 8;
    const u32x4 zero = {0, 0, 0, 0};
    u32x4 raw[U];
    auto kload = [&](int t0) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + 8 * u;
            const u32x4* src = (const u32x4*)(K + (long)t * 64 + lane8 * 8);
            raw[u] = t < pos ? (NT ? __builtin_nontemporal_load(src) : *src) : zero;
        }
    };
    kload(grp);
    {
        // every split's q, k, v partials loaded at once (one memory round trip; <= 16 splits), summed in
        // split order
        const float* p = sl.ws + (long)i * sl.ld + h * 64 + lane;
        float pq[16], pk[16], pv[16];
#pragma unroll
        for (int z = 0; z < 16; z++)
            if (z < sl.splits) {
                const float* pz = p + z * sl.zstride;
                pq[z] = pz[0];
                pk[z] = pz[d];
                pv[z] = pz[2 * d];
            }
        float vq = 0.0f, vk = 0.0f, vv = 0.0f;
#pragma unroll
        for (int z = 0; z < 16; z++)
            if (z < sl.splits) {
                vq += pq[z];
                vk += pk[z];
                vv += pv[z];
            }
        if (sl.bias) {
            vq = vq + sl.bias[h * 64 + lane];
            vk = vk + sl.bias[d + h * 64 + lane];
            vv = vv + sl.bias[2 * d + h * 64 + lane];
        }
        const T tq = (T)(vq * sl.scale), tk = (T)(vk * sl.scale), tv = (T)vv;
        K[(long)pos * 64 + lane] = tk;
        V[(long)pos * 64 + lane] = tv;
        qs[w][lane] = (float)tq;
        ks[w][lane] = (float)tk;
        vs[w][lane] = (float)tv;
    }
    __syncthreads();
    float qv[8];
#pragma unroll
    for (int e = 0; e < 8; e++) qv[e] = qs[w][lane8 * 8 + e];
    // 8 key rows in flight per lane group (16, with the first V chunk issued before the softmax, measured
    // 14.6 vs 13.6 us at 128 clips and 8.3 vs 8.2 at 16)
    float lmax = -INFINITY;
    for (int t0 = grp; t0 < pos; t0 += 8 * U) {
        if (t0 != grp) kload(t0);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + 8 * u;
            const T* ke = (const T*)&raw[u];
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e++) a += qv[e] * (float)ke[e];
            a = sum8(a);
            if (t < pos) {
                if (lane8 == 0) sc[w][t] = a;
                lmax = fmaxf(lmax, a);
            }
        }
    }
    {  // the fresh key (position pos)
        float a = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; e++) a += qv[e] * ks[w][lane8 * 8 + e];
        a = sum8(a);
        if (lane == 0) sc[w][pos] = a;
        lmax = fmaxf(lmax, a);
    }
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    __syncthreads();
    const int n_kv = pos + 1;
    float lsum = 0.0f;
    for (int t = lane; t < n_kv; t += 64) {
        const float e = expf(sc[w][t] - lmax);
        sc[w][t] = e;
        lsum += e;
    }
    for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o);
    const float inv = 1.0f / lsum;
    for (int t = lane; t < n_kv; t += 64) sc[w][t] = (float)(T)(sc[w][t] * inv);  // P rounded as ggml's f16 src1
    __syncthreads();
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] = 0.0f;
    for (int t0 = grp; t0 < pos; t0 += 8 * U) {
        u32x4 vraw[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + 8 * u;
            const u32x4* src = (const u32x4*)(V + (long)t * 64 + lane8 * 8);
            vraw[u] = t < pos ? (NT ? __builtin_nontemporal_load(src) : *src) : zero;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + 8 * u;
            const T* ve = (const T*)&vraw[u];
            const float p = t < pos ? sc[w][t] : 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e++) acc[e] += p * (float)ve[e];
        }
    }
    if (grp == 0) {
        const float p = sc[w][pos];
#pragma unroll
        for (int e = 0; e < 8; e++) acc[e] += p * vs[w][lane8 * 8 + e];
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
        acc[e] += dpp8_f<0x128>(acc[e]);  // row_ror:8 = lane ^ 8 within the 16-lane row
        acc[e] += __shfl_xor(acc[e], 16);
        acc[e] += __shfl_xor(acc[e], 32);
    }
    if (grp == 0) {
        T o8[8];
#pragma unroll
        for (int e = 0; e < 8; e++) o8[e] = (T)acc[e];
        *(u32x4*)(out + (long)i * d + h * 64 + lane8 * 8) = *(const u32x4*)o8;
    }
}

// ------------------------------------------------------------------------------------------------
// Prefill attention (prompts: the app's vocabulary prompt is ~170 tokens per clip, whisper.rs:98-109,
// config.rs:40-42): one workgroup = up to 64 consecutive query tokens of ONE clip (a host-built tile
// list) x one head, 4 waves x 16 query rows, over that clip's cache rows [0, n_kv[i]) (the self cache
// with n_kv = pos + 1, causal, or the cross cache, 1500 rows). Each K/V tile is staged once in LDS for
// all 64 queries (the one-query-per-workgroup kernel above re-reads the clip's whole cache per token).
// Two passes keep ggml's soft_max order (normalise, then round P to the f16 src1 of P.V): pass 1
// S = Q.K^T by MFMA with an online row max and sum; pass 2 S again, P = (T)(exp(S - max) / sum),
// O += P.V by MFMA (K tiles row-major and V tiles transposed in XOR-swizzled LDS images, as
// attn_enc_kernel). Rows of a tile must have non-decreasing n_kv (positions increase).
template <typename T>
__global__ void __launch_bounds__(256) attn_prefill_kernel(const T* __restrict__ q, int q_stride, const T* __restrict__ cache,
                                                           const int* __restrict__ slot, const int* __restrict__ n_kv_arr,
                                                           const int2* __restrict__ tiles, int L, int layer, int H,
                                                           int ctx, int d, T* __restrict__ out) {
    typedef typename Frag<T>::type FT;
    const int2 tl = tiles[blockIdx.x];
    const int i0 = tl.x, cnt = tl.y, h = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long s = slot[i0];
    const T* K = cache + (((s * L + layer) * 2 + 0) * H + h) * (long)ctx * 64;
    const T* V = cache + (((s * L + layer) * 2 + 1) * H + h) * (long)ctx * 64;
    __shared__ u32x4 Ks[64 * 8];
    __shared__ u32x4 Vts[64 * 8];
    __shared__ u32x4 Ps[4][16 * 8];
    const u32x4 zero = {0, 0, 0, 0};
    const int kv_end = n_kv_arr[i0 + cnt - 1];
    FT qf[2];
    {
        const int row = wave * 16 + (lane & 15);
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++) {
            const int ch = s2 * 4 + (lane >> 4);
            const u32x4 v = row < cnt ? *(const u32x4*)(q + (long)(i0 + row) * q_stride + h * 64 + ch * 8) : zero;
            qf[s2] = __builtin_bit_cast(FT, v);
        }
    }
    int nkv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = wave * 16 + (lane >> 4) * 4 + r;
        nkv[r] = row < cnt ? n_kv_arr[i0 + row] : 0;
    }
    const int n_kt = (kv_end + 63) / 64;
    auto stage_k = [&](int kt) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int c = tid + i * 256, key = c >> 3, kc = c & 7, kg = kt * 64 + key;
            Ks[key * 8 + swz(key, kc)] = kg < kv_end ? *(const u32x4*)(K + (long)kg * 64 + kc * 8) : zero;
        }
    };
    auto scores = [&](int kt, f32x4 (&sacc)[4]) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            sacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int row = j * 16 + (lane & 15);
                const FT kf = __builtin_bit_cast(FT, Ks[row * 8 + swz(row, s2 * 4 + (lane >> 4))]);
                sacc[j] = mfma16x16x32(qf[s2], kf, sacc[j]);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int key = kt * 64 + j * 16 + (lane & 15);
                if (key >= nkv[r]) sacc[j][r] = -INFINITY;
            }
        }
    };
    // pass 1: row max and sum (online)
    float m_i[4], l_i[4];
#pragma unroll
    for (int r = 0; r < 4; r++) { m_i[r] = -INFINITY; l_i[r] = 0.0f; }
    for (int kt = 0; kt < n_kt; kt++) {
        __syncthreads();
        stage_k(kt);
        __syncthreads();
        f32x4 sacc[4];
        scores(kt, sacc);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float mx = fmaxf(fmaxf(sacc[0][r], sacc[1][r]), fmaxf(sacc[2][r], sacc[3][r]));
            for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2));
            const float mn = fmaxf(m_i[r], mx);
            float sum = 0.0f;
            if (mn != -INFINITY) {
#pragma unroll
                for (int j = 0; j < 4; j++) sum += expf(sacc[j][r] - mn);
            }
            for (int o2 = 1; o2 < 16; o2 <<= 1) sum += __shfl_xor(sum, o2);
            l_i[r] = (m_i[r] == -INFINITY ? 0.0f : l_i[r] * expf(m_i[r] - mn)) + sum;
            m_i[r] = mn;
        }
    }
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) inv[r] = l_i[r] > 0.0f ? 1.0f / l_i[r] : 0.0f;
    // pass 2: P = (T)(exp(S - max) * (1 / sum)), O += P.V
    f32x4 o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) o[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    T* Vt_el = (T*)Vts;
    T* P_el = (T*)Ps[wave];
    for (int kt = 0; kt < n_kt; kt++) {
        __syncthreads();
        stage_k(kt);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int c = tid + i * 256, key = c >> 3, kc = c & 7, kg = kt * 64 + key;
            const u32x4 vv = kg < kv_end ? *(const u32x4*)(V + (long)kg * 64 + kc * 8) : zero;
            const T* ve = (const T*)&vv;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int dim = kc * 8 + e;
                Vt_el[(dim * 8 + swz(dim, key >> 3)) * 8 + (key & 7)] = ve[e];
            }
        }
        __syncthreads();
        f32x4 sacc[4];
        scores(kt, sacc);
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float p = sacc[j][r] == -INFINITY ? 0.0f : expf(sacc[j][r] - m_i[r]) * inv[r];
                const int row = (lane >> 4) * 4 + r, key = j * 16 + (lane & 15);
                P_el[(row * 8 + swz(row, key >> 3)) * 8 + (key & 7)] = (T)p;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P stores landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++) {
            const int prow = lane & 15;
            const FT pf = __builtin_bit_cast(FT, Ps[wave][prow * 8 + swz(prow, s2 * 4 + (lane >> 4))]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int vrow = j * 16 + (lane & 15);
                const FT vf = __builtin_bit_cast(FT, Vts[vrow * 8 + swz(vrow, s2 * 4 + (lane >> 4))]);
                o[j] = mfma16x16x32(pf, vf, o[j]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = wave * 16 + (lane >> 4) * 4 + r;
        if (row >= cnt) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) out[(long)(i0 + row) * d + h * 64 + j * 16 + (lane & 15)] = (T)o[j][r];
    }
}

void launch_attn_prefill(DType dt, const void* q, int q_stride, const void* cache, const int* slot, const int* n_kv,
                         const void* tiles, int n_tiles, int L, int layer, int H, int ctx, int d, void* out,
                         hipStream_t st) {
    if (n_tiles <= 0) return;
    dim3 grid(n_tiles, H);
    if (dt == DType::F16)
        attn_prefill_kernel<half_t><<<grid, 256, 0, st>>>((const half_t*)q, q_stride, (const half_t*)cache, slot, n_kv,
                                                          (const int2*)tiles, L, layer, H, ctx, d, (half_t*)out);
    else
        attn_prefill_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)q, q_stride, (const bf16_t*)cache, slot, n_kv,
                                                          (const int2*)tiles, L, layer, H, ctx, d, (bf16_t*)out);
}

// XCD-grouped encoder attention grid (attn_enc2_kernel): WHISPER_MI355X_ENC_ATTN_XCD=0 keeps the 3-D grid (A/B)
static bool attn_enc_xcd() {
    static const bool v = !getenv("WHISPER_MI355X_ENC_ATTN_XCD") || atoi(getenv("WHISPER_MI355X_ENC_ATTN_XCD")) != 0;
    return v;
}

void launch_attn_encoder(DType dt, const void* qkv, void* out, int B, int Tn, int d, int H, hipStream_t st,
                         int variant_arg) {
    // variant 6 (attn_enc2_kernel, 128 VGPRs, scalar softmax FMAs) unless a kernel benchmark asks for
    // another (whisper_mi355x_bench_attn_encoder)
    const int variant = variant_arg >= 0 ? variant_arg : 6;
    if (variant == 3 && d == H * 64) {
        dim3 grid(cdiv(Tn, 256), H, B);
        if (dt == DType::F16) attn_enc3_kernel<half_t><<<grid, 512, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d);
        else attn_enc3_kernel<bf16_t><<<grid, 512, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d);
        return;
    }
    if (variant == 6 && d == H * 64) {
        const int nqb = cdiv(Tn, 256);
        if ((long)nqb * H * B % 8 == 0 && attn_enc_xcd()) {
            const int G = nqb * H * B;
            if (dt == DType::F16) attn_enc2_kernel<half_t, 4, false><<<G, 512, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d, nqb, H);
            else attn_enc2_kernel<bf16_t, 4, false><<<G, 512, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d, nqb, H);
            return;
        }
        dim3 grid(nqb, H, B);
        if (dt == DType::F16) attn_enc2_kernel<half_t, 4, false><<<grid, 512, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d);
        else attn_enc2_kernel<bf16_t, 4, false><<<grid, 512, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d);
        return;
    }
    if (variant == 5 && d == H * 64) {
        dim3 grid(cdiv(Tn, 256), H, B);
        if (dt == DType::F16) attn_enc2_kernel<half_t, 4><<<grid, 512, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d);
        else attn_enc2_kernel<bf16_t, 4><<<grid, 512, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d);
        return;
    }
    if (variant == 2 && d == H * 64) {
        dim3 grid(cdiv(Tn, 256), H, B);
        if (dt == DType::F16) attn_enc2_kernel<half_t><<<grid, 512, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d);
        else attn_enc2_kernel<bf16_t><<<grid, 512, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d);
        return;
    }
    dim3 grid(cdiv(Tn, 64), H, B);
    if (dt == DType::F16) attn_enc_kernel<half_t><<<grid, 256, 0, st>>>((const half_t*)qkv, (half_t*)out, Tn, d);
    else attn_enc_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)qkv, (bf16_t*)out, Tn, d);
}

void launch_attn_decode(DType dt, const void* q, int q_stride, const void* cache, const int* slot, const int* n_kv, int n,
                        int L, int layer, int H, int ctx, int d, void* out, int kind, hipStream_t st) {
    if (n <= 0) return;
    if (ctx > 1536) WM_FAIL("attention context %d > 1536", ctx);
    dim3 grid(n, H);
#define WM_ATTN_DEC(TT, KN) \
    KN<TT><<<grid, 256, 0, st>>>((const TT*)q, q_stride, (const TT*)cache, slot, n_kv, L, layer, H, ctx, d, (TT*)out)
    if (dt == DType::F16) {
        if (kind == 2) WM_ATTN_DEC(half_t, attn_cross_prefill_kernel);
        else WM_ATTN_DEC(half_t, attn_self_kernel);
    } else {
        if (kind == 2) WM_ATTN_DEC(bf16_t, attn_cross_prefill_kernel);
        else WM_ATTN_DEC(bf16_t, attn_self_kernel);
    }
#undef WM_ATTN_DEC
}

// WHISPER_MI355X_XWIDE_MAX (default 8, read per call): decode steps of up to this many clips use the
// 1024-thread cache-form kernel (large-v3 bf16, profiles/r05_xwide_ab.txt: 8 clips 633 -> 664 audio-s/s
// with it; 16 clips 1124 -> 1070 and 32 clips 1700 -> 1645 without it stays faster)
int attn_cross_wide_max() {
    const char* e = getenv("WHISPER_MI355X_XWIDE_MAX");
    return e ? atoi(e) : 8;
}

void launch_attn_cross_step(DType dt, const DecSlabs& sl, const void* cache, const int* slot, const int* n_kv, int n,
                            int L, int layer, int H, int ctx, int d, void* out, hipStream_t st) {
    if (n <= 0) return;
    if (ctx > 1536) WM_FAIL("attention context %d > 1536", ctx);
    dim3 grid(n, H);
    if (n <= attn_cross_wide_max()) {
        if (dt == DType::F16)
            attn_cross_step_wide_kernel<half_t><<<grid, 1024, 0, st>>>(sl, (const half_t*)cache, slot, n_kv, L, layer, H, ctx, d, (half_t*)out);
        else
            attn_cross_step_wide_kernel<bf16_t><<<grid, 1024, 0, st>>>(sl, (const bf16_t*)cache, slot, n_kv, L, layer, H, ctx, d, (bf16_t*)out);
        return;
    }
    if (dt == DType::F16)
        attn_cross_step_kernel<half_t><<<grid, 256, 0, st>>>(sl, (const half_t*)cache, slot, n_kv, L, layer, H, ctx, d, (half_t*)out);
    else
        attn_cross_step_kernel<bf16_t><<<grid, 256, 0, st>>>(sl, (const bf16_t*)cache, slot, n_kv, L, layer, H, ctx, d, (bf16_t*)out);
}

void launch_attn_self_step(DType dt, const DecSlabs& sl, void* cache, const int* slot, const int* pos, int n, int L,
                           int layer, int H, int ctx, int d, void* out, hipStream_t st) {
    if (n <= 0) return;
    if (ctx > 448) WM_FAIL("self-attention context %d > 448", ctx);
    // heads (waves) per workgroup: 1 up to 32 clips (16 clips: decode 346.4 -> 342.7 ms per step), 4 above (128
    // clips: the same within noise); profiles/r06_self_hpb_ab.txt. WHISPER_MI355X_SELF_HPB (1 / 2 / 4) forces it for
    // an A/B. The waves of a workgroup share no data, so every value gives the same bits.
    static const int hpb_env = getenv("WHISPER_MI355X_SELF_HPB") ? atoi(getenv("WHISPER_MI355X_SELF_HPB")) : 0;
    const int want = hpb_env > 0 ? hpb_env : (n <= 32 ? 1 : 4);
    const int hpb = want >= 4 && H % 4 == 0 ? 4 : want >= 2 && H % 2 == 0 ? 2 : 1;
    // default-policy K/V reads (non-temporal measured 3048-3053 vs 3050-3057 audio-s/s, not kept)
#define WM_SELF(TT, HB) \
    attn_self_step_kernel<TT, HB, false><<<dim3(n, H / HB), 64 * HB, 0, st>>>(sl, (TT*)cache, slot, pos, L, layer, H, ctx, d, (TT*)out)
#define WM_SELF_H(TT) \
    do { if (hpb == 4) WM_SELF(TT, 4); else if (hpb == 2) WM_SELF(TT, 2); else WM_SELF(TT, 1); } while (0)
    if (dt == DType::F16) WM_SELF_H(half_t);
    else WM_SELF_H(bf16_t);
#undef WM_SELF_H
#undef WM_SELF
}

}  // namespace wm
