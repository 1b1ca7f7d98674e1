// Batched persistent decoder chain (the decode steps of 5-128 clips in the direct cross form: the headline's
// 128-clip batch, BASELINE configs[3], and one rank's 16-clip shard of it at 8 GPUs). SURVEY.md §8a row a10,
// the per-token loop of every whisper_full (whisper.rs:127-129), batched across clips (§8e).
//
// Why (VERDICT r4 "next" #3): at 128 clips a large-v3 decoder layer was ~16 dependent launches: six split-K
// GEMMs with their reduce launches (75.8 us for 46 MB of weights), the Q' projection and the split merge of the
// cross attention (29 us), around the one HBM-bound kernel, the pass over the encoder output E (86 us). The
// launches cost hand-offs through kernel boundaries and split-K slabs, not bytes. Here everything of a layer
// except the E pass runs in ONE launch of 256 workgroups (one per CU, 256 threads), in phases that hand off by
// row group through counters:
//
//   launch (la, lb) = the tail of layer la, then the head of layer lb (la = -1: the embedding; lb = L: the
//   final LayerNorm), between two xattn_step launches (kernels/xattn.hip):
//     T1  split merge of the cross attention + Wv, bv             (row group, head, half of the rows) tasks
//     T2  cross-out projection + bias + residual -> x              GEMM
//     T3  LN2 + FC1 + bias + GELU (ggml's f16 table)               GEMM
//     T4  FC2 + bias + residual -> x                               GEMM (K = 4d: four super-chunks)
//     H1  LN1 + QKV (+ bias, q and k scaled) -> q|k|v, k/v cache   GEMM
//     H2  self attention over the cache + this position            one wave per (clip, head)
//     H3  out projection + bias + residual -> x                    GEMM
//     H4  LN + cross-Q projection (+ bias, scaled)                 GEMM
//     H5  Q' = s Wk_h^T q_h, hi + lo parts (the E pass's operand)   (row group, head, half of the columns) tasks
//
// Tiling. Rows (clips) form row groups of 32 (nrg = ceil(M / 32) <= 4); the 256 workgroups are dealt to row
// groups so that the ones of a row group with equal blockIdx % 8 share an XCD and its L2 (rg = (w >> 3) %
// nrgp, column worker cw = (w & 7) | (w >> (3 + log2 nrgp)) << 3, WPR = 256 / nrgp workers per row group).
// A GEMM phase gives worker cw the 16-column tiles [cw N/16/WPR, (cw+1) N/16/WPR) of its row group's 32 rows over
// the WHOLE K: no split-K partials and no reduction. The 32 x K operand rows are loaded once into LDS (sc1 loads:
// handed off by other workgroups; for the LayerNorm phases the f32 residual rows are normalised on the way in);
// the weight tiles stream through a 6-stage LDS ring by LDS-DMA (non-temporal; stages issued before the hand-off
// wait, since weights do not depend on it). Wave q computes row tile q & 1 for half q >> 1 of the column tiles
// with v_mfma_f32_16x16x32, weights as the A operand so a lane ends with 4 consecutive columns of one row.
//
// Hand-offs (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md "Valid forms", table row 1): every
// handed-off byte is stored with sc1 (write-through) buffer stores; every storing wave waits vmcnt(0), the
// workgroup barrier, then one lane adds 1 to its row group's counter of the phase (agent-scope atomic; 8
// shards by XCD). A consumer's lane 0 polls the 8 shards with sc1 loads (s_sleep between polls) until every
// worker of the row group arrived (WPR / 8 per shard), the workgroup barrier, then EVERY load of handed-off
// bytes is an sc1 buffer load. Counters are per (layer, phase, row group), zeroed by a memset node before each
// step. Every worker of a row group arrives at every phase, with or without work in it. Waits are bounded
// (s_memrealtime, spin_ticks): a workgroup that gives up sets the error word and exits, every other wait sees
// it, later launches of the step exit at once, and the host re-runs the step on the per-kernel path (a give-up,
// counted like the persistent step's).
// Buffers reused inside a launch (x, the activations) are rewritten only behind a wait that transitively
// covers every reader of the previous contents (each phase's producers read their inputs before they arrive).
//
// Numerics (vs oracle/oracle_whisper.cpp): operands rounded to T as ggml's f16 src1, f32 accumulation over the
// whole K in one order (wave-local, k ascending), so a row's results do not depend on the other rows or on M;
// LayerNorm in double sums in one fixed order per row; epilogues as the launch-chain kernels' (gemm.hip
// epilogue: bias, then scale; GELU by ggml's table; residual (v + b) + x). Self attention as
// attn_self_step_kernel (kernels/attn.hip); the split merge and Q' projection as xattn_combine_kernel /
// xattn_qproj_kernel with the k-steps of the Wv product split over 4 waves instead of 8.
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace wm {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
// LDS through address-space-3 pointers only: a generic (flat) access would count in vmcnt too and break the
// counted waits of the weight ring
typedef __attribute__((address_space(3))) char lchar;
typedef __attribute__((address_space(3))) float lfloat;
template <class V>
__device__ __forceinline__ V lget(const lchar* base, int off) { return *(const __attribute__((address_space(3))) V*)(base + off); }
template <class V>
__device__ __forceinline__ void lput(lchar* base, int off, V v) { *(__attribute__((address_space(3))) V*)(base + off) = v; }

constexpr int kG = 256;    // workgroups (one per CU)
constexpr int kNT = 256;   // threads per workgroup
constexpr int kRS = 32;    // rows per row group
constexpr int kSC1 = 16;   // cache-policy bit of sc1 in the buffer intrinsics' aux operand

enum { PH_T1 = 0, PH_T2, PH_T3, PH_T4, PH_T5, PH_H0, PH_H1, PH_H2, PH_H3, PH_H4, PH_H5, PH_H6, kNPH };
enum { BE_QKV = 0, BE_RESID, BE_SCALE, BE_GELU };
enum { AS_T = 0, AS_LN, AS_EMB };  // a GEMM's operand rows: T rows, LayerNorm of x, LayerNorm of the embedding

__device__ __forceinline__ rsrc_t mkr(const void* p, long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)std::min<long>(bytes, 0x7fffffffL), 0x00020000);
}
__device__ __forceinline__ u32x4 ld16(rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1); }
__device__ __forceinline__ void st16(rsrc_t r, uint32_t off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSC1); }
__device__ __forceinline__ void st8(rsrc_t r, uint32_t off, u32x2 v) { __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, kSC1); }

// the thread index as a value the compiler cannot treat as loop-invariant (per-lane addresses are recomputed
// where used instead of being held in registers across the whole kernel; pdec_body.h)
__device__ __forceinline__ int ptid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
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
// whole-wave double sum, every lane the same bits: DPP inside each 16-lane row, then the 4 row sums in order
__device__ __forceinline__ double wave_sum_d(double x) {
    x += dppd<0xB1>(x);
    x += dppd<0x4E>(x);
    x += dppd<0x141>(x);
    x += dppd<0x140>(x);
    return (lane_d(x, 0) + lane_d(x, 16)) + (lane_d(x, 32) + lane_d(x, 48));
}
__device__ __forceinline__ float sum8(float a) {  // over the 8 lanes of a key row (quad xor 1, xor 2, half-row mirror)
    a += dppf<0xB1>(a);
    a += dppf<0x4E>(a);
    return a + dppf<0x141>(a);
}
// a workgroup-uniform value the compiler cannot prove uniform (an argument of a non-inlined callee arrives in a
// VGPR) moved to an SGPR
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
template <class P>
__device__ __forceinline__ P* uni(P* p) {
    const uint64_t v = (uint64_t)p;
    const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((unsigned)v), hi = (uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (P*)(lo | (hi << 32));
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// s_waitcnt vmcnt(n) for a run-time n (the immediate must be a constant)
__device__ __forceinline__ void vm_wait(int n) {
    switch (n) {
#define WM_VW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        WM_VW(0) WM_VW(1) WM_VW(2) WM_VW(3) WM_VW(4) WM_VW(5) WM_VW(6) WM_VW(7) WM_VW(8) WM_VW(9) WM_VW(10)
        WM_VW(11) WM_VW(12) WM_VW(13) WM_VW(14) WM_VW(15) WM_VW(16) WM_VW(17) WM_VW(18) WM_VW(19) WM_VW(20)
        WM_VW(21) WM_VW(22) WM_VW(23) WM_VW(24) WM_VW(25) WM_VW(26) WM_VW(27) WM_VW(28) WM_VW(29) WM_VW(30)
        WM_VW(31) WM_VW(32) WM_VW(33) WM_VW(34) WM_VW(35) WM_VW(36) WM_VW(37) WM_VW(38) WM_VW(39) WM_VW(40)
        WM_VW(41) WM_VW(42) WM_VW(43) WM_VW(44) WM_VW(45) WM_VW(46) WM_VW(47) WM_VW(48) WM_VW(49) WM_VW(50)
        WM_VW(51) WM_VW(52) WM_VW(53) WM_VW(54) WM_VW(55) WM_VW(56) WM_VW(57) WM_VW(58) WM_VW(59) WM_VW(60)
        WM_VW(61) WM_VW(62) WM_VW(63)
#undef WM_VW
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}
// s_waitcnt vmcnt(2 n) for n ring steps of two DMA instructions still allowed in flight, n in [0, NS - 2]
template <int NS>
__device__ __forceinline__ void vm_wait_steps(int n) {
    if (n >= NS - 2) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (NS - 2)) : "memory");
        return;
    }
    vm_wait(2 * n);
}
template <typename T>
__device__ __forceinline__ u32x2 pack4(const float (&v)[4]) {
    T o[4];
#pragma unroll
    for (int r = 0; r < 4; r++) o[r] = (T)v[r];
    return *(const u32x2*)o;
}
// ggml's GELU table lookup (the table lives in gemm.hip: gelu_table_device())
__device__ __forceinline__ float gelu_t(float x, const uint16_t* tab) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return (float)__builtin_bit_cast(half_t, tab[__builtin_bit_cast(uint16_t, (half_t)x)]);
}

template <int D>
struct BG {
    static constexpr int H = D / 64;
    static constexpr int CPR = D / 8;                 // 16-byte chunks per operand row (a super-chunk of K = D)
    static constexpr int A_BYTES = kRS * D * 2;       // operand image [32][D] T
    static constexpr int MAXCT = (D + 255) / 256;     // column tiles per worker at WPR = 64 (FC1: 4D / 16 / 64)
    // one wave's weight ring: a quarter of the rest of the 160 KB, in 1-KB slots (one MFMA fragment each)
    static constexpr int RW = ((160 * 1024 - A_BYTES - 1024) / 4) & ~1023;
    static constexpr int NS = RW / 2048 < 32 ? RW / 2048 : 32;  // its slots of 16 weight rows x 64 k
    static constexpr int RING = 4 * RW;
    static constexpr int LDS = A_BYTES + RING + 64;
};

// operand image [32 rows][D] T, 16-byte chunks XOR-swizzled per 256-byte group by the row (ds_read_b128 of
// 16 rows x one chunk: 16 distinct bank slots)
template <int D>
__device__ __forceinline__ int a_off(int row, int ch) {
    return row * D * 2 + (((ch & ~15) | ((ch & 15) ^ (row & 15))) << 4);
}

}  // namespace

// A phase's copy of the context's coordinates: a member read through `this` is a flat load of the stack object
// whenever the callee is not inlined, and the compiler then waits vmcnt(0) for it, draining the weight ring
// (the workgroup-uniform ones through readfirstlane, so that loop counters and the counted waits stay scalar)
#define BD_LOCALS                                                                                            \
    const int lane = this->lane, tid = this->tid;                                                             \
    const int wave = __builtin_amdgcn_readfirstlane(this->wave), r0 = __builtin_amdgcn_readfirstlane(this->r0); \
    const int cw = __builtin_amdgcn_readfirstlane(this->cw), wpr = __builtin_amdgcn_readfirstlane(this->wpr);   \
    lchar* const lds = this->lds;                                                                            \
    CArgs& a = this->a;                                                                                      \
    (void)lane; (void)wave; (void)tid; (void)r0; (void)cw; (void)wpr; (void)lds

// The launch's arguments read in place from the kernarg segment (constant address space: scalar loads). A
// reference to the by-value kernel parameter would make hipcc copy the whole struct to scratch first.
typedef __attribute__((address_space(4))) const BdecArgs CArgs;
typedef __attribute__((address_space(4))) const BdecLayer CLayer;

// The kernel's per-launch context (workgroup coordinates, LDS carve, the hand-off block).
template <typename T, int D>
struct BdecCtx {
    typedef typename Frag<T>::type FT;
    static constexpr int H = BG<D>::H;
    CArgs& a;
    lchar* lds;
    int w, tid, wave, lane;
    int nrg, lg, wpr, rg, cw, r0;
    bool active;
    unsigned* err;
    __attribute__((address_space(3))) int* lflag;

    __device__ BdecCtx(CArgs& a_, lchar* l) : a(a_), lds(l) {
        w = blockIdx.x;
        tid = ptid();
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        lane = tid & 63;
        nrg = (a.M + kRS - 1) / kRS;
        lg = nrg <= 1 ? 0 : nrg <= 2 ? 1 : 2;
        wpr = kG >> lg;
        rg = (w >> 3) & ((1 << lg) - 1);
        cw = (w & 7) | ((w >> (3 + lg)) << 3);
        r0 = rg * kRS;
        active = rg < nrg;
        err = a.cnt + a.err_index;
        lflag = (__attribute__((address_space(3))) int*)(lds + BG<D>::A_BYTES + BG<D>::RING);
    }
    __device__ unsigned* counter(int layer, int ph, int rgi, int shard) const {
        return a.cnt + (((long)layer * kNPH + ph) * 4 + rgi) * 8 + shard;
    }
    // every storing wave's stores retired, then one lane counts the workgroup in
    __device__ void arrive(int layer, int ph) {
        vm_wait_all();
        __syncthreads();
        if (a.dbg_fence == 2) {
            __threadfence();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (a.dbg_fence && tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (tid == 0) __hip_atomic_fetch_add(counter(layer, ph, rg, w & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // debug timeline (tools/bdec_stamps.py): the 100 MHz clock when phase ph's input arrived (k = 0), its output
    // was published (k = 1), its first operand image was in LDS (k = 2, GEMM phases), per launch and workgroup
    // (a vector store from lane 0)
    __device__ void stamp(int ph, int k) const {
        if (a.stamps && tid == 0) a.stamps[(((long)(a.la + 1) * 3 + k) * kNPH + ph) * kG + w] = __builtin_amdgcn_s_memrealtime();
    }
    // wait until every worker of this row group arrived at (layer, ph); false = give up (the caller returns)
    __device__ bool wait(int layer, int ph) {
        if (tid == 0) {
            const unsigned want = (unsigned)(wpr >> 3);
            bool ok = true;
            long t0 = 0;
            for (int it = 0;; it++) {
                bool done = true;
#pragma unroll
                for (int s = 0; s < 8; s++)
                    done &= __hip_atomic_load(counter(layer, ph, rg, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
                if (done) break;
                const long now = (long)__builtin_amdgcn_s_memrealtime();
                if (it == 0) t0 = now;
                if (now - t0 > a.spin_ticks) {
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
            *lflag = ok ? 1 : 0;
        }
        __syncthreads();
        const bool r = *lflag != 0;
        if (a.dbg_fence) {
            if (a.dbg_fence == 2) __threadfence();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        return r;
    }

    // ---- operand loading into the image ------------------------------------------------------------
    // rows r0.. r0+31 of a T matrix [M][ld] (handed off: sc1 loads), columns [k0, k0 + D)
    __device__ void load_a_t(const T* src, int ld, int k0) {
        BD_LOCALS;
        const rsrc_t r = mkr(src, (long)a.M * ld * 2);  // rows >= M read 0
        constexpr int CPR = BG<D>::CPR, NCH = kRS * CPR / kNT;
        u32x4 v[NCH];
#pragma unroll
        for (int u = 0; u < NCH; u++) {
            const int i = tid + kNT * u, row = i / CPR, c = i - row * CPR;
            v[u] = ld16(r, (uint32_t)(((long)(r0 + row) * ld + k0 + c * 8) * 2));
        }
#pragma unroll
        for (int u = 0; u < NCH; u++) {
            const int i = tid + kNT * u, row = i / CPR, c = i - row * CPR;
            lput<u32x4>(lds, a_off<D>(row, c), v[u]);
        }
    }
    // ---- operand image from LayerNorm rows: wave q normalises rows 8 q .. 8 q + 7 of the f32 residual x (sc1
    // loads; a batch of rows' loads in flight together) or of the token + position embedding (emb), ggml_norm's
    // arithmetic as ln_phase's, and writes them rounded to T into the image
    __device__ void load_a_ln(const float* x, bool emb, const float* gw, const float* gb) {
#pragma clang fp contract(off)
        BD_LOCALS;
        constexpr int NE = D / 256, RB = NE <= 3 ? 4 : 2;
        float g[NE][4], b[NE][4];
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const float4 gv = *(const float4*)(gw + 4 * lane + 256 * e);
            const float4 bv = *(const float4*)(gb + 4 * lane + 256 * e);
            g[e][0] = gv.x; g[e][1] = gv.y; g[e][2] = gv.z; g[e][3] = gv.w;
            b[e][0] = bv.x; b[e][1] = bv.y; b[e][2] = bv.z; b[e][3] = bv.w;
        }
        const rsrc_t rx = mkr(x, (long)a.M * D * 4);
#pragma unroll
        for (int r8 = 0; r8 < 8; r8 += RB) {
            float v[RB][NE][4];
            if (emb) {
#pragma unroll
                for (int rr = 0; rr < RB; rr++) {
                    const int m0 = r0 + wave * 8 + r8 + rr, m = m0 < a.M ? m0 : 0;
                    const long t = a.tok[m], p = a.pos[m];
#pragma unroll
                    for (int e = 0; e < NE; e++) {
                        const int k = 4 * lane + 256 * e;
                        const float4 pv = *(const float4*)(a.pos_d + p * D + k);
                        float tv[4];
                        if (a.te_f32) {
                            const float4 q = *(const float4*)((const float*)a.tok_emb + t * D + k);
                            tv[0] = q.x; tv[1] = q.y; tv[2] = q.z; tv[3] = q.w;
                        } else {
                            const u32x2 q = *(const u32x2*)((const T*)a.tok_emb + t * D + k);
                            const T* qe = (const T*)&q;
#pragma unroll
                            for (int j = 0; j < 4; j++) tv[j] = (float)qe[j];
                        }
                        v[rr][e][0] = tv[0] + pv.x; v[rr][e][1] = tv[1] + pv.y; v[rr][e][2] = tv[2] + pv.z; v[rr][e][3] = tv[3] + pv.w;
                    }
                }
            } else {
                u32x4 q[RB][NE];
#pragma unroll
                for (int rr = 0; rr < RB; rr++)
#pragma unroll
                    for (int e = 0; e < NE; e++)
                        q[rr][e] = ld16(rx, (uint32_t)(((long)(r0 + wave * 8 + r8 + rr) * D + 4 * lane + 256 * e) * 4));
#pragma unroll
                for (int rr = 0; rr < RB; rr++)
#pragma unroll
                    for (int e = 0; e < NE; e++) {
                        // (whole-vector cast: an element-wise cast of a buffer load's lanes lets this compiler narrow the
                        // load to its first dword and broadcast it, see DESIGN.md "toolchain notes")
                        const f32x4 f = __builtin_bit_cast(f32x4, q[rr][e]);
#pragma unroll
                        for (int j = 0; j < 4; j++) v[rr][e][j] = f[j];
                    }
            }
#pragma unroll
            for (int rr = 0; rr < RB; rr++) {
                double s = 0.0;
#pragma unroll
                for (int e = 0; e < NE; e++)
#pragma unroll
                    for (int j = 0; j < 4; j++) s += (double)v[rr][e][j];
                s = wave_sum_d(s);
                const float mean = (float)(s / D);
                double s2 = 0.0;
#pragma unroll
                for (int e = 0; e < NE; e++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        v[rr][e][j] = v[rr][e][j] - mean;
                        s2 += (double)(v[rr][e][j] * v[rr][e][j]);
                    }
                s2 = wave_sum_d(s2);
                const float variance = (float)(s2 / D);
                const float scale = 1.0f / sqrtf(variance + 1e-5f);
                const int row = wave * 8 + r8 + rr;
#pragma unroll
                for (int e = 0; e < NE; e++) {
                    float y[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        float t = v[rr][e][j] * scale;
                        t = t * g[e][j];
                        y[j] = t + b[e][j];
                    }
                    const int k = 4 * lane + 256 * e;
                    lput<u32x2>(lds, a_off<D>(row, k >> 3) + ((k >> 2) & 1) * 8, pack4<T>(y));
                }
            }
        }
    }

    // ---- LayerNorm phase (the final LayerNorm): row r0 + cw of the row group (workers cw < 32, wave 0) ------
    // ggml_norm: double sums, float mean / variance, (v * scale) * w + b separately rounded; lane l holds columns
    // 4 l + 256 e (+ 0..3), summed in e, then j order, then over the lanes by the fixed DPP tree. Input: the f32
    // residual x (sc1 loads) or, for layer 0's head (emb), the token + position embedding, which also becomes
    // x. Output: the row rounded to T (sc1 stores), the next GEMM's operand.
    __device__ bool ln_phase(int layer, int ph, int wait_layer, int wait_ph, bool emb, const float* gw, const float* gb,
                             T* out) {
#pragma clang fp contract(off)
        BD_LOCALS;
        constexpr int NE = D / 256;
        const int m = r0 + cw;
        const bool row = cw < kRS && m < a.M;  // (workgroup-uniform)
        float g[NE][4], b[NE][4];
        if (row && wave == 0) {  // the parameters before the wait
#pragma unroll
            for (int e = 0; e < NE; e++) {
                const float4 gv = *(const float4*)(gw + 4 * lane + 256 * e);
                const float4 bv = *(const float4*)(gb + 4 * lane + 256 * e);
                g[e][0] = gv.x; g[e][1] = gv.y; g[e][2] = gv.z; g[e][3] = gv.w;
                b[e][0] = bv.x; b[e][1] = bv.y; b[e][2] = bv.z; b[e][3] = bv.w;
            }
        }
        if (row && wait_ph >= 0 && !wait(wait_layer, wait_ph)) return false;
        stamp(ph, 0);
        if (row && wave == 0) {
            float v[NE][4];
            const rsrc_t rx = mkr(a.x, (long)a.M * D * 4);
            if (emb) {
                const long t = a.tok[m], p = a.pos[m];
#pragma unroll
                for (int e = 0; e < NE; e++) {
                    const int k = 4 * lane + 256 * e;
                    const float4 pv = *(const float4*)(a.pos_d + p * D + k);
                    float tv[4];
                    if (a.te_f32) {
                        const float4 q = *(const float4*)((const float*)a.tok_emb + t * D + k);
                        tv[0] = q.x; tv[1] = q.y; tv[2] = q.z; tv[3] = q.w;
                    } else {
                        const u32x2 q = *(const u32x2*)((const T*)a.tok_emb + t * D + k);
                        const T* qe = (const T*)&q;
#pragma unroll
                        for (int j = 0; j < 4; j++) tv[j] = (float)qe[j];
                    }
                    v[e][0] = tv[0] + pv.x; v[e][1] = tv[1] + pv.y; v[e][2] = tv[2] + pv.z; v[e][3] = tv[3] + pv.w;
                    u32x4 o;
#pragma unroll
                    for (int j = 0; j < 4; j++) o[j] = __builtin_bit_cast(uint32_t, v[e][j]);
                    st16(rx, (uint32_t)(((long)m * D + k) * 4), o);  // x = the embedding (the residual of H3)
                }
            } else {
                u32x4 q[NE];
#pragma unroll
                for (int e = 0; e < NE; e++) q[e] = ld16(rx, (uint32_t)(((long)m * D + 4 * lane + 256 * e) * 4));
#pragma unroll
                for (int e = 0; e < NE; e++) {
                    // (cast the whole vector: an element-wise cast of a buffer load's lanes lets this compiler
                    // narrow the load to its first dword and broadcast it, see DESIGN.md "toolchain notes")
                    const f32x4 f = __builtin_bit_cast(f32x4, q[e]);
#pragma unroll
                    for (int j = 0; j < 4; j++) v[e][j] = f[j];
                }
            }
            double s = 0.0;
#pragma unroll
            for (int e = 0; e < NE; e++)
#pragma unroll
                for (int j = 0; j < 4; j++) s += (double)v[e][j];
            s = wave_sum_d(s);
            const float mean = (float)(s / D);
            double s2 = 0.0;
#pragma unroll
            for (int e = 0; e < NE; e++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    v[e][j] = v[e][j] - mean;
                    s2 += (double)(v[e][j] * v[e][j]);
                }
            s2 = wave_sum_d(s2);
            const float variance = (float)(s2 / D);
            const float scale = 1.0f / sqrtf(variance + 1e-5f);
            const rsrc_t ro = mkr(out, (long)a.M * D * 2);
#pragma unroll
            for (int e = 0; e < NE; e++) {
                float y[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float t = v[e][j] * scale;
                    t = t * g[e][j];
                    y[j] = t + b[e][j];
                }
                st8(ro, (uint32_t)(((long)m * D + 4 * lane + 256 * e) * 2), pack4<T>(y));
            }
        }
        arrive(layer, ph);
        stamp(ph, 1);
        return true;
    }

    // ---- a GEMM phase: rows r0 .. r0 + 31, this worker's 16-column tiles of W [N][K] over the whole K ----------
    // The operand rows A [M][K] (T, handed off) go into the LDS image one super-chunk of D columns at a time
    // (FC2: four). The weights stream through wave-private rings by LDS-DMA, a slot = 16 weight rows x 64 k
    // (two DMA instructions of 8 whole 128-byte lines; chunks XOR-swizzled by (row >> 1) & 7), so a wave waits
    // only for its own DMA (counted vmcnt) and never for the other waves: no barrier per k-step. The weights use
    // the default cache policy: the row groups' workers with equal blockIdx % 8 share an XCD and read the same
    // columns. Wave q takes the 64-k steps q, q + 4, ... of every super-chunk, tile after tile, and sums them
    // into f32 accumulators; the four waves' partials are added in wave order through LDS at the end, then bias
    // and the epilogue. The summation order depends on K and the tile only, not on M or the other rows.
    template <int EPI, int ASRC>
    __device__ bool gemm(int layer, int ph, int wait_layer, int wait_ph, const T* W, const float* bias, int N, int K,
                         const void* A, void* out, int ldo, const float* gw = nullptr, const float* gb = nullptr) {
        BD_LOCALS;
        layer = uni(layer); N = uni(N); K = uni(K); ldo = uni(ldo);
        W = uni(W); A = uni(A); out = uni(out);
        constexpr int MAXCT = BG<D>::MAXCT, NKI = D / 256;  // a wave's 64-k steps per super-chunk
        constexpr int NS = BG<D>::NS;                          // ring slots
        constexpr int NI = (2 * MAXCT * 64 + kNT - 1) / kNT;   // epilogue items per thread
        const int nct_all = N / 16;
        const int ct0 = (int)((long)cw * nct_all / wpr), nct = (int)((long)(cw + 1) * nct_all / wpr) - ct0;
        const int nsc = K / D;
        const int nstep = nsc * NKI * nct;  // the wave's stream: step (j, t) = j * nct + t, j = its 64-k steps
        const bool skip_w = (a.dbg_skip & 1) != 0, skip_a = (a.dbg_skip & 2) != 0;
        lchar* ring = lds + BG<D>::A_BYTES + wave * BG<D>::RW;
        // DMA lane: row wr (+ 8 in the second instruction) of the slot, the chunk that lands at its position
        const int wr = lane >> 3, wc0 = (lane & 7) ^ ((wr >> 1) & 7), wc1 = (lane & 7) ^ (((wr + 8) >> 1) & 7);
        const T* wl = W + (long)(ct0 * 16 + wr) * K + wc0 * 8 + wave * 64;
        const long wl1 = 8L * K + (wc1 - wc0) * 8;  // the second instruction's source, relative
        // the next step to issue: (ij, it) into slot islot
        int ij = 0, it = 0, islot = 0, nissued = 0;
        auto issue = [&]() {
            if (!skip_w) {
                const T* src = wl + (long)it * 16 * K + (long)ij * 256;
                lchar* dst = ring + islot * 2048;
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)dst, 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(src + wl1), (lds_ptr_t)(dst + 1024), 16, 0, 0);
            }
            nissued++;
            islot = islot == NS - 1 ? 0 : islot + 1;
            if (++it == nct) {
                it = 0;
                ij++;
            }
        };
        // a fragment lane's byte offset in a slot: row lane & 15, chunk 4 s + (lane >> 4) of sub-step s
        const int fr = lane & 15, fo0 = fr * 128 + (((lane >> 4) ^ ((fr >> 1) & 7)) << 4),
                  fo1 = fr * 128 + (((4 + (lane >> 4)) ^ ((fr >> 1) & 7)) << 4);
        const int npre = min(nstep, NS - 1);
        for (int g = 0; g < npre; g++) issue();
        // (a worker without column tiles reads nothing: it arrives without waiting)
        if (nct > 0 && wait_ph >= 0 && !wait(wait_layer, wait_ph)) return false;
        stamp(ph, 0);
        if (nct > 0) {
            const int nit = 2 * nct * 64;
            u32x4 xold[NI];
            if constexpr (EPI == BE_RESID) {  // the residual this worker updates (loaded behind the wait)
                const rsrc_t rx = mkr(out, (long)a.M * ldo * 4);
#pragma unroll
                for (int u = 0; u < NI; u++) {
                    const int i = tid + kNT * u, rt = i / (nct * 64), rem = i - rt * nct * 64, t = rem >> 6, l = rem & 63;
                    const int n = (ct0 + t) * 16 + 4 * (l >> 4), mrow = r0 + rt * 16 + (l & 15);
                    xold[u] = i < nit ? ld16(rx, (uint32_t)(((long)mrow * ldo + n) * 4)) : u32x4{0, 0, 0, 0};
                }
            }
            f32x4 acc[2][MAXCT];
#pragma unroll
            for (int t = 0; t < MAXCT; t++) acc[0][t] = acc[1][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
            int g = 0, slot = 0;
            for (int sc = 0; sc < nsc; sc++) {
                if (sc > 0) lds_barrier();  // every wave is done with the previous image
                if (skip_a) {
                } else if constexpr (ASRC == AS_T) {
                    load_a_t((const T*)A, K, sc * D);
                } else {
                    load_a_ln((const float*)A, ASRC == AS_EMB, gw, gb);
                }
                vm_wait_all();  // (also retires the weight steps issued so far)
                lds_barrier();
                if (sc == 0) stamp(ph, 2);
                for (int jj = 0; jj < NKI; jj++) {
                    // the operand fragments of this 64-k step, shared by the tiles
                    const int ch = (4 * jj + wave) * 8 + (lane >> 4);
                    const FT a00 = lget<FT>(lds, a_off<D>(lane & 15, ch)), a01 = lget<FT>(lds, a_off<D>(lane & 15, ch + 4));
                    const FT a10 = lget<FT>(lds, a_off<D>(16 + (lane & 15), ch)), a11 = lget<FT>(lds, a_off<D>(16 + (lane & 15), ch + 4));
#pragma unroll
                    for (int t = 0; t < MAXCT; t++) {
                        if (t >= nct) break;
                        // step g landed: at most the steps issued after it still in flight
                        vm_wait_steps<NS>(nissued - g - 1);
                        const lchar* sl = ring + slot * 2048;
                        const FT b0 = lget<FT>(sl, fo0), b1 = lget<FT>(sl, fo1);
                        if (nissued < nstep) issue();  // into the slot read one step ago
                        acc[0][t] = mfma16x16x32(b0, a00, acc[0][t]);
                        acc[1][t] = mfma16x16x32(b0, a10, acc[1][t]);
                        acc[0][t] = mfma16x16x32(b1, a01, acc[0][t]);
                        acc[1][t] = mfma16x16x32(b1, a11, acc[1][t]);
                        g++;
                        slot = slot == NS - 1 ? 0 : slot + 1;
                    }
                }
            }
            // the waves' partials -> LDS [wave][rt][t][lane], summed in wave order
            lds_barrier();
            lchar* red = lds + BG<D>::A_BYTES;
#pragma unroll
            for (int t = 0; t < MAXCT; t++) {
                if (t >= nct) break;
#pragma unroll
                for (int rt = 0; rt < 2; rt++) lput<f32x4>(red, (((wave * 2 + rt) * MAXCT + t) * 64 + lane) * 16, acc[rt][t]);
            }
            lds_barrier();
            // epilogue: item (rt, t, l) holds columns n .. n + 3 of row mrow
#pragma unroll
            for (int u = 0; u < NI; u++) {
                const int i = tid + kNT * u, rt = i / (nct * 64), rem = i - rt * nct * 64, t = rem >> 6, l = rem & 63;
                const int n = (ct0 + t) * 16 + 4 * (l >> 4), mrow = r0 + rt * 16 + (l & 15);
                if (i >= nit || mrow >= a.M) continue;
                f32x4 sum = lget<f32x4>(red, ((rt * MAXCT + t) * 64 + l) * 16);
#pragma unroll
                for (int q = 1; q < 4; q++) sum += lget<f32x4>(red, (((q * 2 + rt) * MAXCT + t) * 64 + l) * 16);
                const float4 bb = bias ? *(const float4*)(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
                float v[4] = {sum[0] + bb.x, sum[1] + bb.y, sum[2] + bb.z, sum[3] + bb.w};
                if constexpr (EPI == BE_RESID) {
                    f32x4 xo = __builtin_bit_cast(f32x4, xold[u]);  // (whole-vector cast, as in load_a_ln)
                    if (a.la < 0 && a.lb == 0) {  // layer 0's head launch: the residual is the embedding
                        const long tk = a.tok[mrow], p = a.pos[mrow];
#pragma unroll
                        for (int r = 0; r < 4; r++)
                            xo[r] = (a.te_f32 ? ((const float*)a.tok_emb)[tk * D + n + r] : (float)((const T*)a.tok_emb)[tk * D + n + r]) +
                                    a.pos_d[p * D + n + r];
                    }
                    u32x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = __builtin_bit_cast(uint32_t, v[r] + xo[r]);
                    st16(mkr(out, (long)a.M * ldo * 4), (uint32_t)(((long)mrow * ldo + n) * 4), o);
                } else if constexpr (EPI == BE_QKV) {
                    const int part = n / D;  // 0 q, 1 k, 2 v (a 16-column tile never straddles)
                    if (part < 2) {
#pragma unroll
                        for (int r = 0; r < 4; r++) v[r] = v[r] * a.k_scale;
                    }
                    const u32x2 pk = pack4<T>(v);
                    st8(mkr(out, (long)a.M * ldo * 2), (uint32_t)(((long)mrow * ldo + n) * 2), pk);
                    if (part > 0) {  // the self cache at this position (read by later steps)
                        const int nn = n - part * D, h = nn >> 6, dh = nn & 63;
                        const long sl = a.slot[mrow], pos = a.pos[mrow];
                        T* dst = (T*)a.self_cache + ((((sl * a.L + layer) * 2 + (part - 1)) * H + h) * (long)a.n_text_ctx + pos) * 64 + dh;
                        *(u32x2*)dst = pk;
                    }
                } else if constexpr (EPI == BE_SCALE) {
#pragma unroll
                    for (int r = 0; r < 4; r++) v[r] = v[r] * a.k_scale;
                    st8(mkr(out, (long)a.M * ldo * 2), (uint32_t)(((long)mrow * ldo + n) * 2), pack4<T>(v));
                } else {  // BE_GELU
#pragma unroll
                    for (int r = 0; r < 4; r++) v[r] = gelu_t(v[r], a.gelu_tab);
                    st8(mkr(out, (long)a.M * ldo * 2), (uint32_t)(((long)mrow * ldo + n) * 2), pack4<T>(v));
                }
            }
        }
        arrive(layer, ph);
        stamp(ph, 1);
        return true;
    }

    // ---- T1: merge the cross-attention splits of (row group, head h, half b of the rows) and apply Wv -------
    __device__ bool combine(int layer, CLayer& Lw) {
        BD_LOCALS;
        const int S = a.S;
        const int j = cw, h = j >> 1, half = j & 1;
        const bool task = j < 2 * H;
        lfloat* wgt = (lfloat*)(lds + BG<D>::A_BYTES);          // [16 rows][16 splits] (ring region)
        lfloat* red = (lfloat*)(lds + BG<D>::A_BYTES + 1024);   // [4 waves][32][64]
        const int mb = r0 + 16 * half;                        // first row of the task
        stamp(PH_T1, 0);
        constexpr int KS = D / 32, KW = KS / 4;               // k-steps, per wave
        if (task) {
            if (tid < 16) {
                const int m = mb + tid;
                if (m < a.M) {
                    const float* p = a.ml + ((long)m * S * H + h) * 2;
                    float Mx = -INFINITY;
                    for (int s = 0; s < S; s++) Mx = fmaxf(Mx, p[(long)s * H * 2]);
                    float Ls = 0.0f;
                    for (int s = 0; s < S; s++) Ls += __builtin_amdgcn_exp2f(p[(long)s * H * 2] - Mx) * p[(long)s * H * 2 + 1];
                    const float inv = 1.0f / Ls;
                    for (int s = 0; s < S; s++) wgt[tid * 16 + s] = __builtin_amdgcn_exp2f(p[(long)s * H * 2] - Mx) * inv;
                } else {
                    for (int s = 0; s < S; s++) wgt[tid * 16 + s] = 0.0f;
                }
            }
            __syncthreads();
            // merged E~ = sum_s w_s O_s (f32), split into hi + lo rows of the image (rows 0-15 hi, 16-31 lo); a
            // split's loads of every element of the thread are in flight together (one latency per split)
            constexpr int Q4 = D / 4, NE = 16 * Q4 / kNT;
            {
                f32x4 mg[NE];
#pragma unroll
                for (int u = 0; u < NE; u++) mg[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
                for (int s = 0; s < S; s++) {
                    f32x4 xv[NE];
#pragma unroll
                    for (int u = 0; u < NE; u++) {
                        const int e = tid + kNT * u, t = e / Q4, c = (e - t * Q4) * 4;
                        const int m = min(mb + t, a.M - 1);
                        xv[u] = __builtin_nontemporal_load((const f32x4*)(a.opart + (((long)m * S + s) * H + h) * D + c));
                    }
#pragma unroll
                    for (int u = 0; u < NE; u++) {
                        const int t = (tid + kNT * u) / Q4;
                        const float wt = wgt[t * 16 + s];
#pragma unroll
                        for (int k = 0; k < 4; k++) mg[u][k] += wt * xv[u][k];
                    }
                }
#pragma unroll
                for (int u = 0; u < NE; u++) {
                    const int e = tid + kNT * u, t = e / Q4, c = (e - t * Q4) * 4;
                    float hi[4], lo[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const T th = (T)mg[u][k];
                        hi[k] = (float)th;
                        lo[k] = mg[u][k] - hi[k];
                    }
                    const int ch = c >> 3, hf = ((c >> 2) & 1) * 8;
                    lput<u32x2>(lds, a_off<D>(t, ch) + hf, pack4<T>(hi));
                    lput<u32x2>(lds, a_off<D>(16 + t, ch) + hf, pack4<T>(lo));
                }
            }
            // Wv fragments of this wave's k-steps (ks = wave + 4 u), 4 column tiles (the head's 64 outputs)
            const T* wv = (const T*)Lw.wv;
            FT wf[KW][4];
#pragma unroll
            for (int u = 0; u < KW; u++)
#pragma unroll
                for (int c = 0; c < 4; c++)
                    wf[u][c] = *(const FT*)(wv + ((long)h * 64 + c * 16 + (lane & 15)) * D + (wave + 4 * u) * 32 + 8 * (lane >> 4));
            __syncthreads();
            f32x4 acc[2][4];
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) acc[r][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < KW; u++) {
                const int ks = wave + 4 * u;
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    const FT af = lget<FT>(lds, a_off<D>(r * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
                    for (int c = 0; c < 4; c++) acc[r][c] = mfma16x16x32(wf[u][c], af, acc[r][c]);
                }
            }
            // lane: columns c*16 + 4 (lane >> 4) + i of row (lane & 15) of the hi (r = 0) / lo (r = 1) image
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int c = 0; c < 4; c++)
                    lput<f32x4>((lchar*)red, 4 * ((wave * 32 + r * 16 + (lane & 15)) * 64 + c * 16 + 4 * (lane >> 4)), acc[r][c]);
            __syncthreads();
            {
                const int t = tid >> 4, c4 = (tid & 15) * 4, m = mb + t;
                float v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float s = 0.0f;
#pragma unroll
                    for (int q = 0; q < 4; q++) s += red[(q * 32 + t) * 64 + c4 + k] + red[(q * 32 + 16 + t) * 64 + c4 + k];
                    v[k] = s + Lw.bv[h * 64 + c4 + k];
                }
                if (m < a.M) st8(mkr(a.batt, (long)a.M * D * 2), (uint32_t)(((long)m * D + h * 64 + c4) * 2), pack4<T>(v));
            }
        }
        arrive(layer, PH_T1);
        stamp(PH_T1, 1);
        return true;
    }

    // ---- H2: self attention, one wave per (clip, head) task (attn_self_step_kernel's arithmetic) ----------
    // A task's first 64 cached keys and values (earlier steps' rows: not handed off) are issued with its q / k /
    // v loads, one round trip per task; the wave's first task's before the hand-off wait.
    __device__ bool self_attn(int layer) {
        BD_LOCALS;
        constexpr int U = 8;
        const u32x4 zero = {0, 0, 0, 0};
        const int lane8 = lane & 7, grp = lane >> 3;
        const T* cache = (const T*)a.self_cache;
        const int t_first = cw * 4 + wave, t_step = wpr * 4;
        u32x4 rk[U], rv[U];
        auto kv_first = [&](int t) {
            const int m = r0 + t / H, h = t % H;
            const bool ok = t < kRS * H && m < a.M;
            const int pos = ok ? a.pos[m] : 0;
            const long sl = ok ? a.slot[m] : 0;
            const T* K = cache + (((sl * a.L + layer) * 2 + 0) * H + h) * (long)a.n_text_ctx * 64;
            const T* V = cache + (((sl * a.L + layer) * 2 + 1) * H + h) * (long)a.n_text_ctx * 64;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int tt = grp + 8 * u;
                rk[u] = tt < pos ? __builtin_nontemporal_load((const u32x4*)(K + (long)tt * 64 + lane8 * 8)) : zero;
                rv[u] = tt < pos ? __builtin_nontemporal_load((const u32x4*)(V + (long)tt * 64 + lane8 * 8)) : zero;
            }
        };
        kv_first(t_first);
        if (!wait(layer, PH_H1)) return false;
        stamp(PH_H2, 0);
        lfloat* qs = (lfloat*)lds + wave * (3 * 64 + 448);
        lfloat* ks = qs + 64;
        lfloat* vs = qs + 128;
        lfloat* sc = qs + 192;
        const rsrc_t rq = mkr(a.bq, (long)a.M * 3 * D * 2);
        for (int t = t_first; t < kRS * H; t += t_step) {
            const int m = r0 + t / H, h = t % H;
            if (m >= a.M) break;  // (wave-uniform; tasks are in row order)
            const int pos = a.pos[m];
            const long sl = a.slot[m];
            const T* K = cache + (((sl * a.L + layer) * 2 + 0) * H + h) * (long)a.n_text_ctx * 64;
            const T* V = cache + (((sl * a.L + layer) * 2 + 1) * H + h) * (long)a.n_text_ctx * 64;
            if (t != t_first) kv_first(t);
            // q, k, v of this (clip, head): lanes 0-7 / 8-15 / 16-23 load 8 values each (sc1: handed off)
            if (lane < 24) {
                const int part = lane >> 3, e0 = (lane & 7) * 8;
                const u32x4 raw = ld16(rq, (uint32_t)(((long)m * 3 * D + part * D + h * 64 + e0) * 2));
                const T* re = (const T*)&raw;
#pragma unroll
                for (int e = 0; e < 8; e++) qs[part * 64 + e0 + e] = (float)re[e];
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float qv[8];
#pragma unroll
            for (int e = 0; e < 8; e++) qv[e] = qs[lane8 * 8 + e];
            float lmax = -INFINITY;
            for (int t0 = grp; t0 < pos; t0 += 8 * U) {
                u32x4 raw[U];
                if (t0 == grp) {
#pragma unroll
                    for (int u = 0; u < U; u++) raw[u] = rk[u];
                } else {
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int tt = t0 + 8 * u;
                        raw[u] = tt < pos ? __builtin_nontemporal_load((const u32x4*)(K + (long)tt * 64 + lane8 * 8)) : zero;
                    }
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int tt = t0 + 8 * u;
                    const T* ke = (const T*)&raw[u];
                    float s = 0.0f;
#pragma unroll
                    for (int e = 0; e < 8; e++) s += qv[e] * (float)ke[e];
                    s = sum8(s);
                    if (tt < pos) {
                        if (lane8 == 0) sc[tt] = s;
                        lmax = fmaxf(lmax, s);
                    }
                }
            }
            {  // the fresh key (this position)
                float s = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; e++) s += qv[e] * ks[lane8 * 8 + e];
                s = sum8(s);
                if (lane == 0) sc[pos] = s;
                lmax = fmaxf(lmax, s);
            }
            for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int n_kv = pos + 1;
            float lsum = 0.0f;
            for (int tt = lane; tt < n_kv; tt += 64) {
                const float e = expf(sc[tt] - lmax);
                sc[tt] = e;
                lsum += e;
            }
            for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o);
            const float inv = 1.0f / lsum;
            for (int tt = lane; tt < n_kv; tt += 64) sc[tt] = (float)(T)(sc[tt] * inv);  // P rounded as ggml's f16 src1
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float acc[8];
#pragma unroll
            for (int e = 0; e < 8; e++) acc[e] = 0.0f;
            for (int t0 = grp; t0 < pos; t0 += 8 * U) {
                u32x4 raw[U];
                if (t0 == grp) {
#pragma unroll
                    for (int u = 0; u < U; u++) raw[u] = rv[u];
                } else {
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int tt = t0 + 8 * u;
                        raw[u] = tt < pos ? __builtin_nontemporal_load((const u32x4*)(V + (long)tt * 64 + lane8 * 8)) : zero;
                    }
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int tt = t0 + 8 * u;
                    const T* ve = (const T*)&raw[u];
                    const float p = tt < pos ? sc[tt] : 0.0f;
#pragma unroll
                    for (int e = 0; e < 8; e++) acc[e] += p * (float)ve[e];
                }
            }
            if (grp == 0) {
                const float p = sc[pos];
#pragma unroll
                for (int e = 0; e < 8; e++) acc[e] += p * vs[lane8 * 8 + e];
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                acc[e] += dppf<0x128>(acc[e]);  // row_ror:8 = lane ^ 8 within the 16-lane row
                acc[e] += __shfl_xor(acc[e], 16);
                acc[e] += __shfl_xor(acc[e], 32);
            }
            if (grp == 0) {
                T o8[8];
#pragma unroll
                for (int e = 0; e < 8; e++) o8[e] = (T)acc[e];
                st16(mkr(a.batt, (long)a.M * D * 2), (uint32_t)(((long)m * D + h * 64 + lane8 * 8) * 2), *(const u32x4*)o8);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // qs / sc reused by the next task
        }
        arrive(layer, PH_H2);
        stamp(PH_H2, 1);
        return true;
    }

    // ---- H6: Q'_h = s Wk_h^T q_h (hi + lo) for (row group, head h, half b of the d columns) -----------------
    // The task's Wk_h^T fragments (NPW column tiles per wave) are loaded before the hand-off wait.
    __device__ bool qproj(int layer, CLayer& Lw) {
        BD_LOCALS;
        const int j = cw, h = j >> 1, half = j & 1;
        const bool task = j < 2 * H;
        constexpr int NCT = D / 2 / 16, NPW = NCT / 4;  // column tiles of the half, per wave
        const T* wkt = (const T*)Lw.wkt;  // [H][D][64]
        FT wf[NPW][2];
        if (task) {
#pragma unroll
            for (int u = 0; u < NPW; u++)
#pragma unroll
                for (int ks = 0; ks < 2; ks++)
                    wf[u][ks] = *(const FT*)(wkt + ((long)h * D + half * (D / 2) + (wave + 4 * u) * 16 + (lane & 15)) * 64 + ks * 32 +
                                             8 * (lane >> 4));
        }
        if (!wait(layer, PH_H5)) return false;
        stamp(PH_H6, 0);
        if (!task) return true;
        const rsrc_t rq = mkr(a.bxq, (long)a.M * D * 2);
        FT qf[2][2];
#pragma unroll
        for (int rt = 0; rt < 2; rt++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++) {
                const int m = r0 + rt * 16 + (lane & 15);
                qf[rt][ks] = __builtin_bit_cast(FT, ld16(rq, (uint32_t)(((long)m * D + h * 64 + ks * 32 + 8 * (lane >> 4)) * 2)));
            }
        T* qx = (T*)a.qx;
#pragma unroll
        for (int u = 0; u < NPW; u++) {
            const int c0 = half * (D / 2) + (wave + 4 * u) * 16;
#pragma unroll
            for (int rt = 0; rt < 2; rt++) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ks++) acc = mfma16x16x32(wf[u][ks], qf[rt][ks], acc);
                const int m = r0 + rt * 16 + (lane & 15);
                if (m >= a.M) continue;
                const int c = c0 + 4 * (lane >> 4);
                float hi[4], lo[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float v = acc[r] * a.k_scale;
                    const T th = (T)v;
                    hi[r] = (float)th;
                    lo[r] = v - hi[r];
                }
                *(u32x2*)(qx + ((long)m * 2 * H + h) * D + c) = pack4<T>(hi);
                *(u32x2*)(qx + ((long)m * 2 * H + H + h) * D + c) = pack4<T>(lo);
            }
        }
        stamp(PH_H6, 1);
        return true;
    }
};

template <typename T, int D>
__global__ void __launch_bounds__(kNT, 1) bdec_kernel(const BdecArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    (void)a;
    CArgs& A = *(CArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    BdecCtx<T, D> C(A, (lchar*)smem);
    if (__hip_atomic_load(C.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // an earlier launch gave up
    if (!C.active || (A.dbg_head_only && A.la >= 0)) return;
    CLayer* LT = (CLayer*)A.layers;
    constexpr int d = D;
    if (A.la >= 0) {
        CLayer& W = LT[A.la];
        const int l = A.la;
        if (!C.combine(l, W)) return;
        if (!C.template gemm<BE_RESID, AS_T>(l, PH_T2, l, PH_T1, (const T*)W.wxo, W.bxo, d, d, A.batt, A.x, d)) return;
        if (!C.template gemm<BE_GELU, AS_LN>(l, PH_T4, l, PH_T2, (const T*)W.w1, W.b1, 4 * d, d, A.x, A.bff, 4 * d, W.ln2_w, W.ln2_b)) return;
        if (!C.template gemm<BE_RESID, AS_T>(l, PH_T5, l, PH_T4, (const T*)W.w2, W.b2, d, 4 * d, A.bff, A.x, d)) return;
    }
    if (A.lb < A.L) {
        CLayer& W = LT[A.lb];
        const int l = A.lb;
        bool ok;
        if (A.la < 0) ok = C.template gemm<BE_QKV, AS_EMB>(l, PH_H1, 0, -1, (const T*)W.wqkv, W.bqkv, 3 * d, d, A.x, A.bq, 3 * d, W.ln1_w, W.ln1_b);
        else ok = C.template gemm<BE_QKV, AS_LN>(l, PH_H1, A.la, PH_T5, (const T*)W.wqkv, W.bqkv, 3 * d, d, A.x, A.bq, 3 * d, W.ln1_w, W.ln1_b);
        if (!ok) return;
        if (!C.self_attn(l)) return;
        if (!C.template gemm<BE_RESID, AS_T>(l, PH_H3, l, PH_H2, (const T*)W.wo, W.bo, d, d, A.batt, A.x, d)) return;
        if (!C.template gemm<BE_SCALE, AS_LN>(l, PH_H5, l, PH_H3, (const T*)W.wxq, W.bxq, d, d, A.x, A.bxq, d, W.lnx_w, W.lnx_b)) return;
        C.qproj(l, W);
    } else {  // the final LayerNorm (the logits GEMM's input; counters of the spare layer slot L)
        C.ln_phase(A.L, PH_H0, A.la, PH_T5, false, A.lnd_w, A.lnd_b, (T*)A.out_dh);
    }
}

bool bdec_supported(int d) { return d == 768 || d == 1024 || d == 1280; }

size_t bdec_sync_bytes(int L) { return ((size_t)(L + 1) * kNPH * 4 * 8 + 64) * 4; }

int bdec_err_index(int L) { return (L + 1) * kNPH * 4 * 8; }

template <typename T, int DD>
static void bdec_launch_d(const BdecArgs& a, hipStream_t st) {
    static bool attr = [] {  // dynamic LDS above 64 KB
        WM_CHECK(hipFuncSetAttribute((const void*)bdec_kernel<T, DD>, hipFuncAttributeMaxDynamicSharedMemorySize, BG<DD>::LDS));
        return true;
    }();
    (void)attr;
    bdec_kernel<T, DD><<<kG, kNT, BG<DD>::LDS, st>>>(a);
    WM_CHECK(hipGetLastError());
}
template <typename T>
static void bdec_launch_t(const BdecArgs& a, hipStream_t st) {
#define WM_BD(DD)                 \
    case DD:                      \
        bdec_launch_d<T, DD>(a, st); \
        return;
    switch (a.d) { WM_BD(768) WM_BD(1024) WM_BD(1280) default: break; }
#undef WM_BD
    WM_FAIL("bdec: d %d", a.d);
}

void launch_bdec(DType dt, const BdecArgs& a, hipStream_t st) {
    if (a.M < 1 || a.M > 4 * kRS) WM_FAIL("bdec: %d rows", a.M);
    if (a.S < 1 || a.S > 16) WM_FAIL("bdec: %d splits", a.S);
    if (a.n_text_ctx > 448) WM_FAIL("bdec: text context %d", a.n_text_ctx);
    if (dt == DType::F16) bdec_launch_t<half_t>(a, st);
    else bdec_launch_t<bf16_t>(a, st);
}

}  // namespace wm
