// Device-side whisper_process_logits + whisper_sample_token(best=true).
//
// One 1024-thread workgroup per sequence reads its logits row (V = 51864..51866 f32) once, into
// from L2 and returns only a TokOut record (token id, p, plog, tid, pt, ptsum, no-speech prob),
// so the host never copies a [B, V] logits block per step. Rules, in whisper.cpp's order [ext]:
// temperature divide; suppress_blank (initial step: EOT and " "); <|notimestamps|>; optional
// no_timestamps; sot/nosp/solm/translate/transcribe/prev; the 100 language tokens; timestamp
// pairing; max_initial_ts; monotonic timestamps; log-softmax; "sum(p(timestamps)) > max p(text)
// => timestamp"; probs = exp(logprob). Greedy argmax keeps whisper's first-index tie break over
// the float probs. When temperature > 0 the probs row is also written for host-side sampling
// (std::discrete_distribution, exactly as whisper.cpp samples).
// This file is compiled with -ffp-contract=off.
#include "../common.h"
#include "../kernels.h"

namespace wm {

static constexpr int LT = 1024;

__device__ __forceinline__ float masked_logit(float x, int i, const SeqCtl& c, const VocabIds& v) {
    if (c.temperature > 0.0f) x = x / c.temperature;
    // text tokens (every special id is >= eot): only the blank and the timestamp-pairing rules reach them
    if (i < v.eot) {
        if (c.last_ts && !c.penult_ts) return -INFINITY;
        if (c.suppress_blank && c.is_initial && i == v.space) return -INFINITY;
        return x;
    }
    if (c.suppress_blank && c.is_initial && (i == v.eot || i == v.space)) return -INFINITY;
    if (i == v.not_) return -INFINITY;
    if (c.no_timestamps && i >= v.beg) return -INFINITY;
    if (i == v.sot || i == v.nosp || i == v.solm || i == v.translate || i == v.transcribe || i == v.prev) return -INFINITY;
    if (i > v.sot && i <= v.sot + v.n_lang) return -INFINITY;
    if (c.suppress_eot && i == v.eot) return -INFINITY;
    if (c.last_ts) {
        if (c.penult_ts) { if (i >= v.beg) return -INFINITY; }
        else if (i < v.eot) return -INFINITY;
    }
    if (c.is_initial && c.tid0_initial >= 0 && i >= v.beg + c.tid0_initial + 1) return -INFINITY;
    if (c.has_ts && i >= v.beg && i < v.beg + c.seek_delta / 2) return -INFINITY;
    return x;
}

__device__ float block_max(float x, float* sh) {
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = x;
    __syncthreads();
    float r = sh[0];
    for (int i = 1; i < LT / 64; i++) r = fmaxf(r, sh[i]);
    return r;
}
__device__ float block_sum(float x, float* sh) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = x;
    __syncthreads();
    float r = 0.0f;
    for (int i = 0; i < LT / 64; i++) r += sh[i];
    return r;
}
__device__ double block_sum_d(double x, double* sh) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = x;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < LT / 64; i++) r += sh[i];
    return r;
}
// argmax with first-index tie break: (value larger) or (equal and index smaller)
__device__ void block_argmax(float& v, int& idx, float* shv, int* shi) {
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o);
        const int oi = __shfl_xor(idx, o);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { shv[w] = v; shi[w] = idx; }
    __syncthreads();
    v = shv[0]; idx = shi[0];
    for (int i = 1; i < LT / 64; i++)
        if (shv[i] > v || (shv[i] == v && shi[i] < idx)) { v = shv[i]; idx = shi[i]; }
}

// Per-element exponentials over the whole row use the hardware exp2 (__expf, a few ulp): the GPU's
// logits already differ from the CPU's by ~1e-3, so libm-accurate exp buys no parity there, and its
// ~20-instruction expansion per element made the kernel VALU-bound. The timestamp sum (<= 1501
// elements) uses expf: "sum p(timestamps) > max p(text)" is a threshold decision on that sum alone
// (the log-sum-exp of the row cancels out of it).
// The row is loaded once into registers (NPT values per thread, all loads issued back to back) and
// every pass works on registers: a row re-read per pass from L2 with one load in flight per wave
// made the kernel latency-bound (128 us per step at 128 rows). Per-thread accumulation runs over
// i = tid, tid + LT, ... in ascending order, as before (same bits).
static constexpr int NPT = 51;  // 51 * 1024 >= 51866 (largest Whisper vocabulary)
static constexpr int NPT_LDS = 36;  // values k < NPT_LDS of each thread live in LDS (144 KiB), the rest in VGPRs

// element k of this thread's row slice (compile-time k after unrolling: LDS or a register)
struct RowSlice {
    float* lds;
    float reg[NPT - NPT_LDS];
    __device__ __forceinline__ float get(int k) const { return k < NPT_LDS ? lds[k * LT + threadIdx.x] : reg[k - NPT_LDS]; }
    __device__ __forceinline__ void set(int k, float v) {
        if (k < NPT_LDS) lds[k * LT + threadIdx.x] = v;
        else reg[k - NPT_LDS] = v;
    }
};

__global__ void __launch_bounds__(LT) logits_kernel(const float* __restrict__ logits, long ld, const SeqCtl* __restrict__ ctl,
                                                    VocabIds v, TokOut* __restrict__ out, float* __restrict__ probs) {
    const int s = blockIdx.x;
    const SeqCtl c = ctl[s];
    const float* L = logits + (long)s * ld;
    const int n = v.n_vocab, tid = threadIdx.x;
    __shared__ float shf[LT / 64];
    __shared__ int shi[LT / 64];
    __shared__ double shd[LT / 64];

    extern __shared__ float s_row[];  // [NPT_LDS][LT]
    RowSlice x{s_row};
    // the register part first, then the LDS part in batches of 12 loads in flight (a load -> LDS
    // store pair per element would wait out one memory latency per element)
#pragma unroll
    for (int k = NPT_LDS; k < NPT; k++) {
        const int i = tid + k * LT;
        x.set(k, i < n ? L[i] : -INFINITY);
    }
#pragma unroll
    for (int k0 = 0; k0 < NPT_LDS; k0 += 12) {
        float t[12];
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int i = tid + (k0 + k) * LT;
            t[k] = i < n ? L[i] : -INFINITY;
        }
#pragma unroll
        for (int k = 0; k < 12; k++) x.set(k0 + k, t[k]);
    }
    float nosp_prob = 0.0f;
    if (c.want_nosp) {  // no-speech probability from the raw (unfiltered) logits
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < NPT; k++)
            if (tid + k * LT < n) mx = fmaxf(mx, x.get(k));
        mx = block_max(mx, shf);
        float sm = 0.0f;
#pragma unroll
        for (int k = 0; k < NPT; k++)
            if (tid + k * LT < n) sm += __expf(x.get(k) - mx);
        sm = block_sum(sm, shf);
        const float lse = logf(sm) + mx;
        nosp_prob = expf(L[v.nosp] - lse);
    }
    // filtered logits, in place
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = tid + k * LT;
        if (i < n) x.set(k, masked_logit(x.get(k), i, c, v));
    }
    // log-softmax of the filtered logits
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NPT; k++) mx = fmaxf(mx, x.get(k));
    mx = block_max(mx, shf);
    float sm = 0.0f;
#pragma unroll
    for (int k = 0; k < NPT; k++)
        if (x.get(k) > -INFINITY) sm += __expf(x.get(k) - mx);
    sm = block_sum(sm, shf);
    const float lse = logf(sm) + mx;
    // timestamp rule
    float mts = -INFINITY, mtext = -INFINITY;
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = tid + k * LT;
        const float lp = x.get(k) > -INFINITY ? x.get(k) - lse : -INFINITY;
        if (i >= v.beg) mts = fmaxf(mts, lp); else mtext = fmaxf(mtext, lp);
    }
    mts = block_max(mts, shf);
    mtext = block_max(mtext, shf);
    float sts = 0.0f;
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = tid + k * LT;
        if (i < v.beg) continue;
        const float lp = x.get(k) > -INFINITY ? x.get(k) - lse : -INFINITY;
        if (lp > -INFINITY) sts += expf(lp - mts);  // libm-accurate: this sum decides the timestamp rule
    }
    sts = block_sum(sts, shf);
    const float ts_logprob = sts > 0.0f ? logf(sts) + mts : -INFINITY;
    const bool mask_text = ts_logprob > mtext;
    // probs, argmax (all) and argmax / sum over timestamps
    float best = 0.0f, best_ts = 0.0f;
    int ibest = 0x7fffffff, its = 0x7fffffff;
    double sum_ts = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = tid + k * LT;
        if (i >= n) continue;
        float xv = x.get(k);
        if (mask_text && i < v.beg) xv = -INFINITY;
        const float p = xv == -INFINITY ? 0.0f : __expf(xv - lse);
        if (c.want_probs) {  // [seq][2][V]: probs, logprobs (host sampling at t > 0)
            probs[(long)s * 2 * n + i] = p;
            probs[(long)s * 2 * n + n + i] = xv == -INFINITY ? -INFINITY : xv - lse;
        }
        if (p > best) { best = p; ibest = i; }
        if (i >= v.beg) {
            sum_ts += (double)p;
            if (p > best_ts) { best_ts = p; its = i; }
        }
    }
    block_argmax(best, ibest, shf, shi);
    block_argmax(best_ts, its, shf, shi);
    sum_ts = block_sum_d(sum_ts, shd);
    if (tid == 0) {
        TokOut r;
        r.id = best > 0.0f ? ibest : 0;
        r.p = best;
        {
            float xv = masked_logit(L[r.id], r.id, c, v);
            if (mask_text && r.id < v.beg) xv = -INFINITY;
            r.plog = xv > -INFINITY ? xv - lse : -INFINITY;
        }
        r.tid = best_ts > 0.0f ? its : 0;
        r.pt = (float)((double)best_ts / (sum_ts + 1e-10));
        r.ptsum = (float)sum_ts;
        if (r.id >= v.beg) { r.tid = r.id; r.pt = r.p; }
        r.nosp_prob = nosp_prob;
        r.pad = 0.0f;
        out[s] = r;
    }
}

// ---- split form for few rows (decode steps of <= 16 clips: one 1024-thread workgroup per row leaves
// the chip idle and took 38 us per step at one clip) -------------------------------------------------
// Pass 1: KS workgroups per row, each over a chunk of the vocabulary, write per-chunk statistics of
// the filtered logits x: the max m over all tokens, over the timestamp tokens (m_ts) and over the text
// tokens (m_text), the argmax of all and of the timestamp tokens (lowest index on ties), and the sums
// s = sum exp(x - m), s_ts = sum_ts exp(x - m_ts) (and for no_speech the raw logits' max and sum).
// Pass 2: one workgroup per row combines them in chunk order: lse = log(sum_c s_c e^(m_c - M)) + M,
// the timestamp rule log(S_ts) + M_ts > M_text with S_ts = sum_c s_ts_c e^(m_ts_c - M_ts) (the
// log-softmax shift cancels out of it), the argmax of p = e^(x - lse) as the argmax of x, and
// sum_ts p = S_ts e^(M_ts - lse). The same decisions as logits_kernel; sums associate differently (last
// bits of p, plog, pt), and a near-tie of p under rounding resolves by x instead of by index.
// want_probs rows (sampled attempts) have pass 2 write the probs / logprobs rows as well.
static constexpr int KS = 16, LT2 = 256;
struct LogitRec {
    float m_r, s_r, m, s, m_ts, s_ts, m_text;
    int ix_all, ix_ts, pad;
};

size_t logits_rec_bytes(int n_seq) { return (size_t)std::max(1, n_seq) * KS * sizeof(LogitRec); }

__device__ __forceinline__ void argmax_pair(float& v, int& ix, float ov, int oi) {
    if (ov > v || (ov == v && oi < ix)) { v = ov; ix = oi; }
}

template <int NW>
__device__ float blk_max(float x, float* sh) {
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    float r = sh[0];
    for (int i = 1; i < NW; i++) r = fmaxf(r, sh[i]);
    return r;
}
template <int NW>
__device__ float blk_sum(float x, float* sh) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    float r = 0.0f;
    for (int i = 0; i < NW; i++) r += sh[i];
    return r;
}
template <int NW>
__device__ void blk_argmax(float& v, int& ix, float* shv, int* shi) {
    for (int o = 32; o > 0; o >>= 1) argmax_pair(v, ix, __shfl_xor(v, o), __shfl_xor(ix, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { shv[threadIdx.x >> 6] = v; shi[threadIdx.x >> 6] = ix; }
    __syncthreads();
    v = shv[0]; ix = shi[0];
    for (int i = 1; i < NW; i++) argmax_pair(v, ix, shv[i], shi[i]);
}

__global__ void __launch_bounds__(LT2) logits_part_kernel(const float* __restrict__ logits, long ld,
                                                          const SeqCtl* __restrict__ ctl, VocabIds v,
                                                          LogitRec* __restrict__ rec) {
    constexpr int NW = LT2 / 64, PER = 14;  // 14 * 256 * 16 >= 51866
    const int c = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, n = v.n_vocab;
    const SeqCtl q = ctl[s];
    const float* L = logits + (long)s * ld;
    const int cs = (n + KS - 1) / KS, i0 = c * cs, i1 = min(n, i0 + cs);
    __shared__ float shf[NW];
    __shared__ int shi[NW];
    float raw[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = i0 + tid + k * LT2;
        raw[k] = i < i1 ? L[i] : -INFINITY;
    }
    LogitRec r;
    r.m_r = -INFINITY; r.s_r = 0.0f; r.pad = 0;
    if (q.want_nosp) {
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < PER; k++) mx = fmaxf(mx, raw[k]);
        mx = blk_max<NW>(mx, shf);
        float sm = 0.0f;
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (i0 + tid + k * LT2 < i1) sm += __expf(raw[k] - mx);
        r.m_r = mx;
        r.s_r = blk_sum<NW>(sm, shf);
    }
    float m = -INFINITY, mts = -INFINITY, mtx = -INFINITY;
    int ix = 0x7fffffff, its = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = i0 + tid + k * LT2;
        const float x = i < i1 ? masked_logit(raw[k], i, q, v) : -INFINITY;
        raw[k] = x;
        if (x > -INFINITY) {
            argmax_pair(m, ix, x, i);
            if (i >= v.beg) argmax_pair(mts, its, x, i);
            else mtx = fmaxf(mtx, x);
        }
    }
    blk_argmax<NW>(m, ix, shf, shi);
    blk_argmax<NW>(mts, its, shf, shi);
    mtx = blk_max<NW>(mtx, shf);
    float sm = 0.0f, sts = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = i0 + tid + k * LT2;
        if (raw[k] > -INFINITY) {
            sm += __expf(raw[k] - m);
            if (i >= v.beg) sts += expf(raw[k] - mts);
        }
    }
    r.m = m; r.m_ts = mts; r.m_text = mtx; r.ix_all = ix; r.ix_ts = its;
    r.s = blk_sum<NW>(sm, shf);
    r.s_ts = blk_sum<NW>(sts, shf);
    if (tid == 0) rec[(long)s * KS + c] = r;
}

__global__ void __launch_bounds__(LT2) logits_combine_kernel(const float* __restrict__ logits, long ld,
                                                             const SeqCtl* __restrict__ ctl, VocabIds v,
                                                             const LogitRec* __restrict__ rec, TokOut* __restrict__ out,
                                                             float* __restrict__ probs) {
    const int s = blockIdx.x, tid = threadIdx.x, n = v.n_vocab;
    const SeqCtl q = ctl[s];
    const float* L = logits + (long)s * ld;
    __shared__ float sh_lse;
    __shared__ int sh_mask;
    if (tid == 0) {
        const LogitRec* R = rec + (long)s * KS;
        float M = -INFINITY, Mts = -INFINITY, Mtx = -INFINITY, Mr = -INFINITY;
        int ix = 0x7fffffff, its = 0x7fffffff;
        for (int c = 0; c < KS; c++) {
            argmax_pair(M, ix, R[c].m, R[c].ix_all);
            argmax_pair(Mts, its, R[c].m_ts, R[c].ix_ts);
            Mtx = fmaxf(Mtx, R[c].m_text);
            Mr = fmaxf(Mr, R[c].m_r);
        }
        float S = 0.0f, Sts = 0.0f, Sr = 0.0f;
        for (int c = 0; c < KS; c++) {
            if (R[c].m > -INFINITY) S += R[c].s * expf(R[c].m - M);
            if (R[c].m_ts > -INFINITY) Sts += R[c].s_ts * expf(R[c].m_ts - Mts);
            if (q.want_nosp && R[c].m_r > -INFINITY) Sr += R[c].s_r * expf(R[c].m_r - Mr);
        }
        const float lse = logf(S) + M;
        const float mts = Mts - lse, mtext = Mtx - lse;
        const float ts_logprob = Sts > 0.0f ? logf(Sts) + mts : -INFINITY;
        const bool mask_text = ts_logprob > mtext;
        TokOut r;
        const float xb = mask_text ? Mts : M;
        const int ib = mask_text ? its : ix;
        const float best = xb > -INFINITY ? __expf(xb - lse) : 0.0f;
        r.id = best > 0.0f ? ib : 0;
        r.p = best;
        {
            float xv = masked_logit(L[r.id], r.id, q, v);
            if (mask_text && r.id < v.beg) xv = -INFINITY;
            r.plog = xv > -INFINITY ? xv - lse : -INFINITY;
        }
        const float best_ts = Mts > -INFINITY ? __expf(Mts - lse) : 0.0f;
        const double sum_ts = Mts > -INFINITY ? (double)Sts * (double)expf(Mts - lse) : 0.0;
        r.tid = best_ts > 0.0f ? its : 0;
        r.pt = (float)((double)best_ts / (sum_ts + 1e-10));
        r.ptsum = (float)sum_ts;
        if (r.id >= v.beg) { r.tid = r.id; r.pt = r.p; }
        r.nosp_prob = q.want_nosp ? expf(L[v.nosp] - (logf(Sr) + Mr)) : 0.0f;
        r.pad = 0.0f;
        out[s] = r;
        sh_lse = lse;
        sh_mask = mask_text;
    }
    if (!q.want_probs) return;
    __syncthreads();
    const float lse = sh_lse;
    const bool mask_text = sh_mask;
    for (int i = tid; i < n; i += LT2) {
        float xv = masked_logit(L[i], i, q, v);
        if (mask_text && i < v.beg) xv = -INFINITY;
        probs[(long)s * 2 * n + i] = xv == -INFINITY ? 0.0f : __expf(xv - lse);
        probs[(long)s * 2 * n + n + i] = xv == -INFINITY ? -INFINITY : xv - lse;
    }
}

// rows up to this count take the split form (16 chunk workgroups per row + a combine)
static const int kLogitsSplitMax = 16;

void launch_logits(const float* logits, long ld, const SeqCtl* ctl, int n_seq, const VocabIds& v, TokOut* out, float* probs,
                   void* rec, hipStream_t st) {
    if (n_seq <= 0) return;
    if (v.n_vocab > NPT * LT) WM_FAIL("vocabulary %d > %d", v.n_vocab, NPT * LT);
    if (rec && n_seq <= kLogitsSplitMax && v.n_vocab <= 14 * LT2 * KS) {
        logits_part_kernel<<<dim3(KS, n_seq), LT2, 0, st>>>(logits, ld, ctl, v, (LogitRec*)rec);
        logits_combine_kernel<<<n_seq, LT2, 0, st>>>(logits, ld, ctl, v, (const LogitRec*)rec, out, probs);
        return;
    }
    logits_kernel<<<n_seq, LT, (size_t)NPT_LDS * LT * sizeof(float), st>>>(logits, ld, ctl, v, out, probs);
}

// ---- device-side step advance (pipelined greedy decoding, engine.cpp decode_pipelined) -----------------------
// After a decode step's logits kernel, in stream order: row r's chosen token becomes its next input and its
// position advances (the layout of decoder_upload: tok | pos | slot | nkv_self | nkv_cross, ct entries each),
// its SeqCtl advances exactly as fill_ctl would rebuild it from the job after process_step appended the
// token (is_initial, last_ts = id >= beg, penult_ts = the previous last_ts or true after the first token;
// has_ts / seek_delta from a timestamp above beg), and the step's TokOut (and the persistent launch's error
// word) is copied to the ring slot the host reads while the next step runs.
__global__ void decode_advance_kernel(int n, int ct, int beg, const TokOut* __restrict__ tout, int* __restrict__ ints,
                                      SeqCtl* __restrict__ ctl, TokOut* __restrict__ ring, const unsigned* __restrict__ err,
                                      unsigned* __restrict__ ring_err) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r == 0) *ring_err = err ? *err : 0u;
    if (r >= n) return;
    const TokOut o = tout[r];
    ring[r] = o;
    const int id = o.id;
    ints[r] = id;                       // tok
    const int pos = ints[ct + r] + 1;   // pos
    ints[ct + r] = pos;
    ints[3 * ct + r] = pos + 1;         // nkv_self
    SeqCtl c = ctl[r];
    c.penult_ts = c.is_initial ? 1 : c.last_ts;
    c.last_ts = id >= beg;
    c.is_initial = 0;
    if (id > beg) {
        c.has_ts = 1;
        c.seek_delta = 2 * (id - beg);
    }
    c.want_nosp = 0;
    ctl[r] = c;
}

void launch_decode_advance(int n, int ct, int beg, const TokOut* tout, int* ints, SeqCtl* ctl, TokOut* ring,
                           const unsigned* err, unsigned* ring_err, hipStream_t st) {
    decode_advance_kernel<<<(std::max(n, 1) + 127) / 128, 128, 0, st>>>(n, ct, beg, tout, ints, ctl, ring, err, ring_err);
    WM_CHECK(hipGetLastError());
}

}  // namespace wm
