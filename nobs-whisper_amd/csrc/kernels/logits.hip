// Device-side whisper_process_logits + whisper_sample_token(best=true).
//
// One 1024-thread workgroup per sequence reads its logits row (V = 51864..51866 f32) four times
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

__device__ __forceinline__ float masked_logit(const float* L, int i, const SeqCtl& c, const VocabIds& v) {
    float x = L[i];
    if (c.temperature > 0.0f) x = x / c.temperature;
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

__global__ void __launch_bounds__(LT) logits_kernel(const float* __restrict__ logits, long ld, const SeqCtl* __restrict__ ctl,
                                                    VocabIds v, TokOut* __restrict__ out, float* __restrict__ probs) {
    const int s = blockIdx.x;
    const SeqCtl c = ctl[s];
    const float* L = logits + (long)s * ld;
    const int n = v.n_vocab, tid = threadIdx.x;
    __shared__ float shf[LT / 64];
    __shared__ int shi[LT / 64];
    __shared__ double shd[LT / 64];

    float nosp_prob = 0.0f;
    if (c.want_nosp) {  // no-speech probability from the raw (unfiltered) logits
        float mx = -INFINITY;
        for (int i = tid; i < n; i += LT) mx = fmaxf(mx, L[i]);
        mx = block_max(mx, shf);
        float sm = 0.0f;
        for (int i = tid; i < n; i += LT) sm += expf(L[i] - mx);
        sm = block_sum(sm, shf);
        const float lse = logf(sm) + mx;
        nosp_prob = expf(L[v.nosp] - lse);
    }
    // log-softmax of the filtered logits
    float mx = -INFINITY;
    for (int i = tid; i < n; i += LT) mx = fmaxf(mx, masked_logit(L, i, c, v));
    mx = block_max(mx, shf);
    float sm = 0.0f;
    for (int i = tid; i < n; i += LT) {
        const float x = masked_logit(L, i, c, v);
        if (x > -INFINITY) sm += expf(x - mx);
    }
    sm = block_sum(sm, shf);
    const float lse = logf(sm) + mx;
    // timestamp rule
    float mts = -INFINITY, mtext = -INFINITY;
    for (int i = tid; i < n; i += LT) {
        const float x = masked_logit(L, i, c, v);
        const float lp = x > -INFINITY ? x - lse : -INFINITY;
        if (i >= v.beg) mts = fmaxf(mts, lp); else mtext = fmaxf(mtext, lp);
    }
    mts = block_max(mts, shf);
    mtext = block_max(mtext, shf);
    float sts = 0.0f;
    for (int i = v.beg + tid; i < n; i += LT) {
        const float x = masked_logit(L, i, c, v);
        const float lp = x > -INFINITY ? x - lse : -INFINITY;
        if (lp > -INFINITY) sts += expf(lp - mts);
    }
    sts = block_sum(sts, shf);
    const float ts_logprob = sts > 0.0f ? logf(sts) + mts : -INFINITY;
    const bool mask_text = ts_logprob > mtext;
    // probs, argmax (all) and argmax / sum over timestamps
    float best = 0.0f, best_ts = 0.0f;
    int ibest = 0x7fffffff, its = 0x7fffffff;
    double sum_ts = 0.0;
    for (int i = tid; i < n; i += LT) {
        float x = masked_logit(L, i, c, v);
        if (mask_text && i < v.beg) x = -INFINITY;
        const float p = x == -INFINITY ? 0.0f : expf(x - lse);
        if (c.want_probs) {  // [seq][2][V]: probs, logprobs (host sampling at t > 0)
            probs[(long)s * 2 * n + i] = p;
            probs[(long)s * 2 * n + n + i] = x == -INFINITY ? -INFINITY : x - lse;
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
            float x = masked_logit(L, r.id, c, v);
            if (mask_text && r.id < v.beg) x = -INFINITY;
            r.plog = x > -INFINITY ? x - lse : -INFINITY;
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

void launch_logits(const float* logits, long ld, const SeqCtl* ctl, int n_seq, const VocabIds& v, TokOut* out, float* probs,
                   hipStream_t st) {
    if (n_seq <= 0) return;
    logits_kernel<<<n_seq, LT, 0, st>>>(logits, ld, ctl, v, out, probs);
}

}  // namespace wm
