// The MI355X Whisper engine: workspace, encoder/decoder forward on one HIP stream, and the
// batched window scheduler that reproduces whisper_full_with_state for every clip of a batch
// (reference call site whisper.rs:127-129).
//
// Control flow is whisper.cpp's [ext], restated in oracle/oracle_whisper.cpp `full()` and kept
// per clip here (prompt/temperature/seek/segments live on the host, one small struct per clip);
// the arithmetic is batched across clips: one encoder pass per group of windows, one cross-KV
// GEMM, a ragged prefill, then lockstep decode steps over every clip still decoding. Per step the
// host receives only a 32-byte TokOut per clip (plus the probs row of clips that sample at t>0).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <exception>
#include <thread>

#include "engine.h"

namespace wm {

static size_t esize(DType) { return 2; }

// device buffers: freed and nulled together, so that a workspace whose (re)allocation failed half way
// can be released as a whole (ensure_ws) and the state reused
static void dfree(void*& p) {
    if (p) { void* q = p; p = nullptr; WM_CHECK(hipFree(q)); }
}
template <typename T> static void dfree(T*& p) {
    void* q = (void*)p;
    p = nullptr;
    dfree(q);
}
template <typename T> static void dalloc(T*& p, size_t bytes) {
    void* q = nullptr;
    p = nullptr;
    WM_CHECK(hipMalloc(&q, bytes));
    p = (T*)q;
}

// ---- live kernel timing (HIP events on the state's stream) ------------------------------------------
static hipEvent_t kt_event(whisper_state* s) {
    if (!s->kpool.empty()) { hipEvent_t e = s->kpool.back(); s->kpool.pop_back(); return e; }
    hipEvent_t e;
    WM_CHECK(hipEventCreate(&e));
    return e;
}
// Record a timing event on the state's stream. While a decode step is being captured, the record
// is added as an explicit event-record node of the graph: a stream-captured hipEventRecord does
// not yield a timestamp on replay (hipEventElapsedTime -> invalid handle), an explicit node does
// (tools/probe/graph_events.hip).
static void kt_record(whisper_state* s, hipEvent_t e, hipStream_t st) {
    if (!s->capture_ev) { WM_CHECK(hipEventRecord(e, st)); return; }
    hipStreamCaptureStatus cs;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    WM_CHECK(hipStreamGetCaptureInfo_v2(st, &cs, &id, &g, &deps, &nd));
    hipGraphNode_t node;
    WM_CHECK(hipGraphAddEventRecordNode(&node, g, deps, nd, e));
    WM_CHECK(hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies));
}
// Times the launches of its scope on stream `st` (default: the state's stream) when the class is
// enabled. For K_ATTN_SELF `work` is the share of the step's rows (the bytes grow every step and
// are filled in when the events are read).
struct KT {
    whisper_state* s;
    int cls;
    double work;
    hipStream_t st;
    hipEvent_t a = nullptr;
    KT(whisper_state* s_, int c, double w, hipStream_t st_ = nullptr, bool on = true)
        : s(s_), cls(c), work(w), st(st_ ? st_ : s_->stream) {
        if (on && ((s->ktime_mask >> c) & 1)) { a = kt_event(s); kt_record(s, a, st); }
    }
    ~KT() {
        if (!a) return;
        hipEvent_t b = kt_event(s);
        kt_record(s, b, st);
        (s->capture_ev ? *s->capture_ev : s->kpending).push_back({cls, a, b, work});
    }
};
static void drop_graphs(whisper_state* s) {
    for (auto& g : s->dec_graphs) {
        hipGraphExecDestroy(g.exec);
        for (auto& e : g.ev) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
    }
    s->dec_graphs.clear();
}
// accumulate the timing events of one graph replay (stream already synchronised)
static void kt_flush_graph(whisper_state* s, const whisper_state::DecGraph& g) {
    for (auto& p : g.ev) {
        if (!((s->ktime_mask >> p.cls) & 1)) continue;
        float ms = 0.0f;
        const hipError_t e = hipEventElapsedTime(&ms, p.a, p.b);
        if (e != hipSuccess) {
            static bool warned = false;
            if (!warned) fprintf(stderr, "whisper_mi355x: graph kernel timing unavailable (%s)\n", hipGetErrorString(e));
            warned = true;
            continue;
        }
        s->kstat[p.cls].ms += ms;
        s->kstat[p.cls].work += p.cls == K_ATTN_SELF ? s->cur_self_work * p.work : p.work;
        s->kstat[p.cls].count++;
    }
}
void kt_flush(whisper_state* s) {
    if (s->kpending.empty()) return;
    WM_CHECK(hipStreamSynchronize(s->stream));
    for (auto& p : s->kpending) {
        float ms = 0.0f;
        WM_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
        s->kstat[p.cls].ms += ms;
        s->kstat[p.cls].work += p.cls == K_ATTN_SELF ? s->cur_self_work * p.work : p.work;
        s->kstat[p.cls].count++;
        s->kpool.push_back(p.a);
        s->kpool.push_back(p.b);
    }
    s->kpending.clear();
}
// GEMM launch with its algorithmic work: FLOPs for encoder-side GEMMs (MFMA-bound), HBM bytes
// (weights + activations) for decode-side GEMMs (weight-streaming)
// Decode-step split-K slabs are stored write-through (sc1): the lines leave the XCD's L2 while the
// GEMM runs instead of being written back at the kernel boundary before the reduce can start
// (MI355X_MICROARCH.md price list, "boundary": + dirty bytes / 6 TB/s). Same-box A/B, large-v3 bf16:
// decode 864 -> 824 ms per step at 128 clips, 423 -> 413 at 16 (profiles/r03_envab_slab_gelu.txt).
static void tgemm_ws(whisper_state* s, int cls, DType dt, int epi, const GemmArgs& g0, hipStream_t st, float* ws,
                     long ws_elems) {
    GemmArgs g = g0;
    if (cls == K_GEMM_DEC) { g.splitk_ws = ws; g.splitk_ws_elems = ws_elems; g.slab_wt = 1; }
    const double work = cls == K_GEMM_ENC ? 2.0 * g.M * g.N * g.K
                                          : 2.0 * g.N * g.K + 2.0 * g.M * g.K + 4.0 * g.M * g.N;
    KT kt(s, cls, work, st);
    launch_gemm(dt, epi, g, st);
}
static void tgemm(whisper_state* s, int cls, DType dt, int epi, const GemmArgs& g0, hipStream_t st) {
    tgemm_ws(s, cls, dt, epi, g0, st, s->ws.splitk, s->ws.splitk_elems);
}

static whisper_state* create_state(Context* c) {
    WM_CHECK(hipSetDevice(c->device));
    whisper_state* s = new whisper_state();
    s->ctx = c;
    s->device = c->device;
    try {
        WM_CHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        WM_CHECK(hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking));
        WM_CHECK(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
        WM_CHECK(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
    } catch (...) {
        if (s->ev_join) hipEventDestroy(s->ev_join);
        if (s->ev_fork) hipEventDestroy(s->ev_fork);
        if (s->stream2) hipStreamDestroy(s->stream2);
        if (s->stream) hipStreamDestroy(s->stream);
        delete s;
        throw;
    }
    std::lock_guard<std::mutex> lk(c->pool_mu);
    c->live.push_back(s);
    return s;
}

// A recycled state is a fresh whisper_state to its new owner: everything whisper_init_state would
// start from (prompt_past, the rng, results, mel, timing) is reset; only the device workspace and the
// decode graphs captured over it (keyed by active-clip count) are kept.
static void reset_for_reuse(whisper_state* s) {
    s->direct = false;
    s->results.clear();
    s->lang_ids.clear();
    s->decisions.clear();
    s->prompt_past.clear();
    s->rng = std::mt19937(0);
    s->lang_id = 0;
    s->n_len = s->n_len_org = 0;
    s->logits_host.clear();
    for (double& t : s->phase_ms) t = 0;
    s->decoded_tokens = 0;
    s->last_enc_windows = 0;
    s->mel_ready = false;
    s->ktime_mask = 0;
    for (auto& k : s->kstat) k = KStat();
    s->cur_self_work = 0;
    s->pdec_give_ups = 0;
    s->pdec_lost_ms = 0;
    s->pdec_off_until = 0;
    s->pdec_off = false;
    std::fill(s->ws.cross_fresh.begin(), s->ws.cross_fresh.end(), 0);
}

// states kept per context, and the largest workspace kept (clips): the app's pattern is one clip per
// call (whisper.rs:83-85, state.rs:147); a batch-sized workspace is released, not kept
static int pool_states() {
    const char* e = getenv("WHISPER_MI355X_STATE_POOL");
    return e ? std::max(0, atoi(e)) : 2;
}
static const int kPoolMaxJobs = 16;

whisper_state* new_state(Context* c) {
    {
        std::lock_guard<std::mutex> lk(c->pool_mu);
        if (!c->pool.empty()) {
            whisper_state* s = c->pool.back();
            c->pool.pop_back();
            reset_for_reuse(s);
            s->pooled = true;
            return s;
        }
    }
    return create_state(c);
}

static void free_ws(Workspace& w);

static void destroy_state(whisper_state* s) {
    if (s->twin) {
        destroy_state(s->twin);
        s->twin = nullptr;
    }
    if (Context* c = s->ctx) {
        std::lock_guard<std::mutex> lk(c->pool_mu);
        c->live.erase(std::remove(c->live.begin(), c->live.end(), s), c->live.end());
    }
    hipSetDevice(s->device);
    hipStreamSynchronize(s->stream);
    hipStreamSynchronize(s->stream2);
    drop_graphs(s);
    try { free_ws(s->ws); } catch (const Error&) {}
    for (auto& p : s->kpending) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
    for (hipEvent_t e : s->kpool) hipEventDestroy(e);
    hipEventDestroy(s->ev_fork);
    hipEventDestroy(s->ev_join);
    hipStreamDestroy(s->stream2);
    hipStreamDestroy(s->stream);
    delete s;
}

void free_state(whisper_state* s) {
    if (!s) return;
    Context* c = s->ctx;
    if (!c) {  // its context is gone: nothing to pool into
        destroy_state(s);
        return;
    }
    hipSetDevice(c->device);
    const bool healthy = hipStreamSynchronize(s->stream) == hipSuccess && hipStreamSynchronize(s->stream2) == hipSuccess &&
                         s->kpending.empty();
    if (healthy && s->ws.cap_jobs <= kPoolMaxJobs) {
        std::lock_guard<std::mutex> lk(c->pool_mu);
        if ((int)c->pool.size() < pool_states()) {
            c->pool.push_back(s);
            return;
        }
    }
    destroy_state(s);
}

void drain_state_pool(Context* c) {
    std::vector<whisper_state*> p;
    {
        std::lock_guard<std::mutex> lk(c->pool_mu);
        p.swap(c->pool);
    }
    for (whisper_state* s : p) destroy_state(s);
}

void orphan_states(Context* c) {
    std::lock_guard<std::mutex> lk(c->pool_mu);
    for (whisper_state* s : c->live) s->ctx = nullptr;
    c->live.clear();
}

void recover_state(whisper_state* s) {
    if (!s) return;
    hipSetDevice(s->device);
    for (hipStream_t st : {s->stream, s->stream2}) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
            hipGraph_t g = nullptr;
            hipStreamEndCapture(st, &g);
            if (g) hipGraphDestroy(g);
        }
    }
    s->capture_ev = nullptr;
    hipStreamSynchronize(s->stream);
    hipStreamSynchronize(s->stream2);
    (void)hipGetLastError();
    for (auto& p : s->kpending) { s->kpool.push_back(p.a); s->kpool.push_back(p.b); }
    s->kpending.clear();
}

static void free_ws(Workspace& w) {
    // sub-allocations (pos/slot/.. of tok, win_seek/win_slot of win_job, pcm_ptrs/n_* of mel_ptrs)
    // are freed with their parent
    dfree(w.mel_img); dfree(w.h1); dfree(w.hn); dfree(w.qkv); dfree(w.att); dfree(w.ff); dfree(w.x);
    dfree(w.cross); dfree(w.self); dfree(w.dx); dfree(w.dh); dfree(w.dq); dfree(w.datt); dfree(w.dff);
    dfree(w.lrow); dfree(w.logits); dfree(w.probs); dfree(w.tok); dfree(w.ctl); dfree(w.tout); dfree(w.lrec); dfree(w.win_job);
    dfree(w.pcm); dfree(w.mel); dfree(w.mel_ptrs); dfree(w.splitk); dfree(w.enc); dfree(w.qx); dfree(w.xo);
    dfree(w.xml); dfree(w.kvslot); dfree(w.hs); dfree(w.qtiles); dfree(w.wdq); dfree(w.pd_sync);
    if (w.h_pd_err) hipHostFree(w.h_pd_err);
    if (w.h_ring) hipHostFree(w.h_ring);
    for (auto& e : w.ring_ev)
        if (e) hipEventDestroy(e);
    if (w.h_ints) hipHostFree(w.h_ints);
    if (w.h_qtiles) hipHostFree(w.h_qtiles);
    if (w.h_tout) hipHostFree(w.h_tout);
    if (w.h_ctl) hipHostFree(w.h_ctl);
    w = Workspace();
}

// prefills with at most this many tokens per clip take the direct cross attention; longer prompts
// go through a cross K/V cache computed for their clips on demand
static const int kXDirectMaxTok = 8;
// lazy-rescale threshold of the direct cross attention's online softmax (log2 units: P <= 2^8)
static const float kXattnThr = 8.0f;

// Cross attention form per call. The direct form reads E once per clip and layer (half the bytes of
// the cached K + V) but its split partials are [H][d] per (clip, split) whatever the batch, and it
// adds two launches per layer (Q' projection, combine); at a few clips a step is launch- and
// latency-bound and the cached form (one attention kernel, whisper.cpp's own numerics) wins: the
// cross K/V of a window then costs one GEMM at encode time. WHISPER_MI355X_CROSS=direct|cache
// forces a form; otherwise direct above 32 clips.
static bool pick_direct(Context* c, int n_jobs) {
    if (!c->cross_direct) return false;
    // read per call (tests switch the form per case)
    const char* e = getenv("WHISPER_MI355X_CROSS");
    if (e && strcmp(e, "direct") == 0) return true;
    if (e && strcmp(e, "cache") == 0) return false;
    return n_jobs > 32;
}

// encoder windows per launch group. Round 6: 128 (a whole headline batch per launch): the encoder GEMMs'
// 256 x 256 tiles then fill their last round of 256 CUs (32 windows: QKV 2820 tiles = 11.02 rounds, i.e. a 12th
// round of 4 tiles; 128 windows: 11250 = 43.9), and the encoder attention's grid is 30 whole rounds: encode
// 313.6 -> 304.1 ms per step, 3384 -> 3402 audio-s/s (profiles/r06_encb_ab_*.json; round 2 had measured 32 / 64 /
// 128 the same). ~6.5 GB of encoder activations for large-v3. WHISPER_MI355X_ENC_BATCH overrides it.
static int enc_batch() {
    static const int v = getenv("WHISPER_MI355X_ENC_BATCH") ? std::max(1, atoi(getenv("WHISPER_MI355X_ENC_BATCH"))) : 128;
    return v;
}

// Cross K/V cache for at least `slots` slots (cache form: the call's clips; direct form: the clips
// whose prompts are too long for the direct prefill). Sized by the calls that use it, so a state
// that ran a large direct-form batch does not allocate a cache for all of its slots later.
// A reallocation drops the state's decode graphs first: a captured cache-form step holds the old
// w.cross pointer, and the cross cache is sized apart from cap_jobs (a direct-form call of > 32 clips
// followed by cache-form calls of 8 and then 16 clips regrows it under graphs captured at 8).
static void ensure_cross(Context* c, whisper_state* s, int slots) {
    Workspace& w = s->ws;
    if (w.cross && w.cap_cross >= slots) return;
    const Hparams& hp = c->hp;
    WM_CHECK(hipStreamSynchronize(s->stream));
    WM_CHECK(hipStreamSynchronize(s->stream2));
    drop_graphs(s);
    dfree(w.cross);
    w.cap_cross = 0;
    std::fill(w.cross_fresh.begin(), w.cross_fresh.end(), 0);
    dalloc(w.cross, (size_t)slots * hp.n_text_layer * 2 * hp.n_audio_ctx * hp.n_audio_state * esize(c->dt));
    w.cap_cross = slots;
}

// (Re)allocate the workspace for n_jobs clips. Encoder activations are sized for at most
// enc_batch() windows at once; caches for n_jobs slots. If an allocation fails (out of memory),
// the whole workspace is released and the error propagates: the state stays usable (empty).
static void ensure_ws_impl(Context* c, whisper_state* s, int n_jobs) {
    Workspace& w = s->ws;
    const Hparams& hp = c->hp;
    const size_t d = hp.n_audio_state, nm = hp.n_mels, T = hp.n_audio_ctx, E = esize(c->dt);
    const int n_enc = std::min(n_jobs, enc_batch());
    if (n_enc > w.cap_enc || n_jobs > w.cap_jobs) drop_graphs(s);
    if (n_enc > w.cap_enc) {
        dfree(w.mel_img); dfree(w.h1); dfree(w.hn); dfree(w.qkv); dfree(w.att); dfree(w.ff); dfree(w.x);
        dfree(w.win_job); dfree(w.hs);
        w.cap_enc = 0;
        dalloc(w.mel_img, (size_t)n_enc * 3002 * nm * E);
        dalloc(w.h1, (size_t)n_enc * 3002 * d * E);
        WM_CHECK(hipMemset(w.h1, 0, (size_t)n_enc * 3002 * d * E));  // conv padding rows stay zero
        dalloc(w.hn, (size_t)n_enc * T * d * E);
        dalloc(w.qkv, (size_t)n_enc * T * 3 * d * E);
        dalloc(w.att, (size_t)n_enc * T * d * E);
        dalloc(w.ff, (size_t)n_enc * T * 4 * d * E);
        dalloc(w.x, (size_t)n_enc * T * d * 4);
        if (c->fp8_enc) {
            dalloc(w.hs, (size_t)n_enc * T * sizeof(float));
        }
        dalloc(w.win_job, (size_t)n_enc * 3 * sizeof(int));
        w.win_seek = w.win_job + n_enc;
        w.win_slot = w.win_job + 2 * n_enc;
        w.cap_enc = n_enc;
    }
    if (n_jobs > w.cap_jobs) {
        const int L = hp.n_text_layer;
        const int n_tok = n_jobs * (hp.n_text_ctx / 2 + 8);
        dfree(w.cross); dfree(w.self); dfree(w.dx); dfree(w.dh); dfree(w.dq); dfree(w.datt); dfree(w.dff);
        dfree(w.lrow); dfree(w.logits); dfree(w.probs); dfree(w.tok); dfree(w.ctl); dfree(w.tout); dfree(w.lrec); dfree(w.mel_ptrs);
        dfree(w.splitk); dfree(w.enc); dfree(w.qx); dfree(w.xo); dfree(w.xml); dfree(w.kvslot); dfree(w.qtiles);
        if (w.h_ring) { WM_CHECK(hipHostFree(w.h_ring)); w.h_ring = nullptr; w.ring = nullptr; }
        for (void** h : {(void**)&w.h_qtiles, (void**)&w.h_ints, (void**)&w.h_tout, (void**)&w.h_ctl})
            if (*h) { void* q = *h; *h = nullptr; WM_CHECK(hipHostFree(q)); }
        w.cap_jobs = w.cap_tok = w.cap_cross = w.cap_xq = 0;
        // split-K slabs: decode steps (<= 128 rows per group, two concurrent groups) and the prefill
        // GEMMs below the big-GEMM size (M*N < 2^22), whose split count depends on N and K only
        // (kernels/gemm.hip dec_splits_for: splits * N <= 16384, <= 12 splits)
        w.splitk_elems = std::max(16L * std::min(n_tok, 256) * 4 * (long)d, std::min(16384L * n_tok, 12L << 22));
        dalloc(w.splitk, w.splitk_elems * 4);
        w.cross_fresh.assign(n_jobs, 0);
        {
            std::vector<int> ident(n_jobs);
            for (int k = 0; k < n_jobs; k++) ident[k] = k;
            dalloc(w.kvslot, (size_t)n_jobs * sizeof(int));
            WM_CHECK(hipMemcpy(w.kvslot, ident.data(), (size_t)n_jobs * sizeof(int), hipMemcpyHostToDevice));
        }
        dalloc(w.self, (size_t)n_jobs * L * 2 * hp.n_text_ctx * d * E);
        dalloc(w.dx, (size_t)n_tok * d * 4);
        dalloc(w.dh, (size_t)n_tok * d * E);
        dalloc(w.dq, (size_t)n_tok * d * E);
        dalloc(w.datt, (size_t)n_tok * d * E);
        dalloc(w.dff, (size_t)n_tok * 4 * d * E);
        dalloc(w.lrow, (size_t)n_jobs * d * E);
        dalloc(w.logits, (size_t)n_jobs * hp.n_vocab * 4);
        dalloc(w.probs, (size_t)n_jobs * 2 * hp.n_vocab * 4);
        dalloc(w.tok, ((size_t)5 * n_tok + n_jobs) * sizeof(int));
        w.pos = w.tok + n_tok;
        w.slot = w.tok + 2 * n_tok;
        w.nkv_self = w.tok + 3 * n_tok;
        w.nkv_cross = w.tok + 4 * n_tok;
        w.lrows = w.tok + 5 * n_tok;
        dalloc(w.ctl, (size_t)n_jobs * sizeof(SeqCtl));
        dalloc(w.tout, (size_t)n_jobs * sizeof(TokOut));
        dalloc(w.lrec, logits_rec_bytes(n_jobs));
        dalloc(w.mel_ptrs, (size_t)n_jobs * (2 * sizeof(void*) + 3 * sizeof(int)));
        w.pcm_ptrs = (const float**)(w.mel_ptrs + n_jobs);
        w.n_samp = (int*)(w.pcm_ptrs + n_jobs);
        w.n_len = w.n_samp + n_jobs;
        w.mel_max = w.n_len + n_jobs;
        WM_CHECK(hipHostMalloc((void**)&w.h_ints, ((size_t)5 * n_tok + n_jobs) * sizeof(int) + 64, 0));
        dalloc(w.qtiles, (size_t)n_tok * sizeof(int2));
        WM_CHECK(hipHostMalloc((void**)&w.h_qtiles, (size_t)n_tok * sizeof(int2), 0));
        WM_CHECK(hipHostMalloc((void**)&w.h_tout, (size_t)n_jobs * sizeof(TokOut), 0));
        WM_CHECK(hipHostMalloc((void**)&w.h_ctl, (size_t)n_jobs * sizeof(SeqCtl), 0));
        w.cap_jobs = n_jobs;
        w.cap_tok = n_tok;
    }
    // the buffers of this call's cross attention form (allocated on first use, kept)
    if (s->direct && !w.enc) {
        // no cross K/V cache up front: decode steps (and short prefills) read E directly
        const int H = hp.n_text_head;
        w.cap_xq = std::max(kXDirectMaxTok * w.cap_jobs, 128);
        // n * xattn_splits(n) <= max(n, 255 + n) per row group; two concurrent groups at most double it
        const size_t xo_rows = (size_t)std::max(w.cap_xq, 512) + w.cap_jobs + 512;
        dalloc(w.enc, (size_t)w.cap_jobs * T * d * E);
        dalloc(w.qx, (size_t)w.cap_xq * 2 * H * d * E);
        dalloc(w.xo, xo_rows * H * d * 4);
        dalloc(w.xml, xo_rows * H * 2 * 4);
    }
    if (!s->direct) ensure_cross(c, s, n_jobs);
    if (c->quant && !w.wdq) dalloc(w.wdq, (size_t)16 * d * d * E);
}

static void ensure_ws(Context* c, whisper_state* s, int n_jobs) {
    try {
        ensure_ws_impl(c, s, n_jobs);
    } catch (const Error&) {
        hipStreamSynchronize(s->stream);
        hipStreamSynchronize(s->stream2);
        drop_graphs(s);
        free_ws(s->ws);
        throw;
    }
}

// ---- mel ------------------------------------------------------------------------------------------
static inline int mel_n_len(int n) { return (n + 16000 * 30) / 160; }
static inline int mel_n_len_org(int n) { return 1 + (int)(((int64_t)n + 200 - 400) / 160); }

int compute_mel(Context* c, whisper_state* s, const float* const* pcm, const int* n, int n_jobs, bool on_device) {
    s->direct = pick_direct(c, n_jobs);
    ensure_ws(c, s, n_jobs);
    Workspace& w = s->ws;
    const int nm = c->hp.n_mels;
    size_t pcm_tot = 0, mel_tot = 0;
    int max_frames = 1;
    for (int j = 0; j < n_jobs; j++) {
        pcm_tot += ((size_t)n[j] + 63) & ~(size_t)63;
        mel_tot += (size_t)nm * mel_n_len(n[j]);
        max_frames = std::max(max_frames, std::min((n[j] + 200) / 160 + 1, mel_n_len(n[j])));
    }
    if (!on_device && pcm_tot > w.cap_pcm) {
        dfree(w.pcm);
        w.cap_pcm = 0;
        dalloc(w.pcm, pcm_tot * 4);
        w.cap_pcm = pcm_tot;
    }
    if (mel_tot > w.cap_mel) {
        dfree(w.mel);
        w.cap_mel = 0;
        dalloc(w.mel, mel_tot * 4);
        w.cap_mel = mel_tot;
    }
    std::vector<const float*> pp(n_jobs);
    std::vector<float*> mp(n_jobs);
    std::vector<int> ints(3 * n_jobs);
    size_t po = 0, mo = 0;
    for (int j = 0; j < n_jobs; j++) {
        if (on_device) pp[j] = pcm[j];
        else {
            pp[j] = w.pcm + po;
            if (n[j] > 0) WM_CHECK(hipMemcpyAsync(w.pcm + po, pcm[j], (size_t)n[j] * 4, hipMemcpyHostToDevice, s->stream));
            po += ((size_t)n[j] + 63) & ~(size_t)63;
        }
        mp[j] = w.mel + mo;
        mo += (size_t)nm * mel_n_len(n[j]);
        ints[j] = n[j];
        ints[n_jobs + j] = mel_n_len(n[j]);
    }
    // one host block -> device, laid out as the workspace carves it (ensure_ws: arrays of cap_jobs
    // entries, whatever this call's clip count): [mel ptrs][pcm ptrs][n][n_len] ([max] is the kernel's)
    const size_t cap = w.cap_jobs;
    std::vector<char> blk(cap * (2 * sizeof(void*) + 2 * sizeof(int)));
    memcpy(blk.data(), mp.data(), n_jobs * sizeof(void*));
    memcpy(blk.data() + cap * sizeof(void*), pp.data(), n_jobs * sizeof(void*));
    memcpy(blk.data() + 2 * cap * sizeof(void*), ints.data(), n_jobs * sizeof(int));
    memcpy(blk.data() + 2 * cap * sizeof(void*) + cap * sizeof(int), ints.data() + n_jobs, n_jobs * sizeof(int));
    WM_CHECK(hipMemcpyAsync(w.mel_ptrs, blk.data(), blk.size(), hipMemcpyHostToDevice, s->stream));
    {
        double bytes = 0;
        for (int j = 0; j < n_jobs; j++)
            bytes += 4.0 * n[j] + 4.0 * nm * std::min((n[j] + 200) / 160 + 1, mel_n_len(n[j]));
        KT kt(s, K_MEL, bytes);
        launch_mel(w.pcm_ptrs, w.n_samp, c->w.mel_tab, c->w.filt_t, nm, w.mel_ptrs, w.n_len, w.mel_max, n_jobs, max_frames,
                   s->stream);
    }
    WM_CHECK(hipStreamSynchronize(s->stream));  // blk (pageable) must outlive the copy
    s->n_len = mel_n_len(n[0]);
    s->n_len_org = mel_n_len_org(n[0]);
    s->mel_ready = true;
    return 0;
}

// ---- encoder + cross KV ---------------------------------------------------------------------------
static GemmArgs gemm_plain(const void* A, int M, int K, const void* B, int N, const float* bias, void* out, long ldo) {
    GemmArgs g{};
    g.A = A; g.a_rpb = M > 0 ? M : 1; g.a_bstride = 0; g.a_rstride = K;
    g.B = B; g.bias = bias; g.M = M; g.N = N; g.K = K;
    g.out = out; g.ldo = ldo; g.o_rpb = M > 0 ? M : 1; g.o_bstride = 0; g.o_off = 0;
    g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
    return g;
}

// fp8 mode, decoder half: WHISPER_MI355X_FP8_DEC=1 (read when a context first quantizes its weights).
// Off by default: correct (tests/test_gpu_fp8.py) but slower, because the decode-step GEMMs are
// latency-bound, not bound by their weight bytes (profiles/r02_fp8_decoder_ab.txt: large-v3 fp8 at
// 128 clips decode 849 -> 936 ms per step, turbo fp8 at 256 clips 193 -> 210 ms).
static bool dec_fp8() {
    const char* e = getenv("WHISPER_MI355X_FP8_DEC");
    return e && atoi(e) == 1;
}

// fp8 encoder weights: e4m3 copies of QKV, FC1 and FC2 with per-output-row scales, quantized on the
// device from the bf16 weights once per context (after load or the RCCL weight broadcast); in the
// same arena the decoder's decode-step projections (dec_fp8()).
static void ensure_fp8(Context* c) {
    std::lock_guard<std::mutex> lk(c->fp8_mu);
    if (c->fp8_ready) return;
    const Hparams& hp = c->hp;
    const size_t d = hp.n_audio_state, nl = hp.n_audio_layer;
    const size_t per = 3 * d * d + 4 * d * d + 4 * d * d, per_s = (3 * d + 4 * d + d) * sizeof(float);
    // decoder: wqkv [3t][t], wo / wxq / wxo [t][t], w1 [4t][t], w2 [t][4t] (+ one f32 scale per row)
    const size_t t = hp.n_text_state, nd = dec_fp8() ? hp.n_text_layer : 0;
    const size_t per_d = 14 * t * t, per_ds = (3 * t + 3 * t + 4 * t + t) * sizeof(float);
    WM_CHECK(hipSetDevice(c->device));
    dalloc(c->arena8, nl * (per + per_s) + nd * (per_d + per_ds));
    c->enc8.assign(nl, Context::Fp8Layer{});
    char* p = c->arena8;
    for (size_t l = 0; l < nl; l++) {
        Context::Fp8Layer& f = c->enc8[l];
        const LayerW& L = c->w.enc[l];
        f.wqkv = p; p += 3 * d * d;
        f.w1 = p; p += 4 * d * d;
        f.w2 = p; p += 4 * d * d;
        f.sqkv = (float*)p; p += 3 * d * sizeof(float);
        f.s1 = (float*)p; p += 4 * d * sizeof(float);
        f.s2 = (float*)p; p += d * sizeof(float);
        launch_quant_rows_fp8(c->dt, L.wqkv, 3 * d, (int)d, f.wqkv, f.sqkv, nullptr);
        launch_quant_rows_fp8(c->dt, L.w1, 4 * d, (int)d, f.w1, f.s1, nullptr);
        launch_quant_rows_fp8(c->dt, L.w2, d, (int)(4 * d), f.w2, f.s2, nullptr);
    }
    c->dec8.assign(nd, Context::Fp8Dec{});
    for (size_t l = 0; l < nd; l++) {
        Context::Fp8Dec& f = c->dec8[l];
        const LayerW& L = c->w.dec[l];
        auto q = [&](const void* w, size_t rows, size_t cols, void*& q8, float*& sc) {
            q8 = p; p += rows * cols;
            sc = (float*)p; p += rows * sizeof(float);
            launch_quant_rows_fp8(c->dt, w, (long)rows, (int)cols, q8, sc, nullptr);
        };
        q(L.wqkv, 3 * t, t, f.wqkv, f.sqkv);
        q(L.wo, t, t, f.wo, f.so);
        q(L.wxq, t, t, f.wxq, f.sxq);
        q(L.wxo, t, t, f.wxo, f.sxo);
        q(L.w1, 4 * t, t, f.w1, f.s1);
        q(L.w2, t, 4 * t, f.w2, f.s2);
    }
    WM_CHECK(hipDeviceSynchronize());
    c->fp8_ready = true;
}

// fp8 mode, FC1 -> FC2: the GELU output is re-quantized per row (one pass). An MX hand-off (FC1's
// epilogue quantizing per 32-column block for a block-scaled FC2) measured slower on turbo at 256 clips
// (encode 743-815 vs 578 ms per step: the MX-A FC2 tile spilled past 256 VGPRs) and was removed.
static void tgemm_fp8(whisper_state* s, int epi, const GemmArgs& g, const float* sa, const float* sb, hipStream_t st) {
    KT kt(s, K_GEMM_ENC, 2.0 * g.M * g.N * g.K, st);
    launch_gemm_fp8(s->ctx->dt, epi, g, sa, sb, st);
}

// Encoder FC1 GELU. f16 (whisper.cpp's CPU numerics, the parity mode): ggml's f16 GELU table
// (EPI_GELU), bit-exact with the oracle. bf16: the tanh formula in f32 (EPI_GELU_F; ggml-metal, the
// reference app's back-end (whisper.rs:40 use_gpu), evaluates GELU by formula too, and the epilogue
// stages no 75.8 KB table per tile): encode 340 -> 336 ms per step at 128 clips
// (profiles/r03_envab_slab_gelu.txt).
static int enc_gelu_epi(DType dt) { return dt == DType::BF16 ? EPI_GELU_F : EPI_GELU; }

// Projection weights of one layer in the compute type: the arena's matrices, or, for a block-quantized
// file, the context's expanded copy (ensure_expanded: every projection dequantized once per context,
// 3.2 GB for large-v3, on first use outside a graph capture). The encoder, the prefill and the decode
// steps of many clips are big-M GEMMs that read every weight many times, so they read the copy; the
// decode steps of few clips stream the blocks themselves (gemm_small_kernel, the persistent step).
// Until the copy exists (a first use inside a capture) a layer is dequantized into the state's scratch.
using LayerMats = Context::LayerMats;
// (returns the end of the layer's matrices in p)
static char* dequant_layer(Context* c, const LayerW& L, char* p, LayerMats& m, hipStream_t st) {
    const int d = c->hp.n_audio_state;
    const size_t E = esize(c->dt);
    // one launch for the layer when its blocks share one type (a ggml file quantizes every projection
    // alike), else one per matrix
    DequantJobs J;
    bool one_type = true;
    auto one = [&](const QMat& q, long rows, int K, const void*& dst) {
        if (!q.type) return;
        if (J.n && q.type != J.q[0].type) one_type = false;
        J.q[J.n] = q; J.rows[J.n] = rows; J.K[J.n] = K; J.out[J.n] = p; J.n++;
        dst = p;
        p += (size_t)rows * K * E;
    };
    one(L.qqkv, 3L * d, d, m.wqkv);
    one(L.qo, d, d, m.wo);
    one(L.qxq, d, d, m.wxq);
    one(L.qxo, d, d, m.wxo);
    one(L.q1, 4L * d, d, m.w1);
    one(L.q2, d, 4 * d, m.w2);
    if (one_type) launch_dequant_multi(c->dt, J, st);
    else
        for (int j = 0; j < J.n; j++) launch_dequant(c->dt, J.q[j], J.rows[j], J.K[j], J.out[j], st);
    return p;
}

static void ensure_expanded(Context* c, hipStream_t st) {
    if (!c->quant || c->expanded.load(std::memory_order_acquire)) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    WM_CHECK(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone) return;
    std::lock_guard<std::mutex> lk(c->exp_mu);
    if (c->expanded.load(std::memory_order_relaxed)) return;
    // encoder layers: QKV, out, FC1, FC2 = 12 d^2; decoder layers + cross Q, cross out = 14 d^2
    const size_t d = c->hp.n_audio_state;
    dalloc(c->arena_exp, (12 * c->w.enc.size() + 14 * c->w.dec.size()) * d * d * esize(c->dt));
    char* p = c->arena_exp;
    auto fill = [&](const std::vector<LayerW>& layers, std::vector<LayerMats>& out) {
        out.resize(layers.size());
        for (size_t l = 0; l < layers.size(); l++) {
            const LayerW& L = layers[l];
            out[l] = LayerMats{L.wqkv, L.wo, L.wxq, L.wxo, L.w1, L.w2};
            p = dequant_layer(c, L, p, out[l], st);
        }
    };
    fill(c->w.enc, c->exp_enc);
    fill(c->w.dec, c->exp_dec);
    WM_CHECK(hipStreamSynchronize(st));  // other states' streams read the copy from now on
    c->expanded.store(true, std::memory_order_release);
}

static LayerMats layer_mats(Context* c, whisper_state* s, bool dec, int l, hipStream_t st) {
    const LayerW& L = dec ? c->w.dec[l] : c->w.enc[l];
    LayerMats m{L.wqkv, L.wo, L.wxq, L.wxo, L.w1, L.w2};
    if (!c->quant) return m;
    ensure_expanded(c, st);
    if (c->expanded.load(std::memory_order_acquire)) return dec ? c->exp_dec[l] : c->exp_enc[l];
    dequant_layer(c, L, (char*)s->ws.wdq, m, st);
    return m;
}

int encode_windows(Context* c, whisper_state* s, const int* jobs, const int* seeks, const int* slots, int n_win) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    const int d = hp.n_audio_state, nm = hp.n_mels, T = hp.n_audio_ctx, H = hp.n_audio_head;
    const DType dt = c->dt;
    const size_t E = esize(dt);
    const int KCLS = K_GEMM_ENC;
    const Weights& W = c->w;
    hipStream_t st = s->stream;
    const bool fp8 = c->fp8_enc && d % 128 == 0;
    if (fp8) ensure_fp8(c);
    for (int b0 = 0; b0 < n_win; b0 += w.cap_enc) {
        const int nb = std::min(w.cap_enc, n_win - b0);
        int* hi = w.h_ints;
        for (int i = 0; i < nb; i++) { hi[i] = jobs[b0 + i]; hi[nb + i] = seeks[b0 + i]; hi[2 * nb + i] = slots[b0 + i]; }
        WM_CHECK(hipMemcpyAsync(w.win_job, hi, 3 * nb * sizeof(int), hipMemcpyHostToDevice, st));
        const int* d_job = w.win_job;
        const int* d_seek = w.win_job + nb;
        const int* d_slot = w.win_job + 2 * nb;
        launch_mel_window(dt, w.mel_ptrs, w.n_len, w.n_samp, w.mel_max, d_job, d_seek, nb, nm, w.mel_img, st);
        // conv1 (stride 1, pad 1) + GELU -> h1 rows 1..3000 of each 3002-row image
        {
            GemmArgs g = gemm_plain(w.mel_img, nb * 2 * T, 3 * nm, W.conv1_w, d, W.conv1_b, w.h1, d);
            g.a_rpb = 2 * T; g.a_bstride = (long)3002 * nm; g.a_rstride = nm;
            g.o_rpb = 2 * T; g.o_bstride = 3002; g.o_off = 1;
            tgemm(s, KCLS, dt, EPI_GELU, g, st);
        }
        // conv2 (stride 2, pad 1) + GELU + positional embedding -> residual stream x (f32)
        {
            GemmArgs g = gemm_plain(w.h1, nb * T, 3 * d, W.conv2_w, d, W.conv2_b, w.x, d);
            g.a_rpb = T; g.a_bstride = (long)3002 * d; g.a_rstride = 2 * d;
            g.pos = W.pos_e; g.pos_rows = T;
            tgemm(s, KCLS, dt, EPI_GELU_POS, g, st);
        }
        const int M = nb * T;
        for (int l = 0; l < hp.n_audio_layer; l++) {
            const LayerW& L = W.enc[l];
            if (fp8) {
                // e4m3 path: LN quantized per row into hn (bytes), QKV/FC1/FC2 on the fp8 MFMA; the
                // GELU output is re-quantized per row into the qkv buffer (free again after attention)
                const Context::Fp8Layer& F = c->enc8[l];
                launch_layernorm_fp8(w.x, M, d, L.ln1_w, L.ln1_b, w.hn, w.hs, st);
                tgemm_fp8(s, EPI_STORE, gemm_plain(w.hn, M, d, F.wqkv, 3 * d, L.bqkv, w.qkv, 3 * d), w.hs, F.sqkv, st);
                {
                    KT kt(s, K_ATTN_ENC, 4.0 * nb * H * (double)T * T * 64);
                    launch_attn_encoder(dt, w.qkv, w.att, nb, T, d, H, st);
                }
                tgemm(s, KCLS, dt, EPI_RESID, gemm_plain(w.att, M, d, L.wo, d, L.bo, w.x, d), st);
                launch_layernorm_fp8(w.x, M, d, L.ln2_w, L.ln2_b, w.hn, w.hs, st);
                tgemm_fp8(s, EPI_GELU_F, gemm_plain(w.hn, M, d, F.w1, 4 * d, L.b1, w.ff, 4 * d), w.hs, F.s1, st);
                launch_quant_rows_fp8(dt, w.ff, M, 4 * d, w.qkv, w.hs, st);
                tgemm_fp8(s, EPI_RESID, gemm_plain(w.qkv, M, 4 * d, F.w2, d, L.b2, w.x, d), w.hs, F.s2, st);
                continue;
            }
            const LayerMats Wm = layer_mats(c, s, false, l, st);
            launch_layernorm(dt, w.x, nullptr, M, d, L.ln1_w, L.ln1_b, w.hn, st);
            tgemm(s, KCLS, dt, EPI_STORE, gemm_plain(w.hn, M, d, Wm.wqkv, 3 * d, L.bqkv, w.qkv, 3 * d), st);
            {
                KT kt(s, K_ATTN_ENC, 4.0 * nb * H * (double)T * T * 64);
                launch_attn_encoder(dt, w.qkv, w.att, nb, T, d, H, st);
            }
            tgemm(s, KCLS, dt, EPI_RESID, gemm_plain(w.att, M, d, Wm.wo, d, L.bo, w.x, d), st);
            launch_layernorm(dt, w.x, nullptr, M, d, L.ln2_w, L.ln2_b, w.hn, st);
            tgemm(s, KCLS, dt, enc_gelu_epi(dt), gemm_plain(w.hn, M, d, Wm.w1, 4 * d, L.b1, w.ff, 4 * d), st);
            tgemm(s, KCLS, dt, EPI_RESID, gemm_plain(w.ff, M, 4 * d, Wm.w2, d, L.b2, w.x, d), st);
        }
        launch_layernorm(dt, w.x, nullptr, M, d, W.lnpost_w, W.lnpost_b, w.hn, st);
        if (s->direct) {
            // keep E per slot for the direct cross attention; the slot's cross K/V (if any) is stale
            for (int k = 0; k < nb; k++) {
                WM_CHECK(hipMemcpyAsync((char*)w.enc + (size_t)slots[b0 + k] * T * d * E, (const char*)w.hn + (size_t)k * T * d * E,
                                        (size_t)T * d * E, hipMemcpyDeviceToDevice, st));
                w.cross_fresh[slots[b0 + k]] = 0;
            }
        } else {
            // cross K/V of every decoder layer in one GEMM, scattered into each window's slot
            GemmArgs g = gemm_plain(w.hn, M, d, W.wkv_cross, 2 * hp.n_text_layer * d, W.bkv_cross, nullptr, 0);
            g.scale = c->k_scale;
            g.cache = w.cross; g.row_slot = d_slot; g.L = hp.n_text_layer; g.H = hp.n_text_head; g.ctx = T; g.d = d;
            tgemm(s, KCLS, dt, EPI_CROSSKV, g, st);
            for (int k = 0; k < nb; k++) w.cross_fresh[slots[b0 + k]] = 1;
        }
        WM_CHECK(hipStreamSynchronize(st));  // h_ints reused by the next micro-batch
    }
    s->last_enc_windows = n_win;
    return 0;
}

// ---- decoder --------------------------------------------------------------------------------------
// n_tok tokens (ragged over slots) -> logits of n_rows rows (row r = token lrows[r]) into w.logits.
// Token metadata must already be in w.h_ints: [tok | pos | slot | - | - ] with stride cap_tok and
// lrows at 5*cap_tok.
// token metadata (already in w.h_ints: [tok | pos | slot | - | -], lrows at 5*cap_tok) -> device
static void decoder_upload(Context* c, whisper_state* s, int n_tok, int n_rows, bool tiles) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    int* hi = w.h_ints;
    const int ct = w.cap_tok;
    double self_kv = 0;
    for (int i = 0; i < n_tok; i++) {
        hi[3 * ct + i] = hi[ct + i] + 1;
        hi[4 * ct + i] = hp.n_audio_ctx;
        self_kv += hi[ct + i] + 1;
    }
    s->cur_self_work = self_kv * hp.n_text_head * 64 * 2 * 2;
    WM_CHECK(hipMemcpyAsync(w.tok, hi, ((size_t)5 * ct + n_rows) * sizeof(int), hipMemcpyHostToDevice, s->stream));
    if (!tiles) return;
    // prefill attention tiles: runs of <= 64 consecutive tokens of one slot with increasing positions
    int nt = 0;
    for (int i = 0; i < n_tok; i++) {
        const bool cont = i > 0 && hi[2 * ct + i] == hi[2 * ct + i - 1] && hi[ct + i] > hi[ct + i - 1] &&
                          w.h_qtiles[nt - 1].y < 64;
        if (cont) w.h_qtiles[nt - 1].y++;
        else w.h_qtiles[nt++] = make_int2(i, 1);
    }
    w.n_qtiles = nt;
    WM_CHECK(hipMemcpyAsync(w.qtiles, w.h_qtiles, (size_t)nt * sizeof(int2), hipMemcpyHostToDevice, s->stream));
}

// One group of decoder rows on one stream: rows [r0, r0+n) of the token arrays and activations,
// with its own split-K slab region and cross-attention partials, so that two groups can run at the
// same time (decode steps).
struct DecView {
    int r0, n;
    hipStream_t st;
    float* splitk;
    long splitk_elems;
    float *xo, *xml;
};

// The small-M decode path (decoder_rows_small): every projection one launch (no split-K slabs, no
// reduce launch), LayerNorm in the GEMM prologue. Default for decode steps of <= 4 clips: at one clip
// base f16 471-481 -> 539-540 audio-s/s, large-v3 f16 78 -> 80 (profiles/r03_smallm_b1_ab.txt); at 16
// clips it measured slower (large-v3 bf16: 101 vs 94 us per decoder layer, r03_prof16_smallm{0,1}.md:
// its 80 workgroups of 16 columns pull the weights more slowly than split-K's 200-240, and the
// LayerNorm recomputed by every workgroup costs ~4.7 us per LN-consuming GEMM at 16 rows).
// WHISPER_MI355X_SMALLM=0 off, =1 up to 32 clips, =k up to k clips (read per call). Block-quantized
// files use it up to quant_small_max() clips whatever this says.
static int small_m_max() {
    const char* e = getenv("WHISPER_MI355X_SMALLM");
    if (!e) return 4;
    const int v = atoi(e);
    return v == 1 ? 32 : std::max(0, std::min(32, v));
}

// Decode steps of block-quantized files: up to this many clips the small-M path reads the blocks
// in its GEMMs; above it (its 32-row chunks each re-read the blocks: large-v3-q5_0 at 128 clips decoded
// in 2534 ms per step against 857 for f16) the layer's blocks are dequantized once per step into the
// scratch (one launch) and the split-K path runs as for f16 / bf16 weights. WHISPER_MI355X_QSMALL_MAX.
static int quant_small_max() {
    const char* e = getenv("WHISPER_MI355X_QSMALL_MAX");  // read per call (tests switch it)
    return e ? atoi(e) : 32;
}

// The persistent decode step (kernels/pdec.hip) for decode steps of up to this many clips in the cache
// form: WHISPER_MI355X_PDEC (default 4 = kPdecMaxRows; 0 = off; read per call).
static int pdec_max() {
    const char* e = getenv("WHISPER_MI355X_PDEC");
    return e ? std::max(0, std::min(kPdecMaxRows, atoi(e))) : kPdecMaxRows;
}

// The per-call switches that choose a decode step's kernels, folded into the key of its captured graph.
static int dec_path_sig() {
    return small_m_max() | (std::min(std::max(quant_small_max(), 0), 1023) << 6) |
           (std::min(std::max(attn_cross_wide_max(), 0), 1023) << 16) | (pdec_max() << 26) | ((g_pdec_blocks & 1) << 29);
}

// Quantized files: the persistent step reads the context's expanded compute-type copy when it exists
// (measured faster: the one-wave-per-SIMD kernel pays for the in-register dequantization; large-v3
// q5_0, 1 clip: 2.79 ms per step streaming blocks, 1.52 reading the copy); whisper_mi355x_set_pdec_blocks(1)
// makes it stream the GGML blocks (0.69 bytes per q5_0 weight) instead.
static bool pdec_blocks(Context* c) {
    return c->quant && (g_pdec_blocks || !c->expanded.load(std::memory_order_acquire));
}

// A decode step of n clips runs as one persistent launch when the model shape has a kernel, the
// weights are f16 / bf16 or GGML blocks (not the fp8 decoder copies), the device has the 256 CUs the
// grid is built for, and the step is in the cross K/V cache form.
static bool pdec_use(Context* c, whisper_state* s, int n, bool xdirect) {
    if (xdirect || s->pdec_block || s->pdec_off || n < 1 || n > pdec_max()) return false;
    if (c->fp8_enc && !c->dec8.empty()) return false;
    // one weight form for every decoder matrix (the kernel is built per form)
    const bool quant = c->w.dec[0].qqkv.type != 0;
    for (const LayerW& L : c->w.dec)
        for (const QMat* q : {&L.qqkv, &L.qo, &L.qxq, &L.qxo, &L.q1, &L.q2})
            if ((q->type != 0) != quant) return false;
    const bool blocks = pdec_blocks(c);
    if (blocks && c->dt != DType::F16) return false;
    if (!pdec_supported(c->hp.n_text_state, c->hp.n_text_head, blocks)) return false;
    static const int cus = [] {
        int dev = 0, v = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        return v;
    }();
    return cus == 256;
}

// Device array of the decoder layers' pointers (once per context and weight form): the arena's
// matrices, the GGML blocks of a quantized file, or that file's expanded compute-type copy
static const PdecLayer* pdec_layers(Context* c, bool blocks) {
    std::lock_guard<std::mutex> lk(c->pdec_mu);
    void*& slot = blocks || !c->quant ? c->pdec_layers : c->pdec_layers_exp;
    if (!slot) {
        std::vector<PdecLayer> h(c->hp.n_text_layer);
        for (int l = 0; l < c->hp.n_text_layer; l++) {
            const LayerW& L = c->w.dec[l];
            LayerMats m{L.wqkv, L.wo, L.wxq, L.wxo, L.w1, L.w2};
            if (c->quant && !blocks) m = c->exp_dec[l];
            auto mat = [&](const void* w, const QMat& q) {
                return q.type && blocks ? PdecMat{q.qs, q.qh, q.dm, q.type} : PdecMat{w, nullptr, nullptr, 0};
            };
            h[l] = PdecLayer{mat(m.wqkv, L.qqkv), mat(m.wo, L.qo), mat(m.wxq, L.qxq), mat(m.wxo, L.qxo), mat(m.w1, L.q1),
                             mat(m.w2, L.q2), L.bqkv, L.bo, L.bxq, L.bxo, L.b1, L.b2,
                             L.ln1_w, L.ln1_b, L.lnx_w, L.lnx_b, L.ln2_w, L.ln2_b};
        }
        void* p = nullptr;
        WM_CHECK(hipMalloc(&p, h.size() * sizeof(PdecLayer)));
        WM_CHECK(hipMemcpy(p, h.data(), h.size() * sizeof(PdecLayer), hipMemcpyHostToDevice));
        slot = p;
    }
    return (const PdecLayer*)slot;
}

// Everything a persistent step allocates, before a decode step is captured (no hipMalloc in a capture)
static void pdec_prepare(Context* c, whisper_state* s) {
    Workspace& w = s->ws;
    pdec_layers(c, pdec_blocks(c));
    if (w.pd_sync) return;
    // the hand-off block
    dalloc(w.pd_sync, pdec_granules(c->hp.n_text_state, c->hp.n_text_layer, c->hp.n_text_head).bytes);
    WM_CHECK(hipHostMalloc((void**)&w.h_pd_err, 16, 0));
    *w.h_pd_err = 0;
}

// One decode step of the view's rows as the persistent launch + the logits GEMM (graph-capturable).
// The launch's error word is copied to the host (a node of the step's graph): decode_step checks it
// after the step's synchronisation and re-runs the step on the per-kernel path if the launch gave up.
static void decoder_rows_pdec(Context* c, whisper_state* s, const DecView& v) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    const int d = hp.n_text_state, H = hp.n_text_head, L = hp.n_text_layer, V = hp.n_vocab;
    const int n = v.n;
    hipStream_t st = v.st;
    if (!w.pd_sync) WM_FAIL("pdec: buffers not allocated (pdec_prepare)");
    const bool blocks = pdec_blocks(c);
    PdecArgs a{};
    a.layers = pdec_layers(c, blocks);
    a.L = L; a.M = n; a.d = d; a.n_text_ctx = hp.n_text_ctx; a.n_audio_ctx = hp.n_audio_ctx;
    a.tok_emb = c->w.tok_emb_f32 ? (const void*)c->w.tok_emb_f32 : c->w.tok_emb;
    a.te_f32 = c->w.tok_emb_f32 != nullptr;
    a.pos_d = c->w.pos_d;
    a.lnd_w = c->w.lnd_w; a.lnd_b = c->w.lnd_b;
    a.tok = w.tok + v.r0; a.pos = w.pos + v.r0; a.slot = w.slot + v.r0;
    a.self_cache = w.self; a.cross_cache = w.cross;
    a.k_scale = c->k_scale;
    a.quant = blocks;
    a.s_cross = pdec_cross_splits(H, hp.n_audio_ctx);
    a.sync = w.pd_sync;
    a.gr = pdec_granules(d, L, H);
    a.out_dh = (char*)w.dh + (size_t)v.r0 * d * esize(c->dt);
    a.gelu_tab = gelu_table_device();
    a.spin_ticks = g_pdec_spin_ticks;
    a.stamps = g_pdec_stamps;
    {
        // weights once + cross K/V + self K/V of every row, per launch
        const double bytes = 14.0 * d * d * 2 * L + (double)n * L * 2 * hp.n_audio_ctx * d * 2 + s->cur_self_work;
        KT kt(s, K_PDEC, bytes, st);
        launch_pdec(c->dt, a, st);
    }
    // (a pipelined step graph's advance kernel writes the error word to its ring slot instead)
    if (!s->pipe_capture)
        WM_CHECK(hipMemcpyAsync(w.h_pd_err, (const char*)w.pd_sync + a.gr.err_bytes, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    GemmArgs g = gemm_plain(a.out_dh, n, d, c->w.tok_emb, V, nullptr, w.logits + (size_t)v.r0 * V, V);
    tgemm_ws(s, K_GEMM_DEC, c->dt, EPI_F32, g, st, v.splitk, v.splitk_elems);
}

// Decode step over <= 32 rows (the app's one clip per call, whisper.rs:83-85 / state.rs:147; one
// rank's 16-clip shard of configs[3] at 8 GPUs), kernels only: every projection is ONE launch of
// gemm_small_kernel (no split-K slabs, no reduce launch), and the LayerNorm in front of the QKV,
// cross-Q and FC1 projections runs in that GEMM's prologue from the f32 residual stream. Per layer:
// QKV (raw f32 sums) -> self attention (bias, scale, cache append, attention) -> Wo (+x) -> cross-Q
// -> cross attention -> Wxo (+x) -> FC1 (GELU) -> FC2 (+x): 8 launches in the cache form, against
// 15 on the split-K path. Results per row do not depend on the other rows (batch == single within
// this path); they differ in the last bits from the split-K path's (another summation order).
static void decoder_rows_small(Context* c, whisper_state* s, const DecView& v, bool xdirect, double self_share,
                               int kt_stride) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    const int d = hp.n_text_state, H = hp.n_text_head, V = hp.n_vocab, L = hp.n_text_layer;
    const DType dt = c->dt;
    const Weights& W = c->w;
    const size_t E = esize(dt);
    hipStream_t st = v.st;
    const int n = v.n;
    int* tok = w.tok + v.r0;
    int* pos = w.pos + v.r0;
    int* slot = w.slot + v.r0;
    int* nkv_cross = w.nkv_cross + v.r0;
    float* dx = w.dx + (size_t)v.r0 * d;
    void* dh = (char*)w.dh + (size_t)v.r0 * d * E;
    void* dq = (char*)w.dq + (size_t)v.r0 * d * E;
    void* datt = (char*)w.datt + (size_t)v.r0 * d * E;
    void* dff = (char*)w.dff + (size_t)v.r0 * 4 * d * E;
    void* qx = w.qx ? (void*)((char*)w.qx + (size_t)v.r0 * 2 * H * d * E) : nullptr;
    float* raw = v.splitk;  // f32 projection sums handed to the attention prologues ([n][3d] / [n][d])
    const double kvrow = (double)H * 64 * 2 * 2;
    const QMat* qm = nullptr;  // the layer's block-quantized matrix of the next `small` call (quantized files)
    auto small = [&](int epi, const void* A, int K, const void* Wt, int N, const float* bias, void* out, long ldo,
                     const float* lnw = nullptr, const float* lnb = nullptr) {
        GemmArgs g = gemm_plain(A, n, K, Wt, N, bias, out, ldo);
        g.a_ln_w = lnw;
        g.a_ln_b = lnb;
        if (qm) g.q = *qm;
        qm = nullptr;
        KT kt(s, K_GEMM_DEC, 2.0 * N * K + 2.0 * n * K + 4.0 * n * N, st);
        launch_gemm_small(dt, epi, g, lnw != nullptr, st);
    };
    launch_embed(dt, W.tok_emb_f32 ? (const void*)W.tok_emb_f32 : W.tok_emb, W.tok_emb_f32 != nullptr, W.pos_d, tok, pos, n, d,
                 dx, st);
    for (int l = 0; l < L; l++) {
        const LayerW& Lw = W.dec[l];
        const bool kt_layer = l % kt_stride == 0;
        // self attention: LN1 in the QKV GEMM, raw sums to the attention prologue (+ bias, q/k scale)
        qm = &Lw.qqkv;
        small(EPI_F32, dx, d, Lw.wqkv, 3 * d, nullptr, raw, 3 * d, Lw.ln1_w, Lw.ln1_b);
        {
            const DecSlabs sl{raw, 1, (long)n * 3 * d, 3 * d, Lw.bqkv, c->k_scale};
            KT kt(s, K_ATTN_SELF, self_share, st, kt_layer);
            launch_attn_self_step(dt, sl, w.self, slot, pos, n, L, l, H, hp.n_text_ctx, d, datt, st);
        }
        qm = &Lw.qo;
        small(EPI_RESID, datt, d, Lw.wo, d, Lw.bo, dx, d);
        if (xdirect) {
            GemmArgs g = gemm_plain(dx, n, d, Lw.wxq, d, Lw.bxq, dq, d);
            g.scale = c->k_scale; g.sc_div = d; g.sc_mod = 1; g.sc_lim = 1;
            g.a_ln_w = Lw.lnx_w; g.a_ln_b = Lw.lnx_b;
            g.q = Lw.qxq;
            {
                KT kt(s, K_GEMM_DEC, 2.0 * d * d + 2.0 * n * d + 4.0 * n * d, st);
                launch_gemm_small(dt, EPI_STORE, g, true, st);
            }
            const int Ta = hp.n_audio_ctx, S = xattn_splits(n, Ta);
            {
                KT kt(s, K_GEMM_DEC, 2.0 * d * d + 2.0 * n * d + 4.0 * n * H * d, st);
                launch_xattn_qproj(dt, dq, (const char*)W.wkT + (size_t)l * H * d * 64 * 2, n, d, H, c->k_scale, qx, st);
            }
            {
                KT kt(s, K_ATTN_CROSS, (double)n * Ta * d * 2, st, kt_layer);
                launch_xattn_step(dt, w.enc, slot, qx, n, Ta, d, S, kXattnThr, v.xo, v.xml, st);
            }
            {
                KT kt(s, K_GEMM_DEC, 2.0 * d * d + 4.0 * n * S * d + 2.0 * n * d, st);
                launch_xattn_combine(dt, v.xo, v.xml, S, (const char*)W.wkv_cross + (size_t)(2 * l + 1) * d * d * 2,
                                     W.bkv_cross + (size_t)(2 * l + 1) * d, n, d, H, datt, st);
            }
        } else {
            qm = &Lw.qxq;
            small(EPI_F32, dx, d, Lw.wxq, d, nullptr, raw, d, Lw.lnx_w, Lw.lnx_b);
            const DecSlabs sl{raw, 1, (long)n * d, d, Lw.bxq, c->k_scale};
            KT kt(s, K_ATTN_CROSS, (double)n * hp.n_audio_ctx * kvrow, st, kt_layer);
            launch_attn_cross_step(dt, sl, w.cross, slot, nkv_cross, n, L, l, H, hp.n_audio_ctx, d, datt, st);
        }
        qm = &Lw.qxo;
        small(EPI_RESID, datt, d, Lw.wxo, d, Lw.bxo, dx, d);
        qm = &Lw.q1;
        small(EPI_GELU, dx, d, Lw.w1, 4 * d, Lw.b1, dff, 4 * d, Lw.ln2_w, Lw.ln2_b);
        qm = &Lw.q2;
        small(EPI_RESID, dff, 4 * d, Lw.w2, d, Lw.b2, dx, d);
    }
    launch_layernorm(dt, dx, nullptr, n, d, W.lnd_w, W.lnd_b, dh, st);
    GemmArgs g = gemm_plain(dh, n, d, W.tok_emb, V, nullptr, w.logits + (size_t)v.r0 * V, V);
    tgemm_ws(s, K_GEMM_DEC, dt, EPI_F32, g, st, v.splitk, v.splitk_elems);
}

// The decoder forward over the view's tokens + logits; kernels only (graph-capturable). `fused`
// (decode steps: one token per clip, logits for every row, <= 128 rows per view): every LayerNorm
// is folded into the embedding or into the split-K reduce of the preceding residual GEMM.
// Otherwise (prefill, one view at r0 = 0) logits of n_rows rows (row r = token lrows[r]).
static void decoder_rows(Context* c, whisper_state* s, const DecView& v, int n_rows, bool fused, bool xdirect,
                         double self_share) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    const int d = hp.n_text_state, H = hp.n_text_head, V = hp.n_vocab, L = hp.n_text_layer;
    const DType dt = c->dt;
    const Weights& W = c->w;
    const size_t E = esize(dt);
    hipStream_t st = v.st;
    const int n_tok = v.n;
    const int KCLS = K_GEMM_DEC;
    const double kvrow = (double)H * 64 * 2 * 2;  // K and V row bytes of one position, all heads
    int* tok = w.tok + v.r0;
    int* pos = w.pos + v.r0;
    int* slot = w.slot + v.r0;
    int* nkv_self = w.nkv_self + v.r0;
    int* nkv_cross = w.nkv_cross + v.r0;
    float* dx = w.dx + (size_t)v.r0 * d;
    void* dh = (char*)w.dh + (size_t)v.r0 * d * E;
    void* dq = (char*)w.dq + (size_t)v.r0 * d * E;
    void* datt = (char*)w.datt + (size_t)v.r0 * d * E;
    void* dff = (char*)w.dff + (size_t)v.r0 * 4 * d * E;
    void* qx = w.qx ? (void*)((char*)w.qx + (size_t)v.r0 * 2 * H * d * E) : nullptr;
    auto gemm = [&](int cls, int epi, const GemmArgs& g) { tgemm_ws(s, cls, dt, epi, g, st, v.splitk, v.splitk_elems); };
    // fp8 mode: decode steps read the e4m3 copies of the layer's projection weights
    const bool w8 = fused && c->fp8_enc && !c->dec8.empty();
    auto use8 = [&](GemmArgs g, void* q8, float* sc) {
        if (w8) { g.B = q8; g.w8_scale = sc; }
        return g;
    };
    auto resid = [&](const void* A, int K, const void* Wt, const float* bias, const float* lnw, const float* lnb,
                     void* q8 = nullptr, float* sc = nullptr) {
        GemmArgs g = use8(gemm_plain(A, n_tok, K, Wt, d, bias, dx, d), q8, sc);
        if (fused) { g.ln_w = lnw; g.ln_b = lnb; g.ln_out = dh; }
        gemm(KCLS, EPI_RESID, g);
        if (!fused && lnw) launch_layernorm(dt, dx, nullptr, n_tok, d, lnw, lnb, dh, st);
    };
    // kernel timing (bench roofline): bits 8..15 of the mask = time the per-layer attention launches of
    // every k-th layer only (fewer event nodes in the timed decode graphs; every layer does the same work)
    const int kt_stride = std::max(1, (s->ktime_mask >> 16) & 0xFF);
    if (fused && pdec_use(c, s, n_tok, xdirect)) {
        decoder_rows_pdec(c, s, v);
        return;
    }
    // (the persistent and small-M paths embed the tokens themselves)
    if (fused && !w8 && ((c->quant && n_tok <= quant_small_max()) || n_tok <= small_m_max()) && gemm_small_ok(n_tok, d, true) &&
        gemm_small_ok(n_tok, 4 * d, false)) {
        decoder_rows_small(c, s, v, xdirect, self_share, kt_stride);
        return;
    }
    if (fused) launch_embed_ln(dt, W.tok_emb_f32 ? (const void*)W.tok_emb_f32 : W.tok_emb, W.tok_emb_f32 != nullptr, W.pos_d, tok, pos, n_tok, d, dx, W.dec[0].ln1_w, W.dec[0].ln1_b, dh, st);
    else {
        launch_embed(dt, W.tok_emb_f32 ? (const void*)W.tok_emb_f32 : W.tok_emb, W.tok_emb_f32 != nullptr, W.pos_d, tok, pos, n_tok, d, dx, st);
        launch_layernorm(dt, dx, nullptr, n_tok, d, W.dec[0].ln1_w, W.dec[0].ln1_b, dh, st);
    }
    // decode steps: the QKV (and, cache mode, cross-Q) projections leave split-K partial sums that
    // the attention kernels reduce in their prologue (no separate reduce launch)
    auto partials = [&](const void* A, const void* Wt, int N, const float* bias, float scale, void* q8,
                        float* sc) -> DecSlabs {
        GemmArgs g = use8(gemm_plain(A, n_tok, d, Wt, N, bias, nullptr, N), q8, sc);
        g.splitk_ws = v.splitk;
        g.splitk_ws_elems = v.splitk_elems;
        g.slab_wt = 1;
        KT kt(s, KCLS, 2.0 * g.N * g.K + 2.0 * g.M * g.K + 4.0 * g.M * g.N, st);
        const int splits = launch_gemm_partials(dt, g, st);
        if (splits <= 0 || splits > 16) WM_FAIL("decode partials GEMM not applicable (splits %d)", splits);
        return DecSlabs{v.splitk, splits, (long)n_tok * N, N, bias, scale};
    };
    for (int l = 0; l < L; l++) {
        const int lw = l;
        LayerW Lw = W.dec[lw];
        if (c->quant) {  // prefill / language detection: this layer's blocks dequantized into the scratch
            const LayerMats m = layer_mats(c, s, true, lw, st);
            Lw.wqkv = (void*)m.wqkv; Lw.wo = (void*)m.wo; Lw.wxq = (void*)m.wxq; Lw.wxo = (void*)m.wxo;
            Lw.w1 = (void*)m.w1; Lw.w2 = (void*)m.w2;
        }
        static const Context::Fp8Dec no8{};
        const Context::Fp8Dec& F = w8 ? c->dec8[l] : no8;
        const bool kt_layer = l % kt_stride == 0;
        if (fused) {
            const DecSlabs sl = partials(dh, Lw.wqkv, 3 * d, Lw.bqkv, c->k_scale, F.wqkv, F.sqkv);
            KT kt(s, K_ATTN_SELF, self_share, st, kt_layer);
            launch_attn_self_step(dt, sl, w.self, slot, pos, n_tok, L, l, H, hp.n_text_ctx, d, datt, st);
        } else {
            GemmArgs g = gemm_plain(dh, n_tok, d, Lw.wqkv, 3 * d, Lw.bqkv, dq, d);
            g.scale = c->k_scale;
            g.cache = w.self; g.row_slot = slot; g.row_pos = pos; g.L = L; g.layer = l; g.H = H;
            g.ctx = hp.n_text_ctx; g.d = d;
            gemm(KCLS, EPI_QKV_DEC, g);
            KT kt(s, K_ATTN_SELF, self_share, st, kt_layer);
            launch_attn_prefill(dt, dq, d, w.self, slot, nkv_self, w.qtiles, w.n_qtiles, L, l, H, hp.n_text_ctx, d, datt, st);
        }
        resid(datt, d, Lw.wo, Lw.bo, Lw.lnx_w, Lw.lnx_b, F.wo, F.so);
        if (xdirect) {
            // cross attention from the encoder output (kernels/xattn.hip): q -> Q' = s Wk^T q (hi/lo)
            // -> one pass over E per clip -> split merge + Wv. (Fusing the cross-Q reduce into the Q'
            // projection was bit-identical but slower, 855 vs 848 ms per step at 128 clips: removed.)
            const void* wkt_l = (const char*)W.wkT + (size_t)lw * H * d * 64 * 2;
            {
                GemmArgs g = use8(gemm_plain(dh, n_tok, d, Lw.wxq, d, Lw.bxq, dq, d), F.wxq, F.sxq);
                g.scale = c->k_scale; g.sc_div = d; g.sc_mod = 1; g.sc_lim = 1;
                gemm(KCLS, EPI_STORE, g);
                KT kt(s, KCLS, 2.0 * d * d + 2.0 * n_tok * d + 4.0 * n_tok * H * d, st);
                launch_xattn_qproj(dt, dq, wkt_l, n_tok, d, H, c->k_scale, qx, st);
            }
            const int Ta = hp.n_audio_ctx, S = xattn_splits(n_tok, Ta);
            {
                // the roofline class holds decode steps only (E bytes read once per clip and layer)
                KT kt(s, fused ? K_ATTN_CROSS : K_OTHER, (double)n_tok * Ta * d * 2, st, kt_layer);
                launch_xattn_step(dt, w.enc, slot, qx, n_tok, Ta, d, S, kXattnThr, v.xo, v.xml, st);
            }
            {
                KT kt(s, KCLS, 2.0 * d * d + 4.0 * n_tok * S * d + 2.0 * n_tok * d, st);
                launch_xattn_combine(dt, v.xo, v.xml, S, (const char*)W.wkv_cross + (size_t)(2 * lw + 1) * d * d * 2,
                                     W.bkv_cross + (size_t)(2 * lw + 1) * d, n_tok, d, H, datt, st);
            }
        } else if (fused) {
            const DecSlabs sl = partials(dh, Lw.wxq, d, Lw.bxq, c->k_scale, F.wxq, F.sxq);
            KT kt(s, K_ATTN_CROSS, (double)n_tok * hp.n_audio_ctx * kvrow, st, kt_layer);  // decode steps only
            launch_attn_cross_step(dt, sl, w.cross, slot, nkv_cross, n_tok, L, l, H, hp.n_audio_ctx, d, datt, st);
        } else {
            GemmArgs g = gemm_plain(dh, n_tok, d, Lw.wxq, d, Lw.bxq, dq, d);
            g.scale = c->k_scale; g.sc_div = d; g.sc_mod = 1; g.sc_lim = 1;
            gemm(KCLS, EPI_STORE, g);
            KT kt(s, K_OTHER, (double)n_tok * hp.n_audio_ctx * kvrow, st);
            launch_attn_prefill(dt, dq, d, w.cross, slot, nkv_cross, w.qtiles, w.n_qtiles, L, l, H, hp.n_audio_ctx, d, datt, st);
        }
        resid(datt, d, Lw.wxo, Lw.bxo, Lw.ln2_w, Lw.ln2_b, F.wxo, F.sxo);
        gemm(KCLS, EPI_GELU, use8(gemm_plain(dh, n_tok, d, Lw.w1, 4 * d, Lw.b1, dff, 4 * d), F.w1, F.s1));
        if (l + 1 < L) resid(dff, 4 * d, Lw.w2, Lw.b2, W.dec[l + 1].ln1_w, W.dec[l + 1].ln1_b, F.w2, F.s2);
        else if (fused) resid(dff, 4 * d, Lw.w2, Lw.b2, W.lnd_w, W.lnd_b, F.w2, F.s2);  // dh = final LN of every row
        else resid(dff, 4 * d, Lw.w2, Lw.b2, nullptr, nullptr);
    }
    if (fused) {
        gemm(KCLS, EPI_F32, gemm_plain(dh, n_tok, d, W.tok_emb, V, nullptr, w.logits + (size_t)v.r0 * V, V));
    } else {
        launch_layernorm(dt, w.dx, w.lrows, n_rows, d, W.lnd_w, W.lnd_b, w.lrow, st);
        gemm(KCLS, EPI_F32, gemm_plain(w.lrow, n_rows, d, W.tok_emb, V, nullptr, w.logits, V));
    }
}

// Row groups of a decode step. The fused pass (every LayerNorm folded into a split-K reduce) takes at
// most 128 rows, so a step over n > 128 clips runs as ceil(n / 128) fused groups of near-equal size,
// alternating between the state's two streams (forked from and joined back into the state's stream:
// branches of the step's hipGraph); two groups for 129..256 clips measured the same as the unfused
// path in bf16 (turbo at 256 clips: decode 213 vs 217 ms per step) and the fp8 decoder weights exist
// only on the fused path.
// Splitting steps of 32..128 clips into two concurrent groups measured slower on large-v3 at 128 clips
// (2360-2392 vs 2729-2740 audio-s/s: the cross-attention pass at 64 clips per group reads E at 3.6
// instead of 4.7 TB/s), and so did two separate graphs on two streams (942 vs 843 ms of decode per
// step, profiles/r02_dec_groups_ab.txt); both were removed.
static int dec_groups(int n_tok) { return cdiv(n_tok, 128); }

// The two stream halves of a decode step's scratch: group views on the state's stream use the first
// half of the split-K slabs and cross-attention partials, views on stream2 the second. A group of
// <= gmax rows uses at most gmax * xattn_splits(gmax) partial rows.
static void dec_halves(Context* c, whisper_state* s, int gmax, bool xdirect, DecView& a, DecView& b) {
    Workspace& w = s->ws;
    const int H = c->hp.n_text_head, d = c->hp.n_text_state;
    const long half = w.splitk_elems / 2;
    long xoff = 0;
    if (xdirect)
        for (int n = 1; n <= gmax; n++) xoff = std::max(xoff, (long)n * xattn_splits(n, c->hp.n_audio_ctx));
    a = DecView{0, 0, s->stream, w.splitk, half, w.xo, w.xml};
    b = DecView{0, 0, s->stream2, w.splitk + half, half, w.xo ? w.xo + xoff * H * d : nullptr,
                w.xml ? w.xml + xoff * H * 2 : nullptr};
}

static void decoder_launch(Context* c, whisper_state* s, int n_tok, int n_rows, bool rows_identity, bool xdirect) {
    Workspace& w = s->ws;
    const bool step = rows_identity && n_rows == n_tok;  // a decode step: one token per clip, logits of every row
    const int groups = step ? dec_groups(n_tok) : 1;
    s->step_rows = n_tok;
    if (groups == 1) {
        // prefill / language detection / whisper_decode: the unfused pass over the tiles that
        // decoder_upload built (decoder_forward); decode steps of <= 128 clips: one fused pass
        const DecView v{0, n_tok, s->stream, w.splitk, w.splitk_elems, w.xo, w.xml};
        decoder_rows(c, s, v, n_rows, step, xdirect, 1.0);
        return;
    }
    const int gsz = cdiv(n_tok, groups);
    DecView half[2];
    dec_halves(c, s, gsz, xdirect, half[0], half[1]);
    // block-quantized files before the expanded copy exists: one dequantization scratch per state, so
    // the groups run one after the other on the state's stream
    if (c->quant && !c->expanded.load(std::memory_order_acquire)) half[1] = half[0];
    WM_CHECK(hipEventRecord(s->ev_fork, s->stream));
    WM_CHECK(hipStreamWaitEvent(s->stream2, s->ev_fork, 0));
    for (int g = 0, r0 = 0; r0 < n_tok; g++, r0 += gsz) {
        DecView v = half[g & 1];
        v.r0 = r0;
        v.n = std::min(gsz, n_tok - r0);
        decoder_rows(c, s, v, v.n, true, xdirect, (double)v.n / n_tok);
    }
    WM_CHECK(hipEventRecord(s->ev_join, s->stream2));
    WM_CHECK(hipStreamWaitEvent(s->stream, s->ev_join, 0));
}


// Cross K/V of the given slots (all decoder layers, one GEMM per clip) into the cache, for slots
// whose cache is stale: direct mode computes it only for prompts too long for the direct prefill.
static void ensure_cross_cache(Context* c, whisper_state* s, const std::vector<int>& slots) {
    Workspace& w = s->ws;
    const Hparams& hp = c->hp;
    const int d = hp.n_audio_state, T = hp.n_audio_ctx, L = hp.n_text_layer;
    const size_t E = esize(c->dt);
    std::vector<int> stale;
    int need = 0;
    for (int sl : slots) need = std::max(need, sl + 1);
    ensure_cross(c, s, need);
    for (int sl : slots)
        if (!w.cross_fresh[sl]) stale.push_back(sl);
    std::sort(stale.begin(), stale.end());
    // one GEMM per run of consecutive slots (E is slot-major, so a run is one [k*T][d] matrix)
    for (size_t a = 0; a < stale.size();) {
        size_t b = a + 1;
        while (b < stale.size() && stale[b] == stale[b - 1] + 1) b++;
        const int sl = stale[a], k = (int)(b - a);
        GemmArgs g = gemm_plain((const char*)w.enc + (size_t)sl * T * d * E, k * T, d, c->w.wkv_cross, 2 * L * d,
                                c->w.bkv_cross, nullptr, 0);
        g.scale = c->k_scale;
        g.cache = w.cross; g.row_slot = w.kvslot + sl; g.L = L; g.H = hp.n_text_head; g.ctx = T; g.d = d;
        tgemm(s, K_GEMM_ENC, c->dt, EPI_CROSSKV, g, s->stream);
        for (size_t i = a; i < b; i++) w.cross_fresh[stale[i]] = 1;
        a = b;
    }
}

// Direct cross attention for this forward (tokens/slots already in w.h_ints)? Yes for one-token
// steps and short prompts; otherwise the clips involved get a cross K/V cache first.
static bool choose_xdirect(Context* c, whisper_state* s, int n_tok) {
    if (!s->direct) return false;
    Workspace& w = s->ws;
    const int* slot = w.h_ints + 2 * w.cap_tok;
    std::vector<int> cnt(w.cap_jobs, 0);
    int mx = 0;
    for (int i = 0; i < n_tok; i++) mx = std::max(mx, ++cnt[slot[i]]);
    if (n_tok <= w.cap_xq && mx <= kXDirectMaxTok) return true;
    std::vector<int> used;
    for (int k = 0; k < w.cap_jobs; k++) if (cnt[k]) used.push_back(k);
    ensure_cross_cache(c, s, used);
    return false;
}

static void decoder_forward(Context* c, whisper_state* s, int n_tok, int n_rows, bool rows_identity = false) {
    const bool xdirect = choose_xdirect(c, s, n_tok);
    decoder_upload(c, s, n_tok, n_rows, true);
    decoder_launch(c, s, n_tok, n_rows, rows_identity, xdirect);
}

int decode_tokens(Context* c, whisper_state* s, const int* tokens, const int* pos, const int* slots, int n_tok,
                  const int* logit_rows, int n_logit_rows) {
    Workspace& w = s->ws;
    if (n_tok > w.cap_tok) return -1;
    int* hi = w.h_ints;
    for (int i = 0; i < n_tok; i++) { hi[i] = tokens[i]; hi[w.cap_tok + i] = pos[i]; hi[2 * w.cap_tok + i] = slots[i]; }
    for (int r = 0; r < n_logit_rows; r++) hi[5 * w.cap_tok + r] = logit_rows[r];
    decoder_forward(c, s, n_tok, n_logit_rows);
    return 0;
}

// ---- scheduler ------------------------------------------------------------------------------------
enum Phase { PH_ENCODE, PH_LANG, PH_PREFILL, PH_DECODE, PH_DONE };

struct Job {
    int slot = 0;
    int n_samples = 0, n_len = 0, n_len_org = 0;
    int seek = 0, seek_start = 0, seek_end = 0;
    bool lang_pending = false;
    int lang_id = 0;
    std::vector<int> prompt_init, prompt_past, prompt;
    int temp_idx = 0;
    std::vector<TokenData> tokens;
    int result_len = 0;
    double sum_logprobs_all = 0, sum_logprobs = -INFINITY, avg_logprobs = -INFINITY, entropy = 0, score = -INFINITY;
    int seek_delta = 3000;
    bool has_ts = false, failed = false, completed = false;
    int step = 0;
    float no_speech_prob = 0.0f;
    std::mt19937* rng = nullptr;
    std::mt19937 own_rng{0};
    Phase phase = PH_ENCODE;
    std::vector<Segment> result;
    int n_new_segments = 0;
    whisper_mi355x_window_decision dec{};                // the current window's fallback decisions
    std::vector<whisper_mi355x_window_decision> decisions;
};

struct Sched {
    Context* c;
    whisper_state* s;
    whisper_full_params p;
    FullOpts o;
    std::vector<float> temps;
    std::vector<Job> jobs;
    bool single_api;
    int n_max_steps;
    long decoded = 0;
    double t_mel = 0, t_enc = 0, t_prefill = 0, t_decode = 0, t_logits = 0;
};

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void score_seq(const whisper_full_params& p, Job& j) {
    if (j.result_len == 0) return;
    double result = 0.0;
    for (int i = 0; i < j.result_len; ++i) result += j.tokens[i].plog;
    j.sum_logprobs = result;
    j.avg_logprobs = result / j.result_len;
    double penalty = j.result_len;
    if (p.length_penalty > 0.0f) penalty = pow((5.0 + penalty) / 6.0, p.length_penalty);
    j.score = result / penalty;
    std::map<int, int> counts;
    int cnt = 0;
    for (int i = std::max(0, j.result_len - 32); i < j.result_len; ++i) { counts[j.tokens[i].id]++; cnt++; }
    double entropy = 0.0;
    for (auto& kv : counts) { const double q = kv.second / (double)cnt; entropy -= q * log(q); }
    j.entropy = entropy;
}

static void start_attempt(Sched& S, Job& j) {
    const Vocab& v = S.c->vocab;
    const float t = S.temps[j.temp_idx];
    j.tokens.clear();
    j.result_len = 0;
    j.sum_logprobs_all = 0;
    j.sum_logprobs = j.avg_logprobs = j.score = -INFINITY;
    j.entropy = 0;
    j.seek_delta = 100 * WHISPER_CHUNK_SIZE;
    j.failed = j.completed = j.has_ts = false;
    j.step = 0;
    j.prompt.clear();
    if (!j.prompt_past.empty() && t < 0.5f && S.p.n_max_text_ctx > 0) {
        const int n_take = std::min(std::min(S.p.n_max_text_ctx, S.c->hp.n_text_ctx / 2), (int)j.prompt_past.size());
        j.prompt = {v.token_prev};
        j.prompt.insert(j.prompt.begin() + 1, j.prompt_past.end() - n_take, j.prompt_past.end());
    }
    j.prompt.insert(j.prompt.end(), j.prompt_init.begin(), j.prompt_init.end());
}

static void fill_ctl(Sched& S, Job& j, SeqCtl& ctl, bool want_nosp) {
    const Vocab& v = S.c->vocab;
    const float t = S.temps[j.temp_idx];
    ctl.is_initial = j.tokens.empty();
    ctl.last_ts = j.tokens.size() > 0 && j.tokens.back().id >= v.token_beg;
    ctl.penult_ts = j.tokens.size() < 2 || j.tokens[j.tokens.size() - 2].id >= v.token_beg;
    ctl.has_ts = j.has_ts;
    ctl.seek_delta = j.seek_delta;
    ctl.temperature = t;
    ctl.suppress_blank = S.p.suppress_blank;
    ctl.no_timestamps = S.p.no_timestamps;
    ctl.suppress_eot = S.o.fixed_tokens > 0;
    if (S.p.max_initial_ts > 0.0f) {
        const float precision = float(WHISPER_CHUNK_SIZE) / S.c->hp.n_audio_ctx;
        ctl.tid0_initial = (int)std::round(S.p.max_initial_ts / precision);
    } else ctl.tid0_initial = -1;
    ctl.want_probs = t >= 1e-6f;
    ctl.want_nosp = want_nosp;
}

static void finish_window(Sched& S, Job& j) {
    const Vocab& v = S.c->vocab;
    const whisper_full_params& p = S.p;
    const int seek_delta = j.seek_delta;
    const int result_len = j.result_len;
    const auto& toks = j.tokens;
    const bool is_no_speech = (j.no_speech_prob > p.no_speech_thold && j.avg_logprobs < p.logprob_thold);
    std::vector<int> past;
    if (j.prompt.front() == v.token_prev)
        past.insert(past.end(), j.prompt.begin() + 1, j.prompt.end() - j.prompt_init.size());
    for (int i = 0; i < result_len && !is_no_speech && i < (int)toks.size(); ++i) past.push_back(toks[i].id);
    j.prompt_past.swap(past);
    const size_t n_before = j.result.size();
    if (!toks.empty() && !is_no_speech) {
        int i0 = 0;
        int64_t t0 = j.seek + 2 * (toks.front().tid - v.token_beg);
        std::string text;
        for (int i = 0; i < (int)toks.size(); i++) {
            if (p.print_special || toks[i].id < v.token_eot) text += v.id_to_token[toks[i].id];
            if (toks[i].id > v.token_beg && !p.single_segment) {
                const int64_t t1 = j.seek + 2 * (toks[i].tid - v.token_beg);
                if (!text.empty()) {
                    j.result.push_back({t0, t1, text, j.no_speech_prob, {}});
                    for (int k = i0; k <= i; k++) j.result.back().tokens.push_back(toks[k]);
                }
                text = "";
                while (i < (int)toks.size() && toks[i].id > v.token_beg) i++;
                i--;
                t0 = t1;
                i0 = i + 1;
            }
        }
        if (!text.empty()) {
            const int64_t t1 = j.seek + seek_delta;
            j.result.push_back({t0, t1, text, j.no_speech_prob, {}});
            for (int k = i0; k < (int)toks.size(); k++) j.result.back().tokens.push_back(toks[k]);
        }
    }
    j.n_new_segments = (int)(j.result.size() - n_before);
    j.dec.seek = j.seek;
    j.dec.temp_idx = j.temp_idx;
    j.dec.no_speech = is_no_speech;
    j.dec.no_speech_prob = j.no_speech_prob;
    j.decisions.push_back(j.dec);
    j.seek += seek_delta;
    j.phase = (j.seek + 10 >= j.seek_end) ? PH_DONE : PH_ENCODE;
}

static void attempt_done(Sched& S, Job& j) {
    if (!j.failed) {
        j.tokens.resize(j.result_len);
        score_seq(S.p, j);
        if (j.result_len > 32 && j.entropy < S.p.entropy_thold) j.failed = true;
    }
    if (j.temp_idx == 0) {  // the greedy attempt's outcome (comparable with whisper.cpp bit for bit)
        j.dec = whisper_mi355x_window_decision{};
        j.dec.failed0 = j.failed;
        j.dec.logprob_fail0 = j.avg_logprobs < S.p.logprob_thold;
        j.dec.result_len0 = j.result_len;
        j.dec.avg_logprob0 = (float)j.avg_logprobs;
        j.dec.entropy0 = (float)j.entropy;
    }
    bool success = true;
    if (j.temp_idx != (int)S.temps.size() - 1)
        if (j.failed || j.avg_logprobs < S.p.logprob_thold) success = false;
    if (!success) {
        j.temp_idx++;
        j.phase = PH_PREFILL;
        return;
    }
    finish_window(S, j);
}

// teacher-forcing hook (FullOpts::spot): the raw logits rows of the spot jobs among `act` (row r of
// w.logits belongs to act[r]) for step `step` of each
static void copy_spot_logits(Sched& S, const std::vector<int>& act) {
    if (!S.o.spot_logits || S.o.n_spot <= 0) return;
    Workspace& w = S.s->ws;
    const size_t V = S.c->hp.n_vocab;
    for (int r = 0; r < (int)act.size(); r++)
        for (int k = 0; k < S.o.n_spot; k++)
            if (S.o.spot[k] == act[r]) {
                const int step = S.jobs[act[r]].step;
                if (step < 0 || step >= S.o.fixed_tokens) continue;
                WM_CHECK(hipMemcpyAsync(S.o.spot_logits + ((size_t)step * S.o.n_spot + k) * V, w.logits + (size_t)r * V,
                                        V * 4, hipMemcpyDeviceToHost, S.s->stream));
            }
    WM_CHECK(hipStreamSynchronize(S.s->stream));
}

// one whisper_full "sample + update" iteration for token index j.step; returns true if decoding continues
static bool process_step(Sched& S, Job& j, const TokOut& r, const float* probs_row) {
    const Vocab& v = S.c->vocab;
    const whisper_full_params& p = S.p;
    const int i = j.step;
    const float t = S.temps[j.temp_idx];
    TokenData td;
    td.tid = r.tid; td.pt = r.pt; td.ptsum = r.ptsum;
    if (t < 1e-6f) {
        td.id = r.id; td.p = r.p; td.plog = r.plog;
    } else {
        const int n = v.n_vocab;
        std::discrete_distribution<> dist(probs_row, probs_row + n);
        td.id = dist(*j.rng);
        td.p = probs_row[td.id];
        td.plog = probs_row[n + td.id];
        if (td.id >= v.token_beg) { td.tid = td.id; td.pt = td.p; }
        else { td.tid = r.tid; td.pt = r.pt; }
    }
    if (S.o.forced && S.o.fixed_tokens > 0) td.id = S.o.forced[(long)j.slot * S.o.fixed_tokens + i];
    j.tokens.push_back(td);
    j.sum_logprobs_all += td.plog;
    S.decoded++;
    const int delta_min = 10;
    if (td.id > v.token_beg) {
        const int sd_new = 2 * (td.id - v.token_beg);
        if (j.has_ts && j.seek_delta > sd_new && j.result_len < i && S.o.fixed_tokens <= 0) {
            j.failed = true;
            return false;
        }
        j.seek_delta = sd_new;
        j.result_len = i + 1;
        j.has_ts = true;
    }
    if (S.o.fixed_tokens > 0) {
        if (i == S.n_max_steps - 1) {  // fixed-work mode: one full window per chunk
            j.result_len = S.n_max_steps;
            j.seek_delta = 100 * WHISPER_CHUNK_SIZE;
            j.completed = true;
            return false;
        }
    } else if (td.id == v.token_eot || (p.max_tokens > 0 && i >= p.max_tokens) ||
               (j.has_ts && j.seek + j.seek_delta + delta_min >= j.seek_end)) {
        if (j.result_len == 0 && !p.no_timestamps) {
            if (j.seek + j.seek_delta + delta_min >= j.seek_end) j.result_len = i + 1;
            else { j.failed = true; return false; }
        }
        if (p.single_segment || p.no_timestamps) { j.result_len = i + 1; j.seek_delta = 100 * WHISPER_CHUNK_SIZE; }
        j.completed = true;
        return false;
    }
    if (S.o.fixed_tokens <= 0 && i == S.n_max_steps - 1 &&
        (j.result_len == 0 || j.seek_delta < 100 * WHISPER_CHUNK_SIZE / 2)) {
        j.failed = true;
        return false;
    }
    // whisper.cpp's loop runs i < n_max: after the last iteration nothing more is sampled (its
    // trailing decode cannot change the result, so it is skipped here)
    if (i + 1 >= S.n_max_steps) return false;
    return true;
}

// logits kernel over the rows of `act` jobs (row r of w.logits belongs to act[r]) + D2H
static bool logits_prepare(Sched& S, const std::vector<int>& act, bool want_nosp) {
    Workspace& w = S.s->ws;
    const int n = (int)act.size();
    bool any_probs = false;
    for (int r = 0; r < n; r++) {
        fill_ctl(S, S.jobs[act[r]], w.h_ctl[r], want_nosp);
        any_probs |= w.h_ctl[r].want_probs != 0;
    }
    WM_CHECK(hipMemcpyAsync(w.ctl, w.h_ctl, n * sizeof(SeqCtl), hipMemcpyHostToDevice, S.s->stream));
    return any_probs;
}
static void logits_launch(Context* c, whisper_state* s, int n) {
    Workspace& w = s->ws;
    KT kt(s, K_LOGITS, (double)n * c->hp.n_vocab * 4);
    launch_logits(w.logits, c->hp.n_vocab, w.ctl, n, c->vid, w.tout, w.probs, w.lrec, s->stream);
}
static void logits_finish(Sched& S, int n, bool any_probs, std::vector<std::vector<float>>& probs_rows) {
    Context* c = S.c;
    Workspace& w = S.s->ws;
    hipStream_t st = S.s->stream;
    WM_CHECK(hipMemcpyAsync(w.h_tout, w.tout, n * sizeof(TokOut), hipMemcpyDeviceToHost, st));
    probs_rows.assign(n, {});
    if (any_probs) {  // sampling clips (t > 0): probs and logprobs rows for std::discrete_distribution
        const size_t V = c->hp.n_vocab;
        for (int r = 0; r < n; r++)
            if (w.h_ctl[r].want_probs) {
                probs_rows[r].resize(2 * V);
                WM_CHECK(hipMemcpyAsync(probs_rows[r].data(), w.probs + (size_t)r * 2 * V, 2 * V * 4, hipMemcpyDeviceToHost, st));
            }
    }
    WM_CHECK(hipStreamSynchronize(st));
}
static void run_logits(Sched& S, const std::vector<int>& act, bool want_nosp, std::vector<std::vector<float>>& probs_rows) {
    const bool any = logits_prepare(S, act, want_nosp);
    logits_launch(S.c, S.s, (int)act.size());
    logits_finish(S, (int)act.size(), any, probs_rows);
}

// One decode step (decoder over n active clips + logits kernel) as a replayed hipGraph: the host
// cost of ~11 launches per layer is paid once per distinct n at capture time.
// After a persistent launch gave up, the state's steps take the per-kernel path for this long (a co-tenant
// holding CUs would otherwise cost the 50 ms timeout on every step)
static const double kPdecBackoffMs = 1000.0;

// the persistent launch's error word on the device (null for the launch chain)
static const unsigned* pd_err_ptr(Context* c, whisper_state* s, int pd) {
    const Hparams& hp = c->hp;
    Workspace& w = s->ws;
    if (pd == 1) return (const unsigned*)((const char*)w.pd_sync + pdec_granules(hp.n_text_state, hp.n_text_layer, hp.n_text_head).err_bytes);
    return nullptr;
}
static size_t ring_slot_bytes(const Workspace& w) { return (size_t)w.cap_jobs * sizeof(TokOut) + 16; }

// The decode graph of n rows on the state's current path (pd: 0 launch chain, 1 persistent step, 2 batched
// chain), instance `par` (captured on first use; graphs of a persistent path captured under an older stamps
// pointer / spin limit are retired first). par 0: the per-step path's; par 1, 2: the pipelined path's two
// instances, which end with the device-side advance writing the step's results to ring slot par - 1.
static whisper_state::DecGraph* dec_graph(Context* c, whisper_state* s, int n, int pd, int par) {
    const int sig = dec_path_sig();
    // read once: a setter stores its value before it bumps the generation, so a graph captured below under
    // generation `gen` holds that generation's (or a newer) stamps pointer and spin limit, and is retired later
    const int gen = g_pdec_gen.load(std::memory_order_acquire);
    for (size_t i = 0; i < s->dec_graphs.size();) {
        auto& g = s->dec_graphs[i];
        if (g.pdec && g.gen != gen) {
            hipGraphExecDestroy(g.exec);
            for (auto& e : g.ev) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
            s->dec_graphs.erase(s->dec_graphs.begin() + i);
        } else {
            i++;
        }
    }
    for (auto& g : s->dec_graphs)
        if (g.n_tok == n && g.n_rows == n && g.mask == s->ktime_mask && g.direct == s->direct && g.sig == sig && g.pdec == pd &&
            g.par == par)
            return &g;
    whisper_state::DecGraph g{n, n, s->ktime_mask, s->direct, sig, pd, gen, par, nullptr, {}};
    hipGraph_t graph;
    s->capture_ev = &g.ev;
    s->pipe_capture = par > 0;
    WM_CHECK(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
    decoder_launch(c, s, n, n, true, s->direct);
    logits_launch(c, s, n);
    s->pipe_capture = false;
    if (par > 0) {
        Workspace& w = s->ws;
        char* slot = w.ring + (par - 1) * ring_slot_bytes(w);
        launch_decode_advance(n, w.cap_tok, c->vid.beg, w.tout, w.tok, w.ctl, (TokOut*)slot, pd_err_ptr(c, s, pd),
                              (unsigned*)(slot + (size_t)w.cap_jobs * sizeof(TokOut)), s->stream);
    }
    WM_CHECK(hipStreamEndCapture(s->stream, &graph));
    s->capture_ev = nullptr;
    WM_CHECK(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
    WM_CHECK(hipGraphDestroy(graph));
    s->dec_graphs.push_back(std::move(g));
    return &s->dec_graphs.back();
}

// persistent launches of different states of this process on one device never overlap: two of them could hold
// half the CUs each. A pipelined run holds its device's lock for the whole run (a step is always in flight), so
// persistent steps of other threads on that device wait for it (documented). A caller's
// abort callback runs under the lock; if it calls back into the library on the same device from the same thread,
// that thread already holds the lock and does not take it again (g_pdec_held): its persistent launch then relies
// on the launch's bounded waits (a launch whose workgroups cannot all become resident gives up and the step
// re-runs on the per-kernel path) instead of deadlocking the thread on itself.
static std::mutex g_pdec_run_mu[16];
static thread_local unsigned g_pdec_held = 0;  // devices whose lock this thread holds (bit per device & 15)
struct PdecRunLock {
    int dev;
    bool owns = false;
    explicit PdecRunLock(int device, bool take = true) : dev(device & 15) {
        if (take) lock();
    }
    void lock() {
        if (owns || (g_pdec_held >> dev & 1)) return;
        g_pdec_run_mu[dev].lock();
        g_pdec_held |= 1u << dev;
        owns = true;
    }
    ~PdecRunLock() {
        if (!owns) return;
        g_pdec_held &= ~(1u << dev);
        g_pdec_run_mu[dev].unlock();
    }
};

// the decode path of a step of n rows (and its buffers prepared)
static int dec_path_prepare(Context* c, whisper_state* s, int n) {
    s->pdec_off = s->pdec_give_ups > 0 && now_ms() < s->pdec_off_until;
    s->step_rows = n;
    const int pd = pdec_use(c, s, n, s->direct) ? 1 : 0;
    if (pd) pdec_prepare(c, s);
    return pd;
}

static void decode_step(Sched& S, const std::vector<int>& act, std::vector<std::vector<float>>& probs_rows) {
    Context* c = S.c;
    whisper_state* s = S.s;
    const int n = (int)act.size();
    decoder_upload(c, s, n, n, false);
    const bool any = logits_prepare(S, act, false);
    const double t_step = now_ms();
    const int pd = dec_path_prepare(c, s, n);
    whisper_state::DecGraph* G = dec_graph(c, s, n, pd, 0);
    if (!G->pdec) {
        WM_CHECK(hipGraphLaunch(G->exec, s->stream));
        logits_finish(S, n, any, probs_rows);
        kt_flush_graph(s, *G);
        return;
    }
    // A persistent launch (the one-launch step, or the chain's launches) needs its 256 workgroups resident
    // together: persistent steps of different states (threads) of this process on one device never overlap,
    // so two of them cannot hold half the CUs each (steps on different devices do not wait for each other)
    bool gave_up;
    {
        PdecRunLock lk(c->device);
        WM_CHECK(hipGraphLaunch(G->exec, s->stream));
        logits_finish(S, n, any, probs_rows);
        gave_up = *s->ws.h_pd_err != 0;
    }
    kt_flush_graph(s, *G);
    if (!gave_up) return;
    // the launch gave up (a wait timed out: not every workgroup became resident): the step again on
    // the per-kernel path, which rewrites everything the launch may have written (the self K/V rows of
    // this position); counted (whisper_mi355x_pdec_give_ups) and followed by kPdecBackoffMs of steps on
    // the per-kernel path
    static bool warned = false;
    if (!warned) fprintf(stderr, "whisper_mi355x: persistent decode step timed out; step re-run on the per-kernel path\n");
    warned = true;
    *s->ws.h_pd_err = 0;
    s->pdec_block = true;
    try {
        decoder_launch(c, s, n, n, true, s->direct);
        logits_launch(c, s, n);
        logits_finish(S, n, any, probs_rows);
    } catch (...) {
        s->pdec_block = false;
        throw;
    }
    s->pdec_block = false;
    s->pdec_give_ups++;
    g_pdec_give_ups_total++;
    s->pdec_off_until = now_ms() + kPdecBackoffMs;
    s->pdec_lost_ms += now_ms() - t_step;
}

// Pipelined greedy decoding. The per-step path waits for a step's 32-byte results before it launches the next
// step, so every step pays the host's round trip (copy, synchronise, process_step, upload, launch: ~40-60 us,
// a fifth of a base-model persistent step). Here a small kernel advances every row's input token, position and
// logits-rule state on the device after the step (launch_decode_advance: the token the logits kernel chose, as
// process_step + fill_ctl would), the next step's graph is launched at once, and the host processes step k
// while step k + 1 runs. The results are the per-step path's bits: the same graphs on the same inputs. A row
// whose attempt ends at step k has had step k + 1 computed for it (its self-K/V row at the next position, never
// read: a new attempt prefills over it); the other rows' step k + 1 results are used, since a row's results
// do not depend on the other rows. Taken only where the host has nothing to decide per step: greedy attempts
// (no sampling), no forced tokens or logits hooks, no other job in another phase, and attempts that already
// decoded pipe_min_step() tokens (24; the speculative step at an attempt's end costs one step, which pays off only
// over a long attempt). WHISPER_MI355X_PIPE=0 turns it off.
static int pipe_min_step() {  // kPipeMinStep, or WHISPER_MI355X_PIPE_MIN (tests: exercise short attempts)
    const char* e = getenv("WHISPER_MI355X_PIPE_MIN");
    return e ? atoi(e) : 24;
}
static bool pipe_on() {  // (read per call: tests compare both paths in one process)
    const char* e = getenv("WHISPER_MI355X_PIPE");
    return !e || atoi(e) != 0;
}

static bool pipe_ok(Sched& S, const std::vector<int>& act) {
    if (!pipe_on() || S.o.forced || (S.o.spot_logits && S.o.n_spot > 0)) return false;
    for (size_t k = 0; k < S.jobs.size(); k++) {
        const Job& j = S.jobs[k];
        if (j.phase == PH_DONE) continue;
        if (j.phase != PH_DECODE) return false;
        if (S.temps[j.temp_idx] >= 1e-6f || j.step < pipe_min_step()) return false;
    }
    return !act.empty();
}

// Everything about a decode step of n rows that can change a row's bits with n: the path (persistent step,
// small-M GEMMs, launch chain), the cache-form cross-attention kernel (the wide one up to
// attn_cross_wide_max() rows), the direct form's key-split count (xattn_splits), the logits GEMM's kernel
// (gemm.hip launch_t: the unsplit 64-row kernel up to 64 rows, gemm_dec_kernel above) and the number of
// 128-row groups (dec_groups). Equal keys: a row's results at n and at n' rows are the same bits.
static long step_variant(Context* c, whisper_state* s, int n) {
    const int pd = pdec_use(c, s, n, s->direct) ? 1 : 0;
    const bool small = (c->quant && n <= quant_small_max()) || n <= small_m_max();
    const bool wide = !s->direct && n <= attn_cross_wide_max();
    const int sp = s->direct ? xattn_splits(n, c->hp.n_audio_ctx) : 0;
    const bool lg64 = n <= 64;
    return pd | (long)small << 2 | (long)wide << 3 | (long)sp << 4 | (long)lg64 << 9 | (long)dec_groups(n) << 10;
}

// the host inputs of a decode step of the `act` jobs (their next token, position, slot, logits row)
static void step_inputs(Sched& S, const std::vector<int>& act) {
    Workspace& w = S.s->ws;
    int* hi = w.h_ints;
    for (int r = 0; r < (int)act.size(); r++) {
        const Job& j = S.jobs[act[r]];
        hi[r] = j.tokens.back().id;
        hi[w.cap_tok + r] = (int)j.prompt.size() + j.step;
        hi[2 * w.cap_tok + r] = j.slot;
        hi[5 * w.cap_tok + r] = r;
    }
}

// Re-run the step of the `act` rows on the per-kernel path after its persistent launch gave up (the device
// inputs as uploaded by `upload`); results in w.h_tout. Counted like decode_step's give-ups.
static void pipe_give_up(Sched& S, const std::vector<int>& act, bool upload, double t0) {
    Context* c = S.c;
    whisper_state* s = S.s;
    const int n = (int)act.size();
    WM_CHECK(hipStreamSynchronize(s->stream));
    static bool warned = false;
    if (!warned) fprintf(stderr, "whisper_mi355x: persistent decode step timed out; step re-run on the per-kernel path\n");
    warned = true;
    if (upload) {
        step_inputs(S, act);
        decoder_upload(c, s, n, n, false);
        logits_prepare(S, act, false);
    }
    *s->ws.h_pd_err = 0;
    std::vector<std::vector<float>> probs_rows;
    s->pdec_block = true;
    try {
        decoder_launch(c, s, n, n, true, s->direct);
        logits_launch(c, s, n);
        logits_finish(S, n, false, probs_rows);
    } catch (...) {
        s->pdec_block = false;
        throw;
    }
    s->pdec_block = false;
    s->pdec_give_ups++;
    g_pdec_give_ups_total++;
    s->pdec_off_until = now_ms() + kPdecBackoffMs;
    s->pdec_lost_ms += now_ms() - t0;
}

// Decode the `act` jobs step after step with the next step in flight while the host processes the last one,
// until an attempt ends (or the caller's abort callback fires: returns true); the jobs are left exactly as the
// per-step path leaves them: every step it ran is processed, except the one in flight when the callback asked
// to abort (the per-step path would not have started it). The callback is asked after every step; when an
// attempt ended, the main loop asks it again before its next step (one call more than the per-step path).
static bool decode_pipelined(Sched& S, const std::vector<int>& act) {
    Context* c = S.c;
    whisper_state* s = S.s;
    Workspace& w = s->ws;
    const whisper_full_params& p = S.p;
    const int n = (int)act.size();
    hipStream_t st = s->stream;
    const size_t slot_b = ring_slot_bytes(w);
    if (!w.h_ring) {  // written by the advance kernel over the bus (coherent pinned memory), read after the event
        WM_CHECK(hipHostMalloc((void**)&w.h_ring, 2 * slot_b, hipHostMallocCoherent | hipHostMallocMapped));
        WM_CHECK(hipHostGetDevicePointer((void**)&w.ring, w.h_ring, 0));
    }
    for (auto& e : w.ring_ev)
        if (!e) WM_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    step_inputs(S, act);
    decoder_upload(c, s, n, n, false);
    logits_prepare(S, act, false);
    const int pd = dec_path_prepare(c, s, n);
    dec_graph(c, s, n, pd, 1);
    dec_graph(c, s, n, pd, 2);  // (may grow dec_graphs: the pointers are taken after both exist)
    whisper_state::DecGraph* G[2] = {dec_graph(c, s, n, pd, 1), dec_graph(c, s, n, pd, 2)};
    PdecRunLock lk(c->device, pd != 0);
    double t_step = now_ms();
    WM_CHECK(hipGraphLaunch(G[0]->exec, st));
    WM_CHECK(hipEventRecord(w.ring_ev[0], st));
    for (int k = 0;; k++) {
        const int par = k & 1;
        char* hslot = w.h_ring + par * slot_b;
        // step k produces token j.step + 1 of each job; a job continues past it only if j.step + 2 < n_max. Step
        // k + 1 runs for every row, also for a row whose attempt ends at step k, so it is launched only when every
        // row's next position fits the self cache and the positional table (prompt + step + 1 < n_text_ctx: a
        // 229-token prompt at the 220-token limit would write row 448); otherwise the main loop's
        // per-step path decodes the rows that continue
        bool more = false, fits = true;
        for (int r = 0; r < n; r++) {
            const Job& j = S.jobs[act[r]];
            more |= j.step + 2 < S.n_max_steps;
            fits &= (int)j.prompt.size() + j.step + 1 < c->hp.n_text_ctx;
        }
        more = more && fits;
        if (more) {
            WM_CHECK(hipGraphLaunch(G[par ^ 1]->exec, st));
            WM_CHECK(hipEventRecord(w.ring_ev[par ^ 1], st));
        }
        s->cur_self_work += (double)n * c->hp.n_text_head * 64 * 2 * 2;  // (kernel timing: one more key per row)
        WM_CHECK(hipEventSynchronize(w.ring_ev[par]));
        kt_flush_graph(s, *G[par]);
        const TokOut* out = (const TokOut*)hslot;
        if (pd && *(const unsigned*)(hslot + (size_t)w.cap_jobs * sizeof(TokOut))) {
            // step k gave up: re-run it on the per-kernel path from the host's inputs, then leave
            pipe_give_up(S, act, true, t_step);
            for (int r = 0; r < n; r++) S.jobs[act[r]].step++;
            for (int r = 0; r < n; r++) {
                Job& j = S.jobs[act[r]];
                if (!process_step(S, j, w.h_tout[r], nullptr)) attempt_done(S, j);
            }
            return false;
        }
        for (int r = 0; r < n; r++) S.jobs[act[r]].step++;
        bool ended = false;
        for (int r = 0; r < n; r++) {
            Job& j = S.jobs[act[r]];
            if (!process_step(S, j, out[r], nullptr)) {
                attempt_done(S, j);
                ended = true;
            }
        }
        const bool aborted = p.abort_callback && p.abort_callback(p.abort_callback_user_data);
        if (!ended && !aborted && more) {
            t_step = now_ms();
            continue;
        }
        if (more) {
            // step k + 1 ran for every row: its results stand for the rows still decoding if a step of that
            // many rows computes the same bits (step_variant); otherwise the main loop runs step k + 1 again
            // for them from the host's inputs (the speculative one only wrote their self-K/V rows at the
            // next position, which the re-run writes again)
            WM_CHECK(hipMemcpyAsync(w.h_tout, w.tout, (size_t)n * sizeof(TokOut), hipMemcpyDeviceToHost, st));
            WM_CHECK(hipStreamSynchronize(st));
            kt_flush_graph(s, *G[par ^ 1]);
            if (aborted) {
                if (pd) *w.h_pd_err = 0;
                return true;
            }
            std::vector<int> still;
            for (int r = 0; r < n; r++)
                if (S.jobs[act[r]].phase == PH_DECODE) still.push_back(r);
            if (still.empty() || step_variant(c, s, (int)still.size()) != step_variant(c, s, n)) {
                if (pd) *w.h_pd_err = 0;  // (a discarded step's give-up is not one)
                return false;
            }
            if (pd && *(const unsigned*)(w.h_ring + (par ^ 1) * slot_b + (size_t)w.cap_jobs * sizeof(TokOut))) {
                // its persistent launch gave up: the step again, for all n rows, from the host's inputs (the
                // graph's own advance has moved the device's past step k + 1)
                pipe_give_up(S, act, true, now_ms());
            }
            for (int r : still) {
                Job& j = S.jobs[act[r]];
                j.step++;
                if (!process_step(S, j, w.h_tout[r], nullptr)) attempt_done(S, j);
            }
        }
        return aborted;
    }
}

// Batches above kPairMin clips run as two independent halves at
// once: the first on this state, the second on a twin state (its own streams, workspace and decode
// graphs, kept with this state for later calls) from a second host thread, and the twin's per-clip
// results are appended. Each half is exactly a batch of its own clips (the same bits as two separate
// calls), and one half's launch chain runs in the other's latency gaps: two 128-chunk large-v3 batches
// in flight measured 3720 vs 3201 audio-s/s back to back (profiles/r03_overlap_two_batches.txt),
// where one 256-row decode step ran as two lockstep row groups before.
static const int kPairMin = 128;
std::atomic<long> g_decoded_tokens_total{0};

static int full_batch_one(Context* c, whisper_state* s, const whisper_full_params& p, const float* const* pcm, const int* n,
                          int n_jobs, bool on_device, const FullOpts& o, bool single_api);

int full_batch(Context* c, whisper_state* s, const whisper_full_params& p, const float* const* pcm, const int* n,
               int n_jobs, bool on_device, const FullOpts& o, bool single_api) {
    if (single_api || n_jobs <= kPairMin) return full_batch_one(c, s, p, pcm, n, n_jobs, on_device, o, single_api);
    WM_CHECK(hipSetDevice(c->device));
    if (!s->twin) s->twin = create_state(c);
    whisper_state* t = s->twin;
    t->ktime_mask = s->ktime_mask;
    const int na = (n_jobs + 1) / 2;
    int ra = 0, rb = 0;
    std::exception_ptr ea, eb;
    // the caller's abort callback need not be thread-safe: both halves reach it through one mutex
    whisper_full_params pp = p;
    struct AbortGate { std::mutex mu; ggml_abort_callback cb; void* ud; } gate{{}, p.abort_callback, p.abort_callback_user_data};
    if (p.abort_callback) {
        pp.abort_callback = [](void* u) -> bool {
            AbortGate* g = (AbortGate*)u;
            std::lock_guard<std::mutex> lk(g->mu);
            return g->cb(g->ud);
        };
        pp.abort_callback_user_data = &gate;
    }
    // teacher forcing (a parity-test hook) by halves: each half sees its own jobs' forced rows, and the spot
    // jobs of the other half never match (-1); both write their own rows of the caller's spot_logits
    FullOpts oa = o, ob = o;
    std::vector<int> spot_a, spot_b;
    if (o.n_spot > 0 && o.spot) {
        for (int k = 0; k < o.n_spot; k++) {
            spot_a.push_back(o.spot[k] < na ? o.spot[k] : -1);
            spot_b.push_back(o.spot[k] >= na ? o.spot[k] - na : -1);
        }
        oa.spot = spot_a.data();
        ob.spot = spot_b.data();
    }
    if (o.forced) ob.forced = o.forced + (long)na * o.fixed_tokens;
    std::thread th([&] {
        try {
            rb = full_batch_one(c, t, pp, pcm + na, n + na, n_jobs - na, on_device, ob, false);
        } catch (...) {
            eb = std::current_exception();
        }
    });
    try {
        ra = full_batch_one(c, s, pp, pcm, n, na, on_device, oa, false);
    } catch (...) {
        ea = std::current_exception();
    }
    th.join();
    if (eb) recover_state(t);
    if (ea) std::rethrow_exception(ea);
    if (eb) std::rethrow_exception(eb);
    if (ra) return ra;
    if (rb) return rb;
    for (int j = 0; j < n_jobs - na; j++) {
        s->results.push_back(std::move(t->results[j]));
        s->lang_ids.push_back(t->lang_ids[j]);
        s->decisions.push_back(std::move(t->decisions[j]));
    }
    s->decoded_tokens += t->decoded_tokens;
    s->pdec_give_ups += t->pdec_give_ups;
    s->pdec_lost_ms += t->pdec_lost_ms;
    t->pdec_give_ups = 0;
    t->pdec_lost_ms = 0;
    // the halves ran concurrently: a phase lasted as long as its slower half; kernel time adds up
    for (int k = 0; k < 5; k++) s->phase_ms[k] = std::max(s->phase_ms[k], t->phase_ms[k]);
    for (int k = 0; k < K_NCLASS; k++) {
        s->kstat[k].ms += t->kstat[k].ms;
        s->kstat[k].work += t->kstat[k].work;
        s->kstat[k].count += t->kstat[k].count;
        t->kstat[k] = KStat();
    }
    return 0;
}

static int full_batch_one(Context* c, whisper_state* s, const whisper_full_params& p, const float* const* pcm, const int* n,
                          int n_jobs, bool on_device, const FullOpts& o, bool single_api) {
    WM_CHECK(hipSetDevice(c->device));
    if (p.strategy != WHISPER_SAMPLING_GREEDY) {
        fprintf(stderr, "whisper_mi355x: beam search is not implemented (the reference uses Greedy, whisper.rs:88)\n");
        return -100;
    }
    if (p.greedy.best_of > 1) {
        // whisper.cpp uses best_of only for sampled (t > 0) fallback attempts: t = 0 is unaffected.
        // Sampled attempts here run one candidate per clip (the reference's Greedy{best_of: 1}).
        static bool warned = false;
        if (!warned) fprintf(stderr, "whisper_mi355x: greedy best_of=%d: fallback attempts sample 1 candidate\n", p.greedy.best_of);
        warned = true;
    }
    ensure_expanded(c, s->stream);  // quantized files: before anything is captured
    Sched S;
    S.c = c; S.s = s; S.p = p; S.o = o; S.single_api = single_api;
    const Vocab& v = c->vocab;
    const Hparams& hp = c->hp;
    s->results.assign(n_jobs, {});
    s->lang_ids.assign(n_jobs, 0);
    s->decisions.assign(n_jobs, {});
    s->decoded_tokens = 0;
    double t0 = now_ms();
    s->direct = pick_direct(c, n_jobs);
    ensure_ws(c, s, n_jobs);
    compute_mel(c, s, pcm, n, n_jobs, on_device);
    S.t_mel = now_ms() - t0;

    if (p.temperature_inc > 0.0f && o.fixed_tokens <= 0)
        for (float t = p.temperature; t < 1.0f + 1e-6f; t += p.temperature_inc) S.temps.push_back(t);
    if (S.temps.empty()) S.temps.push_back(p.temperature);
    const int n_max = hp.n_text_ctx / 2 - 4;
    S.n_max_steps = o.fixed_tokens > 0 ? o.fixed_tokens : n_max;
    const bool need_lang = p.language == nullptr || strlen(p.language) == 0 || strcmp(p.language, "auto") == 0 || p.detect_language;
    std::vector<int> init_prompt_tokens;
    if (!p.prompt_tokens && p.initial_prompt) init_prompt_tokens = tokenize(v, p.initial_prompt);
    else if (p.prompt_tokens && p.prompt_n_tokens > 0) init_prompt_tokens.assign(p.prompt_tokens, p.prompt_tokens + p.prompt_n_tokens);
    const bool is_distil = hp.n_text_layer == 2 && hp.n_vocab != 51866;
    const bool no_ts = p.no_timestamps || is_distil;
    S.p.no_timestamps = no_ts;

    S.jobs.resize(n_jobs);
    for (int k = 0; k < n_jobs; k++) {
        Job& j = S.jobs[k];
        j.slot = k;
        j.n_samples = n[k];
        j.n_len = mel_n_len(n[k]);
        j.n_len_org = mel_n_len_org(n[k]);
        j.seek_start = p.offset_ms / 10;
        j.seek_end = p.duration_ms == 0 ? j.n_len_org : j.seek_start + p.duration_ms / 10;
        j.seek = j.seek_start;
        j.rng = single_api ? &s->rng : &j.own_rng;
        if (single_api) j.prompt_past = s->prompt_past;
        if (p.no_context) j.prompt_past.clear();
        if (!init_prompt_tokens.empty()) {
            for (int t : init_prompt_tokens) j.prompt_past.push_back(t);
            std::rotate(j.prompt_past.begin(), j.prompt_past.end() - init_prompt_tokens.size(), j.prompt_past.end());
        }
        if (need_lang && 0 >= j.n_len_org) {  // whisper_full_with_state: failed auto-detect -> -3
            if (single_api) return -3;
            j.phase = PH_DONE;
            continue;
        }
        if (j.seek_end < j.seek_start + 10) { j.phase = PH_DONE; continue; }
        j.lang_pending = need_lang;
        if (!need_lang) j.lang_id = lang_index(p.language);
        j.phase = PH_ENCODE;
    }
    auto build_prompt_init = [&](Job& j) -> bool {
        j.prompt_init = {v.token_sot};
        if (v.is_multilingual()) {
            if (j.lang_id < 0) return false;
            j.prompt_init.push_back(v.token_sot + 1 + j.lang_id);
            j.prompt_init.push_back(p.translate ? v.token_translate : v.token_transcribe);
        }
        if (no_ts) j.prompt_init.push_back(v.token_not);
        return true;
    };
    for (auto& j : S.jobs)
        if (j.phase != PH_DONE && !j.lang_pending && !build_prompt_init(j)) return -7;

    Workspace& w = s->ws;
    std::vector<std::vector<float>> probs_rows;
    bool aborted = false;
    while (!aborted) {
        bool any = false;
        for (auto& j : S.jobs) any |= j.phase != PH_DONE;
        if (!any) break;
        // ---- encode every window that is due
        {
            std::vector<int> wj, ws_, wsl;
            for (int k = 0; k < n_jobs; k++) {
                Job& j = S.jobs[k];
                if (j.phase != PH_ENCODE) continue;
                if (single_api && p.progress_callback) {
                    const int prog = (100 * (j.seek - j.seek_start)) / std::max(1, j.seek_end - j.seek_start);
                    p.progress_callback(c->owner, s, prog, p.progress_callback_user_data);
                }
                if (j.seek + 10 >= j.seek_end && !j.lang_pending) { j.phase = PH_DONE; continue; }
                if (single_api && p.encoder_begin_callback &&
                    !p.encoder_begin_callback(c->owner, s, p.encoder_begin_callback_user_data)) {
                    aborted = true;
                    break;
                }
                if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) { aborted = true; break; }
                wj.push_back(k);
                ws_.push_back(j.lang_pending ? 0 : j.seek);
                wsl.push_back(j.slot);
            }
            if (aborted) break;
            if (!wj.empty()) {
                const double te = now_ms();
                encode_windows(c, s, wj.data(), ws_.data(), wsl.data(), (int)wj.size());
                S.t_enc += now_ms() - te;
                for (int k : wj) {
                    Job& j = S.jobs[k];
                    if (j.lang_pending) { j.phase = PH_LANG; continue; }
                    if (j.seek > j.seek_start && j.seek + 500 >= j.seek_end) j.prompt_past.clear();
                    j.temp_idx = 0;
                    j.phase = PH_PREFILL;
                }
            }
        }
        // ---- language detection: decode [sot] at pos 0, argmax over the language logits
        {
            std::vector<int> act;
            for (int k = 0; k < n_jobs; k++) if (S.jobs[k].phase == PH_LANG) act.push_back(k);
            if (!act.empty()) {
                const double tp = now_ms();
                const int na = (int)act.size();
                int* hi = w.h_ints;
                for (int r = 0; r < na; r++) {
                    hi[r] = v.token_sot; hi[w.cap_tok + r] = 0; hi[2 * w.cap_tok + r] = S.jobs[act[r]].slot;
                    hi[5 * w.cap_tok + r] = r;
                }
                decoder_forward(c, s, na, na);
                std::vector<float> lg((size_t)na * 100);
                for (int r = 0; r < na; r++)
                    WM_CHECK(hipMemcpyAsync(lg.data() + r * 100, w.logits + (size_t)r * hp.n_vocab + v.token_sot + 1, 100 * 4,
                                            hipMemcpyDeviceToHost, s->stream));
                WM_CHECK(hipStreamSynchronize(s->stream));
                S.t_prefill += now_ms() - tp;
                for (int r = 0; r < na; r++) {
                    Job& j = S.jobs[act[r]];
                    // whisper_lang_auto_detect_with_state: iterate g_lang (std::map, key order), sort desc
                    std::map<std::string, int> g_lang;
                    for (int i = 0; i < 100; i++) g_lang[k_lang_codes[i]] = i;
                    std::vector<std::pair<float, int>> ids;
                    for (auto& kv : g_lang) ids.emplace_back(lg[r * 100 + kv.second], kv.second);
                    std::sort(ids.begin(), ids.end(), [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first > b.first; });
                    j.lang_id = ids[0].second;
                    j.lang_pending = false;
                    if (!build_prompt_init(j)) return -7;
                    if (p.detect_language) { j.phase = PH_DONE; continue; }
                    if (j.seek == 0) {
                        j.temp_idx = 0;
                        j.phase = PH_PREFILL;
                    } else j.phase = PH_ENCODE;
                }
            }
        }
        // ---- prefill every attempt that is due
        {
            std::vector<int> act;
            for (int k = 0; k < n_jobs; k++) if (S.jobs[k].phase == PH_PREFILL) act.push_back(k);
            if (!act.empty()) {
                if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) { aborted = true; break; }
                const double tp = now_ms();
                int* hi = w.h_ints;
                int nt = 0;
                for (int r = 0; r < (int)act.size(); r++) {
                    Job& j = S.jobs[act[r]];
                    start_attempt(S, j);
                    for (int t = 0; t < (int)j.prompt.size(); t++) {
                        hi[nt] = j.prompt[t]; hi[w.cap_tok + nt] = t; hi[2 * w.cap_tok + nt] = j.slot;
                        nt++;
                    }
                    hi[5 * w.cap_tok + r] = nt - 1;
                }
                decoder_forward(c, s, nt, (int)act.size());
                run_logits(S, act, true, probs_rows);
                S.t_prefill += now_ms() - tp;
                copy_spot_logits(S, act);
                for (int r = 0; r < (int)act.size(); r++) {
                    Job& j = S.jobs[act[r]];
                    j.no_speech_prob = w.h_tout[r].nosp_prob;
                    if (process_step(S, j, w.h_tout[r], probs_rows[r].empty() ? nullptr : probs_rows[r].data())) j.phase = PH_DECODE;
                    else attempt_done(S, j);
                }
            }
        }
        // ---- one decode step for every clip that is decoding
        {
            std::vector<int> act;
            for (int k = 0; k < n_jobs; k++) if (S.jobs[k].phase == PH_DECODE) act.push_back(k);
            if (!act.empty() && pipe_ok(S, act)) {
                if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) { aborted = true; break; }
                const double td = now_ms();
                const bool ab = decode_pipelined(S, act);
                S.t_decode += now_ms() - td;
                if (ab) { aborted = true; break; }
            } else if (!act.empty()) {
                if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) { aborted = true; break; }
                const double td = now_ms();
                int* hi = w.h_ints;
                const int na = (int)act.size();
                for (int r = 0; r < na; r++) {
                    Job& j = S.jobs[act[r]];
                    hi[r] = j.tokens.back().id;
                    hi[w.cap_tok + r] = (int)j.prompt.size() + j.step;
                    hi[2 * w.cap_tok + r] = j.slot;
                    hi[5 * w.cap_tok + r] = r;
                }
                decode_step(S, act, probs_rows);
                S.t_decode += now_ms() - td;
                for (int r = 0; r < na; r++) S.jobs[act[r]].step++;
                copy_spot_logits(S, act);
                for (int r = 0; r < na; r++) {
                    Job& j = S.jobs[act[r]];
                    if (!process_step(S, j, w.h_tout[r], probs_rows[r].empty() ? nullptr : probs_rows[r].data())) attempt_done(S, j);
                }
            }
        }
        // ---- new-segment callback (whisper.h single-clip API)
        if (single_api && p.new_segment_callback) {
            Job& j = S.jobs[0];
            if (j.n_new_segments > 0) {
                s->results[0] = j.result;
                p.new_segment_callback(c->owner, s, j.n_new_segments,
                                       p.new_segment_callback_user_data);
                j.n_new_segments = 0;
            }
        }
    }
    for (int k = 0; k < n_jobs; k++) {
        s->results[k] = std::move(S.jobs[k].result);
        s->lang_ids[k] = S.jobs[k].lang_id;
        s->decisions[k] = std::move(S.jobs[k].decisions);
    }
    if (single_api && n_jobs > 0) {
        s->prompt_past = S.jobs[0].prompt_past;
        s->lang_id = S.jobs[0].lang_id;
    }
    kt_flush(s);
    s->decoded_tokens = S.decoded;
    g_decoded_tokens_total += S.decoded;
    s->phase_ms[0] = S.t_mel; s->phase_ms[1] = S.t_enc; s->phase_ms[2] = S.t_prefill; s->phase_ms[3] = S.t_decode;
    s->phase_ms[4] = S.t_logits;
    std::lock_guard<std::mutex> lk(c->timings_mu);
    c->timings.encode_ms += (float)S.t_enc;
    c->timings.decode_ms += (float)S.t_decode;
    c->timings.prompt_ms += (float)S.t_prefill;
    return 0;
}

}  // namespace wm
