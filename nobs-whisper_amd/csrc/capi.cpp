// extern "C" whisper.h entry points (include/whisper.h) and the MI355X extensions
// (include/whisper_mi355x.h). See include/whisper.h for the whisper.rs call site of each.
#include <cmath>
#include <cstring>
#include <string>
#include <thread>

#include <rccl/rccl.h>

#include "../../include/whisper_mi355x.h"
#include "engine.h"

namespace wm { extern int g_gemm_variant; extern int g_dec_splits; extern int g_dec_bm; extern unsigned long long* g_gemm_stamps; }
using namespace wm;

static Context* C(whisper_context* ctx) { return ctx ? &ctx->c : nullptr; }

// Engine errors (wm::Error: a HIP error such as out of memory, an unsupported shape) end the call
// with WHISPER_MI355X_ERR_RUNTIME and leave the context and the state usable; whisper-rs turns the
// non-zero return into WhisperError (whisper.rs:127-129) and the app logs and skips the chunk
// (state.rs:157-159).
template <typename F> static int guarded(whisper_state* s, F&& f) {
    try {
        return f();
    } catch (const wm::Error&) {
    } catch (const std::bad_alloc&) {
        fprintf(stderr, "whisper_mi355x: host out of memory\n");
    }
    if (s) recover_state(s);
    return WHISPER_MI355X_ERR_RUNTIME;
}

static DType env_dtype(DType def) {
    const char* e = getenv("WHISPER_MI355X_DTYPE");
    if (!e) return def;
    return (strcmp(e, "bf16") == 0 || strcmp(e, "BF16") == 0) ? DType::BF16 : DType::F16;
}

static whisper_context* make_ctx(const char* path, whisper_context_params cp, int dtype, bool load) {
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0) {
        fprintf(stderr, "whisper_mi355x: no HIP device available (this engine has no CPU path)\n");
        return nullptr;
    }
    const int dev = cp.gpu_device >= 0 && cp.gpu_device < n_dev ? cp.gpu_device : 0;
    whisper_context* w = new whisper_context();
    // dtype 2 = bf16 with the fp8 encoder GEMMs (large-v3-turbo fp8 config)
    w->c.fp8_enc = dtype == 2;
    if (dtype == 2) dtype = (int)DType::BF16;
    bool ok = false;
    try {
        ok = load_context(&w->c, path, dev, (DType)dtype, load);
    } catch (const wm::Error&) {
    } catch (const std::bad_alloc&) {
    }
    if (!ok) {
        free_context(&w->c);
        delete w;
        return nullptr;
    }
    if (w->c.quant && w->c.fp8_enc) {  // the e4m3 weights are quantized from compute-type matrices
        fprintf(stderr, "whisper_mi355x: fp8 mode needs an f16 model file; %s is block-quantized, fp8 off\n", path);
        w->c.fp8_enc = false;
    }
    w->c.owner = w;
    return w;
}

extern "C" {

const char* whisper_version(void) { return "1.7.6-mi355x"; }

struct whisper_context_params whisper_context_default_params(void) {
    whisper_context_params r;
    memset(&r, 0, sizeof(r));
    r.use_gpu = true;
    r.flash_attn = false;
    r.gpu_device = 0;
    r.dtw_token_timestamps = false;
    r.dtw_aheads_preset = WHISPER_AHEADS_NONE;
    r.dtw_n_top = -1;
    r.dtw_aheads.n_heads = 0;
    r.dtw_aheads.heads = nullptr;
    r.dtw_mem_size = 1024 * 1024 * 128;
    return r;
}
struct whisper_context_params* whisper_context_default_params_by_ref(void) {
    return new whisper_context_params(whisper_context_default_params());
}
void whisper_free_context_params(struct whisper_context_params* p) { delete p; }

struct whisper_full_params whisper_full_default_params(enum whisper_sampling_strategy strategy) {
    whisper_full_params r;
    memset(&r, 0, sizeof(r));
    r.strategy = strategy;
    r.n_threads = std::min(4, (int)std::thread::hardware_concurrency());
    r.n_max_text_ctx = 16384;
    r.offset_ms = 0;
    r.duration_ms = 0;
    r.translate = false;
    r.no_context = true;
    r.no_timestamps = false;
    r.single_segment = false;
    r.print_special = false;
    r.print_progress = true;
    r.print_realtime = false;
    r.print_timestamps = true;
    r.token_timestamps = false;
    r.thold_pt = 0.01f;
    r.thold_ptsum = 0.01f;
    r.max_len = 0;
    r.split_on_word = false;
    r.max_tokens = 0;
    r.debug_mode = false;
    r.audio_ctx = 0;
    r.tdrz_enable = false;
    r.suppress_regex = nullptr;
    r.initial_prompt = nullptr;
    r.prompt_tokens = nullptr;
    r.prompt_n_tokens = 0;
    r.language = "en";
    r.detect_language = false;
    r.suppress_blank = true;
    r.suppress_nst = false;
    r.temperature = 0.0f;
    r.max_initial_ts = 1.0f;
    r.length_penalty = -1.0f;
    r.temperature_inc = 0.2f;
    r.entropy_thold = 2.4f;
    r.logprob_thold = -1.0f;
    r.no_speech_thold = 0.6f;
    r.greedy.best_of = -1;
    r.beam_search.beam_size = -1;
    r.beam_search.patience = -1.0f;
    r.grammar_penalty = 100.0f;
    r.vad = false;
    r.vad_model_path = nullptr;
    r.vad_params.threshold = 0.5f;
    r.vad_params.min_speech_duration_ms = 250;
    r.vad_params.min_silence_duration_ms = 100;
    r.vad_params.max_speech_duration_s = INFINITY;
    r.vad_params.speech_pad_ms = 30;
    r.vad_params.samples_overlap = 0.1f;
    if (strategy == WHISPER_SAMPLING_GREEDY) r.greedy.best_of = 5;
    else { r.beam_search.beam_size = 5; r.beam_search.patience = -1.0f; }
    return r;
}
struct whisper_full_params* whisper_full_default_params_by_ref(enum whisper_sampling_strategy s) {
    return new whisper_full_params(whisper_full_default_params(s));
}
void whisper_free_params(struct whisper_full_params* p) { delete p; }

// ---- init / free ----------------------------------------------------------------------------------
struct whisper_context* whisper_init_from_file_with_params_no_state(const char* path, struct whisper_context_params p) {
    return make_ctx(path, p, (int)env_dtype(DType::F16), true);
}
struct whisper_context* whisper_init_from_file_with_params(const char* path, struct whisper_context_params p) {
    whisper_context* w = whisper_init_from_file_with_params_no_state(path, p);
    if (w) w->c.default_state = whisper_init_state(w);
    if (w && !w->c.default_state) { whisper_free(w); return nullptr; }
    return w;
}
struct whisper_context* whisper_init_from_buffer_with_params_no_state(void*, size_t, struct whisper_context_params) {
    fprintf(stderr, "whisper_mi355x: init from buffer is not supported; use a model file\n");
    return nullptr;
}
struct whisper_context* whisper_init_from_buffer_with_params(void* b, size_t n, struct whisper_context_params p) {
    return whisper_init_from_buffer_with_params_no_state(b, n, p);
}
struct whisper_context* whisper_init_with_params_no_state(struct whisper_model_loader*, struct whisper_context_params) {
    fprintf(stderr, "whisper_mi355x: custom model loaders are not supported; use a model file\n");
    return nullptr;
}
struct whisper_context* whisper_init_with_params(struct whisper_model_loader* l, struct whisper_context_params p) {
    return whisper_init_with_params_no_state(l, p);
}
struct whisper_state* whisper_init_state(struct whisper_context* ctx) {
    if (!ctx) return nullptr;
    whisper_state* s = nullptr;
    guarded(nullptr, [&] { s = new_state(&ctx->c); return 0; });
    return s;
}
int whisper_ctx_init_openvino_encoder_with_state(struct whisper_context*, struct whisper_state*, const char*, const char*, const char*) { return 1; }
int whisper_ctx_init_openvino_encoder(struct whisper_context*, const char*, const char*, const char*) { return 1; }
void whisper_free_state(struct whisper_state* s) { free_state(s); }
void whisper_free(struct whisper_context* ctx) {
    if (!ctx) return;
    if (ctx->c.default_state) free_state(ctx->c.default_state);
    ctx->c.default_state = nullptr;
    drain_state_pool(&ctx->c);
    orphan_states(&ctx->c);  // states the caller still holds stay valid to whisper_free_state
    free_context(&ctx->c);  // weight arena + the fp8 arena
    delete ctx;
}

// ---- mel / encode / decode ------------------------------------------------------------------------
int whisper_pcm_to_mel_with_state(struct whisper_context* ctx, struct whisper_state* s, const float* samples, int n, int) {
    if (!ctx || !s) return -1;
    hipSetDevice(ctx->c.device);
    const float* pp[1] = {samples};
    int nn[1] = {n};
    return guarded(s, [&] { return compute_mel(&ctx->c, s, pp, nn, 1, false); });
}
int whisper_pcm_to_mel(struct whisper_context* ctx, const float* samples, int n, int t) {
    return whisper_pcm_to_mel_with_state(ctx, ctx ? ctx->c.default_state : nullptr, samples, n, t);
}
int whisper_set_mel_with_state(struct whisper_context*, struct whisper_state*, const float*, int, int) {
    fprintf(stderr, "whisper_mi355x: whisper_set_mel is not supported (mel is computed on device)\n");
    return -1;
}
int whisper_set_mel(struct whisper_context* ctx, const float* d, int n, int m) { return whisper_set_mel_with_state(ctx, nullptr, d, n, m); }
int whisper_encode_with_state(struct whisper_context* ctx, struct whisper_state* s, int offset, int) {
    if (!ctx || !s || !s->mel_ready) return -1;
    hipSetDevice(ctx->c.device);
    int job = 0, slot = 0;
    return guarded(s, [&] { return encode_windows(&ctx->c, s, &job, &offset, &slot, 1); });
}
int whisper_encode(struct whisper_context* ctx, int offset, int t) {
    return whisper_encode_with_state(ctx, ctx ? ctx->c.default_state : nullptr, offset, t);
}
int whisper_decode_with_state(struct whisper_context* ctx, struct whisper_state* s, const whisper_token* tokens, int n_tokens,
                              int n_past, int) {
    if (!ctx || !s || !s->mel_ready || n_tokens <= 0) return -1;
    if (n_past + n_tokens > ctx->c.hp.n_text_ctx) return -1;
    hipSetDevice(ctx->c.device);
    std::vector<int> pos(n_tokens), slot(n_tokens, 0);
    for (int i = 0; i < n_tokens; i++) pos[i] = n_past + i;
    int row = n_tokens - 1;
    return guarded(s, [&] {
        if (decode_tokens(&ctx->c, s, tokens, pos.data(), slot.data(), n_tokens, &row, 1) != 0) return -1;
        const int V = ctx->c.hp.n_vocab;
        s->logits_host.assign((size_t)n_tokens * V, 0.0f);
        WM_CHECK(hipMemcpyAsync(s->logits_host.data() + (size_t)(n_tokens - 1) * V, s->ws.logits, (size_t)V * 4,
                                hipMemcpyDeviceToHost, s->stream));
        WM_CHECK(hipStreamSynchronize(s->stream));
        return 0;
    });
}
int whisper_decode(struct whisper_context* ctx, const whisper_token* t, int n, int n_past, int th) {
    return whisper_decode_with_state(ctx, ctx ? ctx->c.default_state : nullptr, t, n, n_past, th);
}
float* whisper_get_logits_from_state(struct whisper_state* s) { return s ? s->logits_host.data() : nullptr; }
float* whisper_get_logits(struct whisper_context* ctx) {
    return ctx && ctx->c.default_state ? ctx->c.default_state->logits_host.data() : nullptr;
}

// ---- tokens / languages ---------------------------------------------------------------------------
int whisper_tokenize(struct whisper_context* ctx, const char* text, whisper_token* tokens, int n_max) {
    if (!ctx || !text) return -1;
    std::vector<int> t = tokenize(ctx->c.vocab, text);
    if (n_max < (int)t.size()) return -(int)t.size();
    for (size_t i = 0; i < t.size(); i++) tokens[i] = t[i];
    return (int)t.size();
}
int whisper_token_count(struct whisper_context* ctx, const char* text) { return -whisper_tokenize(ctx, text, nullptr, 0); }
int whisper_lang_max_id(void) { return 99; }
int whisper_lang_id(const char* lang) { return lang_index(lang); }
const char* whisper_lang_str(int id) { return id >= 0 && id < 100 ? k_lang_codes[id] : nullptr; }
const char* whisper_lang_str_full(int id) { return id >= 0 && id < 100 ? k_lang_names[id] : nullptr; }
int whisper_lang_auto_detect_with_state(struct whisper_context* ctx, struct whisper_state* s, int offset_ms, int, float* probs) {
    if (!ctx || !s || !s->mel_ready) return -1;
    const int seek = offset_ms / 10;
    if (seek < 0 || seek >= s->n_len_org) return -2;
    hipSetDevice(ctx->c.device);
    int job = 0, slot = 0;
    const Vocab& v = ctx->c.vocab;
    std::vector<float> lg(100);
    const int rc = guarded(s, [&] {
        if (encode_windows(&ctx->c, s, &job, &seek, &slot, 1) != 0) return -6;
        int tok = v.token_sot, pos = 0, row = 0;
        if (decode_tokens(&ctx->c, s, &tok, &pos, &slot, 1, &row, 1) != 0) return -7;
        WM_CHECK(hipMemcpy(lg.data(), s->ws.logits + v.token_sot + 1, 100 * 4, hipMemcpyDeviceToHost));
        return 0;
    });
    if (rc != 0) return rc;
    std::map<std::string, int> g_lang;
    for (int i = 0; i < 100; i++) g_lang[k_lang_codes[i]] = i;
    std::vector<std::pair<float, int>> ids;
    for (auto& kv : g_lang) ids.emplace_back(lg[kv.second], kv.second);
    std::sort(ids.begin(), ids.end(), [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first > b.first; });
    const float mx = ids[0].first;
    double sum = 0.0;
    for (auto& kv : ids) { kv.first = exp(kv.first - mx); sum += kv.first; }
    for (auto& kv : ids) kv.first /= sum;
    if (probs) for (auto& kv : ids) probs[kv.second] = kv.first;
    return ids[0].second;
}
int whisper_lang_auto_detect(struct whisper_context* ctx, int offset_ms, int t, float* probs) {
    return whisper_lang_auto_detect_with_state(ctx, ctx ? ctx->c.default_state : nullptr, offset_ms, t, probs);
}

int whisper_n_len_from_state(struct whisper_state* s) { return s ? s->n_len_org : 0; }
int whisper_n_len(struct whisper_context* ctx) { return ctx && ctx->c.default_state ? ctx->c.default_state->n_len_org : 0; }
int whisper_n_vocab(struct whisper_context* ctx) { return ctx->c.vocab.n_vocab; }
int whisper_n_text_ctx(struct whisper_context* ctx) { return ctx->c.hp.n_text_ctx; }
int whisper_n_audio_ctx(struct whisper_context* ctx) { return ctx->c.hp.n_audio_ctx; }
int whisper_is_multilingual(struct whisper_context* ctx) { return ctx->c.vocab.is_multilingual() ? 1 : 0; }
int whisper_model_n_vocab(struct whisper_context* ctx) { return ctx->c.hp.n_vocab; }
int whisper_model_n_audio_ctx(struct whisper_context* ctx) { return ctx->c.hp.n_audio_ctx; }
int whisper_model_n_audio_state(struct whisper_context* ctx) { return ctx->c.hp.n_audio_state; }
int whisper_model_n_audio_head(struct whisper_context* ctx) { return ctx->c.hp.n_audio_head; }
int whisper_model_n_audio_layer(struct whisper_context* ctx) { return ctx->c.hp.n_audio_layer; }
int whisper_model_n_text_ctx(struct whisper_context* ctx) { return ctx->c.hp.n_text_ctx; }
int whisper_model_n_text_state(struct whisper_context* ctx) { return ctx->c.hp.n_text_state; }
int whisper_model_n_text_head(struct whisper_context* ctx) { return ctx->c.hp.n_text_head; }
int whisper_model_n_text_layer(struct whisper_context* ctx) { return ctx->c.hp.n_text_layer; }
int whisper_model_n_mels(struct whisper_context* ctx) { return ctx->c.hp.n_mels; }
int whisper_model_ftype(struct whisper_context* ctx) { return ctx->c.hp.ftype; }
int whisper_model_type(struct whisper_context* ctx) {
    const int L = ctx->c.hp.n_audio_layer;
    return L == 4 ? 1 : L == 6 ? 2 : L == 12 ? 3 : L == 24 ? 4 : 5;
}
const char* whisper_model_type_readable(struct whisper_context* ctx) { return ctx->c.model_type.c_str(); }

const char* whisper_token_to_str(struct whisper_context* ctx, whisper_token t) {
    if (!ctx || t < 0 || t >= (int)ctx->c.vocab.id_to_token.size()) return nullptr;
    return ctx->c.vocab.id_to_token[t].c_str();
}
whisper_token whisper_token_eot(struct whisper_context* ctx) { return ctx->c.vocab.token_eot; }
whisper_token whisper_token_sot(struct whisper_context* ctx) { return ctx->c.vocab.token_sot; }
whisper_token whisper_token_solm(struct whisper_context* ctx) { return ctx->c.vocab.token_solm; }
whisper_token whisper_token_prev(struct whisper_context* ctx) { return ctx->c.vocab.token_prev; }
whisper_token whisper_token_nosp(struct whisper_context* ctx) { return ctx->c.vocab.token_nosp; }
whisper_token whisper_token_not(struct whisper_context* ctx) { return ctx->c.vocab.token_not; }
whisper_token whisper_token_beg(struct whisper_context* ctx) { return ctx->c.vocab.token_beg; }
whisper_token whisper_token_lang(struct whisper_context* ctx, int id) { return ctx->c.vocab.token_sot + 1 + id; }
whisper_token whisper_token_translate(struct whisper_context* ctx) { return ctx->c.vocab.token_translate; }
whisper_token whisper_token_transcribe(struct whisper_context* ctx) { return ctx->c.vocab.token_transcribe; }

struct whisper_timings* whisper_get_timings(struct whisper_context* ctx) { return ctx ? &ctx->c.timings : nullptr; }
void whisper_print_timings(struct whisper_context* ctx) {
    if (!ctx) return;
    const whisper_timings& t = ctx->c.timings;
    fprintf(stderr, "whisper_mi355x: encode %.2f ms, prompt %.2f ms, decode %.2f ms\n", t.encode_ms, t.prompt_ms, t.decode_ms);
}
void whisper_reset_timings(struct whisper_context* ctx) { if (ctx) ctx->c.timings = whisper_timings{}; }
const char* whisper_print_system_info(void) { return "HIP = 1 | gfx950 | MFMA = 1 | RCCL = 1 | "; }

// ---- full ----------------------------------------------------------------------------------------
int whisper_full_with_state(struct whisper_context* ctx, struct whisper_state* s, struct whisper_full_params p,
                            const float* samples, int n_samples) {
    if (!ctx || !s) return -1;
    const float* pp[1] = {samples};
    int nn[1] = {n_samples};
    FullOpts o;
    return guarded(s, [&] { return full_batch(&ctx->c, s, p, pp, nn, 1, false, o, true); });
}
int whisper_full(struct whisper_context* ctx, struct whisper_full_params p, const float* samples, int n) {
    return whisper_full_with_state(ctx, ctx ? ctx->c.default_state : nullptr, p, samples, n);
}
int whisper_full_parallel(struct whisper_context* ctx, struct whisper_full_params p, const float* samples, int n, int) {
    return whisper_full(ctx, p, samples, n);
}

static const Segment* seg(whisper_state* s, int job, int i) {
    if (!s || job < 0 || job >= (int)s->results.size() || i < 0 || i >= (int)s->results[job].size()) return nullptr;
    return &s->results[job][i];
}
int whisper_full_n_segments_from_state(struct whisper_state* s) { return s && !s->results.empty() ? (int)s->results[0].size() : 0; }
int whisper_full_n_segments(struct whisper_context* ctx) { return whisper_full_n_segments_from_state(ctx ? ctx->c.default_state : nullptr); }
int whisper_full_lang_id_from_state(struct whisper_state* s) { return s ? s->lang_id : -1; }
int whisper_full_lang_id(struct whisper_context* ctx) { return whisper_full_lang_id_from_state(ctx ? ctx->c.default_state : nullptr); }
int64_t whisper_full_get_segment_t0_from_state(struct whisper_state* s, int i) { auto g = seg(s, 0, i); return g ? g->t0 : 0; }
int64_t whisper_full_get_segment_t0(struct whisper_context* ctx, int i) { return whisper_full_get_segment_t0_from_state(ctx->c.default_state, i); }
int64_t whisper_full_get_segment_t1_from_state(struct whisper_state* s, int i) { auto g = seg(s, 0, i); return g ? g->t1 : 0; }
int64_t whisper_full_get_segment_t1(struct whisper_context* ctx, int i) { return whisper_full_get_segment_t1_from_state(ctx->c.default_state, i); }
bool whisper_full_get_segment_speaker_turn_next_from_state(struct whisper_state*, int) { return false; }
bool whisper_full_get_segment_speaker_turn_next(struct whisper_context*, int) { return false; }
const char* whisper_full_get_segment_text_from_state(struct whisper_state* s, int i) { auto g = seg(s, 0, i); return g ? g->text.c_str() : nullptr; }
const char* whisper_full_get_segment_text(struct whisper_context* ctx, int i) { return whisper_full_get_segment_text_from_state(ctx->c.default_state, i); }
int whisper_full_n_tokens_from_state(struct whisper_state* s, int i) { auto g = seg(s, 0, i); return g ? (int)g->tokens.size() : 0; }
int whisper_full_n_tokens(struct whisper_context* ctx, int i) { return whisper_full_n_tokens_from_state(ctx->c.default_state, i); }
const char* whisper_full_get_token_text_from_state(struct whisper_context* ctx, struct whisper_state* s, int i, int t) {
    auto g = seg(s, 0, i);
    if (!g || t < 0 || t >= (int)g->tokens.size()) return nullptr;
    return whisper_token_to_str(ctx, g->tokens[t].id);
}
const char* whisper_full_get_token_text(struct whisper_context* ctx, int i, int t) {
    return whisper_full_get_token_text_from_state(ctx, ctx->c.default_state, i, t);
}
whisper_token whisper_full_get_token_id_from_state(struct whisper_state* s, int i, int t) {
    auto g = seg(s, 0, i);
    return g && t >= 0 && t < (int)g->tokens.size() ? g->tokens[t].id : -1;
}
whisper_token whisper_full_get_token_id(struct whisper_context* ctx, int i, int t) { return whisper_full_get_token_id_from_state(ctx->c.default_state, i, t); }
static whisper_token_data tdata(const Segment* g, int t) {
    whisper_token_data r;
    memset(&r, 0, sizeof(r));
    if (!g || t < 0 || t >= (int)g->tokens.size()) { r.id = -1; return r; }
    const TokenData& x = g->tokens[t];
    r.id = x.id; r.tid = x.tid; r.p = x.p; r.plog = x.plog; r.pt = x.pt; r.ptsum = x.ptsum;
    r.t0 = -1; r.t1 = -1; r.t_dtw = -1; r.vlen = 0.0f;
    return r;
}
whisper_token_data whisper_full_get_token_data_from_state(struct whisper_state* s, int i, int t) { return tdata(seg(s, 0, i), t); }
whisper_token_data whisper_full_get_token_data(struct whisper_context* ctx, int i, int t) { return tdata(seg(ctx->c.default_state, 0, i), t); }
float whisper_full_get_token_p_from_state(struct whisper_state* s, int i, int t) { return tdata(seg(s, 0, i), t).p; }
float whisper_full_get_token_p(struct whisper_context* ctx, int i, int t) { return tdata(seg(ctx->c.default_state, 0, i), t).p; }
float whisper_full_get_segment_no_speech_prob_from_state(struct whisper_state* s, int i) { auto g = seg(s, 0, i); return g ? g->no_speech_prob : 0.0f; }
float whisper_full_get_segment_no_speech_prob(struct whisper_context* ctx, int i) { return whisper_full_get_segment_no_speech_prob_from_state(ctx->c.default_state, i); }

int whisper_bench_memcpy(int) { return 0; }
const char* whisper_bench_memcpy_str(int) { return "whisper_mi355x: memcpy benchmark not implemented\n"; }
int whisper_bench_ggml_mul_mat(int) { return 0; }
const char* whisper_bench_ggml_mul_mat_str(int) { return "whisper_mi355x: ggml mul_mat benchmark not applicable (no ggml)\n"; }
void whisper_log_set(ggml_log_callback, void*) {}

// ---- MI355X extensions -----------------------------------------------------------------------------
struct whisper_context* whisper_mi355x_init(const char* path, struct whisper_context_params p, int dtype, bool load) {
    return make_ctx(path, p, dtype, load);
}
int whisper_mi355x_weight_arena(struct whisper_context* ctx, void** ptr, size_t* bytes) {
    if (!ctx) return -1;
    *ptr = ctx->c.arena;
    *bytes = ctx->c.arena_bytes;
    return 0;
}
int whisper_mi355x_rccl_unique_id(char out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    memcpy(out, &id, 128);
    return 0;
}
// One ncclBroadcast of the packed weight arena from rank 0 over xGMI.
int whisper_mi355x_broadcast_weights(struct whisper_context* ctx, const char uid[128], int rank, int world) {
    if (!ctx) return -1;
    if (world <= 1) return 0;
    hipSetDevice(ctx->c.device);
    ncclUniqueId id;
    memcpy(&id, uid, 128);
    ncclComm_t comm;
    if (ncclCommInitRank(&comm, world, id, rank) != ncclSuccess) return -2;
    hipStream_t st = nullptr;
    ncclResult_t r = ncclInternalError;
    const int rc = guarded(nullptr, [&] {
        WM_CHECK(hipStreamCreate(&st));
        r = ncclBroadcast(ctx->c.arena, ctx->c.arena, ctx->c.arena_bytes, ncclChar, 0, comm, st);
        WM_CHECK(hipStreamSynchronize(st));
        return 0;
    });
    if (st) hipStreamDestroy(st);
    ncclCommDestroy(comm);
    if (rc != 0) return rc;
    return r == ncclSuccess ? 0 : -3;
}

int whisper_mi355x_full_batch(struct whisper_context* ctx, struct whisper_state* s, struct whisper_full_params p,
                              const float* const* pcm, const int* n, int n_jobs, bool on_device, int fixed_tokens) {
    // fixed work decodes at most a window's n_max = n_text_ctx / 2 - 4 tokens (whisper.cpp's limit: a 229-token
    // prompt + 220 tokens ends at the last self-cache row)
    if (!ctx || !s || n_jobs <= 0 || fixed_tokens > ctx->c.hp.n_text_ctx / 2 - 4) return -1;
    FullOpts o;
    o.fixed_tokens = fixed_tokens;
    return guarded(s, [&] { return full_batch(&ctx->c, s, p, pcm, n, n_jobs, on_device, o, false); });
}
int whisper_mi355x_full_batch_forced(struct whisper_context* ctx, struct whisper_state* s, struct whisper_full_params p,
                                     const float* const* pcm, const int* n, int n_jobs, bool on_device, int fixed_tokens,
                                     const int* forced, const int* spot, int n_spot, float* spot_logits) {
    if (!ctx || !s || n_jobs <= 0 || fixed_tokens <= 0 || fixed_tokens > ctx->c.hp.n_text_ctx / 2 - 4 || !forced || n_spot < 0 ||
        (n_spot && (!spot || !spot_logits)))
        return -1;
    for (int k = 0; k < n_spot; k++)
        if (spot[k] < 0 || spot[k] >= n_jobs) return -1;
    FullOpts o;
    o.fixed_tokens = fixed_tokens;
    o.forced = forced;
    o.spot = spot;
    o.n_spot = n_spot;
    o.spot_logits = spot_logits;
    return guarded(s, [&] { return full_batch(&ctx->c, s, p, pcm, n, n_jobs, on_device, o, false); });
}
int whisper_mi355x_batch_n_segments(struct whisper_state* s, int job) {
    return s && job >= 0 && job < (int)s->results.size() ? (int)s->results[job].size() : 0;
}
const char* whisper_mi355x_batch_segment_text(struct whisper_state* s, int job, int i) { auto g = seg(s, job, i); return g ? g->text.c_str() : nullptr; }
int64_t whisper_mi355x_batch_segment_t0(struct whisper_state* s, int job, int i) { auto g = seg(s, job, i); return g ? g->t0 : 0; }
int64_t whisper_mi355x_batch_segment_t1(struct whisper_state* s, int job, int i) { auto g = seg(s, job, i); return g ? g->t1 : 0; }
int whisper_mi355x_batch_segment_n_tokens(struct whisper_state* s, int job, int i) { auto g = seg(s, job, i); return g ? (int)g->tokens.size() : 0; }
whisper_token_data whisper_mi355x_batch_token_data(struct whisper_state* s, int job, int i, int t) { return tdata(seg(s, job, i), t); }
int whisper_mi355x_batch_lang_id(struct whisper_state* s, int job) {
    return s && job >= 0 && job < (int)s->lang_ids.size() ? s->lang_ids[job] : -1;
}
long whisper_mi355x_batch_decoded_tokens(struct whisper_state* s) { return s ? s->decoded_tokens : 0; }
int whisper_mi355x_window_decisions(struct whisper_state* s, int job, struct whisper_mi355x_window_decision* out, int cap) {
    if (!s || job < 0 || job >= (int)s->decisions.size()) return 0;
    const auto& d = s->decisions[job];
    if ((int)d.size() > cap) return -(int)d.size();
    for (size_t i = 0; i < d.size(); i++) out[i] = d[i];
    return (int)d.size();
}
int whisper_mi355x_phase_ms(struct whisper_state* s, double out[5]) {
    if (!s) return -1;
    for (int i = 0; i < 5; i++) out[i] = s->phase_ms[i];
    return 0;
}
int whisper_mi355x_get_mel(struct whisper_state* s, float* out, int cap) {
    return guarded(nullptr, [&]() -> int {
        if (!s || !s->ctx || !s->ws.mel) return -1;  // orphan state: its context was freed
        Context* c = s->ctx;
        const int nm = c->hp.n_mels, nl = s->n_len;
        if ((long)nm * nl > cap) return -nm * nl;
        hipSetDevice(c->device);
        // recompute n_samples from n_len: n_len = (n + 480000) / 160 is not invertible; keep it via n_len_org
        int n_samp = 0;
        WM_CHECK(hipMemcpy(&n_samp, s->ws.n_samp, sizeof(int), hipMemcpyDeviceToHost));
        float* tmp;
        WM_CHECK(hipMalloc((void**)&tmp, (size_t)nm * nl * 4));
        launch_mel_normalize(s->ws.mel, nl, n_samp, s->ws.mel_max, nm, tmp, s->stream);
        WM_CHECK(hipMemcpyAsync(out, tmp, (size_t)nm * nl * 4, hipMemcpyDeviceToHost, s->stream));
        WM_CHECK(hipStreamSynchronize(s->stream));
        WM_CHECK(hipFree(tmp));
        return nl;
    });
}
int whisper_mi355x_get_encoder_out(struct whisper_state* s, float* out, int cap) {
    return guarded(nullptr, [&]() -> int {
        if (!s || !s->ctx || !s->ws.hn || s->last_enc_windows < 1) return -1;  // orphan state: -1
        Context* c = s->ctx;
        const long n = (long)c->hp.n_audio_ctx * c->hp.n_audio_state;
        if (n > cap) return -1;
        hipSetDevice(c->device);
        std::vector<uint16_t> h(n);
        WM_CHECK(hipMemcpy(h.data(), s->ws.hn, n * 2, hipMemcpyDeviceToHost));
        for (long i = 0; i < n; i++) {
            if (c->dt == DType::F16) out[i] = h2f(h[i]);
            else { uint32_t u = (uint32_t)h[i] << 16; memcpy(&out[i], &u, 4); }
        }
        return 0;
    });
}
int whisper_mi355x_state_info(struct whisper_state* s, int out[5]) {
    if (!s || !out) return -1;
    out[0] = s->direct ? 1 : 0;
    out[1] = s->ws.cap_jobs;
    out[2] = s->ws.cap_cross;
    out[3] = (int)s->dec_graphs.size();
    out[4] = s->pooled ? 1 : 0;
    return 5;
}
void* whisper_mi355x_state_stream(struct whisper_state* s) { return s ? (void*)s->stream : nullptr; }
int whisper_mi355x_kernel_timing(struct whisper_state* s, int class_mask) {
    if (!s) return -1;
    s->ktime_mask = class_mask;
    for (auto& k : s->kstat) k = KStat();
    return 0;
}
int whisper_mi355x_kernel_stats(struct whisper_state* s, int cls, double out[3]) {
    if (s && cls == WHISPER_MI355X_KSTAT_PDEC_GIVE_UPS) {
        out[0] = s->pdec_lost_ms;
        out[1] = (double)s->pdec_give_ups;
        out[2] = 0.0;
        return 0;
    }
    if (!s || cls < 0 || cls >= K_NCLASS) return -1;
    out[0] = s->kstat[cls].ms;
    out[1] = (double)s->kstat[cls].count;
    out[2] = s->kstat[cls].work;
    return 0;
}
// ---- kernel-level test/tuning hooks ---------------------------------------------------------------

void whisper_mi355x_set_gemm_variant(int v) { wm::g_gemm_variant = v; }
void whisper_mi355x_set_gemm_stamps(void* dev) { wm::g_gemm_stamps = (unsigned long long*)dev; }
void whisper_mi355x_set_dec_splits(int splits) { wm::g_dec_splits = splits; }
void whisper_mi355x_set_dec_bm(int rows) { wm::g_dec_bm = rows; }
void whisper_mi355x_set_pdec_spin(long ticks) {
    wm::g_pdec_spin_ticks = ticks;
    wm::g_pdec_gen.fetch_add(1, std::memory_order_release);
}
void whisper_mi355x_set_pdec_stamps(void* dev) {
    wm::g_pdec_stamps = (unsigned long long*)dev;
    wm::g_pdec_gen.fetch_add(1, std::memory_order_release);
}
// debug: device pointers of the state's decode workspace: 0 x (f32 [rows][d]), 1 final LN rows, 2 (unused), 3
// attention outputs, 4 GELU rows, 5 cross q, 6 Q', 7 cross partials, 8 their {m, l}
void* whisper_mi355x_debug_ws(struct whisper_state* s, int which) {
    if (!s) return nullptr;
    const wm::Workspace& w = s->ws;
    void* p[9] = {w.dx, w.dh, nullptr, w.datt, w.dff, w.dq, w.qx, w.xo, w.xml};
    return which >= 0 && which < 9 ? p[which] : nullptr;
}
long whisper_mi355x_decoded_tokens_total(void) { return wm::g_decoded_tokens_total.load(); }
long whisper_mi355x_pdec_give_ups(struct whisper_state* s) { return s ? s->pdec_give_ups : wm::g_pdec_give_ups_total.load(); }
void whisper_mi355x_set_pdec_blocks(int on) { wm::g_pdec_blocks = on != 0; }
// out[M][N] (f32 for epi EPI_F32 / EPI_RESID, else the context dtype) = A[M][K] . B[N][K]^T + bias,
// all device pointers; runs `reps` times and returns the average ms per launch in *ms.
int whisper_mi355x_debug_gemm(struct whisper_context* ctx, int epi, const void* A, int M, int K, const void* B, int N,
                              const float* bias, void* out, int reps, float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx) return -1;
        hipSetDevice(ctx->c.device);
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        GemmArgs g{};
        g.A = A; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = out; g.ldo = N; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
        if (M <= 128) {  // decode-step shapes take the split-K path, as in the engine
            g.splitk_ws_elems = 64L * M * N;
            WM_CHECK(hipMalloc(&g.splitk_ws, g.splitk_ws_elems * sizeof(float)));
        }
        int* dslot = nullptr;
        if (epi == EPI_CROSSKV) {  // out = a cross cache [M / n_audio_ctx][N / 2K][2][K / 64][n_audio_ctx][64], slots in order
            const int T = ctx->c.hp.n_audio_ctx;
            if (M % T != 0 || K % 64 != 0 || N % (2 * K) != 0) return -1;
            std::vector<int> hs(M / T);
            for (int i = 0; i < M / T; i++) hs[i] = i;
            WM_CHECK(hipMalloc((void**)&dslot, hs.size() * sizeof(int)));
            WM_CHECK(hipMemcpy(dslot, hs.data(), hs.size() * sizeof(int), hipMemcpyHostToDevice));
            g.cache = out; g.row_slot = dslot; g.d = K; g.H = K / 64; g.ctx = T; g.L = N / (2 * K); g.layer = 0;
        }
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        launch_gemm(ctx->c.dt, epi, g, st);  // warm
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) launch_gemm(ctx->c.dt, epi, g, st);
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = reps > 0 ? t / reps : 0.0f;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        if (g.splitk_ws) hipFree(g.splitk_ws);
        if (dslot) hipFree(dslot);
        return 0;
    });
}
int whisper_mi355x_debug_gemm_small(struct whisper_context* ctx, int epi, const void* A, int M, int K, const void* B,
                                    int N, const float* bias, void* out, const float* ln_w, const float* ln_b, int reps,
                                    float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx || !gemm_small_ok(M, K, ln_w != nullptr)) return -1;
        hipSetDevice(ctx->c.device);
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        GemmArgs g{};
        g.A = A; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = out; g.ldo = N; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
        g.a_ln_w = ln_w; g.a_ln_b = ln_b;
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        launch_gemm_small(ctx->c.dt, epi, g, ln_w != nullptr, st);
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) launch_gemm_small(ctx->c.dt, epi, g, ln_w != nullptr, st);
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = reps > 0 ? t / reps : 0.0f;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        return 0;
    });
}
int whisper_mi355x_debug_gemm_fp8(struct whisper_context* ctx, int epi, const void* A8, const float* a_scale, int M,
                                  int K, const void* B8, const float* b_scale, int N, const float* bias, void* out,
                                  int reps, float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx) return -1;
        hipSetDevice(ctx->c.device);
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        GemmArgs g{};
        g.A = A8; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B8; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = out; g.ldo = N; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        launch_gemm_fp8(ctx->c.dt, epi, g, a_scale, b_scale, st);
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) launch_gemm_fp8(ctx->c.dt, epi, g, a_scale, b_scale, st);
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = reps > 0 ? t / reps : 0.0f;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        return 0;
    });
}
int whisper_mi355x_debug_gemm_w8(struct whisper_context* ctx, int epi, const void* A, int M, int K, const void* B8,
                                 const float* b_scale, int N, const float* bias, void* out, const float* ln_w,
                                 const float* ln_b, void* y) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx || !b_scale || M < 1 || M > 128 || K % 64) return -1;
        hipSetDevice(ctx->c.device);
        GemmArgs g{};
        g.A = A; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B8; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = out; g.ldo = N; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
        g.w8_scale = b_scale;
        if (epi == EPI_RESID) {
            if (!ln_w || !y) return -1;
            g.ln_w = ln_w; g.ln_b = ln_b; g.ln_out = y;
        }
        g.splitk_ws_elems = 16L * M * N;
        WM_CHECK(hipMalloc(&g.splitk_ws, g.splitk_ws_elems * sizeof(float)));
        launch_gemm(ctx->c.dt, epi, g, nullptr);
        WM_CHECK(hipDeviceSynchronize());
        hipFree(g.splitk_ws);
        return 0;
    });
}
int whisper_mi355x_debug_quant_fp8(struct whisper_context* ctx, const void* x, long rows, int K, void* q, float* s) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx) return -1;
        hipSetDevice(ctx->c.device);
        launch_quant_rows_fp8(ctx->c.dt, x, rows, K, q, s, nullptr);
        WM_CHECK(hipDeviceSynchronize());
        return 0;
    });
}
int whisper_mi355x_debug_attn_encoder(struct whisper_context* ctx, const void* qkv, int B, int T, int d, int H,
                                      int variant, void* out, int reps, float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx || B < 1 || T < 1 || d != 64 * H || variant < 1 || variant > 6 || variant == 4) return -1;
        hipSetDevice(ctx->c.device);
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        launch_attn_encoder(ctx->c.dt, qkv, out, B, T, d, H, st, variant);
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) launch_attn_encoder(ctx->c.dt, qkv, out, B, T, d, H, st, variant);
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = reps > 0 ? t / reps : 0.0f;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        return 0;
    });
}

int whisper_mi355x_debug_gemm_ln(struct whisper_context* ctx, const void* A, int M, int K, const void* B, int N,
                                 const float* bias, float* x, const float* ln_w, const float* ln_b, void* y, int reps,
                                 float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx || M > 128) return -1;
        hipSetDevice(ctx->c.device);
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        GemmArgs g{};
        g.A = A; g.a_rpb = M; g.a_bstride = 0; g.a_rstride = K;
        g.B = B; g.bias = bias; g.M = M; g.N = N; g.K = K;
        g.out = x; g.ldo = N; g.o_rpb = M; g.o_bstride = 0; g.o_off = 0;
        g.sc_div = 0; g.sc_mod = 1; g.sc_lim = 0; g.scale = 1.0f;
        g.ln_w = ln_w; g.ln_b = ln_b; g.ln_out = y;
        g.splitk_ws_elems = 64L * M * N;
        WM_CHECK(hipMalloc(&g.splitk_ws, g.splitk_ws_elems * sizeof(float)));
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < std::max(1, reps); r++) launch_gemm(ctx->c.dt, EPI_RESID, g, st);
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = t / std::max(1, reps);
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        hipFree(g.splitk_ws);
        return 0;
    });
}
// Direct cross attention (kernels/xattn.hip: Q' projection, one pass over E, split merge + Wv) on
// caller data, all device pointers in the context dtype: enc [slots][n_ctx][d], slot [n] int,
// q [n][d] (already scaled), wkt [H][d][64], wv [d][d], bv [d] f32 -> out [n][d].
int whisper_mi355x_debug_xattn(struct whisper_context* ctx, const void* enc, const int* slot, const void* q,
                               const void* wkt, const void* wv, const float* bv, int n, int n_ctx, int d, float scale,
                               int splits, float rescale_thr, void* out, int reps, float* ms) {
    return guarded(nullptr, [&]() -> int {
        if (!ctx || n <= 0 || !xattn_supported(d)) return -1;
        hipSetDevice(ctx->c.device);
        const DType dt = ctx->c.dt;
        const int H = d / 64;
        if (splits <= 0) splits = xattn_splits(n, n_ctx);
        void* qx = nullptr;
        float *op = nullptr, *ml = nullptr;
        WM_CHECK(hipMalloc(&qx, (size_t)n * 2 * H * d * 2));
        WM_CHECK(hipMalloc((void**)&op, (size_t)n * splits * H * d * 4));
        WM_CHECK(hipMalloc((void**)&ml, (size_t)n * splits * H * 2 * 4));
        hipStream_t st;
        WM_CHECK(hipStreamCreate(&st));
        auto run = [&] {
            launch_xattn_qproj(dt, q, wkt, n, d, H, scale, qx, st);
            launch_xattn_step(dt, enc, slot, qx, n, n_ctx, d, splits, rescale_thr, op, ml, st);
            launch_xattn_combine(dt, op, ml, splits, wv, bv, n, d, H, out, st);
        };
        hipEvent_t e0, e1;
        WM_CHECK(hipEventCreate(&e0));
        WM_CHECK(hipEventCreate(&e1));
        run();
        WM_CHECK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) run();
        WM_CHECK(hipEventRecord(e1, st));
        WM_CHECK(hipStreamSynchronize(st));
        float t = 0;
        WM_CHECK(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = reps > 0 ? t / reps : 0.0f;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        hipStreamDestroy(st);
        hipFree(qx);
        hipFree(op);
        hipFree(ml);
        return 0;
    });
}
// ABI self-description (no device needed): sizes/offsets that a binding generator must agree on.
int whisper_mi355x_abi_layout(size_t out[8]) {
    out[0] = sizeof(whisper_full_params);
    out[1] = sizeof(whisper_context_params);
    out[2] = sizeof(whisper_token_data);
    out[3] = offsetof(whisper_full_params, initial_prompt);
    out[4] = offsetof(whisper_full_params, language);
    out[5] = offsetof(whisper_full_params, greedy);
    out[6] = offsetof(whisper_full_params, new_segment_callback);
    out[7] = offsetof(whisper_full_params, vad_params);
    return 8;
}
void* whisper_mi355x_dev_alloc(struct whisper_context* ctx, size_t bytes) {
    void* p = nullptr;
    hipSetDevice(ctx->c.device);
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}
void whisper_mi355x_dev_free(struct whisper_context* ctx, void* p) { hipSetDevice(ctx->c.device); hipFree(p); }
int whisper_mi355x_memcpy(struct whisper_context* ctx, void* dst, const void* src, size_t bytes, int kind) {
    hipSetDevice(ctx->c.device);
    return hipMemcpy(dst, src, bytes, (hipMemcpyKind)kind) == hipSuccess ? 0 : -1;
}

}  // extern "C"
