// Engine internals: model (weights in one HBM arena), vocabulary/tokenizer, per-state workspace,
// and the batched window scheduler that implements whisper_full semantics for many clips at once.
#pragma once
#include <map>
#include <atomic>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/whisper_mi355x.h"
#include "common.h"
#include "kernels.h"

namespace wm {

struct Hparams {
    int32_t n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int32_t n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels, ftype;
};

// whisper.cpp's whisper_vocab semantics (special ids shift for multilingual files, extra
// tokens synthesised up to n_vocab) — SURVEY.md §8a rows a4, a12.
struct Vocab {
    int n_vocab = 51864;
    int token_eot = 50256, token_sot = 50257, token_translate = 50357, token_transcribe = 50358;
    int token_solm = 50359, token_prev = 50360, token_nosp = 50361, token_not = 50362, token_beg = 50363;
    std::map<std::string, int> token_to_id;
    std::vector<std::string> id_to_token;
    bool is_multilingual() const { return n_vocab >= 51865; }
    int num_languages() const { return n_vocab - 51765 - (is_multilingual() ? 1 : 0); }
};

extern const char* const k_lang_codes[100];
extern const char* const k_lang_names[100];
int lang_index(const char* code);
std::vector<int> tokenize(const Vocab& v, const std::string& text);

struct LayerW {
    float *ln1_w, *ln1_b;
    void* wqkv; float* bqkv;
    void* wo; float* bo;
    float *lnx_w, *lnx_b;     // decoder cross-attn LN
    void* wxq; float* bxq;    // decoder cross-attn query
    void* wxo; float* bxo;    // decoder cross-attn out
    float *ln2_w, *ln2_b;
    void* w1; float* b1;
    void* w2; float* b2;
    // block-quantized GGML files: the projection weights as the file's blocks (the compute-type
    // pointers above are null then, except where a layer's matrix was stored unquantized)
    QMat qqkv, qo, qxq, qxo, q1, q2;
};

struct Weights {
    void* conv1_w; float* conv1_b;
    void* conv2_w; float* conv2_b;
    float* pos_e;
    float *lnpost_w, *lnpost_b;
    void* tok_emb; float* pos_d;
    float* tok_emb_f32 = nullptr;       // quantized GGML embedding: exact f32 rows for the lookups
    float *lnd_w, *lnd_b;
    void* wkv_cross; float* bkv_cross;  // [L_d][2][d][d], bias [L_d][2][d] (K part zero)
    void* wkT = nullptr;                // [L_d][H][d][64]: cross K per head, transposed (direct cross attention)
    std::vector<LayerW> enc, dec;
    void* mel_tab;    // MelTablesDev (sin, cos, hann)
    float* filt_t;    // [201][n_mels]
};

struct Context {
    Hparams hp;
    Vocab vocab;
    VocabIds vid;
    DType dt = DType::F16;
    int device = 0;
    std::string path;
    int filt_n_mel = 0, filt_n_fft = 0;
    std::vector<float> filters;
    Weights w;
    char* arena = nullptr;
    size_t arena_bytes = 0;
    whisper_timings timings{};
    std::mutex timings_mu;  // states on different threads add their phase times here
    whisper_state* default_state = nullptr;  // whisper_init_from_file_with_params (with state)
    float k_scale = 0.0f;                    // d_head^-0.25
    // Cross attention straight from the encoder output (kernels/xattn.hip) is available for this
    // model (its per-head transposed Wk is in the arena); each call picks direct or cached form.
    bool cross_direct = false;
    // block-quantized file (ggml type of its projection matrices, 0 = f16/f32 file) kept quantized in
    // the arena: decode steps of few clips read the blocks (gemm_small_kernel, the persistent step);
    // the big-M GEMMs (encoder, prefill, decode steps of many clips) read a compute-type copy of every
    // projection, expanded once per context on first use (ensure_expanded, engine.cpp)
    int quant = 0;
    struct LayerMats { const void *wqkv, *wo, *wxq, *wxo, *w1, *w2; };
    std::mutex exp_mu;
    std::atomic<bool> expanded{false};
    char* arena_exp = nullptr;
    std::vector<LayerMats> exp_enc, exp_dec;
    std::string model_type;
    whisper_context* owner = nullptr;  // the whisper.h handle wrapping this context
    // fp8 encoder (large-v3-turbo fp8 config): QKV, FC1 and FC2 as e4m3 GEMMs with per-row scales.
    // The e4m3 weights are quantized from the loaded (or broadcast) bf16 weights on first use.
    struct Fp8Layer { void* wqkv = nullptr; float* sqkv = nullptr; void* w1 = nullptr; float* s1 = nullptr;
                      void* w2 = nullptr; float* s2 = nullptr; };
    bool fp8_enc = false;
    bool fp8_ready = false;
    std::mutex fp8_mu;
    std::vector<Fp8Layer> enc8;
    char* arena8 = nullptr;
    // fp8 mode, decoder: the decode-step projections (self QKV, self out, cross Q, cross out, FC1, FC2)
    // read e4m3 weights with per-output-row scales (same quantizer, same arena); the token embedding
    // (logits), the cross-attention K/V weights and prefill keep the compute type
    struct Fp8Dec { void *wqkv, *wo, *wxq, *wxo, *w1, *w2; float *sqkv, *so, *sxq, *sxo, *s1, *s2; };
    std::vector<Fp8Dec> dec8;
    // persistent decode step (kernels/pdec.hip): the decoder layers' pointers as a device array
    std::mutex pdec_mu;
    void* pdec_layers = nullptr;
    void* pdec_layers_exp = nullptr;  // (a quantized file's expanded copy)
    // States released by whisper_free_state, kept with their workspace and captured decode graphs
    // for the next whisper_init_state: whisper.rs:83-85 creates (and drops) a state on every
    // transcribe call, which would otherwise pay ~30 hipMallocs and a graph capture per call.
    std::mutex pool_mu;
    std::vector<whisper_state*> pool;
    // every state of this context that is alive (pooled or held by a caller), under pool_mu:
    // whisper_free orphans the ones a caller still holds, so a later whisper_free_state does not touch
    // the freed context (a garbage collector may finalise a context before its states)
    std::vector<whisper_state*> live;
};

struct TokenData {
    int id, tid;
    float p, plog, pt, ptsum;
};

struct Segment {
    int64_t t0, t1;
    std::string text;
    float no_speech_prob;
    std::vector<TokenData> tokens;
};

// Workspace sized for a batch of up to `cap_jobs` clips; grows on demand, never shrinks.
struct Workspace {
    int cap_jobs = 0, cap_enc = 0, cap_tok = 0;
    int cap_cross = 0;  // slots of the cross K/V cache (sized by the calls that use it, not cap_jobs)
    size_t cap_mel = 0, cap_pcm = 0;
    // encoder (cap_enc windows)
    void *mel_img = nullptr, *h1 = nullptr, *hn = nullptr, *qkv = nullptr, *att = nullptr, *ff = nullptr;
    float* x = nullptr;
    float* hs = nullptr;  // fp8 encoder: per-row scales of the quantized GEMM inputs
    // caches (cap_jobs slots). In direct mode `cross` is allocated on first use (prompts too long
    // for the direct prefill) and cross_fresh[slot] says whether a slot's cross K/V match enc.
    void *cross = nullptr, *self = nullptr;
    std::vector<char> cross_fresh;
    int* kvslot = nullptr;  // identity [cap_jobs]: row_slot of a one-clip cross-KV GEMM
    void* wdq = nullptr;    // quantized files: one layer's projection weights dequantized (16 d^2)
    // direct cross attention: encoder output per slot [cap_jobs][T][d], Q' [cap_xq][2H][d],
    // split partials [xo_rows][H][d] f32 + [xo_rows][H][2]
    void *enc = nullptr, *qx = nullptr;
    float *xo = nullptr, *xml = nullptr;
    int cap_xq = 0;
    // decoder (cap_tok tokens)
    float* dx = nullptr;
    void *dh = nullptr, *dq = nullptr, *datt = nullptr, *dff = nullptr, *lrow = nullptr;
    float *logits = nullptr, *probs = nullptr;
    float* splitk = nullptr;  // split-K partial slabs for decode-step GEMMs
    long splitk_elems = 0;
    int *tok = nullptr, *pos = nullptr, *slot = nullptr, *nkv_self = nullptr, *nkv_cross = nullptr, *lrows = nullptr;
    SeqCtl* ctl = nullptr;
    TokOut* tout = nullptr;
    void* lrec = nullptr;  // split logits kernel: per-chunk records
    int *win_job = nullptr, *win_seek = nullptr, *win_slot = nullptr;
    // persistent decode step: the hand-off block (granules + error word) and the error word's host copy
    // (shared with the batched chain's error word)
    unsigned* pd_sync = nullptr;
    unsigned* h_pd_err = nullptr;
    // pipelined greedy decoding (engine.cpp decode_pipelined): two ring slots of [cap_jobs TokOut][16-byte error
    // word] on the device and in pinned host memory, and the event after each slot's copy
    char* ring = nullptr;
    char* h_ring = nullptr;
    hipEvent_t ring_ev[2] = {nullptr, nullptr};
    // mel / pcm
    float* pcm = nullptr;
    float* mel = nullptr;
    float** mel_ptrs = nullptr;
    const float** pcm_ptrs = nullptr;
    int *n_samp = nullptr, *n_len = nullptr, *mel_max = nullptr;
    // host pinned staging
    int* h_ints = nullptr;
    int2* qtiles = nullptr;   // prefill attention tiles {first token, count} (cap_tok), device
    int2* h_qtiles = nullptr; // the same, pinned host staging
    int n_qtiles = 0;
    TokOut* h_tout = nullptr;
    SeqCtl* h_ctl = nullptr;
};

struct Job;

// Live per-kernel-class timing with HIP events on the state's stream (bench.py's roofline leg).
// `work` is the algorithmic FLOPs (MFMA-bound classes) or HBM bytes (HBM-bound classes).
enum KClass { K_GEMM_ENC = 0, K_ATTN_ENC, K_ATTN_CROSS, K_ATTN_SELF, K_GEMM_DEC, K_LOGITS, K_MEL, K_PDEC, K_OTHER, K_NCLASS };
struct KStat { double ms = 0, work = 0; long count = 0; };

}  // namespace wm

struct whisper_state {
    wm::Context* ctx = nullptr;  // nullptr once the context was freed before the state (orphan)
    int device = 0;
    hipStream_t stream = nullptr;
    // second stream + fork/join events: decode steps run their rows as two groups concurrently
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    wm::Workspace ws;
    // cross attention form of the current call: straight from the encoder output (large batches) or
    // through a per-clip cross K/V cache (small batches, and whisper.cpp's own form)
    bool direct = false;
    // whisper.h single-clip results (job 0 of the last call) + batch results
    std::vector<std::vector<wm::Segment>> results;
    std::vector<int> lang_ids;
    std::vector<std::vector<whisper_mi355x_window_decision>> decisions;  // per job, per window
    std::vector<int> prompt_past;  // persists across whisper_full calls on this state
    std::mt19937 rng{0};           // decoder 0's rng: created with the state, never reset
    int lang_id = 0;
    int n_len = 0, n_len_org = 0;  // last mel
    std::vector<float> logits_host;
    double phase_ms[5] = {0, 0, 0, 0, 0};
    long decoded_tokens = 0;
    // standalone encode/decode API support
    int last_enc_windows = 0;
    bool mel_ready = false;  // whisper_pcm_to_mel (or a full call) has run on this state
    bool pooled = false;     // this state was recycled from the context's pool (workspace + graphs kept)
    // kernel timing (off unless whisper_mi355x_kernel_timing enabled it)
    int ktime_mask = 0;  // bit k: time kernel class k
    wm::KStat kstat[wm::K_NCLASS];
    struct KPending { int cls; hipEvent_t a, b; double work; };
    std::vector<KPending> kpending;
    std::vector<hipEvent_t> kpool;
    // decode steps replayed as hipGraphs, one per (active-clip count, timing mask, cross form, path
    // signature): `sig` encodes the per-call switches that pick the step's kernels (dec_path_sig), so a
    // changed setting never replays a graph captured for another path
    // (gen: g_pdec_gen when a persistent step was captured; its graph holds the stamps pointer and spin limit of
    // that time, so a setter call retires it)
    // pdec: 0 = launch chain, 1 = the persistent step (kernels/pdec.hip)
    // (par: 0 for the per-step path; the pipelined path alternates two instances, 0 and 1, so that one step's
    // graph events are read while the other instance runs)
    struct DecGraph { int n_tok, n_rows, mask; bool direct; int sig; int pdec; int gen; int par; hipGraphExec_t exec; std::vector<KPending> ev; };
    std::vector<DecGraph> dec_graphs;
    std::vector<KPending>* capture_ev = nullptr;  // non-null while a decode step is being captured
    bool pipe_capture = false;  // capturing a pipelined step graph (its advance kernel copies the error word)
    double cur_self_work = 0;                     // self-attention bytes of the current step
    whisper_state* twin = nullptr;                // second half of a paired batch (full_batch)
    bool pdec_block = false;                      // re-running a step whose persistent launch gave up
    int step_rows = 0;                            // rows of the decode step being built (all row groups)
    // persistent launches of this state that gave up (a wait timed out: not all 256 workgroups resident, e.g.
    // beside another process's kernels) and were re-run on the per-kernel path; after one, the state's steps
    // take the per-kernel path for kPdecBackoffMs (pdec_off) instead of paying the timeout on every step
    long pdec_give_ups = 0;
    double pdec_lost_ms = 0;    // wall time of the given-up launches (wait until give-up + the re-run)
    double pdec_off_until = 0;  // now_ms() clock
    bool pdec_off = false;
};

struct whisper_context {
    wm::Context c;
};

namespace wm {
bool load_context(Context* c, const char* path, int device, DType dt, bool load_weights);
void free_context(Context* c);
whisper_state* new_state(Context* c);
void free_state(whisper_state* s);
// after an engine error (wm::Error) mid-call: end a half-done graph capture, drain both streams and
// return pending timing events, so that the state and its context stay usable
void recover_state(whisper_state* s);
// frees the states kept in the context's pool (whisper_free)
void drain_state_pool(Context* c);
void orphan_states(Context* c);

struct FullOpts {
    int fixed_tokens = 0;
    // teacher forcing (fixed-work mode only; a parity-test hook): the token chosen at step i of job j is
    // replaced by forced[j * fixed_tokens + i] after the logits rules ran, so every later step decodes
    // the given sequence through the same kernels; the raw logits of jobs spot[0..n_spot) are copied
    // to spot_logits[(i * n_spot + k) * n_vocab] at every step i (prefill = step 0)
    const int* forced = nullptr;
    const int* spot = nullptr;
    int n_spot = 0;
    float* spot_logits = nullptr;
};
// whisper_full over n_jobs clips. B=1 with the state's own prompt_past/rng reproduces
// whisper_full_with_state; B>1 treats every clip as a fresh state.
// tokens decoded by every whisper_full / full_batch call of the process (whisper_mi355x_decoded_tokens_total)
extern std::atomic<long> g_decoded_tokens_total;
int full_batch(Context* c, whisper_state* s, const whisper_full_params& p, const float* const* pcm, const int* n,
               int n_jobs, bool on_device, const FullOpts& o, bool single_api);

// pieces exposed for whisper.h's low-level API
int compute_mel(Context* c, whisper_state* s, const float* const* pcm, const int* n, int n_jobs, bool on_device);
int encode_windows(Context* c, whisper_state* s, const int* jobs, const int* seeks, const int* slots, int n_win);
int decode_tokens(Context* c, whisper_state* s, const int* tokens, const int* pos, const int* slots, int n_tok,
                  const int* logit_rows, int n_logit_rows);
}  // namespace wm
