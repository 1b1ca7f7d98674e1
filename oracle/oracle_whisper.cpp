// TEST INFRASTRUCTURE ONLY (see oracle_common.h for what this restates and how it is pinned).
//
// CPU restatement of whisper.cpp ≈v1.7.x [ext]: GGML model load (`whisper_model_load`), encoder
// graph (`whisper_build_graph_conv` + `whisper_build_graph_encoder`), cross-KV graph
// (`whisper_build_graph_cross`), decoder graph (`whisper_build_graph_decoder`), logits filters
// (`whisper_process_logits`), sampling (`whisper_sample_token`), scoring
// (`whisper_sequence_score`), tokenizer (`tokenize`), language detection
// (`whisper_lang_auto_detect_with_state`) and the window / temperature-fallback / segmentation
// loop of `whisper_full_with_state`, run with the reference's FullParams
// (src-tauri/src/whisper.rs:88-124).
//
// Numerics mode GGML (mode=1) reproduces ggml-cpu's roundings: matmul inputs rounded to f16
// (vec_dot_type of an f16 weight), K/V caches f16, attention probabilities rounded to f16 before
// P·V, GELU through the f16 lookup table (GGML_GELU_FP16), LayerNorm sums in double, softmax sum
// in double, f32 accumulation. Mode F32 (mode=0) removes every rounding so the forward can be
// compared with HF transformers at fp32 (tests/golden/make_golden.py).
#include "oracle_common.h"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <regex>
#include <string>
#include <vector>
#include <omp.h>

namespace oracle {
int mel_compute(const float* samples, int n_samples, const float* filters, int n_mel, int n_fft_bins,
                std::vector<float>& mel, int* n_len_org_out, int n_threads);
}

using namespace oracle;

// ------------------------------------------------------------------------------------------------
// language table: whisper.cpp g_lang (std::map keyed by code; ids are the Whisper order)
static const char* k_lang_codes[] = {
    "en","zh","de","es","ru","ko","fr","ja","pt","tr","pl","ca","nl","ar","sv","it","id","hi","fi","vi",
    "he","uk","el","ms","cs","ro","da","hu","ta","no","th","ur","hr","bg","lt","la","mi","ml","cy","sk",
    "te","fa","lv","bn","sr","az","sl","kn","et","mk","br","eu","is","hy","ne","mn","bs","kk","sq","sw",
    "gl","mr","pa","si","km","sn","yo","so","af","oc","ka","be","tg","sd","gu","am","yi","lo","uz","fo",
    "ht","ps","tk","nn","mt","sa","lb","my","bo","tl","mg","as","tt","haw","ln","ha","ba","jw","su","yue"};
static const int k_n_lang = 100;

static int lang_id(const char* code) {
    for (int i = 0; i < k_n_lang; i++) if (strcmp(k_lang_codes[i], code) == 0) return i;
    return -1;
}

// ------------------------------------------------------------------------------------------------
struct Hparams {
    int n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels, ftype;
};

struct Vocab {
    int n_vocab = 51864;
    int token_eot = 50256, token_sot = 50257, token_translate = 50357, token_transcribe = 50358;
    int token_solm = 50359, token_prev = 50360, token_nosp = 50361, token_not = 50362, token_beg = 50363;
    std::map<std::string, int> token_to_id;
    std::vector<std::string> id_to_token;
    bool is_multilingual() const { return n_vocab >= 51865; }
    int num_languages() const { return n_vocab - 51765 - (is_multilingual() ? 1 : 0); }
};

struct Tensor { std::vector<int> ne; std::vector<float> data; int type = 0; };

// [ext] ggml dequantize_row_q4_0/q4_1/q5_0/q5_1/q8_0: blocks of 32, y = q*d (+ m), exact in f32
static int block_bytes(int type) {
    switch (type) { case 2: return 18; case 3: return 20; case 6: return 22; case 7: return 24; case 8: return 34; }
    return 0;
}
static void dequant_block(int type, const uint8_t* b, float* y) {
    auto hf = [](const uint8_t* p) { uint16_t h; memcpy(&h, p, 2); return f16_to_f32(h); };
    if (type == 8) { const float d = hf(b); for (int j = 0; j < 32; j++) y[j] = (float)(int8_t)b[2 + j] * d; return; }
    const bool has_m = type == 3 || type == 7, has_h = type == 6 || type == 7;
    const float d = hf(b), m = has_m ? hf(b + 2) : 0.0f;
    const uint8_t* qs = b + (has_m ? 4 : 2);
    uint32_t qh = 0;
    if (has_h) { memcpy(&qh, qs, 4); qs += 4; }
    const int off = has_m ? 0 : (has_h ? 16 : 8);
    for (int j = 0; j < 16; j++) {
        int x0 = qs[j] & 0x0F, x1 = qs[j] >> 4;
        if (has_h) { x0 |= ((qh >> j) << 4) & 0x10; x1 |= (qh >> (j + 12)) & 0x10; }
        y[j] = has_m ? (float)x0 * d + m : (float)(x0 - off) * d;
        y[j + 16] = has_m ? (float)x1 * d + m : (float)(x1 - off) * d;
    }
}

struct Layer {  // pointers into the tensor map
    const float *attn_ln_w, *attn_ln_b, *q_w, *q_b, *k_w, *v_w, *v_b, *o_w, *o_b;
    const float *x_ln_w, *x_ln_b, *xq_w, *xq_b, *xk_w, *xv_w, *xv_b, *xo_w, *xo_b;
    const float *mlp_ln_w, *mlp_ln_b, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
};

struct Model {
    Hparams hp;
    int mode = 1;  // 1 = ggml f16 numerics, 0 = pure f32
    int n_threads = 8;
    int filt_n_mel = 0, filt_n_fft = 0;
    std::vector<float> filters;
    Vocab vocab;
    std::map<std::string, Tensor> t;
    std::vector<Layer> enc, dec;
    const float *conv1_w, *conv1_b, *conv2_w, *conv2_b, *e_pe, *e_ln_w, *e_ln_b;
    const float *d_pe, *d_te, *d_ln_w, *d_ln_b;
    // token embedding rows for the lookup: == d_te, except for a quantized embedding, whose
    // ggml_get_rows rows are the exact f32 dequantization while its matmul (the logits) reads the
    // blocks dequantized into f16 tiles (ggml's GPU back-ends; mode 1)
    std::vector<float> te_lookup;
    const float* d_te_lookup = nullptr;
};

static const float* T(Model& m, const std::string& name) {
    auto it = m.t.find(name);
    if (it == m.t.end()) { fprintf(stderr, "oracle: missing tensor %s\n", name.c_str()); abort(); }
    return it->second.data.data();
}

// [ext] whisper_model_load: header, mel filters, vocab (+ special-token shift and synthesis of
// the extra tokens up to n_vocab), tensors (f16 -> f32 here; every value stays f16-exact).
static Model* load_model(const char* path, int mode, int n_threads) {
    FILE* f = fopen(path, "rb");
    if (!f) return nullptr;
    auto rd = [&](void* p, size_t n) { if (fread(p, 1, n, f) != n) throw 1; };
    Model* m = new Model();
    m->mode = mode; m->n_threads = n_threads;
    try {
        uint32_t magic; rd(&magic, 4);
        if (magic != 0x67676d6c) throw 1;
        rd(&m->hp, sizeof(Hparams));
        m->hp.ftype %= 1000;  // + 1000 * GGML_QNT_VERSION on quantized files
        rd(&m->filt_n_mel, 4); rd(&m->filt_n_fft, 4);
        m->filters.resize((size_t)m->filt_n_mel * m->filt_n_fft);
        rd(m->filters.data(), m->filters.size() * 4);
        int32_t n_vocab_file; rd(&n_vocab_file, 4);
        Vocab& v = m->vocab;
        v.n_vocab = m->hp.n_vocab;
        v.id_to_token.assign(m->hp.n_vocab, "");
        for (int i = 0; i < n_vocab_file; i++) {
            uint32_t len; rd(&len, 4);
            std::string w(len, '\0');
            if (len) rd(&w[0], len);
            v.token_to_id[w] = i;
            if (i < (int)v.id_to_token.size()) v.id_to_token[i] = w; else v.id_to_token.push_back(w);
        }
        if (v.is_multilingual()) {
            v.token_eot++; v.token_sot++;
            const int dt = v.num_languages() - 98;
            v.token_translate += dt; v.token_transcribe += dt; v.token_solm += dt; v.token_prev += dt;
            v.token_nosp += dt; v.token_not += dt; v.token_beg += dt;
        }
        for (int i = n_vocab_file; i < m->hp.n_vocab; i++) {
            std::string w;
            if (i > v.token_beg) w = "[_TT_" + std::to_string(i - v.token_beg) + "]";
            else if (i == v.token_eot) w = "[_EOT_]";
            else if (i == v.token_sot) w = "[_SOT_]";
            else if (i == v.token_translate) w = "[_TRANSLATE_]";
            else if (i == v.token_transcribe) w = "[_TRANSCRIBE_]";
            else if (i == v.token_solm) w = "[_SOLM_]";
            else if (i == v.token_prev) w = "[_PREV_]";
            else if (i == v.token_nosp) w = "[_NOSP_]";
            else if (i == v.token_not) w = "[_NOT_]";
            else if (i == v.token_beg) w = "[_BEG_]";
            else if (i > v.token_sot && i <= v.token_sot + v.num_languages())
                w = "[_LANG_" + std::string(k_lang_codes[i - v.token_sot - 1]) + "]";
            else w = "[_extra_token_" + std::to_string(i) + "]";
            v.token_to_id[w] = i;
            v.id_to_token[i] = w;
        }
        while (true) {
            int32_t n_dims, name_len, ttype;
            if (fread(&n_dims, 4, 1, f) != 1) break;
            rd(&name_len, 4); rd(&ttype, 4);
            Tensor tt; tt.ne.resize(n_dims);
            size_t nel = 1;
            for (int i = 0; i < n_dims; i++) { rd(&tt.ne[i], 4); nel *= tt.ne[i]; }
            std::string name(name_len, '\0'); rd(&name[0], name_len);
            tt.data.resize(nel);
            tt.type = ttype;
            if (ttype == 0) rd(tt.data.data(), nel * 4);
            else if (ttype == 1) {
                std::vector<uint16_t> h(nel); rd(h.data(), nel * 2);
                for (size_t i = 0; i < nel; i++) tt.data[i] = f16_to_f32(h[i]);
            } else if (block_bytes(ttype) && nel % 32 == 0) {
                std::vector<uint8_t> q(nel / 32 * block_bytes(ttype));
                rd(q.data(), q.size());
                for (size_t blk = 0; blk < nel / 32; blk++) dequant_block(ttype, q.data() + blk * block_bytes(ttype), &tt.data[blk * 32]);
            } else throw 2;
            m->t[name] = std::move(tt);
        }
    } catch (...) { fclose(f); delete m; return nullptr; }
    fclose(f);
    Model& M = *m;
    M.conv1_w = T(M, "encoder.conv1.weight"); M.conv1_b = T(M, "encoder.conv1.bias");
    M.conv2_w = T(M, "encoder.conv2.weight"); M.conv2_b = T(M, "encoder.conv2.bias");
    M.e_pe = T(M, "encoder.positional_embedding");
    M.e_ln_w = T(M, "encoder.ln_post.weight"); M.e_ln_b = T(M, "encoder.ln_post.bias");
    M.d_pe = T(M, "decoder.positional_embedding"); M.d_te = T(M, "decoder.token_embedding.weight");
    M.d_ln_w = T(M, "decoder.ln.weight"); M.d_ln_b = T(M, "decoder.ln.bias");
    M.d_te_lookup = M.d_te;
    for (auto& kv : M.t) {
        if (kv.second.type < 2) continue;
        if (kv.first == "decoder.token_embedding.weight") {
            M.te_lookup = kv.second.data;
            M.d_te_lookup = M.te_lookup.data();
        }
        if (M.mode) for (auto& x : kv.second.data) x = round_f16(x);  // f16 tiles of the GPU matmul
    }
    for (int i = 0; i < M.hp.n_audio_layer; i++) {
        std::string p = "encoder.blocks." + std::to_string(i) + ".";
        Layer L{};
        L.attn_ln_w = T(M, p + "attn_ln.weight"); L.attn_ln_b = T(M, p + "attn_ln.bias");
        L.q_w = T(M, p + "attn.query.weight"); L.q_b = T(M, p + "attn.query.bias");
        L.k_w = T(M, p + "attn.key.weight");
        L.v_w = T(M, p + "attn.value.weight"); L.v_b = T(M, p + "attn.value.bias");
        L.o_w = T(M, p + "attn.out.weight"); L.o_b = T(M, p + "attn.out.bias");
        L.mlp_ln_w = T(M, p + "mlp_ln.weight"); L.mlp_ln_b = T(M, p + "mlp_ln.bias");
        L.fc1_w = T(M, p + "mlp.0.weight"); L.fc1_b = T(M, p + "mlp.0.bias");
        L.fc2_w = T(M, p + "mlp.2.weight"); L.fc2_b = T(M, p + "mlp.2.bias");
        M.enc.push_back(L);
    }
    for (int i = 0; i < M.hp.n_text_layer; i++) {
        std::string p = "decoder.blocks." + std::to_string(i) + ".";
        Layer L{};
        L.attn_ln_w = T(M, p + "attn_ln.weight"); L.attn_ln_b = T(M, p + "attn_ln.bias");
        L.q_w = T(M, p + "attn.query.weight"); L.q_b = T(M, p + "attn.query.bias");
        L.k_w = T(M, p + "attn.key.weight");
        L.v_w = T(M, p + "attn.value.weight"); L.v_b = T(M, p + "attn.value.bias");
        L.o_w = T(M, p + "attn.out.weight"); L.o_b = T(M, p + "attn.out.bias");
        L.x_ln_w = T(M, p + "cross_attn_ln.weight"); L.x_ln_b = T(M, p + "cross_attn_ln.bias");
        L.xq_w = T(M, p + "cross_attn.query.weight"); L.xq_b = T(M, p + "cross_attn.query.bias");
        L.xk_w = T(M, p + "cross_attn.key.weight");
        L.xv_w = T(M, p + "cross_attn.value.weight"); L.xv_b = T(M, p + "cross_attn.value.bias");
        L.xo_w = T(M, p + "cross_attn.out.weight"); L.xo_b = T(M, p + "cross_attn.out.bias");
        L.mlp_ln_w = T(M, p + "mlp_ln.weight"); L.mlp_ln_b = T(M, p + "mlp_ln.bias");
        L.fc1_w = T(M, p + "mlp.0.weight"); L.fc1_b = T(M, p + "mlp.0.bias");
        L.fc2_w = T(M, p + "mlp.2.weight"); L.fc2_b = T(M, p + "mlp.2.bias");
        M.dec.push_back(L);
    }
    return m;
}

// ------------------------------------------------------------------------------------------------
// numerics helpers
static inline float rnd(const Model& m, float x) { return m.mode ? round_f16(x) : x; }
static void rnd_vec(const Model& m, std::vector<float>& v) { if (m.mode) for (auto& x : v) x = round_f16(x); }

// Y[M][N] = X[M][K] . W[N][K]^T (+ bias[N]); f32 accumulation (ggml mul_mat + ggml_add).
static void gemm_nt(const Model& m, const float* X, int M, int K, const float* W, int N, const float* bias, float* Y) {
    const int MB = 8, NB = 32;
#pragma omp parallel for collapse(2) schedule(dynamic) num_threads(m.n_threads)
    for (int i0 = 0; i0 < M; i0 += MB)
        for (int j0 = 0; j0 < N; j0 += NB) {
            const int i1 = std::min(M, i0 + MB), j1 = std::min(N, j0 + NB);
            for (int j = j0; j < j1; j++) {
                const float* w = W + (size_t)j * K;
                for (int i = i0; i < i1; i++) {
                    const float* x = X + (size_t)i * K;
                    float acc = 0.0f;
#pragma omp simd reduction(+ : acc)
                    for (int k = 0; k < K; k++) acc += x[k] * w[k];
                    Y[(size_t)i * N + j] = bias ? acc + bias[j] : acc;
                }
            }
        }
}

// ggml_norm (double sums) then ggml_mul(w) and ggml_add(b); output optionally f16-rounded for
// the following matmul's src1 conversion.
static void layer_norm(const Model& m, const float* x, int M, int D, const float* w, const float* b, float* y) {
#pragma omp parallel for num_threads(m.n_threads)
    for (int i = 0; i < M; i++) {
        const float* xr = x + (size_t)i * D;
        float* yr = y + (size_t)i * D;
        double sum = 0.0;
        for (int k = 0; k < D; k++) sum += (double)xr[k];
        float mean = sum / D;
        double sum2 = 0.0;
        for (int k = 0; k < D; k++) { float v = xr[k] - mean; yr[k] = v; sum2 += (double)(v * v); }
        float variance = sum2 / D;
        const float scale = 1.0f / sqrtf(variance + 1e-5f);
        for (int k = 0; k < D; k++) { float t = yr[k] * scale; t = t * w[k]; yr[k] = t + b[k]; }
    }
}

static inline float gelu_f32(float x) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
}

// ggml_vec_gelu_f32 with GGML_GELU_FP16: table of f16(gelu(f16 x)); |x| >= 10 shortcuts.
static std::vector<uint16_t> g_gelu_table;
static inline float gelu_ggml(const Model& m, float x) {
    if (!m.mode) return gelu_f32(x);
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return f16_to_f32(g_gelu_table[f32_to_f16(x)]);
}

// softmax_ext over n values (scale then max, expf, double sum, multiply by 1/sum)
static void softmax_row(float* s, int n, float scale) {
    float mx = -INFINITY;
    for (int i = 0; i < n; i++) { s[i] *= scale; mx = std::max(mx, s[i]); }
    double sum = 0.0;
    for (int i = 0; i < n; i++) { float v = (s[i] == -INFINITY) ? 0.0f : expf(s[i] - mx); sum += (double)v; s[i] = v; }
    const float inv = (float)(1.0 / sum);
    for (int i = 0; i < n; i++) s[i] *= inv;
}

// ------------------------------------------------------------------------------------------------
// encoder: mel window [n_mels][2*n_ctx] -> embd_enc [n_ctx][d]
static void encode(Model& m, const std::vector<float>& mel, int n_len, int seek, std::vector<float>& out) {
    const int n_mels = m.hp.n_mels, d = m.hp.n_audio_state, n_ctx = m.hp.n_audio_ctx, H = m.hp.n_audio_head;
    const int T2 = 2 * n_ctx, dh = d / H;
    // window copy with zero fill past n_len (whisper_encode_internal input set)
    std::vector<float> win((size_t)n_mels * T2, 0.0f);
    const int i0 = std::min(seek, n_len), i1 = std::min(seek + T2, n_len);
    for (int j = 0; j < n_mels; j++)
        for (int i = i0; i < i1; i++) win[(size_t)j * T2 + (i - i0)] = mel[(size_t)j * n_len + i];
    // conv1: im2col (f16) [T2][n_mels*3], pad 1
    std::vector<float> col((size_t)T2 * n_mels * 3);
    for (int t = 0; t < T2; t++)
        for (int c = 0; c < n_mels; c++)
            for (int k = 0; k < 3; k++) {
                int ti = t + k - 1;
                col[((size_t)t * n_mels + c) * 3 + k] = (ti >= 0 && ti < T2) ? rnd(m, win[(size_t)c * T2 + ti]) : 0.0f;
            }
    std::vector<float> h1((size_t)T2 * d);
    gemm_nt(m, col.data(), T2, n_mels * 3, m.conv1_w, d, nullptr, h1.data());
    for (int t = 0; t < T2; t++) for (int o = 0; o < d; o++) {
        float v = h1[(size_t)t * d + o] + m.conv1_b[o];
        h1[(size_t)t * d + o] = gelu_ggml(m, v);
    }
    // conv2: stride 2, pad 1; im2col over h1 (time-major here: h1[t][c])
    col.assign((size_t)n_ctx * d * 3, 0.0f);
    for (int t = 0; t < n_ctx; t++)
        for (int c = 0; c < d; c++)
            for (int k = 0; k < 3; k++) {
                int ti = 2 * t + k - 1;
                col[((size_t)t * d + c) * 3 + k] = (ti >= 0 && ti < T2) ? rnd(m, h1[(size_t)ti * d + c]) : 0.0f;
            }
    std::vector<float> x((size_t)n_ctx * d);
    gemm_nt(m, col.data(), n_ctx, d * 3, m.conv2_w, d, nullptr, x.data());
    for (int t = 0; t < n_ctx; t++) for (int o = 0; o < d; o++) {
        float v = x[(size_t)t * d + o] + m.conv2_b[o];
        v = gelu_ggml(m, v);
        x[(size_t)t * d + o] = v + m.e_pe[(size_t)t * d + o];
    }
    std::vector<float> h((size_t)n_ctx * d), q((size_t)n_ctx * d), k((size_t)n_ctx * d), v((size_t)n_ctx * d),
        att((size_t)n_ctx * d), tmp((size_t)n_ctx * d), ff((size_t)n_ctx * 4 * d);
    const float KQscale = 1.0f / sqrtf(float(dh));
    for (const Layer& L : m.enc) {
        layer_norm(m, x.data(), n_ctx, d, L.attn_ln_w, L.attn_ln_b, h.data());
        rnd_vec(m, h);
        gemm_nt(m, h.data(), n_ctx, d, L.q_w, d, L.q_b, q.data());
        gemm_nt(m, h.data(), n_ctx, d, L.k_w, d, nullptr, k.data());
        gemm_nt(m, h.data(), n_ctx, d, L.v_w, d, L.v_b, v.data());
        rnd_vec(m, q); rnd_vec(m, k); rnd_vec(m, v);
#pragma omp parallel num_threads(m.n_threads)
        {
            std::vector<float> s(n_ctx);
#pragma omp for collapse(2) schedule(dynamic)
            for (int hh = 0; hh < H; hh++)
                for (int i = 0; i < n_ctx; i++) {
                    const float* qi = &q[(size_t)i * d + hh * dh];
                    for (int j = 0; j < n_ctx; j++) {
                        const float* kj = &k[(size_t)j * d + hh * dh];
                        float acc = 0.0f;
                        for (int c = 0; c < dh; c++) acc += qi[c] * kj[c];
                        s[j] = acc;
                    }
                    softmax_row(s.data(), n_ctx, KQscale);
                    for (int j = 0; j < n_ctx; j++) s[j] = rnd(m, s[j]);
                    float* o = &att[(size_t)i * d + hh * dh];
                    for (int c = 0; c < dh; c++) o[c] = 0.0f;
                    for (int j = 0; j < n_ctx; j++) {
                        const float* vj = &v[(size_t)j * d + hh * dh];
                        const float p = s[j];
                        for (int c = 0; c < dh; c++) o[c] += p * vj[c];
                    }
                }
        }
        rnd_vec(m, att);
        gemm_nt(m, att.data(), n_ctx, d, L.o_w, d, L.o_b, tmp.data());
        for (size_t i = 0; i < x.size(); i++) x[i] = tmp[i] + x[i];
        layer_norm(m, x.data(), n_ctx, d, L.mlp_ln_w, L.mlp_ln_b, h.data());
        rnd_vec(m, h);
        gemm_nt(m, h.data(), n_ctx, d, L.fc1_w, 4 * d, L.fc1_b, ff.data());
        for (auto& f : ff) f = rnd(m, gelu_ggml(m, f));
        gemm_nt(m, ff.data(), n_ctx, 4 * d, L.fc2_w, d, L.fc2_b, tmp.data());
        for (size_t i = 0; i < x.size(); i++) x[i] = tmp[i] + x[i];
    }
    out.resize((size_t)n_ctx * d);
    layer_norm(m, x.data(), n_ctx, d, m.e_ln_w, m.e_ln_b, out.data());
}

// ------------------------------------------------------------------------------------------------
struct TokenData { int id, tid; float p, plog, pt, ptsum; };

struct Sequence {
    std::vector<TokenData> tokens;
    int result_len = 0;
    double sum_logprobs_all = 0, sum_logprobs = -INFINITY, avg_logprobs = -INFINITY, entropy = 0, score = -INFINITY;
};

struct Decoder {
    Sequence sequence;
    int seek_delta = 3000;
    bool failed = false, completed = false, has_ts = false;
    std::vector<float> probs, logits, logprobs;
    std::mt19937 rng{0};
    float ts_gap = 1e9f;  // |timestamp logprob mass - best text logprob| of the last step (a close call too)
};

struct Segment { int64_t t0, t1; std::string text; float no_speech_prob; std::vector<TokenData> tokens; };

struct State {
    std::vector<float> mel; int n_len = 0, n_len_org = 0;
    std::vector<float> enc;                  // [n_ctx][d]
    std::vector<std::vector<float>> ck, cv;  // cross K/V per layer [n_ctx][d] (f16-rounded in ggml mode)
    std::vector<std::vector<float>> sk, sv;  // self K/V per layer [n_text_ctx][d]
    std::vector<float> logits;               // last decode: [n_tokens][V]
    Decoder decoder;
    std::vector<Segment> result;
    std::vector<int> prompt_past;
    int lang_id = 0;
    float no_speech_prob = 0.0f;
    // diagnostics for tests: per greedy step the top-2 log-probability gap of the chosen token
    std::vector<float> step_margin;
    std::vector<int> step_token, step_seek;  // the greedy choice of each such step and its window's seek
    std::vector<int> seg_seek;               // per result segment: the seek of the window it came from
    // fixed-work mode only: the raw logits row of every step (prefill's last row, then each decode), the
    // rows a teacher-forced pass along the greedy sequence would produce (tests compare GPU logits with them)
    std::vector<float> step_logits;
    int cur_seek = 0;
    // per decoded window: the temperature-fallback decisions (the record whisper_mi355x.h exposes)
    struct Decision { int seek, temp_idx, failed0, logprob_fail0, result_len0, no_speech; float avg_logprob0, entropy0, no_speech_prob, pad; };
    std::vector<Decision> decisions;
};

static void compute_cross(Model& m, State& s) {
    const int d = m.hp.n_text_state, n_ctx = m.hp.n_audio_ctx, dh = d / m.hp.n_text_head;
    const float Kscale = powf(float(dh), -0.25f);
    std::vector<float> h = s.enc;
    rnd_vec(m, h);
    s.ck.assign(m.hp.n_text_layer, {}); s.cv.assign(m.hp.n_text_layer, {});
    for (int l = 0; l < m.hp.n_text_layer; l++) {
        const Layer& L = m.dec[l];
        s.ck[l].resize((size_t)n_ctx * d); s.cv[l].resize((size_t)n_ctx * d);
        gemm_nt(m, h.data(), n_ctx, d, L.xk_w, d, nullptr, s.ck[l].data());
        gemm_nt(m, h.data(), n_ctx, d, L.xv_w, d, L.xv_b, s.cv[l].data());
        for (auto& x : s.ck[l]) x = rnd(m, x * Kscale);
        rnd_vec(m, s.cv[l]);
    }
}

// decode n tokens for one sequence at positions n_past.. ; fills s.logits [n][V]
static void decode(Model& m, State& s, const int* tokens, int n, int n_past) {
    const int d = m.hp.n_text_state, H = m.hp.n_text_head, dh = d / H, V = m.hp.n_vocab;
    const int n_ctx_a = m.hp.n_audio_ctx;
    const float KQscale = powf(float(dh), -0.25f);
    if (s.sk.empty()) {
        s.sk.assign(m.hp.n_text_layer, std::vector<float>((size_t)m.hp.n_text_ctx * d, 0.0f));
        s.sv.assign(m.hp.n_text_layer, std::vector<float>((size_t)m.hp.n_text_ctx * d, 0.0f));
    }
    std::vector<float> x((size_t)n * d), h((size_t)n * d), q((size_t)n * d), k((size_t)n * d), v((size_t)n * d),
        att((size_t)n * d), tmp((size_t)n * d), ff((size_t)n * 4 * d);
    for (int i = 0; i < n; i++)
        for (int c = 0; c < d; c++)
            x[(size_t)i * d + c] = m.d_te_lookup[(size_t)tokens[i] * d + c] + m.d_pe[(size_t)(n_past + i) * d + c];
    auto attend = [&](const float* Q, const float* K, const float* Vv, int n_kv_of_i_base, bool causal, float* O) {
        // Q [n][d] (already scaled + rounded), K/V [n_kv][d]
#pragma omp parallel num_threads(m.n_threads)
        {
            std::vector<float> sc(std::max(n_ctx_a, m.hp.n_text_ctx));
#pragma omp for collapse(2)
            for (int hh = 0; hh < H; hh++)
                for (int i = 0; i < n; i++) {
                    const int n_kv = causal ? (n_kv_of_i_base + i + 1) : n_kv_of_i_base;
                    const float* qi = Q + (size_t)i * d + hh * dh;
                    for (int j = 0; j < n_kv; j++) {
                        const float* kj = K + (size_t)j * d + hh * dh;
                        float acc = 0.0f;
                        for (int c = 0; c < dh; c++) acc += qi[c] * kj[c];
                        sc[j] = acc;
                    }
                    softmax_row(sc.data(), n_kv, 1.0f);
                    float* o = O + (size_t)i * d + hh * dh;
                    for (int c = 0; c < dh; c++) o[c] = 0.0f;
                    for (int j = 0; j < n_kv; j++) {
                        const float p = rnd(m, sc[j]);
                        const float* vj = Vv + (size_t)j * d + hh * dh;
                        for (int c = 0; c < dh; c++) o[c] += p * vj[c];
                    }
                }
        }
    };
    for (int l = 0; l < m.hp.n_text_layer; l++) {
        const Layer& L = m.dec[l];
        layer_norm(m, x.data(), n, d, L.attn_ln_w, L.attn_ln_b, h.data());
        rnd_vec(m, h);
        gemm_nt(m, h.data(), n, d, L.q_w, d, L.q_b, q.data());
        gemm_nt(m, h.data(), n, d, L.k_w, d, nullptr, k.data());
        gemm_nt(m, h.data(), n, d, L.v_w, d, L.v_b, v.data());
        for (auto& t : q) t = rnd(m, t * KQscale);
        for (int i = 0; i < n; i++)
            for (int c = 0; c < d; c++) {
                s.sk[l][(size_t)(n_past + i) * d + c] = rnd(m, k[(size_t)i * d + c] * KQscale);
                s.sv[l][(size_t)(n_past + i) * d + c] = rnd(m, v[(size_t)i * d + c]);
            }
        attend(q.data(), s.sk[l].data(), s.sv[l].data(), n_past, true, att.data());
        rnd_vec(m, att);
        gemm_nt(m, att.data(), n, d, L.o_w, d, L.o_b, tmp.data());
        for (size_t i = 0; i < x.size(); i++) x[i] = tmp[i] + x[i];
        layer_norm(m, x.data(), n, d, L.x_ln_w, L.x_ln_b, h.data());
        rnd_vec(m, h);
        gemm_nt(m, h.data(), n, d, L.xq_w, d, L.xq_b, q.data());
        for (auto& t : q) t = rnd(m, t * KQscale);
        attend(q.data(), s.ck[l].data(), s.cv[l].data(), n_ctx_a, false, att.data());
        rnd_vec(m, att);
        gemm_nt(m, att.data(), n, d, L.xo_w, d, L.xo_b, tmp.data());
        for (size_t i = 0; i < x.size(); i++) x[i] = tmp[i] + x[i];
        layer_norm(m, x.data(), n, d, L.mlp_ln_w, L.mlp_ln_b, h.data());
        rnd_vec(m, h);
        gemm_nt(m, h.data(), n, d, L.fc1_w, 4 * d, L.fc1_b, ff.data());
        for (auto& f : ff) f = rnd(m, gelu_ggml(m, f));
        gemm_nt(m, ff.data(), n, 4 * d, L.fc2_w, d, L.fc2_b, tmp.data());
        for (size_t i = 0; i < x.size(); i++) x[i] = tmp[i] + x[i];
    }
    layer_norm(m, x.data(), n, d, m.d_ln_w, m.d_ln_b, h.data());
    rnd_vec(m, h);
    s.logits.resize((size_t)n * V);
    gemm_nt(m, h.data(), n, d, m.d_te, V, nullptr, s.logits.data());
}

// ------------------------------------------------------------------------------------------------
// [ext] tokenize(): GPT-2 regex pre-split, then greedy longest-prefix match in token_to_id.
static std::vector<int> tokenize(const Vocab& vocab, const std::string& text) {
    std::vector<std::string> words;
    {
        std::string str = text;
        std::string pat = R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)";
        std::regex re(pat);
        std::smatch mm;
        while (std::regex_search(str, mm, re)) {
            for (auto x : mm) words.push_back(x);
            str = mm.suffix();
        }
    }
    std::vector<int> tokens;
    for (const auto& word : words) {
        if (word.empty()) continue;
        int i = 0, n = (int)word.size();
        while (i < n) {
            int j = n;
            bool found = false;
            while (j > i) {
                auto it = vocab.token_to_id.find(word.substr(i, j - i));
                if (it != vocab.token_to_id.end()) { tokens.push_back(it->second); i = j; found = true; break; }
                --j;
            }
            if (!found) ++i;
        }
    }
    return tokens;
}

// ------------------------------------------------------------------------------------------------
struct OracleParams {      // the whisper_full_params fields the reference sets (+ defaults)
    const char* language;  // NULL / "" / "auto" => auto-detect
    const char* initial_prompt;
    int n_max_text_ctx, offset_ms, duration_ms;
    int translate, no_context, no_timestamps, single_segment, print_special, suppress_blank, max_tokens;
    float temperature, temperature_inc, max_initial_ts, length_penalty, entropy_thold, logprob_thold, no_speech_thold;
    int best_of;
    int fixed_tokens;      // mi355x extension: >0 => fixed-work mode (EOT suppressed, no fallback)
};

static void compute_logprobs(const std::vector<float>& logits, int n, std::vector<float>& logprobs) {
    const float logit_max = *std::max_element(logits.begin(), logits.begin() + n);
    float lse = 0.0f;
    for (int i = 0; i < n; ++i) if (logits[i] > -INFINITY) lse += expf(logits[i] - logit_max);
    lse = logf(lse) + logit_max;
    for (int i = 0; i < n; ++i) logprobs[i] = logits[i] > -INFINITY ? logits[i] - lse : -INFINITY;
}
static void compute_probs(const std::vector<float>& logits, int n, const std::vector<float>& logprobs, std::vector<float>& probs) {
    for (int i = 0; i < n; ++i) probs[i] = logits[i] == -INFINITY ? 0.0f : expf(logprobs[i]);
}

// [ext] whisper_process_logits
static void process_logits(Model& m, State& s, Decoder& dec, const OracleParams& p, float temperature, const float* row) {
    const Vocab& vocab = m.vocab;
    const auto& toks = dec.sequence.tokens;
    const bool is_initial = toks.empty();
    const int n = vocab.n_vocab;
    dec.logits.assign(row, row + n);
    dec.probs.resize(n); dec.logprobs.resize(n);
    auto& logits = dec.logits;
    if (temperature > 0.0f) for (int i = 0; i < n; i++) logits[i] /= temperature;
    if (p.suppress_blank && is_initial) {
        logits[vocab.token_eot] = -INFINITY;
        logits[vocab.token_to_id.at(" ")] = -INFINITY;
    }
    logits[vocab.token_not] = -INFINITY;
    if (p.no_timestamps) for (int i = vocab.token_beg; i < n; ++i) logits[i] = -INFINITY;
    logits[vocab.token_sot] = -INFINITY;
    logits[vocab.token_nosp] = -INFINITY;
    logits[vocab.token_solm] = -INFINITY;  // tdrz disabled
    logits[vocab.token_translate] = -INFINITY;
    logits[vocab.token_transcribe] = -INFINITY;
    logits[vocab.token_prev] = -INFINITY;
    for (int i = 0; i < k_n_lang; ++i) logits[vocab.token_sot + 1 + i] = -INFINITY;
    logits[vocab.token_prev] = -INFINITY;
    if (p.fixed_tokens > 0) logits[vocab.token_eot] = -INFINITY;  // fixed-work mode only
    {
        const bool last_was_ts = toks.size() > 0 && toks.back().id >= vocab.token_beg;
        const bool penult_was_ts = toks.size() < 2 || toks[toks.size() - 2].id >= vocab.token_beg;
        if (last_was_ts) {
            if (penult_was_ts) for (int i = vocab.token_beg; i < n; ++i) logits[i] = -INFINITY;
            else for (int i = 0; i < vocab.token_eot; ++i) logits[i] = -INFINITY;
        }
    }
    if (is_initial && p.max_initial_ts > 0.0f) {
        const float precision = float(30) / m.hp.n_audio_ctx;
        const int tid0 = std::round(p.max_initial_ts / precision);
        for (int i = vocab.token_beg + tid0 + 1; i < n; ++i) logits[i] = -INFINITY;
    }
    if (dec.has_ts) {
        const int tid0 = dec.seek_delta / 2;
        for (int i = vocab.token_beg; i < vocab.token_beg + tid0; ++i) logits[i] = -INFINITY;
    }
    compute_logprobs(logits, n, dec.logprobs);
    {
        float ts_logprob = -INFINITY;
        {
            float lse = 0.0f;
            const float mx = *std::max_element(dec.logprobs.begin() + vocab.token_beg, dec.logprobs.end());
            for (int i = vocab.token_beg; i < n; ++i) if (dec.logprobs[i] > -INFINITY) lse += expf(dec.logprobs[i] - mx);
            if (lse > 0.0f) ts_logprob = logf(lse) + mx;
        }
        const float max_text = *std::max_element(dec.logprobs.begin(), dec.logprobs.begin() + vocab.token_beg);
        dec.ts_gap = ts_logprob > -INFINITY && max_text > -INFINITY ? fabsf(ts_logprob - max_text) : 1e9f;
        if (ts_logprob > max_text)
            for (int i = 0; i < vocab.token_beg; ++i) { logits[i] = -INFINITY; dec.logprobs[i] = -INFINITY; }
    }
    compute_probs(logits, n, dec.logprobs, dec.probs);
}

// [ext] whisper_sample_token
static TokenData sample_token(Model& m, State& s, Decoder& dec, bool best) {
    TokenData r = {0, 0, 0.0f, 0.0f, 0.0f, 0.0f};
    const Vocab& vocab = m.vocab;
    const int n = vocab.n_vocab;
    const auto& probs = dec.probs;
    {
        double sum_ts = 0.0, max_ts = 0.0;
        for (int i = vocab.token_beg; i < n; i++) {
            if (probs[i] == -INFINITY) continue;
            sum_ts += probs[i];
            if (max_ts < probs[i]) { max_ts = probs[i]; r.tid = i; }
        }
        r.pt = max_ts / (sum_ts + 1e-10);
        r.ptsum = sum_ts;
    }
    if (best) {
        float second = 0.0f;
        for (int i = 0; i < n; ++i) {
            if (r.p < probs[i]) { second = r.p; r.id = i; r.p = probs[i]; r.plog = dec.logprobs[i]; }
            else if (second < probs[i]) second = probs[i];
        }
        // how far the greedy choice is from flipping: its top-2 log-probability gap, or the gap of the
        // timestamp rule (timestamp mass vs best text token) that shaped this step's candidates
        s.step_margin.push_back(std::min(second > 0.0f ? logf(r.p) - logf(second) : 1e9f, dec.ts_gap));
        s.step_token.push_back(r.id);
        s.step_seek.push_back(s.cur_seek);
    } else {
        std::discrete_distribution<> dist(probs.begin(), probs.end());
        r.id = dist(dec.rng);
        r.p = probs[r.id];
        r.plog = dec.logprobs[r.id];
    }
    if (r.id >= vocab.token_beg) { r.tid = r.id; r.pt = r.p; }
    return r;
}

// [ext] whisper_sequence_score (length_penalty default -1 => penalty = result_len)
static void sequence_score(const OracleParams& p, Sequence& seq) {
    if (seq.result_len == 0) return;
    double result = 0.0;
    for (int i = 0; i < seq.result_len; ++i) result += seq.tokens[i].plog;
    seq.sum_logprobs = result;
    seq.avg_logprobs = result / seq.result_len;
    double penalty = seq.result_len;
    if (p.length_penalty > 0.0f) penalty = pow((5.0 + penalty) / 6.0, p.length_penalty);
    seq.score = result / penalty;
    std::map<int, int> counts;
    int cnt = 0;
    for (int i = std::max(0, seq.result_len - 32); i < seq.result_len; ++i) { counts[seq.tokens[i].id]++; cnt++; }
    double entropy = 0.0;
    for (auto& kv : counts) { const double q = kv.second / (double)cnt; entropy -= q * log(q); }
    seq.entropy = entropy;
}

// [ext] whisper_lang_auto_detect_with_state (encoder at seek 0, decode [sot], argmax over g_lang)
static int lang_auto_detect(Model& m, State& s) {
    std::vector<float> enc_save;
    encode(m, s.mel, s.n_len, 0, s.enc);
    compute_cross(m, s);
    int sot = m.vocab.token_sot;
    decode(m, s, &sot, 1, 0);
    std::vector<std::pair<float, int>> ids;
    std::vector<std::string> codes(k_lang_codes, k_lang_codes + k_n_lang);
    std::map<std::string, int> g_lang;
    for (int i = 0; i < k_n_lang; i++) g_lang[codes[i]] = i;
    for (auto& kv : g_lang) ids.emplace_back(s.logits[m.vocab.token_sot + 1 + kv.second], kv.second);
    std::sort(ids.begin(), ids.end(), [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first > b.first; });
    return ids[0].second;
}

// [ext] whisper_full_with_state, greedy strategy (whisper-rs Greedy{best_of:1}, whisper.rs:88)
static int full(Model& m, State& s, OracleParams p, const float* samples, int n_samples) {
    s.result.clear();
    s.seg_seek.clear();
    s.step_margin.clear();
    s.step_token.clear();
    s.step_seek.clear();
    s.step_logits.clear();
    s.decisions.clear();
    if (n_samples > 0) s.n_len = mel_compute(samples, n_samples, m.filters.data(), m.filt_n_mel, m.filt_n_fft, s.mel, &s.n_len_org, m.n_threads);
    const Vocab& vocab = m.vocab;
    std::string lang_str;
    if (p.language == nullptr || strlen(p.language) == 0 || strcmp(p.language, "auto") == 0) {
        s.lang_id = lang_auto_detect(m, s);
        lang_str = k_lang_codes[s.lang_id];
        p.language = lang_str.c_str();
    }
    const int seek_start = p.offset_ms / 10;
    const int seek_end = p.duration_ms == 0 ? s.n_len_org : seek_start + p.duration_ms / 10;
    const int delta_min = 10;
    if (seek_end < seek_start + delta_min) return 0;
    std::vector<float> temperatures;
    if (p.temperature_inc > 0.0f && p.fixed_tokens <= 0)
        for (float t = p.temperature; t < 1.0f + 1e-6f; t += p.temperature_inc) temperatures.push_back(t);
    if (temperatures.empty()) temperatures.push_back(p.temperature);
    // best_of only affects sampled (t > 0) attempts; one candidate is sampled (Greedy{best_of:1})
    auto& prompt_past = s.prompt_past;
    if (p.no_context) prompt_past.clear();
    if (p.initial_prompt) {
        std::vector<int> pt = tokenize(vocab, p.initial_prompt);
        for (int t : pt) prompt_past.push_back(t);
        std::rotate(prompt_past.begin(), prompt_past.end() - pt.size(), prompt_past.end());
    }
    std::vector<int> prompt_init = {vocab.token_sot};
    if (vocab.is_multilingual()) {
        const int lid = lang_id(p.language);
        if (lid < 0) return -7;
        s.lang_id = lid;
        prompt_init.push_back(vocab.token_sot + 1 + lid);
        prompt_init.push_back(p.translate ? vocab.token_translate : vocab.token_transcribe);
    }
    {
        const bool is_distil = m.hp.n_text_layer == 2 && m.hp.n_vocab != 51866;
        if (is_distil && !p.no_timestamps) p.no_timestamps = 1;
    }
    if (p.no_timestamps) prompt_init.push_back(vocab.token_not);

    int seek = seek_start;
    std::vector<int> prompt;
    Decoder& dec = s.decoder;
    dec.rng = std::mt19937(0);
    const int n_max = m.hp.n_text_ctx / 2 - 4;
    const int n_steps = p.fixed_tokens > 0 ? p.fixed_tokens : n_max;
    while (true) {
        if (seek + delta_min >= seek_end) break;
        encode(m, s.mel, s.n_len, seek, s.enc);
        compute_cross(m, s);
        s.cur_seek = seek;
        if (seek > seek_start && seek + 500 >= seek_end) prompt_past.clear();
        State::Decision dn{};
        dn.seek = seek;
        for (int it = 0; it < (int)temperatures.size(); ++it) {
            const float t_cur = temperatures[it];
            dec.sequence = Sequence();
            dec.seek_delta = 100 * 30;
            dec.failed = dec.completed = dec.has_ts = false;
            prompt.clear();
            if (!prompt_past.empty() && t_cur < 0.5f && p.n_max_text_ctx > 0) {
                int n_take = std::min(std::min(p.n_max_text_ctx, m.hp.n_text_ctx / 2), (int)prompt_past.size());
                prompt = {vocab.token_prev};
                prompt.insert(prompt.begin() + 1, prompt_past.end() - n_take, prompt_past.end());
            }
            prompt.insert(prompt.end(), prompt_init.begin(), prompt_init.end());
            s.sk.clear(); s.sv.clear();
            decode(m, s, prompt.data(), (int)prompt.size(), 0);
            const int V = vocab.n_vocab;
            const float* last = s.logits.data() + (size_t)(prompt.size() - 1) * V;
            {   // no_speech probability before any filter (row = last prompt token)
                std::vector<float> lg(last, last + V), lp(V), pr(V);
                compute_logprobs(lg, V, lp);
                compute_probs(lg, V, lp, pr);
                s.no_speech_prob = pr[vocab.token_nosp];
            }
            if (p.fixed_tokens > 0) s.step_logits.insert(s.step_logits.end(), last, last + V);
            process_logits(m, s, dec, p, t_cur, last);
            for (int i = 0; i < n_steps; ++i) {
                dec.sequence.tokens.push_back(sample_token(m, s, dec, t_cur < 1e-6f));
                dec.sequence.sum_logprobs_all += dec.sequence.tokens.back().plog;
                {
                    const TokenData& tok = dec.sequence.tokens.back();
                    if (tok.id > vocab.token_beg) {
                        const int sd_new = 2 * (tok.id - vocab.token_beg);
                        if (dec.has_ts && dec.seek_delta > sd_new && dec.sequence.result_len < i && p.fixed_tokens <= 0) {
                            dec.failed = true;
                            break;
                        }
                        dec.seek_delta = sd_new;
                        dec.sequence.result_len = i + 1;
                        dec.has_ts = true;
                    }
                    if (p.fixed_tokens > 0) {
                        if (i == n_steps - 1) { dec.sequence.result_len = n_steps; dec.seek_delta = 3000; dec.completed = true; break; }
                    } else if (tok.id == vocab.token_eot || (p.max_tokens > 0 && i >= p.max_tokens) ||
                               (dec.has_ts && seek + dec.seek_delta + delta_min >= seek_end)) {
                        if (dec.sequence.result_len == 0 && !p.no_timestamps) {
                            if (seek + dec.seek_delta + delta_min >= seek_end) dec.sequence.result_len = i + 1;
                            else { dec.failed = true; break; }
                        }
                        if (p.single_segment || p.no_timestamps) { dec.sequence.result_len = i + 1; dec.seek_delta = 100 * 30; }
                        dec.completed = true;
                        break;
                    }
                }
                if (p.fixed_tokens <= 0 && i == n_max - 1 && (dec.sequence.result_len == 0 || dec.seek_delta < 100 * 30 / 2)) { dec.failed = true; break; }
                const int tok = dec.sequence.tokens.back().id;
                decode(m, s, &tok, 1, (int)prompt.size() + i);
                if (p.fixed_tokens > 0) s.step_logits.insert(s.step_logits.end(), s.logits.begin(), s.logits.begin() + V);
                process_logits(m, s, dec, p, t_cur, s.logits.data());
            }
            bool success = true;
            if (!dec.failed) {
                dec.sequence.tokens.resize(dec.sequence.result_len);
                sequence_score(p, dec.sequence);
                if (dec.sequence.result_len > 32 && dec.sequence.entropy < p.entropy_thold) dec.failed = true;
            }
            if (it == 0) {
                dn.failed0 = dec.failed;
                dn.logprob_fail0 = dec.sequence.avg_logprobs < p.logprob_thold;
                dn.result_len0 = dec.sequence.result_len;
                dn.avg_logprob0 = (float)dec.sequence.avg_logprobs;
                dn.entropy0 = (float)dec.sequence.entropy;
            }
            dn.temp_idx = it;
            if (it != (int)temperatures.size() - 1)
                if (dec.failed || dec.sequence.avg_logprobs < p.logprob_thold) success = false;
            if (success) break;
        }
        {
            int seek_delta = dec.seek_delta;
            const int result_len = dec.sequence.result_len;
            const auto& toks = dec.sequence.tokens;
            const bool is_no_speech = (s.no_speech_prob > p.no_speech_thold && dec.sequence.avg_logprobs < p.logprob_thold);
            dn.no_speech = is_no_speech;
            dn.no_speech_prob = s.no_speech_prob;
            s.decisions.push_back(dn);
            prompt_past.clear();
            if (prompt.front() == vocab.token_prev)
                prompt_past.insert(prompt_past.end(), prompt.begin() + 1, prompt.end() - prompt_init.size());
            for (int i = 0; i < result_len && !is_no_speech && i < (int)toks.size(); ++i) prompt_past.push_back(toks[i].id);
            if (!toks.empty() && !is_no_speech) {
                int i0 = 0;
                int64_t t0 = seek + 2 * (toks.front().tid - vocab.token_beg);
                std::string text;
                for (int i = 0; i < (int)toks.size(); i++) {
                    if (p.print_special || toks[i].id < vocab.token_eot) text += vocab.id_to_token[toks[i].id];
                    if (toks[i].id > vocab.token_beg && !p.single_segment) {
                        const int64_t t1 = seek + 2 * (toks[i].tid - vocab.token_beg);
                        if (!text.empty()) {
                            s.result.push_back({t0, t1, text, s.no_speech_prob, {}});
                            for (int j = i0; j <= i; j++) s.result.back().tokens.push_back(toks[j]);
                        }
                        text = "";
                        while (i < (int)toks.size() && toks[i].id > vocab.token_beg) i++;
                        i--;
                        t0 = t1;
                        i0 = i + 1;
                    }
                }
                if (!text.empty()) {
                    const int64_t t1 = seek + seek_delta;
                    s.result.push_back({t0, t1, text, s.no_speech_prob, {}});
                    for (int j = i0; j < (int)toks.size(); j++) s.result.back().tokens.push_back(toks[j]);
                }
            }
            s.seg_seek.resize(s.result.size(), seek);
            seek += seek_delta;
        }
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
// C API for ctypes (tests, golden generation, bench cpu_baseline)
extern "C" {

void* oracle_load(const char* path, int mode, int n_threads) {
    if (g_gelu_table.empty()) {
        g_gelu_table.resize(1 << 16);
        for (int i = 0; i < (1 << 16); i++) g_gelu_table[i] = f32_to_f16(gelu_f32(f16_to_f32((uint16_t)i)));
    }
    return load_model(path, mode, n_threads);
}
void oracle_free(void* m) { delete (Model*)m; }
// a loaded tensor as the oracle computes with it (dequantized; f16-rounded in mode 1), or with
// lookup != 0 the token-embedding rows of the decoder's lookup. Returns the element count.
long oracle_tensor(void* mp, const char* name, int lookup, float* out, long cap) {
    Model& m = *(Model*)mp;
    auto it = m.t.find(name);
    if (it == m.t.end()) return -1;
    const long n = (long)it->second.data.size();
    const float* src = lookup ? m.d_te_lookup : it->second.data.data();
    if (out && cap >= n) std::copy(src, src + n, out);
    return n;
}
void oracle_set_threads(void* m, int n) { ((Model*)m)->n_threads = n; }
void* oracle_state_new(void* m) { (void)m; return new State(); }
void oracle_state_free(void* s) { delete (State*)s; }

int oracle_token(void* mp, const char* which) {
    Vocab& v = ((Model*)mp)->vocab;
    std::string w(which);
    if (w == "eot") return v.token_eot;
    if (w == "sot") return v.token_sot;
    if (w == "beg") return v.token_beg;
    if (w == "not") return v.token_not;
    if (w == "prev") return v.token_prev;
    if (w == "nosp") return v.token_nosp;
    if (w == "solm") return v.token_solm;
    if (w == "transcribe") return v.token_transcribe;
    if (w == "translate") return v.token_translate;
    return -1;
}

// mel of full PCM into state; returns n_len (and n_len_org via ptr). copy out with oracle_state_mel
int oracle_mel(void* mp, void* sp, const float* pcm, int n, int* n_len_org) {
    Model& m = *(Model*)mp; State& s = *(State*)sp;
    s.n_len = mel_compute(pcm, n, m.filters.data(), m.filt_n_mel, m.filt_n_fft, s.mel, &s.n_len_org, m.n_threads);
    if (n_len_org) *n_len_org = s.n_len_org;
    return s.n_len;
}
void oracle_state_mel(void* sp, float* out) { State& s = *(State*)sp; std::copy(s.mel.begin(), s.mel.end(), out); }
void oracle_set_mel(void* mp, void* sp, const float* mel, int n_len) {
    Model& m = *(Model*)mp; State& s = *(State*)sp;
    s.mel.assign(mel, mel + (size_t)m.hp.n_mels * n_len); s.n_len = n_len;
}
// encoder at seek over the state's mel -> out [1500][d]; also computes the cross KV
void oracle_encode(void* mp, void* sp, int seek, float* out) {
    Model& m = *(Model*)mp; State& s = *(State*)sp;
    encode(m, s.mel, s.n_len, seek, s.enc);
    compute_cross(m, s);
    if (out) std::copy(s.enc.begin(), s.enc.end(), out);
}
void oracle_cross_kv(void* mp, void* sp, int layer, float* k_out, float* v_out) {
    State& s = *(State*)sp; (void)mp;
    std::copy(s.ck[layer].begin(), s.ck[layer].end(), k_out);
    std::copy(s.cv[layer].begin(), s.cv[layer].end(), v_out);
}
void oracle_kv_clear(void* sp) { State& s = *(State*)sp; s.sk.clear(); s.sv.clear(); }
// decode n tokens at n_past; logits_out [n][V]
void oracle_decode(void* mp, void* sp, const int* tokens, int n, int n_past, float* logits_out) {
    Model& m = *(Model*)mp; State& s = *(State*)sp;
    decode(m, s, tokens, n, n_past);
    if (logits_out) std::copy(s.logits.begin(), s.logits.end(), logits_out);
}
int oracle_tokenize(void* mp, const char* text, int* out, int cap) {
    auto t = tokenize(((Model*)mp)->vocab, text);
    if ((int)t.size() > cap) return -(int)t.size();
    std::copy(t.begin(), t.end(), out);
    return (int)t.size();
}
const char* oracle_token_str(void* mp, int id) { return ((Model*)mp)->vocab.id_to_token[id].c_str(); }
int oracle_lang_detect(void* mp, void* sp) { return lang_auto_detect(*(Model*)mp, *(State*)sp); }

int oracle_full(void* mp, void* sp, const OracleParams* p, const float* pcm, int n) {
    return full(*(Model*)mp, *(State*)sp, *p, pcm, n);
}
int oracle_n_segments(void* sp) { return (int)((State*)sp)->result.size(); }
const char* oracle_segment_text(void* sp, int i) { return ((State*)sp)->result[i].text.c_str(); }
void oracle_segment_t(void* sp, int i, int64_t* t0, int64_t* t1) { *t0 = ((State*)sp)->result[i].t0; *t1 = ((State*)sp)->result[i].t1; }
int oracle_segment_n_tokens(void* sp, int i) { return (int)((State*)sp)->result[i].tokens.size(); }
int oracle_segment_token(void* sp, int i, int j) { return ((State*)sp)->result[i].tokens[j].id; }
int oracle_lang(void* sp) { return ((State*)sp)->lang_id; }
float oracle_no_speech(void* sp) { return ((State*)sp)->no_speech_prob; }
int oracle_n_decisions(void* sp) { return (int)((State*)sp)->decisions.size(); }
void oracle_decisions(void* sp, void* out) {
    auto& d = ((State*)sp)->decisions;
    memcpy(out, d.data(), d.size() * sizeof(State::Decision));
}
int oracle_n_steps(void* sp) { return (int)((State*)sp)->step_margin.size(); }
// per greedy step (all windows, in decode order): the chosen token and the seek of its window
void oracle_step_tokens(void* sp, int* tok, int* seek) {
    const State& s = *(State*)sp;
    std::copy(s.step_token.begin(), s.step_token.end(), tok);
    std::copy(s.step_seek.begin(), s.step_seek.end(), seek);
}
// fixed-work mode: the raw logits rows of the last full() call ([rows][V]); returns the row count (copies
// only when cap >= rows * V)
long oracle_step_logits(void* mp, void* sp, float* out, long cap) {
    const State& s = *(State*)sp;
    const long V = ((Model*)mp)->vocab.n_vocab;
    const long n = (long)s.step_logits.size();
    if (out && cap >= n) std::copy(s.step_logits.begin(), s.step_logits.end(), out);
    return n / V;
}
int oracle_segment_seek(void* sp, int i) { return ((State*)sp)->seg_seek.at(i); }
void oracle_step_margins(void* sp, float* out) { auto& v = ((State*)sp)->step_margin; std::copy(v.begin(), v.end(), out); }
// last decoder attempt's full token list (ids) before result_len truncation is not kept; expose the final
int oracle_decoder_tokens(void* sp, int* out, int cap) {
    auto& t = ((State*)sp)->decoder.sequence.tokens;
    int n = std::min(cap, (int)t.size());
    for (int i = 0; i < n; i++) out[i] = t[i].id;
    return (int)t.size();
}

}  // extern "C"
