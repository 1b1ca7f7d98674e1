// GGML model file -> device weight arena (reference entry
// WhisperEngine::load_model -> WhisperContext::new_with_params, src-tauri/src/whisper.rs:36-52).
//
// The file layout is whisper.cpp's (`whisper_model_load` [ext], documented in
// tools/make_model.py). Weights are converted once on the host into the engine's layout and
// copied into ONE hipMalloc'ed arena so a multi-GPU node can broadcast them with a single RCCL
// call. Layout decisions (all K-contiguous [out][in] so every projection is an NT GEMM):
//   * Q,K,V of each self-attention concatenated into one [3d][d] matrix (K bias = 0);
//   * all decoder layers' cross-attention K,V concatenated into one [L_d*2*d][d] matrix, so the
//     whole cross-KV precompute is one GEMM per batch of windows;
//   * conv weights reordered [out][in][tap] -> [out][tap][in] (implicit im2col over a time-major
//     input);
//   * mel filterbank transposed to [201][n_mels] for coalesced reads in the mel kernel.
#include <cmath>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "engine.h"

namespace wm {

const char* const k_lang_codes[100] = {
    "en","zh","de","es","ru","ko","fr","ja","pt","tr","pl","ca","nl","ar","sv","it","id","hi","fi","vi",
    "he","uk","el","ms","cs","ro","da","hu","ta","no","th","ur","hr","bg","lt","la","mi","ml","cy","sk",
    "te","fa","lv","bn","sr","az","sl","kn","et","mk","br","eu","is","hy","ne","mn","bs","kk","sq","sw",
    "gl","mr","pa","si","km","sn","yo","so","af","oc","ka","be","tg","sd","gu","am","yi","lo","uz","fo",
    "ht","ps","tk","nn","mt","sa","lb","my","bo","tl","mg","as","tt","haw","ln","ha","ba","jw","su","yue"};
const char* const k_lang_names[100] = {
    "english","chinese","german","spanish","russian","korean","french","japanese","portuguese","turkish",
    "polish","catalan","dutch","arabic","swedish","italian","indonesian","hindi","finnish","vietnamese",
    "hebrew","ukrainian","greek","malay","czech","romanian","danish","hungarian","tamil","norwegian",
    "thai","urdu","croatian","bulgarian","lithuanian","latin","maori","malayalam","welsh","slovak",
    "telugu","persian","latvian","bengali","serbian","azerbaijani","slovenian","kannada","estonian","macedonian",
    "breton","basque","icelandic","armenian","nepali","mongolian","bosnian","kazakh","albanian","swahili",
    "galician","marathi","punjabi","sinhala","khmer","shona","yoruba","somali","afrikaans","occitan",
    "georgian","belarusian","tajik","sindhi","gujarati","amharic","yiddish","lao","uzbek","faroese",
    "haitian creole","pashto","turkmen","nynorsk","maltese","sanskrit","luxembourgish","myanmar","tibetan","tagalog",
    "malagasy","assamese","tatar","hawaiian","lingala","hausa","bashkir","javanese","sundanese","cantonese"};

int lang_index(const char* code) {
    if (!code) return -1;
    for (int i = 0; i < 100; i++)
        if (strcmp(k_lang_codes[i], code) == 0 || strcmp(k_lang_names[i], code) == 0) return i;
    return -1;
}

namespace {

struct TensorRef {
    int type;  // 0 f32, 1 f16, or a GGML block-quantized type (2 q4_0, 3 q4_1, 6 q5_0, 7 q5_1, 8 q8_0)
    std::vector<int> ne;
    const char* data;
    size_t nel;
};

// GGML block quantization [ext, ggml-common.h / ggml-quants.c dequantize_row_*]: blocks of 32 weights,
// y = q * d (q5_0: q - 16, q4_0: q - 8, q8_0: signed bytes) or q * d + m (q5_1, q4_1); q * d is exact
// in f32 (<= 8-bit q times an f16 d). The app's catalog ships q5_1 and q5_0 files (model.rs:153-186).
int block_bytes(int type) {
    switch (type) {
        case 2: return 18; case 3: return 20; case 6: return 22; case 7: return 24; case 8: return 34;
        default: return 0;
    }
}
float hf(const uint8_t* p) { uint16_t h; memcpy(&h, p, 2); return h2f(h); }
void dequant_block(int type, const uint8_t* b, float* y) {
    if (type == 8) {
        const float d = hf(b);
        for (int j = 0; j < 32; j++) y[j] = (float)(int8_t)b[2 + j] * d;
        return;
    }
    const bool has_m = type == 3 || type == 7, has_h = type == 6 || type == 7;
    const float d = hf(b), m = has_m ? hf(b + 2) : 0.0f;
    const uint8_t* p = b + (has_m ? 4 : 2);
    uint32_t qh = 0;
    if (has_h) { memcpy(&qh, p, 4); p += 4; }
    const int off = has_m ? 0 : (has_h ? 16 : 8);
    for (int j = 0; j < 16; j++) {
        int x0 = p[j] & 0x0F, x1 = p[j] >> 4;
        if (has_h) { x0 |= ((qh >> j) << 4) & 0x10; x1 |= (qh >> (j + 12)) & 0x10; }
        y[j] = has_m ? (float)x0 * d + m : (float)(x0 - off) * d;
        y[j + 16] = has_m ? (float)x1 * d + m : (float)(x1 - off) * d;
    }
}

struct Reader {
    const char* p;
    const char* end;
    bool ok = true;
    template <typename X> X get() {
        X x{};
        if (p + sizeof(X) > end) { ok = false; return x; }
        memcpy(&x, p, sizeof(X));
        p += sizeof(X);
        return x;
    }
    const char* take(size_t n) {
        if (p + n > end) { ok = false; return nullptr; }
        const char* r = p;
        p += n;
        return r;
    }
};

// Host images of the device tensors. A rank that receives its weights by RCCL broadcast
// (load_weights = false) records sizes only: no host conversion, no H2D copy.
struct Arena {
    struct Item { void** target; size_t size; std::vector<char> bytes; };
    std::vector<Item> items;
    void add(void** target, size_t size, std::vector<char>&& bytes) {
        items.push_back({target, size, std::move(bytes)});
    }
};

float elem(const TensorRef& t, size_t i) {
    if (t.type == 0) { float f; memcpy(&f, t.data + 4 * i, 4); return f; }
    if (t.type == 1) { uint16_t h; memcpy(&h, t.data + 2 * i, 2); return h2f(h); }
    float y[32];
    dequant_block(t.type, (const uint8_t*)t.data + (i / 32) * block_bytes(t.type), y);
    return y[i % 32];
}
// row r (cols values) of a 2-D tensor as f32
void row_f32(const TensorRef& t, long r, long cols, float* out) {
    if (t.type == 0 || t.type == 1) {
        for (long k = 0; k < cols; k++) out[k] = elem(t, r * cols + k);
        return;
    }
    const uint8_t* b = (const uint8_t*)t.data + (r * cols / 32) * block_bytes(t.type);
    for (long k = 0; k < cols; k += 32) dequant_block(t.type, b + (k / 32) * block_bytes(t.type), out + k);
}

}  // namespace

static void build_vocab(Vocab& v, int n_vocab, Reader& r) {
    const int32_t n_file = r.get<int32_t>();
    v.n_vocab = n_vocab;
    v.id_to_token.assign(std::max(n_vocab, n_file), "");
    for (int i = 0; i < n_file && r.ok; i++) {
        const uint32_t len = r.get<uint32_t>();
        const char* b = len ? r.take(len) : nullptr;
        std::string w = b ? std::string(b, len) : std::string();
        v.token_to_id[w] = i;
        v.id_to_token[i] = w;
    }
    if (v.is_multilingual()) {
        v.token_eot++; v.token_sot++;
        const int dt = v.num_languages() - 98;
        v.token_translate += dt; v.token_transcribe += dt; v.token_solm += dt; v.token_prev += dt;
        v.token_nosp += dt; v.token_not += dt; v.token_beg += dt;
    }
    for (int i = n_file; i < n_vocab; i++) {
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
}

bool load_context(Context* c, const char* path, int device, DType dt, bool load_weights) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) { fprintf(stderr, "whisper_mi355x: cannot open %s\n", path); return false; }
    struct stat st;
    fstat(fd, &st);
    const size_t fsize = st.st_size;
    void* map = mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (map == MAP_FAILED) return false;
    Reader r{(const char*)map, (const char*)map + fsize};
    auto fail = [&](const char* why) -> bool {
        fprintf(stderr, "whisper_mi355x: invalid model file %s (%s)\n", path, why);
        munmap(map, fsize);
        return false;
    };
    if (r.get<uint32_t>() != 0x67676d6cu) return fail("bad magic");
    c->path = path;
    c->dt = dt;
    c->device = device;
    c->hp = r.get<Hparams>();
    c->hp.ftype %= 1000;  // GGML_QNT_VERSION * GGML_QNT_VERSION_FACTOR rides on a quantized file's ftype
    const Hparams& hp = c->hp;
    if (hp.n_audio_state != hp.n_text_state || hp.n_audio_state % 64 || hp.n_audio_state / hp.n_audio_head != 64 ||
        hp.n_text_state / hp.n_text_head != 64 || hp.n_mels % 8) {
        return fail("unsupported hparams (need d_head 64, n_mels % 8 == 0)");
    }
    c->filt_n_mel = r.get<int32_t>();
    c->filt_n_fft = r.get<int32_t>();
    if (c->filt_n_fft != 201 || c->filt_n_mel != hp.n_mels) { return fail("mel filters"); }
    c->filters.resize((size_t)c->filt_n_mel * c->filt_n_fft);
    memcpy(c->filters.data(), r.take(c->filters.size() * 4), c->filters.size() * 4);
    build_vocab(c->vocab, hp.n_vocab, r);
    std::map<std::string, TensorRef> tens;
    while (r.ok && r.p < r.end) {
        const int32_t n_dims = r.get<int32_t>(), name_len = r.get<int32_t>(), ttype = r.get<int32_t>();
        if (!r.ok) break;
        TensorRef t;
        t.type = ttype;
        t.nel = 1;
        for (int i = 0; i < n_dims; i++) { t.ne.push_back(r.get<int32_t>()); t.nel *= t.ne.back(); }
        const char* nm = r.take(name_len);
        if (!nm) break;
        size_t bytes;
        if (ttype == 0 || ttype == 1) bytes = t.nel * (ttype == 0 ? 4 : 2);
        else if (block_bytes(ttype) && n_dims >= 1 && t.ne[0] % 32 == 0) bytes = t.nel / 32 * block_bytes(ttype);
        else return fail("unsupported tensor type (f32, f16, q4_0, q4_1, q5_0, q5_1, q8_0)");
        t.data = r.take(bytes);
        if (!t.data) break;
        tens[std::string(nm, name_len)] = t;
    }
    if (!r.ok) { return fail("truncated"); }

    const int d = hp.n_audio_state, nm = hp.n_mels, V = hp.n_vocab, Le = hp.n_audio_layer, Ld = hp.n_text_layer;
    c->k_scale = (float)pow(64.0, -0.25);
    {
        static const char* types[] = {"tiny", "base", "small", "medium", "large"};
        int ti = Le == 4 ? 0 : Le == 6 ? 1 : Le == 12 ? 2 : Le == 24 ? 3 : 4;
        c->model_type = types[ti];
    }
    // special ids for the logits kernel
    Vocab& v = c->vocab;
    c->vid = VocabIds{v.n_vocab, v.token_eot, v.token_sot, v.token_translate, v.token_transcribe, v.token_solm,
                      v.token_prev, v.token_nosp, v.token_not, v.token_beg,
                      v.token_to_id.count(" ") ? v.token_to_id.at(" ") : -1, 100};

    auto need = [&](const std::string& n) -> const TensorRef* {
        auto it = tens.find(n);
        if (it == tens.end()) { fprintf(stderr, "whisper_mi355x: missing tensor %s\n", n.c_str()); return nullptr; }
        return &it->second;
    };
    // ---- build the host images of every device tensor --------------------------------------
    Arena A;
    const size_t esz = 2;
    // Block-quantized files keep the projection matrices as their blocks (QMat: quant bytes, q5 high
    // bits and f16 scales regrouped by field; no expansion to 16 bits). WHISPER_MI355X_QUANT_EXPAND=1
    // dequantizes them at load instead (the round-2 layout, kept for A/B).
    const bool keep_blocks = !(getenv("WHISPER_MI355X_QUANT_EXPAND") && atoi(getenv("WHISPER_MI355X_QUANT_EXPAND")) == 1);
    auto qmat = [&](QMat* q, const std::vector<const TensorRef*>& parts, long rows_total, long cols,
                    const std::vector<long>& rows_each) -> bool {
        if (!q || !keep_blocks || cols % 32) return false;
        const int type = parts[0] ? parts[0]->type : 0;
        if (!block_bytes(type)) return false;
        for (auto* t : parts)
            if (!t || t->type != type) return false;
        const long nbk = cols / 32;
        const int bb = block_bytes(type);
        const bool q8 = type == 8, has_m = type == 3 || type == 7, has_h = type == 6 || type == 7;
        const int dmb = has_m ? 4 : 2;  // bytes of {d, m} (q4_1, q5_1) or d per block
        const size_t qs_sz = (size_t)rows_total * (q8 ? cols : cols / 2), qh_sz = has_h ? (size_t)rows_total * nbk * 4 : 0,
                     dm_sz = (size_t)rows_total * nbk * dmb;
        std::vector<char> qs(load_weights ? qs_sz : 0), qh(load_weights ? qh_sz : 0), dm(load_weights ? dm_sz : 0);
        if (load_weights) {
            long row0 = 0;
            for (size_t pi = 0; pi < parts.size(); pi++) {
                for (long rr = 0; rr < rows_each[pi]; rr++)
                    for (long b = 0; b < nbk; b++) {
                        const uint8_t* blk = (const uint8_t*)parts[pi]->data + (rr * nbk + b) * bb;
                        const long r = row0 + rr, bi = r * nbk + b;
                        memcpy(dm.data() + bi * dmb, blk, dmb);  // d, or d and m
                        const uint8_t* p = blk + (has_m ? 4 : 2);
                        if (has_h) { memcpy(qh.data() + bi * 4, p, 4); p += 4; }
                        if (q8) memcpy(qs.data() + r * cols + b * 32, p, 32);
                        else memcpy(qs.data() + r * (cols / 2) + b * 16, p, 16);
                    }
                row0 += rows_each[pi];
            }
        }
        q->type = type;
        A.add((void**)&q->qs, qs_sz, std::move(qs));
        if (has_h) A.add((void**)&q->qh, qh_sz, std::move(qh));
        A.add((void**)&q->dm, dm_sz, std::move(dm));
        c->quant = type;
        return true;
    };
    auto mat = [&](void** dst, const std::vector<const TensorRef*>& parts, long rows_total, long cols,
                   const std::vector<long>& rows_each, bool conv_reorder, int taps_in, QMat* q = nullptr) {
        if (qmat(q, parts, rows_total, cols, rows_each)) { *dst = nullptr; return; }
        const size_t sz = (size_t)rows_total * cols * esz;
        if (!load_weights) { A.add(dst, sz, {}); return; }
        std::vector<char> b(sz);
        uint16_t* o = (uint16_t*)b.data();
        long row0 = 0;
        std::vector<float> rowbuf(cols);
        for (size_t pi = 0; pi < parts.size(); pi++) {
            const TensorRef* t = parts[pi];
            const long nr = rows_each[pi];
            if (t && t->type != 0 && t->type != 1) {
                // quantized: dequantize each row (exact f32), round once to the compute type, as ggml's
                // GPU matmuls do when they dequantize blocks into f16 tiles
                for (long rr = 0; rr < nr; rr++) {
                    row_f32(*t, rr, cols, rowbuf.data());
                    for (long k = 0; k < cols; k++) {
                        const float f = rowbuf[k];
                        uint16_t out;
                        if (dt == DType::F16) { _Float16 hf16 = (_Float16)f; memcpy(&out, &hf16, 2); }
                        else out = f2bf(f);
                        o[(row0 + rr) * cols + k] = out;
                    }
                }
                row0 += nr;
                continue;
            }
            for (long rr = 0; rr < nr; rr++)
                for (long k = 0; k < cols; k++) {
                    long src_k = k;
                    if (conv_reorder) {  // dst k = tap*in + c  <- src [c][tap]
                        const long tap = k / taps_in, ci = k % taps_in;
                        src_k = ci * 3 + tap;
                    }
                    uint16_t out;
                    if (t) {
                        if (t->type == 1 && dt == DType::F16) memcpy(&out, t->data + 2 * (rr * cols + src_k), 2);
                        else {
                            const float f = elem(*t, rr * cols + src_k);
                            if (dt == DType::F16) { _Float16 hf = (_Float16)f; memcpy(&out, &hf, 2); }
                            else out = f2bf(f);
                        }
                    } else out = 0;
                    o[(row0 + rr) * cols + k] = out;
                }
            row0 += nr;
        }
        A.add(dst, sz, std::move(b));
    };
    auto vecf = [&](float** dst, const std::vector<const TensorRef*>& parts, const std::vector<long>& n_each) {
        long tot = 0;
        for (long x : n_each) tot += x;
        if (!load_weights) { A.add((void**)dst, tot * 4, {}); return; }
        std::vector<char> b(tot * 4);
        float* o = (float*)b.data();
        long off = 0;
        for (size_t pi = 0; pi < parts.size(); pi++) {
            for (long i = 0; i < n_each[pi]; i++) o[off + i] = parts[pi] ? elem(*parts[pi], i) : 0.0f;
            off += n_each[pi];
        }
        A.add((void**)dst, tot * 4, std::move(b));
    };
    Weights& W = c->w;
    bool ok = true;
#define NEED(var, name) const TensorRef* var = need(name); if (!var) ok = false;
    {
        NEED(c1w, "encoder.conv1.weight") NEED(c1b, "encoder.conv1.bias") NEED(c2w, "encoder.conv2.weight")
        NEED(c2b, "encoder.conv2.bias") NEED(pe, "encoder.positional_embedding") NEED(lpw, "encoder.ln_post.weight")
        NEED(lpb, "encoder.ln_post.bias") NEED(te, "decoder.token_embedding.weight") NEED(pd, "decoder.positional_embedding")
        NEED(ldw, "decoder.ln.weight") NEED(ldb, "decoder.ln.bias")
        if (!ok) { munmap(map, fsize); return false; }
        mat(&W.conv1_w, {c1w}, d, 3 * nm, {d}, true, nm);
        vecf(&W.conv1_b, {c1b}, {d});
        mat(&W.conv2_w, {c2w}, d, 3 * d, {d}, true, d);
        vecf(&W.conv2_b, {c2b}, {d});
        vecf(&W.pos_e, {pe}, {(long)hp.n_audio_ctx * d});
        vecf(&W.lnpost_w, {lpw}, {d});
        vecf(&W.lnpost_b, {lpb}, {d});
        mat(&W.tok_emb, {te}, V, d, {V}, false, 0);
        if (te->type != 0 && te->type != 1) {
            // ggml_get_rows dequantizes a quantized embedding to exact f32 rows (the decoder input),
            // while the logits matmul reads the f16-rounded blocks: keep both
            const size_t sz = (size_t)V * d * 4;
            std::vector<char> eb(load_weights ? sz : 0);
            for (long rr = 0; rr < V && load_weights; rr++) row_f32(*te, rr, d, (float*)eb.data() + rr * d);
            A.add((void**)&W.tok_emb_f32, sz, std::move(eb));
        }
        vecf(&W.pos_d, {pd}, {(long)hp.n_text_ctx * d});
        vecf(&W.lnd_w, {ldw}, {d});
        vecf(&W.lnd_b, {ldb}, {d});
    }
    W.enc.resize(Le);
    W.dec.resize(Ld);
    for (int l = 0; l < Le && ok; l++) {
        const std::string p = "encoder.blocks." + std::to_string(l) + ".";
        LayerW& L = W.enc[l];
        NEED(qw, p + "attn.query.weight") NEED(qb, p + "attn.query.bias") NEED(kw, p + "attn.key.weight")
        NEED(vw, p + "attn.value.weight") NEED(vb, p + "attn.value.bias") NEED(ow, p + "attn.out.weight")
        NEED(ob, p + "attn.out.bias") NEED(l1w, p + "attn_ln.weight") NEED(l1b, p + "attn_ln.bias")
        NEED(f1w, p + "mlp.0.weight") NEED(f1b, p + "mlp.0.bias") NEED(f2w, p + "mlp.2.weight") NEED(f2b, p + "mlp.2.bias")
        NEED(l2w, p + "mlp_ln.weight") NEED(l2b, p + "mlp_ln.bias")
        if (!ok) break;
        vecf(&L.ln1_w, {l1w}, {d}); vecf(&L.ln1_b, {l1b}, {d});
        mat(&L.wqkv, {qw, kw, vw}, 3 * d, d, {d, d, d}, false, 0, &L.qqkv);
        vecf(&L.bqkv, {qb, nullptr, vb}, {d, d, d});
        mat(&L.wo, {ow}, d, d, {d}, false, 0, &L.qo); vecf(&L.bo, {ob}, {d});
        vecf(&L.ln2_w, {l2w}, {d}); vecf(&L.ln2_b, {l2b}, {d});
        mat(&L.w1, {f1w}, 4 * d, d, {4 * d}, false, 0, &L.q1); vecf(&L.b1, {f1b}, {4 * d});
        mat(&L.w2, {f2w}, d, 4 * d, {d}, false, 0, &L.q2); vecf(&L.b2, {f2b}, {d});
    }
    std::vector<const TensorRef*> xkv;
    std::vector<const TensorRef*> xkvb;
    std::vector<long> xrows, xbn;
    for (int l = 0; l < Ld && ok; l++) {
        const std::string p = "decoder.blocks." + std::to_string(l) + ".";
        LayerW& L = W.dec[l];
        NEED(qw, p + "attn.query.weight") NEED(qb, p + "attn.query.bias") NEED(kw, p + "attn.key.weight")
        NEED(vw, p + "attn.value.weight") NEED(vb, p + "attn.value.bias") NEED(ow, p + "attn.out.weight")
        NEED(ob, p + "attn.out.bias") NEED(l1w, p + "attn_ln.weight") NEED(l1b, p + "attn_ln.bias")
        NEED(xqw, p + "cross_attn.query.weight") NEED(xqb, p + "cross_attn.query.bias")
        NEED(xkw, p + "cross_attn.key.weight") NEED(xvw, p + "cross_attn.value.weight") NEED(xvb, p + "cross_attn.value.bias")
        NEED(xow, p + "cross_attn.out.weight") NEED(xob, p + "cross_attn.out.bias")
        NEED(lxw, p + "cross_attn_ln.weight") NEED(lxb, p + "cross_attn_ln.bias")
        NEED(f1w, p + "mlp.0.weight") NEED(f1b, p + "mlp.0.bias") NEED(f2w, p + "mlp.2.weight") NEED(f2b, p + "mlp.2.bias")
        NEED(l2w, p + "mlp_ln.weight") NEED(l2b, p + "mlp_ln.bias")
        if (!ok) break;
        vecf(&L.ln1_w, {l1w}, {d}); vecf(&L.ln1_b, {l1b}, {d});
        mat(&L.wqkv, {qw, kw, vw}, 3 * d, d, {d, d, d}, false, 0, &L.qqkv);
        vecf(&L.bqkv, {qb, nullptr, vb}, {d, d, d});
        mat(&L.wo, {ow}, d, d, {d}, false, 0, &L.qo); vecf(&L.bo, {ob}, {d});
        vecf(&L.lnx_w, {lxw}, {d}); vecf(&L.lnx_b, {lxb}, {d});
        mat(&L.wxq, {xqw}, d, d, {d}, false, 0, &L.qxq); vecf(&L.bxq, {xqb}, {d});
        mat(&L.wxo, {xow}, d, d, {d}, false, 0, &L.qxo); vecf(&L.bxo, {xob}, {d});
        vecf(&L.ln2_w, {l2w}, {d}); vecf(&L.ln2_b, {l2b}, {d});
        mat(&L.w1, {f1w}, 4 * d, d, {4 * d}, false, 0, &L.q1); vecf(&L.b1, {f1b}, {4 * d});
        mat(&L.w2, {f2w}, d, 4 * d, {d}, false, 0, &L.q2); vecf(&L.b2, {f2b}, {d});
        xkv.push_back(xkw); xkv.push_back(xvw);
        xrows.push_back(d); xrows.push_back(d);
        xkvb.push_back(nullptr); xkvb.push_back(xvb);
        xbn.push_back(d); xbn.push_back(d);
    }
#undef NEED
    if (!ok) { munmap(map, fsize); return false; }
    mat(&W.wkv_cross, xkv, (long)2 * Ld * d, d, xrows, false, 0);
    vecf(&W.bkv_cross, xkvb, xbn);
    c->cross_direct = xattn_supported(d) && hp.n_text_head * 64 == d;
    if (c->cross_direct) {
        // cross K weights per head, transposed: wkT[l][h][c][j] = Wk_l[h*64 + j][c], the B operand of
        // the Q' projection Q'_h = s * Wk_h^T q_h (kernels/xattn.hip)
        const int H = hp.n_text_head;
        const size_t sz = (size_t)Ld * H * d * 64 * esz;
        std::vector<char> b(load_weights ? sz : 0);
        uint16_t* o = (uint16_t*)b.data();
        std::vector<float> rows;
        for (int l = 0; l < Ld && load_weights; l++) {
            const TensorRef* t = xkv[2 * l];
            const bool q = t->type != 0 && t->type != 1;
            if (q) {
                rows.resize((size_t)d * d);
                for (long rr = 0; rr < d; rr++) row_f32(*t, rr, d, rows.data() + rr * d);
            }
            for (int h = 0; h < H; h++)
                for (int j = 0; j < 64; j++)
                    for (int k = 0; k < d; k++) {
                        const size_t src = (size_t)(h * 64 + j) * d + k;
                        uint16_t out;
                        if (t->type == 1 && dt == DType::F16) memcpy(&out, t->data + 2 * src, 2);
                        else {
                            const float f = q ? rows[src] : elem(*t, src);
                            if (dt == DType::F16) { _Float16 hf = (_Float16)f; memcpy(&out, &hf, 2); }
                            else out = f2bf(f);
                        }
                        o[(((size_t)l * H + h) * d + k) * 64 + j] = out;
                    }
        }
        A.add(&W.wkT, sz, std::move(b));
    }
    // mel tables (identical libm expressions to whisper.cpp's whisper_global_cache) + filters^T
    {
        std::vector<char> b(3 * 400 * 4);
        float* f = (float*)b.data();
        for (int i = 0; i < 400; i++) {
            double theta = (2 * M_PI * i) / 400;
            f[i] = sinf(theta);
            f[400 + i] = cosf(theta);
        }
        for (int i = 0; i < 400; i++) f[800 + i] = 0.5 * (1.0 - cosf((2.0 * M_PI * i) / (400 + 0)));
        A.add(&W.mel_tab, b.size(), std::move(b));
        std::vector<char> ft(201 * nm * 4);
        float* o = (float*)ft.data();
        for (int j = 0; j < nm; j++)
            for (int k = 0; k < 201; k++) o[k * nm + j] = c->filters[j * 201 + k];
        A.add((void**)&W.filt_t, ft.size(), std::move(ft));
    }
    munmap(map, fsize);
    // ---- one arena, 256-B aligned sub-allocations ------------------------------------------
    size_t total = 0;
    std::vector<size_t> offs;
    for (auto& it : A.items) {
        offs.push_back(total);
        total += (it.size + 255) & ~(size_t)255;
    }
    WM_CHECK(hipSetDevice(device));
    init_gelu_table();
    WM_CHECK(hipMalloc((void**)&c->arena, total));
    c->arena_bytes = total;
    for (size_t i = 0; i < A.items.size(); i++) {
        *A.items[i].target = c->arena + offs[i];
        if (!A.items[i].bytes.empty())
            WM_CHECK(hipMemcpy(c->arena + offs[i], A.items[i].bytes.data(), A.items[i].size, hipMemcpyHostToDevice));
    }
    return true;
}

void free_context(Context* c) {
    if (c && c->arena) { hipSetDevice(c->device); hipFree(c->arena); c->arena = nullptr; }
    if (c && c->arena8) { hipSetDevice(c->device); hipFree(c->arena8); c->arena8 = nullptr; }
    if (c && c->arena_exp) { hipSetDevice(c->device); hipFree(c->arena_exp); c->arena_exp = nullptr; }
    if (c && c->pdec_layers) { hipSetDevice(c->device); hipFree(c->pdec_layers); c->pdec_layers = nullptr; }
    if (c && c->pdec_layers_exp) { hipSetDevice(c->device); hipFree(c->pdec_layers_exp); c->pdec_layers_exp = nullptr; }
}

}  // namespace wm
