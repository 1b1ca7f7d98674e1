// See whisper_engine.h. Reference: src-tauri/src/whisper.rs (file:line cited per function).
#include "whisper_engine.h"

#include <cstdint>
#include <cstring>

#include "../../include/whisper.h"

namespace nobs {

namespace {

// UTF-8 <-> code points (the Rust side works on `char`s)
std::vector<uint32_t> decode_utf8(const std::string& s) {
    std::vector<uint32_t> out;
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = s[i];
        uint32_t cp;
        int n;
        if (c < 0x80) { cp = c; n = 1; }
        else if ((c >> 5) == 6) { cp = c & 0x1f; n = 2; }
        else if ((c >> 4) == 14) { cp = c & 0x0f; n = 3; }
        else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
        else { cp = 0xfffd; n = 1; }
        if (i + n > s.size()) { out.push_back(0xfffd); break; }
        for (int k = 1; k < n; k++) cp = (cp << 6) | (s[i + k] & 0x3f);
        out.push_back(cp);
        i += n;
    }
    return out;
}
std::string encode_utf8(const std::vector<uint32_t>& cps, size_t b, size_t e) {
    std::string s;
    for (size_t i = b; i < e; i++) {
        const uint32_t c = cps[i];
        if (c < 0x80) s += (char)c;
        else if (c < 0x800) { s += (char)(0xc0 | (c >> 6)); s += (char)(0x80 | (c & 0x3f)); }
        else if (c < 0x10000) { s += (char)(0xe0 | (c >> 12)); s += (char)(0x80 | ((c >> 6) & 0x3f)); s += (char)(0x80 | (c & 0x3f)); }
        else { s += (char)(0xf0 | (c >> 18)); s += (char)(0x80 | ((c >> 12) & 0x3f)); s += (char)(0x80 | ((c >> 6) & 0x3f)); s += (char)(0x80 | (c & 0x3f)); }
    }
    return s;
}
// Rust char::is_whitespace (Unicode White_Space)
bool is_ws(uint32_t c) {
    return (c >= 0x09 && c <= 0x0d) || c == 0x20 || c == 0x85 || c == 0xa0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200a) ||
           c == 0x2028 || c == 0x2029 || c == 0x202f || c == 0x205f || c == 0x3000;
}
bool is_ascii_punct(uint32_t c) {
    return (c >= 0x21 && c <= 0x2f) || (c >= 0x3a && c <= 0x40) || (c >= 0x5b && c <= 0x60) || (c >= 0x7b && c <= 0x7e);
}
// Rust str::to_lowercase for the scripts a transcript realistically carries (ASCII, Latin-1,
// Latin Extended-A, Greek, Cyrillic); CJK/Hangul/kana have no case.
uint32_t lower(uint32_t c) {
    if (c >= 'A' && c <= 'Z') return c + 32;
    if ((c >= 0xc0 && c <= 0xde) && c != 0xd7) return c + 32;
    if (c >= 0x100 && c <= 0x17f && c != 0x130 && c != 0x138 && c != 0x149 && c != 0x17f) {
        if ((c >= 0x139 && c <= 0x148) || (c >= 0x179 && c <= 0x17e)) return (c & 1) ? c + 1 : c;
        return (c & 1) ? c : c + 1;
    }
    if (c >= 0x391 && c <= 0x3ab && c != 0x3a2) return c + 32;
    if (c >= 0x410 && c <= 0x42f) return c + 32;
    if (c >= 0x400 && c <= 0x40f) return c + 80;
    return c;
}

const char* const kHallucinationPhrases[] = {  // whisper.rs:202-230
    "thank you for watching", "thanks for watching", "thank you for listening", "thanks for listening",
    "subscribe to my channel", "please subscribe", "like and subscribe", "see you in the next video",
    "see you next time", "please like and subscribe", "don't forget to subscribe", "hit the bell",
    "leave a comment", "check out my other videos", "thanks for tuning in",
    "\xec\x8b\x9c\xec\xb2\xad\xed\x95\xb4 \xec\xa3\xbc\xec\x85\x94\xec\x84\x9c \xea\xb0\x90\xec\x82\xac\xed\x95\xa9\xeb\x8b\x88\xeb\x8b\xa4",
    "\xea\xb5\xac\xeb\x8f\x85\xea\xb3\xbc \xec\xa2\x8b\xec\x95\x84\xec\x9a\x94",
    "\xea\xb5\xac\xeb\x8f\x85 \xeb\xb6\x80\xed\x83\x81\xeb\x93\x9c\xeb\xa6\xbd\xeb\x8b\x88\xeb\x8b\xa4",
    "\xe3\x81\x94\xe8\xa6\x96\xe8\x81\xb4\xe3\x81\x82\xe3\x82\x8a\xe3\x81\x8c\xe3\x81\xa8\xe3\x81\x86\xe3\x81\x94\xe3\x81\x96\xe3\x81\x84\xe3\x81\xbe\xe3\x81\x97\xe3\x81\x9f",
    "\xe6\x84\x9f\xe8\xb0\xa2\xe6\x94\xb6\xe7\x9c\x8b",
    "\xe8\xb0\xa2\xe8\xb0\xa2\xe8\xa7\x82\xe7\x9c\x8b",
    "you",
    "MBC \xeb\x89\xb4\xec\x8a\xa4 \xec\x9d\xb4\xeb\x8d\x95\xec\x98\x81\xec\x9e\x85\xeb\x8b\x88\xeb\x8b\xa4",
};

}  // namespace

// String::from_utf8_lossy (what whisper-rs's WhisperSegment::to_str_lossy returns, whisper.rs:137):
// every maximal ill-formed subsequence (Unicode "substitution of maximal subparts") becomes one
// U+FFFD, valid sequences are copied.
std::string utf8_lossy(const std::string& in) {
    std::string out;
    const size_t n = in.size();
    auto b = [&](size_t i) { return (unsigned char)in[i]; };
    for (size_t i = 0; i < n;) {
        const unsigned char c = b(i);
        if (c < 0x80) { out += (char)c; i++; continue; }
        int len = 0;
        unsigned char lo = 0x80, hi = 0xbf;  // allowed range of the second byte
        if (c >= 0xc2 && c <= 0xdf) len = 2;
        else if (c == 0xe0) { len = 3; lo = 0xa0; }
        else if ((c >= 0xe1 && c <= 0xec) || c == 0xee || c == 0xef) len = 3;
        else if (c == 0xed) { len = 3; hi = 0x9f; }
        else if (c == 0xf0) { len = 4; lo = 0x90; }
        else if (c >= 0xf1 && c <= 0xf3) len = 4;
        else if (c == 0xf4) { len = 4; hi = 0x8f; }
        if (len == 0) { out += "\xef\xbf\xbd"; i++; continue; }
        size_t k = 1;
        for (; k < (size_t)len && i + k < n; k++) {
            const unsigned char x = b(i + k);
            const bool ok = k == 1 ? (x >= lo && x <= hi) : (x >= 0x80 && x <= 0xbf);
            if (!ok) break;
        }
        if (k == (size_t)len) out.append(in, i, len);
        else out += "\xef\xbf\xbd";
        i += k;
    }
    return out;
}

// initial_prompt of whisper.rs:98-105: "{vocab} {ctx}" / vocab / ctx / none
bool build_initial_prompt(const char* vocabulary, const char* context, std::string* out) {
    const bool has_vocab = vocabulary != nullptr, has_ctx = context != nullptr;
    if (has_vocab && has_ctx && vocabulary[0] != '\0') { *out = std::string(vocabulary) + " " + context; return true; }
    if (has_vocab && !has_ctx && vocabulary[0] != '\0') { *out = vocabulary; return true; }
    if (has_ctx) { *out = context; return true; }
    return false;
}

std::string trim(const std::string& s) {
    auto cp = decode_utf8(s);
    size_t b = 0, e = cp.size();
    while (b < e && is_ws(cp[b])) b++;
    while (e > b && is_ws(cp[e - 1])) e--;
    return encode_utf8(cp, b, e);
}

std::string filter_hallucinations(const std::string& text) {
    const std::string trimmed = trim(text);
    if (trimmed.empty()) return std::string();
    const auto cps = decode_utf8(trimmed);
    bool all_punct = true;
    for (uint32_t c : cps)
        if (!(is_ascii_punct(c) || c == 0x2026 || c == 0x266a || c == 0x266b || c == 0x266c)) { all_punct = false; break; }
    if (all_punct) return std::string();
    std::vector<uint32_t> lw(cps.size());
    for (size_t i = 0; i < cps.size(); i++) lw[i] = lower(cps[i]);
    size_t e = lw.size();
    while (e > 0 && (is_ascii_punct(lw[e - 1]) || lw[e - 1] == 0x2026 || lw[e - 1] == 0x266a)) e--;
    const std::string stripped = encode_utf8(lw, 0, e);
    for (const char* phrase : kHallucinationPhrases) {
        auto pc = decode_utf8(phrase);
        for (auto& c : pc) c = lower(c);
        if (stripped == encode_utf8(pc, 0, pc.size())) return std::string();
    }
    return trimmed;
}

WhisperEngine::~WhisperEngine() { unload_model(); }

std::unique_ptr<WhisperEngine> WhisperEngine::from_file(const std::string& path, WhisperError* err, std::string* msg) {
    std::unique_ptr<WhisperEngine> e(new WhisperEngine());
    *err = e->load_model(path, msg);
    if (*err != WhisperError::Ok) e.reset();
    return e;
}

WhisperError WhisperEngine::load_model(const std::string& path, std::string* msg) {
    whisper_context_params params = whisper_context_default_params();
    params.use_gpu = true;  // whisper.rs:40
    whisper_context* ctx = whisper_init_from_file_with_params_no_state(path.c_str(), params);
    if (!ctx) {
        if (msg) *msg = "Failed to load model: failed to create context";
        return WhisperError::LoadError;
    }
    unload_model();
    ctx_ = ctx;
    model_path_ = path;
    return WhisperError::Ok;
}

void WhisperEngine::unload_model() {
    if (ctx_) whisper_free(ctx_);
    ctx_ = nullptr;
    model_path_.clear();
}

WhisperError WhisperEngine::transcribe(const float* audio, size_t n, const char* language, const char* vocabulary,
                                       const char* context, std::string* out, std::string* msg) const {
    if (!ctx_) return WhisperError::NoModel;
    whisper_state* state = whisper_init_state(ctx_);  // whisper.rs:83-85
    if (!state) {
        if (msg) *msg = "Transcription failed: failed to create state";
        return WhisperError::TranscriptionError;
    }
    whisper_full_params params = whisper_full_default_params(WHISPER_SAMPLING_GREEDY);  // whisper.rs:88
    params.greedy.best_of = 1;
    params.language = language;  // None => NULL => auto-detect (whisper.rs:91-95)
    std::string prompt;  // whisper.rs:98-109
    if (build_initial_prompt(vocabulary, context, &prompt)) params.initial_prompt = prompt.c_str();
    params.print_special = false;  // whisper.rs:112-124
    params.print_progress = false;
    params.print_realtime = false;
    params.print_timestamps = false;
    params.translate = false;
    params.no_context = false;
    params.single_segment = false;
    params.suppress_blank = true;
    params.no_speech_thold = 0.6f;
    params.entropy_thold = 2.4f;
    params.logprob_thold = -1.0f;
    const int rc = whisper_full_with_state(ctx_, state, params, audio, (int)n);  // whisper.rs:127-129
    if (rc != 0) {
        whisper_free_state(state);
        if (msg) *msg = "Transcription failed: whisper_full returned " + std::to_string(rc);
        return WhisperError::TranscriptionError;
    }
    std::string result;  // whisper.rs:132-141 (to_str_lossy of each segment)
    const int n_seg = whisper_full_n_segments_from_state(state);
    for (int i = 0; i < n_seg; i++) {
        const char* t = whisper_full_get_segment_text_from_state(state, i);
        if (t) result += utf8_lossy(t);  // per segment, as whisper-rs
    }
    whisper_free_state(state);
    *out = filter_hallucinations(trim(result));  // whisper.rs:143-144
    return WhisperError::Ok;
}

WhisperError WhisperEngine::transcribe_chunked(const std::vector<std::vector<float>>& chunks, const char* language,
                                               const char* vocabulary, std::string* out, std::string* msg) const {
    std::vector<std::string> results;
    std::string last_context;
    bool have_ctx = false;
    for (const auto& chunk : chunks) {
        std::string text;
        const WhisperError e = transcribe(chunk.data(), chunk.size(), language, vocabulary,
                                          have_ctx ? last_context.c_str() : nullptr, &text, msg);
        if (e != WhisperError::Ok) return e;
        if (!text.empty()) {
            last_context = text;
            have_ctx = true;
            results.push_back(text);
        }
    }
    std::string combined;
    for (size_t i = 0; i < results.size(); i++) combined += (i ? " " : "") + results[i];
    *out = combined;
    return WhisperError::Ok;
}

}  // namespace nobs

// C entry points so the parity tests (tests/, ctypes) can drive the mirror exactly as the app does.
extern "C" {
__attribute__((visibility("default"))) void* nobs_engine_new(void) { return new nobs::WhisperEngine(); }
__attribute__((visibility("default"))) void nobs_engine_free(void* e) { delete (nobs::WhisperEngine*)e; }
__attribute__((visibility("default"))) int nobs_engine_load(void* e, const char* path) {
    std::string msg;
    return (int)((nobs::WhisperEngine*)e)->load_model(path, &msg);
}
__attribute__((visibility("default"))) int nobs_engine_is_loaded(void* e) { return ((nobs::WhisperEngine*)e)->is_loaded(); }
__attribute__((visibility("default"))) int nobs_engine_transcribe(void* e, const float* audio, int n, const char* lang,
                                                                 const char* vocab, const char* ctx, char* out, int cap) {
    std::string text, msg;
    const auto r = ((nobs::WhisperEngine*)e)->transcribe(audio, (size_t)n, lang, vocab, ctx, &text, &msg);
    if (r != nobs::WhisperError::Ok) return -(int)r;
    if ((int)text.size() + 1 > cap) return -100;
    memcpy(out, text.c_str(), text.size() + 1);
    return (int)text.size();
}
__attribute__((visibility("default"))) int nobs_engine_transcribe_chunked(void* e, const float* const* chunks,
                                                                         const int* n, int n_chunks, const char* lang,
                                                                         const char* vocab, char* out, int cap) {
    std::vector<std::vector<float>> cs(n_chunks);
    for (int i = 0; i < n_chunks; i++) cs[i].assign(chunks[i], chunks[i] + n[i]);
    std::string text, msg;
    const auto r = ((nobs::WhisperEngine*)e)->transcribe_chunked(cs, lang, vocab, &text, &msg);
    if (r != nobs::WhisperError::Ok) return -(int)r;
    if ((int)text.size() + 1 > cap) return -100;
    memcpy(out, text.c_str(), text.size() + 1);
    return (int)text.size();
}
__attribute__((visibility("default"))) int nobs_build_initial_prompt(const char* vocab, const char* ctx, char* out, int cap) {
    std::string p;
    if (!nobs::build_initial_prompt(vocab, ctx, &p)) return -1;  // None
    if ((int)p.size() + 1 > cap) return -100;
    memcpy(out, p.c_str(), p.size() + 1);
    return (int)p.size();
}
__attribute__((visibility("default"))) int nobs_utf8_lossy(const char* in, int n, char* out, int cap) {
    const std::string r = nobs::utf8_lossy(std::string(in, n));
    if ((int)r.size() + 1 > cap) return -1;
    memcpy(out, r.c_str(), r.size() + 1);
    return (int)r.size();
}
__attribute__((visibility("default"))) int nobs_filter_hallucinations(const char* in, char* out, int cap) {
    const std::string r = nobs::filter_hallucinations(in);
    if ((int)r.size() + 1 > cap) return -1;
    memcpy(out, r.c_str(), r.size() + 1);
    return (int)r.size();
}
}
