// C++ mirror of the reference's boundary caller, src-tauri/src/whisper.rs (`WhisperEngine`).
//
// The reference's host language is Rust; cargo/rustc are absent offline, so the caller above the
// C ABI is restated in C++ against include/whisper.h exactly as whisper.rs drives whisper-rs:
// same FullParams (whisper.rs:88-124), same segment concatenation, trim and hallucination filter
// (whisper.rs:132-144, 200-260), same error kinds (whisper.rs:6-14). It links only the whisper.h
// ABI of libwhisper_mi355x.so, so it also documents what the Rust side would bind.
#pragma once
#include <memory>
#include <string>
#include <vector>

struct whisper_context;

namespace nobs {

enum class WhisperError { Ok = 0, LoadError = 1, TranscriptionError = 2, NoModel = 3 };

class WhisperEngine {
  public:
    WhisperEngine() = default;
    ~WhisperEngine();
    WhisperEngine(const WhisperEngine&) = delete;
    WhisperEngine& operator=(const WhisperEngine&) = delete;

    static std::unique_ptr<WhisperEngine> from_file(const std::string& path, WhisperError* err, std::string* msg);
    WhisperError load_model(const std::string& path, std::string* msg);  // whisper.rs:36-52
    void unload_model();                                                 // whisper.rs:55-59
    bool is_loaded() const { return ctx_ != nullptr; }                   // whisper.rs:62-64

    // whisper.rs:66-148. language/vocabulary/context may be null (Rust `None`).
    WhisperError transcribe(const float* audio, size_t n, const char* language, const char* vocabulary,
                            const char* context, std::string* out, std::string* msg) const;
    // whisper.rs:150-197
    WhisperError transcribe_chunked(const std::vector<std::vector<float>>& chunks, const char* language,
                                    const char* vocabulary, std::string* out, std::string* msg) const;

  private:
    whisper_context* ctx_ = nullptr;
    std::string model_path_;
};

// whisper.rs:200-260
std::string filter_hallucinations(const std::string& text);
// String::from_utf8_lossy: each maximal ill-formed subsequence -> U+FFFD (segment.to_str_lossy(), whisper.rs:137)
std::string utf8_lossy(const std::string& bytes);
// str::trim (Unicode White_Space at both ends)
std::string trim(const std::string& s);
// whisper.rs:98-105 initial prompt; false = None
bool build_initial_prompt(const char* vocabulary, const char* context, std::string* out);

}  // namespace nobs
