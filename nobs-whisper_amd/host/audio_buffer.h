// C++ mirror of the reference's streaming capture path:
//   * AudioBuffer      — src-tauri/src/audio.rs:29-241 (real-time VAD chunker with adaptive noise floor,
//                        silence-split and forced-split chunk extraction, 200 ms overlap carry);
//   * StreamingSession — src-tauri/src/state.rs:113-168 (transcription worker), 585-606 (the input
//                        callback: stereo down-mix, push, dispatch a chunk) and 655-798 (stop: join the
//                        worker, transcribe the remaining audio, split at silences above 30 s, join).
//
// The buffer runs on the host by design: it sees one capture callback (~10 ms of audio)
// at a time, far below what a GPU launch pays off for. The chunks it dispatches are resampled and
// transcribed on the GPU (whisper_mi355x_resample_chunk, WhisperEngine over libwhisper_mi355x.so);
// the end-of-recording split uses whisper_mi355x_find_silence_boundaries.
//
// Arithmetic follows the Rust source operation for operation in f32 (sequential sums, no contraction,
// f32 constants), so chunk boundaries are identical to the app's for the same callback sequence.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace nobs {

class WhisperEngine;

// audio.rs:364-370 calculate_rms
float calculate_rms(const float* x, size_t n);

class AudioBuffer {
  public:
    explicit AudioBuffer(uint32_t sample_rate = 48000);  // audio.rs:45-58

    void push_samples(const float* x, size_t n);          // audio.rs:60-87
    std::vector<float> take();                            // audio.rs:89-93
    bool has_silence_boundary() const;                    // audio.rs:97-106
    bool take_chunk_at_silence(std::vector<float>* out);  // audio.rs:111-156 (false = None)
    bool take_forced_chunk(std::vector<float>* out);      // audio.rs:161-225 (false = None)

    size_t len() const { return samples_.size(); }
    bool is_empty() const { return samples_.empty(); }
    float noise_floor() const { return noise_floor_; }
    uint32_t sample_rate() const { return sample_rate_; }
    size_t overlap_len() const { return overlap_.size(); }
    size_t last_speech_pos() const { return last_speech_pos_; }
    size_t noise_floor_frames() const { return noise_floor_frames_; }

  private:
    void emit_chunk(size_t split_point, std::vector<float>* out);

    std::vector<float> samples_;
    size_t last_speech_pos_ = 0;
    uint32_t sample_rate_;
    float noise_floor_;
    size_t noise_floor_frames_ = 0;
    std::vector<float> overlap_;
};

// audio.rs:469-507 split_at_silences_with_overlap
std::vector<std::vector<float>> split_at_silences_with_overlap(const std::vector<float>& audio,
                                                               const std::vector<int>& boundaries,
                                                               uint32_t sample_rate);

class StreamingSession {
  public:
    // state.rs:515-558: buffer at the device rate, worker spawned when a model is loaded. language /
    // vocabulary may be null (config "auto" / empty vocabulary).
    StreamingSession(const WhisperEngine* engine, uint32_t input_rate, int channels, const char* language,
                     const char* vocabulary, int device);
    ~StreamingSession();

    // state.rs:587-606, one input callback of interleaved frames. Returns 1 when it dispatched a chunk.
    int on_input(const float* data, size_t n);
    // state.rs:655-798 without the UI: the final combined text.
    std::string stop();

    std::vector<int> dispatched_lengths() const;  // samples at the input rate, in dispatch order
    std::vector<std::string> results() const;     // the worker's non-empty texts, then the remaining audio's
    int errors() const { return errors_; }

  private:
    void worker();
    bool resample(const std::vector<float>& in, uint32_t rate, std::vector<float>* out) const;
    void transcribe_into(const std::vector<float>& pcm16k, const char* prev, std::vector<std::string>* res);

    const WhisperEngine* engine_;
    uint32_t rate_;
    int channels_;
    bool has_lang_, has_vocab_;
    std::string lang_, vocab_;
    int device_;

    std::mutex buf_mu_;  // the app's Arc<Mutex<AudioBuffer>>
    AudioBuffer buf_;

    mutable std::mutex q_mu_;  // the app's mpsc channel + results mutex
    std::condition_variable q_cv_;
    std::deque<std::vector<float>> queue_;
    bool closed_ = false;
    std::vector<int> dispatched_;
    std::vector<std::string> results_;
    std::string last_context_;
    bool has_last_context_ = false;
    std::atomic<int> errors_{0};
    bool stopped_ = false;
    std::thread worker_;
};

}  // namespace nobs
