// C++ mirror of the reference's capture-side chunker:
//   * AudioBuffer — src-tauri/src/audio.rs:29-241 (real-time VAD chunker with adaptive noise floor,
//                   silence-split and forced-split chunk extraction, 200 ms overlap carry).
// The app's recording / worker / stop-thread machinery around it (state.rs) is UI state, out of scope
// (SURVEY.md §2 row 4): it is not restated.
//
// The buffer runs on the host by design: it sees one capture callback (~10 ms of audio)
// at a time, far below what a GPU launch pays off for. The chunks it dispatches are resampled and
// transcribed on the GPU (whisper_mi355x_resample_chunk, WhisperEngine over libwhisper_mi355x.so);
// the end-of-recording split uses whisper_mi355x_find_silence_boundaries.
//
// Arithmetic follows the Rust source operation for operation in f32 (sequential sums, no contraction,
// f32 constants), so chunk boundaries are identical to the app's for the same callback sequence.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace nobs {

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

}  // namespace nobs
