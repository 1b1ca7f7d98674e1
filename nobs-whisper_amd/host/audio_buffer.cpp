// See audio_buffer.h. Built with -ffp-contract=off: every f32 product and sum is rounded on its own,
// as rustc emits them.
#include "audio_buffer.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>


namespace nobs {

namespace {
// audio.rs:7-15, 338-361
constexpr uint32_t kWhisperRate = 16000;
constexpr uint32_t kMaxBufferS = 25;
constexpr uint32_t kOverlapMs = 200;
constexpr float kSilenceThreshold = 0.01f;
constexpr uint32_t kMinSilenceMs = 700;
constexpr size_t kNoiseFloorMaxFrames = 100;
constexpr float kAdaptiveFactor = 3.0f;
constexpr float kMinThresholdFactor = 0.5f;
constexpr float kEmaDecay = 0.95f;
constexpr float kUpdateFactor = 0.5f;
}  // namespace

float calculate_rms(const float* x, size_t n) {
    if (n == 0) return 0.0f;
    float s = 0.0f;
    for (size_t i = 0; i < n; i++) {
        const float sq = x[i] * x[i];
        s = s + sq;
    }
    return std::sqrt(s / (float)n);
}

AudioBuffer::AudioBuffer(uint32_t sample_rate) : sample_rate_(sample_rate), noise_floor_(kSilenceThreshold) {}

void AudioBuffer::push_samples(const float* x, size_t n) {
    const size_t start = samples_.size();
    samples_.insert(samples_.end(), x, x + n);
    const size_t w = sample_rate_ / 50;  // 20 ms
    const float min_thr = kSilenceThreshold * kMinThresholdFactor;
    const float one_minus = 1.0f - kEmaDecay;
    size_t i = 0;
    for (size_t off = 0; off < n; off += w, i++) {
        const float rms = calculate_rms(x + off, std::min(w, n - off));
        if (rms < noise_floor_ * kUpdateFactor && noise_floor_frames_ < kNoiseFloorMaxFrames) {
            const float a = noise_floor_ * kEmaDecay;
            const float b = rms * one_minus;
            noise_floor_ = a + b;
            noise_floor_frames_++;
        }
        const float thr = std::fmax(noise_floor_ * kAdaptiveFactor, min_thr);
        if (rms >= thr) last_speech_pos_ = start + (i + 1) * w;
    }
}

std::vector<float> AudioBuffer::take() {
    last_speech_pos_ = 0;
    overlap_.clear();
    std::vector<float> out;
    out.swap(samples_);
    return out;
}

bool AudioBuffer::has_silence_boundary() const {
    if (samples_.empty() || last_speech_pos_ == 0) return false;
    const size_t silence = samples_.size() > last_speech_pos_ ? samples_.size() - last_speech_pos_ : 0;
    const size_t min_silence = (size_t)(sample_rate_ * kMinSilenceMs / 1000);
    return silence >= min_silence;
}

// The common tail of audio.rs:130-142 and 197-208: overlap + samples[..split] out, the last 200 ms of
// that span kept as the next overlap, the span drained.
void AudioBuffer::emit_chunk(size_t split, std::vector<float>* out) {
    const size_t ov = (size_t)(sample_rate_ * kOverlapMs / 1000);
    out->clear();
    out->reserve(overlap_.size() + split);
    out->insert(out->end(), overlap_.begin(), overlap_.end());
    out->insert(out->end(), samples_.begin(), samples_.begin() + split);
    const size_t ov_start = split > ov ? split - ov : 0;
    overlap_.assign(samples_.begin() + ov_start, samples_.begin() + split);
    samples_.erase(samples_.begin(), samples_.begin() + split);
}

bool AudioBuffer::take_chunk_at_silence(std::vector<float>* out) {
    if (!has_silence_boundary()) return false;
    if (last_speech_pos_ < (size_t)(sample_rate_ / 2)) return false;  // < 0.5 s of content
    const size_t silence_start = last_speech_pos_;
    const size_t split = silence_start + (samples_.size() - silence_start) / 2;
    emit_chunk(split, out);
    last_speech_pos_ = 0;
    return true;
}

bool AudioBuffer::take_forced_chunk(std::vector<float>* out) {
    const size_t max_samples = (size_t)(sample_rate_ * kMaxBufferS);
    if (samples_.size() <= max_samples) return false;
    const size_t search = (size_t)(sample_rate_ * 5);
    const size_t w = sample_rate_ / 50;
    const size_t n = samples_.size();
    const size_t search_start = n > search ? n - search : 0;
    size_t quietest = search_start;
    float quietest_rms = FLT_MAX;
    for (size_t pos = search_start; pos + w <= n; pos += w) {
        const float rms = calculate_rms(samples_.data() + pos, w);
        if (rms < quietest_rms) {
            quietest_rms = rms;
            quietest = pos;
        }
    }
    const size_t split = std::min(quietest + w / 2, n);
    if (split < (size_t)(sample_rate_ / 2)) return false;
    emit_chunk(split, out);
    last_speech_pos_ = last_speech_pos_ > split ? last_speech_pos_ - split : 0;
    return true;
}

std::vector<std::vector<float>> split_at_silences_with_overlap(const std::vector<float>& audio,
                                                               const std::vector<int>& boundaries,
                                                               uint32_t sample_rate) {
    if (boundaries.empty()) return {audio};
    const size_t ov = (size_t)(sample_rate * kOverlapMs / 1000);
    std::vector<std::vector<float>> chunks;
    size_t start = 0;
    for (int bi : boundaries) {
        const size_t b = (size_t)bi;
        if (b > start && b < audio.size()) {
            const size_t cs = start > ov ? start - ov : 0;
            chunks.emplace_back(audio.begin() + cs, audio.begin() + b);
            start = b;
        }
    }
    if (start < audio.size()) {
        const size_t cs = start > ov ? start - ov : 0;
        chunks.emplace_back(audio.begin() + cs, audio.end());
    }
    return chunks;
}

}  // namespace nobs

// ---- C ABI (what a Rust or Python caller binds) ---------------------------------------------------

#define NOBS_API extern "C" __attribute__((visibility("default")))

NOBS_API void* nobs_audio_buffer_new(unsigned sample_rate) {
    if (sample_rate < 50) return nullptr;  // 20 ms window of 0 samples (Rust: chunks(0) panics)
    return new nobs::AudioBuffer(sample_rate);
}
NOBS_API void nobs_audio_buffer_free(void* b) { delete (nobs::AudioBuffer*)b; }
NOBS_API void nobs_audio_buffer_push(void* b, const float* x, long n) {
    ((nobs::AudioBuffer*)b)->push_samples(x, (size_t)n);
}
NOBS_API int nobs_audio_buffer_has_silence_boundary(void* b) {
    return ((nobs::AudioBuffer*)b)->has_silence_boundary();
}
// kind 0: take_chunk_at_silence, 1: take_forced_chunk, 2: take. Returns the chunk length (0 = None) or
// -1 when cap is below the possible chunk length (nothing taken). cap >= len() + overlap_len() always fits.
NOBS_API long nobs_audio_buffer_take(void* b, int kind, float* out, long cap) {
    auto* B = (nobs::AudioBuffer*)b;
    if ((size_t)cap < B->len() + B->overlap_len()) return -1;
    std::vector<float> c;
    bool got;
    if (kind == 0) got = B->take_chunk_at_silence(&c);
    else if (kind == 1) got = B->take_forced_chunk(&c);
    else { c = B->take(); got = true; }
    if (!got) return 0;
    if (!c.empty()) memcpy(out, c.data(), c.size() * sizeof(float));
    return (long)c.size();
}
// out[0] len, out[1] last_speech_pos, out[2] overlap_len, out[3] noise_floor_frames; *noise_floor
NOBS_API void nobs_audio_buffer_info(void* b, long* out, float* noise_floor) {
    auto* B = (nobs::AudioBuffer*)b;
    out[0] = (long)B->len();
    out[1] = (long)B->last_speech_pos();
    out[2] = (long)B->overlap_len();
    out[3] = (long)B->noise_floor_frames();
    if (noise_floor) *noise_floor = B->noise_floor();
}
NOBS_API float nobs_calculate_rms(const float* x, long n) { return nobs::calculate_rms(x, (size_t)n); }


