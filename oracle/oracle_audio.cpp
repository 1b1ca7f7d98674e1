// TEST INFRASTRUCTURE ONLY (see oracle_common.h): CPU restatement of the reference app's audio
// front-end, src-tauri/src/audio.rs, for the GPU front-end's parity tests.
//
//  - calculate_rms (audio.rs:364-370), estimate_noise_floor (:373-397), find_silence_boundaries
//    (:400-467), split_at_silences_with_overlap (:474-507): scalar f32 code in the reference's
//    operation order (sequential f32 sums, f32 constants), so window RMS values and boundaries are
//    exact. Pinned by the reference's own tests (audio.rs:569-831), replayed in tests/test_audio.py.
//  - resample_audio (:509-563) = rubato 0.15.0 FftFixedIn(rate_in, 16000, 1024, 2, 1) [ext, a
//    Cargo.lock dependency absent from /root/reference]: restated from rubato's published algorithm,
//    literally (1024-sample calls, saved-frame carry-over, per-block zero-padded FFT, filter
//    multiply, spectrum truncation, inverse FFT, overlap-add, final truncation), in double
//    precision with direct DFTs. The reference pins only its output length (audio.rs:569-583);
//    its values are "parity unpinned" beyond this restatement.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

namespace {

const float SILENCE_THRESHOLD = 0.01f;
const unsigned MIN_SILENCE_DURATION_MS = 700;
const unsigned MIN_CHUNK_DURATION_MS = 1000;
const float ADAPTIVE_THRESHOLD_NOISE_FACTOR = 3.0f;
const float MIN_THRESHOLD_FACTOR = 0.5f;
const size_t NOISE_FLOOR_ESTIMATION_WINDOWS = 25;
const float NOISE_FLOOR_PERCENTILE = 0.1f;
const float MIN_NOISE_FLOOR_FACTOR = 0.3f;
const unsigned CHUNK_OVERLAP_MS = 200;

float calculate_rms(const float* s, size_t n) {
    if (n == 0) return 0.0f;
    float sum = 0.0f;  // Iterator::sum over f32: a sequential fold
    for (size_t i = 0; i < n; i++) {
        const float sq = s[i] * s[i];
        sum = sum + sq;
    }
    return std::sqrt(sum / (float)n);
}

float estimate_noise_floor(const float* a, size_t n, unsigned sr) {
    const size_t ws = sr / 50;
    std::vector<float> v;
    for (size_t i = 0; i < NOISE_FLOOR_ESTIMATION_WINDOWS; i++) {
        const size_t start = i * ws;
        if (start + ws <= n) v.push_back(calculate_rms(a + start, ws));
    }
    if (v.empty()) return SILENCE_THRESHOLD;
    std::stable_sort(v.begin(), v.end());
    const size_t idx = (size_t)((float)v.size() * NOISE_FLOOR_PERCENTILE);
    const float nf = idx < v.size() ? v[idx] : SILENCE_THRESHOLD;
    return std::max(nf, SILENCE_THRESHOLD * MIN_NOISE_FLOOR_FACTOR);
}

// rubato FftFixedIn sizes and filter (see nobs-whisper_amd/csrc/audio_frontend.cpp for the product)
void sizes(int rate_in, int* fsi, int* fso) {
    const int g = std::gcd(rate_in, 16000);
    const int chunks = (int)std::ceil((float)(1024 / 2) / (float)(rate_in / g));
    *fsi = chunks * (rate_in / g);
    *fso = chunks * (16000 / g);
}

std::vector<float> sinc_filter(int npoints, float cutoff) {
    const float pi = 3.14159265358979323846f;
    std::vector<float> y(npoints);
    float sum = 0.0f;
    for (int x = 0; x < npoints; x++) {
        const float xf = (float)x, np = (float)npoints;
        float w = 0.35875f - 0.48829f * cosf(2.0f * pi * xf / np) + 0.14128f * cosf(4.0f * pi * xf / np) -
                  0.01168f * cosf(6.0f * pi * xf / np);
        w = w * w;  // BlackmanHarris2
        const float v = (xf - (float)(npoints / 2)) * cutoff;
        y[x] = w * (v == 0.0f ? 1.0f : sinf(v * pi) / (v * pi));
        sum += y[x];
    }
    for (float& e : y) e /= sum;
    return y;
}

struct FftResampler {
    int fsi, fso, new_len;
    std::vector<double> hr, hi;  // filter spectrum bins [0, new_len)
    FftResampler(int fsi_, int fso_) : fsi(fsi_), fso(fso_) {
        const float cutoff = fsi > fso ? powf(0.4f, 16.0f / (float)fsi) * (float)fso / (float)fsi
                                       : powf(0.4f, 16.0f / (float)fsi);
        const std::vector<float> s = sinc_filter(fsi, cutoff);
        new_len = fsi < fso ? fsi + 1 : fso;
        hr.assign(new_len, 0.0); hi.assign(new_len, 0.0);
        for (int k = 0; k < new_len; k++)
            for (int t = 0; t < fsi; t++) {
                const double a = -2.0 * M_PI * (double)k * t / (2.0 * fsi);
                const double f = (double)(s[t] / (float)(2 * fsi));
                hr[k] += f * cos(a); hi[k] += f * sin(a);
            }
    }
    // FftResampler::resample_unit
    void unit(const float* in, float* out, std::vector<double>& overlap) const {
        std::vector<double> yr(new_len), yi(new_len);
        for (int k = 0; k < new_len; k++) {
            double xr = 0.0, xi = 0.0;  // input_buf = [in, zeros(fsi)]: forward real FFT bin k
            for (int t = 0; t < fsi; t++) {
                const double a = -2.0 * M_PI * (double)k * t / (2.0 * fsi);
                xr += in[t] * cos(a); xi += in[t] * sin(a);
            }
            yr[k] = xr * hr[k] - xi * hi[k];
            yi[k] = xr * hi[k] + xi * hr[k];
        }
        std::vector<double> y(2 * fso);
        for (int n = 0; n < 2 * fso; n++) {  // unnormalised inverse real FFT, bins >= new_len zero
            double acc = yr[0];
            for (int k = 1; k < new_len; k++) {
                const double a = 2.0 * M_PI * (double)k * n / (2.0 * fso);
                acc += (k == fso ? 1.0 : 2.0) * (yr[k] * cos(a) - yi[k] * sin(a));
            }
            y[n] = acc;
        }
        for (int j = 0; j < fso; j++) out[j] = (float)(y[j] + overlap[j]);
        for (int j = 0; j < fso; j++) overlap[j] = y[fso + j];
    }
};

}  // namespace

extern "C" {

float oracle_calculate_rms(const float* s, int n) { return calculate_rms(s, (size_t)std::max(n, 0)); }

float oracle_estimate_noise_floor(const float* a, int n, int sr) {
    return estimate_noise_floor(a, (size_t)std::max(n, 0), (unsigned)sr);
}

int oracle_find_silence_boundaries(const float* a, int n_, int sr_, int* out, int cap) {
    const size_t n = (size_t)std::max(n_, 0);
    const unsigned sr = (unsigned)sr_;
    const size_t min_sil = sr * MIN_SILENCE_DURATION_MS / 1000;
    const size_t min_chunk = sr * MIN_CHUNK_DURATION_MS / 1000;
    const size_t ws = sr / 50;
    const float nf = estimate_noise_floor(a, n, sr);
    const float thr = std::max(nf * ADAPTIVE_THRESHOLD_NOISE_FACTOR, SILENCE_THRESHOLD * MIN_THRESHOLD_FACTOR);
    std::vector<size_t> b;
    bool in_sil = false;
    size_t sil_start = 0, last = 0;
    auto try_add = [&](size_t s0, size_t s1) {
        const size_t dur = s1 - s0;
        if (dur >= min_sil) {
            const size_t split = s0 + dur / 2;
            if (split - last >= min_chunk) { b.push_back(split); last = split; }
        }
    };
    for (size_t pos = 0; pos + ws <= n; pos += ws) {
        const float rms = calculate_rms(a + pos, ws);
        if (rms < thr) {
            if (!in_sil) { in_sil = true; sil_start = pos; }
        } else {
            if (in_sil) try_add(sil_start, pos);
            in_sil = false;
        }
    }
    if (in_sil) try_add(sil_start, n);
    for (size_t i = 0; i < b.size() && (int)i < cap; i++) out[i] = (int)b[i];
    return (int)b.size();
}

// split_at_silences_with_overlap: chunk i = audio[starts[i], ends[i]); returns the chunk count
int oracle_split_at_silences(int n, const int* bounds, int nb, int sr, int* starts, int* ends, int cap) {
    const int overlap = (int)((unsigned)sr * CHUNK_OVERLAP_MS / 1000);
    int k = 0;
    auto push = [&](int s, int e) { if (k < cap) { starts[k] = s; ends[k] = e; } k++; };
    if (nb == 0) { push(0, n); return k; }
    int start = 0;
    for (int i = 0; i < nb; i++) {
        const int b = bounds[i];
        if (b > start && b < n) { push(std::max(start - overlap, 0), b); start = b; }
    }
    if (start < n) push(std::max(start - overlap, 0), n);
    return k;
}

// resample_audio(audio, rate_in, 16000): returns the output length (stored up to cap)
int oracle_resample(const float* audio, int n, int rate_in, float* out, int cap) {
    if (rate_in == 16000) {
        for (int i = 0; i < n && i < cap; i++) out[i] = audio[i];
        return n;
    }
    int fsi, fso;
    sizes(rate_in, &fsi, &fso);
    const FftResampler R(fsi, fso);
    std::vector<double> overlap(fso, 0.0);
    std::vector<float> buf(1024 + fsi, 0.0f), res;
    int saved = 0;
    for (int pos = 0; pos < n; pos += 1024) {  // resample_audio's loop; FftFixedIn::process
        const int end = std::min(pos + 1024, n);
        for (int i = 0; i < 1024; i++) buf[saved + i] = pos + i < end ? audio[pos + i] : 0.0f;
        const int ready = (1024 + saved) / fsi;
        std::vector<float> blk(fso);
        for (int m = 0; m < ready; m++) {
            R.unit(&buf[(size_t)m * fsi], blk.data(), overlap);
            res.insert(res.end(), blk.begin(), blk.end());
        }
        const int extra = 1024 + saved - ready * fsi;
        std::copy(buf.begin() + ready * fsi, buf.begin() + ready * fsi + extra, buf.begin());
        saved = extra;
    }
    const size_t expected = (size_t)((double)n * (16000.0 / (double)rate_in));
    if (res.size() > expected) res.resize(expected);
    for (size_t i = 0; i < res.size() && (int)i < cap; i++) out[i] = res[i];
    return (int)res.size();
}

}  // extern "C"
