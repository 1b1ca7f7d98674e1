// TEST INFRASTRUCTURE ONLY (see oracle_common.h). Compiled with -ffp-contract=off so that every
// product/sum below rounds exactly as written; the HIP mel kernel is built the same way and is
// checked bit-exact against this file.
//
// Restates whisper.cpp ≈v1.7.x `log_mel_spectrogram` + `log_mel_spectrogram_worker_thread` +
// `fft`/`dft` + `whisper_global_cache` [ext]: periodic Hann(400), reflective 200-sample pre-pad,
// 30 s of zeros appended, hop 160, mixed radix-2 / 25-point DFT with 400-entry sin/cos tables,
// power = re²+im², filterbank dot summed in double (4 float products per group), log10 of
// max(sum,1e-10), global (max - 8) clamp, (x + 4) / 4.
#include <algorithm>
#include <cmath>
#include <vector>
#include <omp.h>

namespace oracle {

static const int N_FFT = 400;
static const int HOP = 160;
static const int SIN_COS_N = 400;

struct MelTables {
    float sin_vals[SIN_COS_N], cos_vals[SIN_COS_N], hann[N_FFT];
    MelTables() {
        for (int i = 0; i < SIN_COS_N; i++) {
            double theta = (2 * M_PI * i) / SIN_COS_N;
            sin_vals[i] = sinf(theta);
            cos_vals[i] = cosf(theta);
        }
        for (int i = 0; i < N_FFT; i++) hann[i] = 0.5 * (1.0 - cosf((2.0 * M_PI * i) / (N_FFT + 0)));
    }
};
static const MelTables g_tab;

extern "C" void oracle_mel_tables(float* sin_out, float* cos_out, float* hann_out) {
    std::copy(g_tab.sin_vals, g_tab.sin_vals + SIN_COS_N, sin_out);
    std::copy(g_tab.cos_vals, g_tab.cos_vals + SIN_COS_N, cos_out);
    std::copy(g_tab.hann, g_tab.hann + N_FFT, hann_out);
}

static void dft(const float* in, int N, float* out) {
    const int step = SIN_COS_N / N;
    for (int k = 0; k < N; k++) {
        float re = 0, im = 0;
        for (int n = 0; n < N; n++) {
            int idx = (k * n * step) % SIN_COS_N;
            re += in[n] * g_tab.cos_vals[idx];
            im -= in[n] * g_tab.sin_vals[idx];
        }
        out[k * 2 + 0] = re;
        out[k * 2 + 1] = im;
    }
}

static void fft(float* in, int N, float* out) {
    if (N == 1) { out[0] = in[0]; out[1] = 0; return; }
    const int half_N = N / 2;
    if (N - half_N * 2 == 1) { dft(in, N, out); return; }
    float* even = in + N;
    for (int i = 0; i < half_N; ++i) even[i] = in[2 * i];
    float* even_fft = out + 2 * N;
    fft(even, half_N, even_fft);
    float* odd = even;
    for (int i = 0; i < half_N; ++i) odd[i] = in[2 * i + 1];
    float* odd_fft = even_fft + N;
    fft(odd, half_N, odd_fft);
    const int step = SIN_COS_N / N;
    for (int k = 0; k < half_N; k++) {
        int idx = k * step;
        float re = g_tab.cos_vals[idx];
        float im = -g_tab.sin_vals[idx];
        float re_odd = odd_fft[2 * k + 0];
        float im_odd = odd_fft[2 * k + 1];
        out[2 * k + 0] = even_fft[2 * k + 0] + re * re_odd - im * im_odd;
        out[2 * k + 1] = even_fft[2 * k + 1] + re * im_odd + im * re_odd;
        out[2 * (k + half_N) + 0] = even_fft[2 * k + 0] - re * re_odd + im * im_odd;
        out[2 * (k + half_N) + 1] = even_fft[2 * k + 1] - re * im_odd - im * re_odd;
    }
}

// mel out: [n_mel][n_len] row-major (whisper_mel.data layout). Returns n_len; n_len_org via ptr.
int mel_compute(const float* samples, int n_samples, const float* filters, int n_mel, int n_fft_bins,
                std::vector<float>& mel, int* n_len_org_out, int n_threads) {
    const int64_t stage_1_pad = 16000 * 30;
    const int64_t stage_2_pad = N_FFT / 2;
    std::vector<float> padded(n_samples + stage_1_pad + stage_2_pad * 2, 0.0f);
    std::copy(samples, samples + n_samples, padded.begin() + stage_2_pad);
    std::reverse_copy(samples + 1, samples + 1 + stage_2_pad, padded.begin());

    const int n_len = (int)((padded.size() - N_FFT) / HOP);
    *n_len_org_out = 1 + (n_samples + (int)stage_2_pad - N_FFT) / HOP;
    mel.assign((size_t)n_mel * n_len, 0.0f);

    const int n_in = n_samples + (int)stage_2_pad;  // what the worker treats as "n_samples"
    const int n_fft_frames = std::min(n_in / HOP + 1, n_len);
    const float* hann = g_tab.hann;
#pragma omp parallel num_threads(n_threads)
    {
        std::vector<float> fft_in(N_FFT * 2, 0.0f), fft_out(N_FFT * 2 * 2 * 2);
#pragma omp for schedule(static)
        for (int i = 0; i < n_fft_frames; i++) {
            const int offset = i * HOP;
            std::fill(fft_in.begin(), fft_in.end(), 0.0f);
            const int nw = std::min(N_FFT, n_in - offset);
            for (int j = 0; j < nw; j++) fft_in[j] = hann[j] * padded[offset + j];
            fft(fft_in.data(), N_FFT, fft_out.data());
            for (int j = 0; j < n_fft_bins; j++)
                fft_out[j] = (fft_out[2 * j + 0] * fft_out[2 * j + 0] + fft_out[2 * j + 1] * fft_out[2 * j + 1]);
            for (int j = 0; j < n_mel; j++) {
                double sum = 0.0;
                int k = 0;
                for (k = 0; k < n_fft_bins - 3; k += 4) {
                    sum += fft_out[k + 0] * filters[j * n_fft_bins + k + 0] +
                           fft_out[k + 1] * filters[j * n_fft_bins + k + 1] +
                           fft_out[k + 2] * filters[j * n_fft_bins + k + 2] +
                           fft_out[k + 3] * filters[j * n_fft_bins + k + 3];
                }
                for (; k < n_fft_bins; k++) sum += fft_out[k] * filters[j * n_fft_bins + k];
                sum = log10(std::max(sum, 1e-10));
                mel[(size_t)j * n_len + i] = sum;
            }
        }
    }
    const double empty = log10(1e-10);
    for (int i = n_fft_frames; i < n_len; i++)
        for (int j = 0; j < n_mel; j++) mel[(size_t)j * n_len + i] = empty;

    double mmax = -1e20;
    for (size_t i = 0; i < mel.size(); i++) if (mel[i] > mmax) mmax = mel[i];
    mmax -= 8.0;
    for (size_t i = 0; i < mel.size(); i++) {
        if (mel[i] < mmax) mel[i] = mmax;
        mel[i] = (mel[i] + 4.0) / 4.0;
    }
    return n_len;
}

}  // namespace oracle
