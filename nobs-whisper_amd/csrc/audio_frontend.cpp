// Audio front-end C ABI (include/whisper_mi355x.h): the reference app's silence
// chunking and 16 kHz resampling (src-tauri/src/audio.rs) for a batch of clips on one GPU, kernels
// in kernels/audio.hip. Host side: the resampler operator (rubato 0.15.0 FftFixedIn's whole FFT
// pipeline folded into one matrix, computed once per input rate in double precision from the
// f32 filter rubato designs), per-device scratch, pointer tables.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <vector>

#include "../../include/whisper_mi355x.h"
#include "common.h"
#include "kernels.h"

namespace wm {
namespace {

constexpr int kRate = 16000;       // WHISPER_SAMPLE_RATE (audio.rs:7)
constexpr int kChunkIn = 1024;     // resample_audio: chunk_size (audio.rs:515)
constexpr int kSubChunks = 2;      // FftFixedIn::new(.., 1024, 2, 1) (audio.rs:517-523)

// rubato FftFixedIn::new sizes [ext, rubato 0.15.0 synchro.rs]
struct FftSizes { int fsi, fso; };
FftSizes fft_sizes(int rate_in) {
    const int g = std::gcd(rate_in, kRate);
    const int min_chunk_in = rate_in / g;
    const int wanted = kChunkIn / kSubChunks;
    const int fft_chunks = (int)std::ceil((float)wanted / (float)min_chunk_in);
    return {fft_chunks * min_chunk_in, fft_chunks * kRate / g};
}

// rubato make_sincs(npoints, 1, cutoff, BlackmanHarris2) in f32 [ext, rubato sinc.rs / windows.rs]:
// Blackman-Harris window squared times sinc((x - npoints/2) * cutoff), normalised to unit sum
std::vector<float> rubato_sinc(int npoints, float cutoff) {
    const float pi = 3.14159265358979323846f;
    const float pi2 = 2.0f * pi, pi4 = 4.0f * pi, pi6 = 6.0f * pi;
    const float np_f = (float)npoints;
    std::vector<float> y(npoints);
    float sum = 0.0f;
    for (int x = 0; x < npoints; x++) {
        const float xf = (float)x;
        float w = 0.35875f - 0.48829f * cosf(pi2 * xf / np_f) + 0.14128f * cosf(pi4 * xf / np_f) -
                  0.01168f * cosf(pi6 * xf / np_f);
        w = w * w;
        const float v = (xf - (float)(npoints / 2)) * cutoff;
        const float s = v == 0.0f ? 1.0f : sinf(v * pi) / (v * pi);
        y[x] = w * s;
        sum += y[x];
    }
    for (float& v : y) v /= sum;
    return y;
}

// The FftFixedIn map from the 2*fsi samples x[(m-1)*fsi, (m+1)*fsi) to output block m, as
// W[t][j] (row stride ldw). FftResampler::resample_unit [ext]: block -> zero-pad to 2*fsi -> real
// FFT -> * filter spectrum (filter_t = sinc / (2*fsi), zero-padded) -> keep bins [0, new_len) ->
// unnormalised real inverse FFT at 2*fso points -> first fso values + previous block's last fso.
std::vector<float> fft_fixed_in_operator(int fsi, int fso, int ldw) {
    const float cutoff = fsi > fso ? powf(0.4f, 16.0f / (float)fsi) * (float)fso / (float)fsi
                                   : powf(0.4f, 16.0f / (float)fsi);
    const std::vector<float> sinc = rubato_sinc(fsi, cutoff);
    const int n_in = 2 * fsi, n_out = 2 * fso;
    std::vector<double> ci(n_in), si(n_in), co(n_out), so(n_out);
    for (int i = 0; i < n_in; i++) { ci[i] = cos(2.0 * M_PI * i / n_in); si[i] = sin(2.0 * M_PI * i / n_in); }
    for (int i = 0; i < n_out; i++) { co[i] = cos(2.0 * M_PI * i / n_out); so[i] = sin(2.0 * M_PI * i / n_out); }
    const int new_len = fsi < fso ? fsi + 1 : fso;
    // filter spectrum H[k], k < new_len
    std::vector<double> hr(new_len, 0.0), hi(new_len, 0.0);
    for (int k = 0; k < new_len; k++)
        for (int t = 0; t < fsi; t++) {
            const double f = (double)(sinc[t] / (float)(2 * fsi));
            const int p = (int)(((long)k * t) % n_in);
            hr[k] += f * ci[p];
            hi[k] -= f * si[p];
        }
    std::vector<float> W((size_t)2 * fsi * ldw, 0.0f);
    std::vector<double> yr(new_len), yi(new_len), y(n_out);
    for (int t = 0; t < fsi; t++) {
        for (int k = 0; k < new_len; k++) {  // Y[k] = e^{-2 pi i k t / n_in} H[k]
            const int p = (int)(((long)k * t) % n_in);
            yr[k] = ci[p] * hr[k] + si[p] * hi[k];
            yi[k] = ci[p] * hi[k] - si[p] * hr[k];
        }
        for (int n = 0; n < n_out; n++) {
            double acc = yr[0];
            for (int k = 1; k < new_len; k++) {
                const int p = (int)(((long)k * n) % n_out);
                const double re = yr[k] * co[p] - yi[k] * so[p];
                acc += (k == fso ? 1.0 : 2.0) * re;
            }
            y[n] = acc;
        }
        for (int j = 0; j < fso; j++) {
            W[(size_t)(fsi + t) * ldw + j] = (float)y[j];   // x_m[t] -> first half of block m
            W[(size_t)t * ldw + j] = (float)y[fso + j];     // x_{m-1}[t] -> overlap into block m
        }
    }
    return W;
}

struct ResampleOp { int fsi = 0, fso = 0, ldw = 0; float* dW = nullptr; };

struct DeviceScratch {
    std::mutex mu;
    hipStream_t st = nullptr;
    std::map<int, ResampleOp> ops;  // by input rate
    void* buf = nullptr;
    size_t cap = 0;
    char* get(size_t bytes) {
        if (bytes > cap) {
            if (buf) WM_CHECK(hipFree(buf));
            cap = bytes + (bytes >> 2);
            WM_CHECK(hipMalloc(&buf, cap));
        }
        return (char*)buf;
    }
};

std::mutex g_dev_mu;
std::map<int, DeviceScratch*> g_dev;

DeviceScratch* scratch(int device) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto& p = g_dev[device];
    if (!p) {
        p = new DeviceScratch();
        WM_CHECK(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
    }
    return p;
}

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int d) { WM_CHECK(hipGetDevice(&prev)); WM_CHECK(hipSetDevice(d)); }
    ~DeviceGuard() { hipSetDevice(prev); }
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Host PCM staged into one device buffer, or caller device pointers; returns the device pointer
// table (in scratch at *off). `ptrs` is the host side of the table: it must outlive the stream
// work (async copies from pageable memory).
const float* const* stage_inputs(DeviceScratch* S, char* base, size_t* off, const float* const* pcm, const int* n,
                                 int n_clips, bool on_device, std::vector<const float*>& ptrs) {
    ptrs.resize(n_clips);
    if (on_device) {
        for (int c = 0; c < n_clips; c++) ptrs[c] = pcm[c];
    } else {
        for (int c = 0; c < n_clips; c++) {
            float* d = (float*)(base + *off);
            if (n[c] > 0) WM_CHECK(hipMemcpyAsync(d, pcm[c], (size_t)n[c] * 4, hipMemcpyHostToDevice, S->st));
            ptrs[c] = d;
            *off += align256((size_t)std::max(n[c], 1) * 4);
        }
    }
    const float** tab = (const float**)(base + *off);
    WM_CHECK(hipMemcpyAsync(tab, ptrs.data(), sizeof(float*) * n_clips, hipMemcpyHostToDevice, S->st));
    *off += align256(sizeof(float*) * n_clips);
    return tab;
}

}  // namespace
}  // namespace wm

using namespace wm;

// engine errors (a HIP error, a rate whose 20 ms window does not fit the kernel's LDS) -> -1
template <typename F> static int guarded(F&& f) {
    try {
        return f();
    } catch (const wm::Error&) {
    } catch (const std::bad_alloc&) {
    }
    return -1;
}

extern "C" {

int whisper_mi355x_find_silence_boundaries(int device, const float* const* pcm, const int* n_samples, int n_clips,
                                           int sample_rate, bool pcm_on_device, int* counts, int* boundaries, int cap,
                                           float* noise_floor, float* rms_out, int rms_stride) {
    return guarded([&]() -> int {
        if (n_clips <= 0) return 0;
        if (!pcm || !n_samples || !counts || cap < 0 || sample_rate < 50) return -1;
        const int ws = sample_rate / 50;
        int max_n = 0;
        size_t in_bytes = 0;
        for (int c = 0; c < n_clips; c++) {
            if (n_samples[c] < 0) return -1;
            max_n = std::max(max_n, n_samples[c]);
            in_bytes += align256((size_t)std::max(n_samples[c], 1) * 4);
        }
        const int max_win = std::max(1, max_n / ws);
        if (rms_out && rms_stride < max_n / ws) return -1;
        DeviceGuard g(device);
        DeviceScratch* S = scratch(device);
        std::lock_guard<std::mutex> lk(S->mu);
        const size_t bytes = (pcm_on_device ? 0 : in_bytes) + align256(sizeof(float*) * n_clips) +
                             align256((size_t)n_clips * max_win * 4) + 2 * align256((size_t)n_clips * 4) +
                             align256((size_t)n_clips * std::max(cap, 1) * 4);
        char* base = S->get(bytes);
        size_t off = 0;
        std::vector<const float*> ptrs;
        const float* const* d_pcm = stage_inputs(S, base, &off, pcm, n_samples, n_clips, pcm_on_device, ptrs);
        int* d_n = (int*)(base + off); off += align256((size_t)n_clips * 4);
        float* d_rms = (float*)(base + off); off += align256((size_t)n_clips * max_win * 4);
        int* d_counts = (int*)(base + off); off += align256((size_t)n_clips * 4);
        float* d_floor = (float*)(base + off); off += align256((size_t)n_clips * 4);
        int* d_b = (int*)(base + off);
        WM_CHECK(hipMemcpyAsync(d_n, n_samples, (size_t)n_clips * 4, hipMemcpyHostToDevice, S->st));
        launch_silence_boundaries(d_pcm, d_n, n_clips, max_n, sample_rate, d_rms, max_win, d_counts, d_b, std::max(cap, 1),
                                  d_floor, S->st);
        WM_CHECK(hipMemcpyAsync(counts, d_counts, (size_t)n_clips * 4, hipMemcpyDeviceToHost, S->st));
        if (cap > 0 && boundaries)
            WM_CHECK(hipMemcpyAsync(boundaries, d_b, (size_t)n_clips * cap * 4, hipMemcpyDeviceToHost, S->st));
        if (noise_floor) WM_CHECK(hipMemcpyAsync(noise_floor, d_floor, (size_t)n_clips * 4, hipMemcpyDeviceToHost, S->st));
        if (rms_out)
            WM_CHECK(hipMemcpy2DAsync(rms_out, (size_t)rms_stride * 4, d_rms, (size_t)max_win * 4, (size_t)(max_n / ws) * 4,
                                      n_clips, hipMemcpyDeviceToHost, S->st));
        WM_CHECK(hipStreamSynchronize(S->st));
        return 0;
    });
}

int whisper_mi355x_resample_len(int n_in, int rate_in) {
    if (n_in <= 0 || rate_in <= 0) return 0;
    if (rate_in == kRate) return n_in;
    const FftSizes z = fft_sizes(rate_in);
    const long total = ((long)n_in + kChunkIn - 1) / kChunkIn * kChunkIn;  // last chunk zero-padded
    const long produced = total / z.fsi * z.fso;
    const long expected = (long)((double)n_in * ((double)kRate / (double)rate_in));
    return (int)std::min(produced, expected);
}

int whisper_mi355x_resample_chunk(int device, const float* const* audio, const int* n_in, int n_clips, int rate_in,
                                  bool on_device, float* const* out) {
    return guarded([&]() -> int {
        if (n_clips <= 0) return 0;
        if (!audio || !n_in || !out || rate_in <= 0) return -1;
        DeviceGuard g(device);
        DeviceScratch* S = scratch(device);
        std::lock_guard<std::mutex> lk(S->mu);
        std::vector<int> n_out(n_clips);
        int max_out = 0;
        size_t in_bytes = 0, out_bytes = 0;
        for (int c = 0; c < n_clips; c++) {
            if (n_in[c] < 0) return -1;
            n_out[c] = whisper_mi355x_resample_len(n_in[c], rate_in);
            max_out = std::max(max_out, n_out[c]);
            in_bytes += align256((size_t)std::max(n_in[c], 1) * 4);
            out_bytes += align256((size_t)std::max(n_out[c], 1) * 4);
        }
        if (rate_in == kRate) {  // resample_chunk returns the audio unchanged (audio.rs:332-334)
            for (int c = 0; c < n_clips; c++) {
                if (n_in[c] <= 0) continue;
                if (on_device) WM_CHECK(hipMemcpyAsync(out[c], audio[c], (size_t)n_in[c] * 4, hipMemcpyDeviceToDevice, S->st));
                else std::memcpy(out[c], audio[c], (size_t)n_in[c] * 4);
            }
            WM_CHECK(hipStreamSynchronize(S->st));
            return 0;
        }
        ResampleOp& op = S->ops[rate_in];
        if (!op.dW) {
            const FftSizes z = fft_sizes(rate_in);
            op.fsi = z.fsi; op.fso = z.fso; op.ldw = (z.fso + 63) / 64 * 64;
            const std::vector<float> W = fft_fixed_in_operator(op.fsi, op.fso, op.ldw);
            WM_CHECK(hipMalloc((void**)&op.dW, W.size() * 4));
            WM_CHECK(hipMemcpy(op.dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
        }
        const size_t bytes = (on_device ? 0 : in_bytes + out_bytes) + 2 * align256(sizeof(float*) * n_clips) +
                             2 * align256((size_t)n_clips * 4);
        char* base = S->get(bytes);
        size_t off = 0;
        std::vector<const float*> ptrs;
        const float* const* d_in = stage_inputs(S, base, &off, audio, n_in, n_clips, on_device, ptrs);
        std::vector<float*> optr(n_clips);
        for (int c = 0; c < n_clips; c++) {
            if (on_device) optr[c] = out[c];
            else { optr[c] = (float*)(base + off); off += align256((size_t)std::max(n_out[c], 1) * 4); }
        }
        float** d_out = (float**)(base + off); off += align256(sizeof(float*) * n_clips);
        int* d_nin = (int*)(base + off); off += align256((size_t)n_clips * 4);
        int* d_nout = (int*)(base + off);
        WM_CHECK(hipMemcpyAsync(d_out, optr.data(), sizeof(float*) * n_clips, hipMemcpyHostToDevice, S->st));
        WM_CHECK(hipMemcpyAsync(d_nin, n_in, (size_t)n_clips * 4, hipMemcpyHostToDevice, S->st));
        WM_CHECK(hipMemcpyAsync(d_nout, n_out.data(), (size_t)n_clips * 4, hipMemcpyHostToDevice, S->st));
        launch_resample(d_in, d_nin, n_clips, max_out, op.dW, op.ldw, op.fsi, op.fso, d_out, d_nout, S->st);
        if (!on_device)
            for (int c = 0; c < n_clips; c++)
                if (n_out[c] > 0)
                    WM_CHECK(hipMemcpyAsync(out[c], optr[c], (size_t)n_out[c] * 4, hipMemcpyDeviceToHost, S->st));
        WM_CHECK(hipStreamSynchronize(S->st));
        return 0;
    });
}

int whisper_mi355x_resample_operator(int rate_in, int* fsi, int* fso, float* W, long cap) {
    if (rate_in <= 0 || rate_in == kRate) return -1;
    const FftSizes z = fft_sizes(rate_in);
    if (fsi) *fsi = z.fsi;
    if (fso) *fso = z.fso;
    if (!W) return 0;
    if (cap < (long)2 * z.fsi * z.fso) return -1;
    const std::vector<float> full = fft_fixed_in_operator(z.fsi, z.fso, z.fso);
    std::memcpy(W, full.data(), full.size() * 4);
    return 0;
}

}  // extern "C"
