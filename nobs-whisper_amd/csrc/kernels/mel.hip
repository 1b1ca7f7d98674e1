// Log-mel spectrogram for a batch of PCM jobs — HIP kernel #1.
//
// Reproduces whisper.cpp's CPU algorithm bit-for-bit ([ext] `log_mel_spectrogram` +
// `log_mel_spectrogram_worker_thread` + recursive `fft`/`dft`, restated in
// oracle/oracle_mel.cpp): same Hann/sin/cos tables (computed on the host with the same libm
// calls and uploaded), same radix-2 recursion down to 25-point DFT leaves, same operation order,
// no FMA contraction (this file is compiled with -ffp-contract=off), filterbank dot summed in
// double in groups of four float products, log10 in double. One workgroup = 4 frames of one job;
// the recursion is flattened into LDS levels (16 leaves x 25 -> 8 x 50 -> 4 x 100 -> 2 x 200 ->
// 1 x 400 complex values per frame), one thread per output value.
//
// Roofline: HBM-bound in principle (1.92 MB PCM in + n_mels*3000*4 B out per 30 s chunk) but
// the 25-point DFT leaves (20 kFLOP/frame) and the double-precision filterbank make it a small
// VALU kernel; it is <1% of a chunk's time either way.
#include "../common.h"
#include "../kernels.h"

namespace wm {

static constexpr int MEL_FPW = 4;     // frames per workgroup
static constexpr int MEL_THREADS = 256;

struct MelTablesDev { float sinv[400], cosv[400], hann[400]; };

__device__ __forceinline__ float padded_sample(const float* x, int n, int p) {
    // whisper.cpp samples_padded: [reverse(samples[1..200])] + samples + zeros
    if (p < 200) { const int i = 200 - p; return i < n ? x[i] : 0.0f; }
    const int i = p - 200;
    return i < n ? x[i] : 0.0f;
}

__device__ __forceinline__ int ordered_key(float f) {
    int b = __float_as_int(f);
    return b >= 0 ? b : (b ^ 0x7fffffff);
}

// leaf index = path bits (b1 b2 b3 b4) as b1 | b2<<1 | b3<<2 | b4<<3 ; its samples are x[16n + leaf]
__global__ void __launch_bounds__(MEL_THREADS)
mel_kernel(const float* const* __restrict__ pcm, const int* __restrict__ n_samples,
           const MelTablesDev* __restrict__ tab, const float* __restrict__ filt_t,  // [n_fft][n_mel]
           int n_mel, float* const* __restrict__ mel_out, const int* __restrict__ n_len,
           int* __restrict__ max_key) {
    const int job = blockIdx.y;
    const int n = n_samples[job];
    const int nl = n_len[job];
    const int n_fft_frames = min((n + 200) / 160 + 1, nl);
    const int f0 = blockIdx.x * MEL_FPW;
    if (f0 >= n_fft_frames) return;
    const float* x = pcm[job];

    __shared__ float s_sin[400], s_cos[400];
    __shared__ float s_in[MEL_FPW][400];
    __shared__ float s_a[MEL_FPW][800], s_b[MEL_FPW][800];
    __shared__ int s_max;
    const int tid = threadIdx.x;
    if (tid == 0) s_max = ordered_key(-INFINITY);
    for (int i = tid; i < 400; i += MEL_THREADS) { s_sin[i] = tab->sinv[i]; s_cos[i] = tab->cosv[i]; }
    const int n_in = n + 200;
    for (int i = tid; i < MEL_FPW * 400; i += MEL_THREADS) {
        const int f = i / 400, j = i % 400, fr = f0 + f;
        const int off = fr * 160;
        float v = 0.0f;
        if (fr < n_fft_frames && j < n_in - off) v = tab->hann[j] * padded_sample(x, n, off + j);
        s_in[f][j] = v;
    }
    __syncthreads();
    // leaves: 16 leaves x 25 outputs, dft with step 16 (table index (k*m*16) % 400)
    for (int i = tid; i < MEL_FPW * 400; i += MEL_THREADS) {
        const int f = i / 400, r = i % 400, leaf = r / 25, k = r % 25;
        float re = 0, im = 0;
        for (int m = 0; m < 25; m++) {
            const int idx = (k * m * 16) % 400;
            const float v = s_in[f][16 * m + leaf];
            re += v * s_cos[idx];
            im -= v * s_sin[idx];
        }
        s_a[f][2 * r + 0] = re;
        s_a[f][2 * r + 1] = im;
    }
    __syncthreads();
    // combine levels: node size N = 50, 100, 200, 400. Nodes of the previous level (size N/2) are
    // indexed by path prefix; node p of size N/2 at level L is stored at offset p*(N/2) complex.
    // Child ordering: at the leaf level, leaf id = b1 | b2<<1 | b3<<2 | b4<<3 where b4 is the LAST
    // split; a node at size N with prefix q (bits b1..b_l) has children q (b_{l+1}=0) and
    // q + (1<<l) (b_{l+1}=1).
    float* src = &s_a[0][0];
    float* dst = &s_b[0][0];
    int n_nodes = 8;  // nodes at the new level
    for (int N = 50; N <= 400; N *= 2) {
        const int half = N / 2;
        const int step = 400 / N;
        for (int i = tid; i < MEL_FPW * n_nodes * half; i += MEL_THREADS) {
            const int f = i / (n_nodes * half);
            const int rem = i % (n_nodes * half);
            const int q = rem / half, k = rem % half;
            const float* E = src + f * 800 + 2 * (q * half);
            const float* O = src + f * 800 + 2 * ((q + n_nodes) * half);
            float* out = dst + f * 800 + 2 * (q * N);
            const int idx = k * step;
            const float re = s_cos[idx];
            const float im = -s_sin[idx];
            const float re_odd = O[2 * k + 0], im_odd = O[2 * k + 1];
            out[2 * k + 0] = E[2 * k + 0] + re * re_odd - im * im_odd;
            out[2 * k + 1] = E[2 * k + 1] + re * im_odd + im * re_odd;
            out[2 * (k + half) + 0] = E[2 * k + 0] - re * re_odd + im * im_odd;
            out[2 * (k + half) + 1] = E[2 * k + 1] - re * im_odd - im * re_odd;
        }
        __syncthreads();
        float* t = src; src = dst; dst = t;
        n_nodes /= 2;
    }
    // src holds the 400-point spectrum; power for bins 0..200 into dst[f][0..200]
    for (int i = tid; i < MEL_FPW * 201; i += MEL_THREADS) {
        const int f = i / 201, j = i % 201;
        const float re = src[f * 800 + 2 * j], im = src[f * 800 + 2 * j + 1];
        dst[f * 800 + j] = (re * re + im * im);
    }
    __syncthreads();
    float* out = mel_out[job];
    int local_max = ordered_key(-INFINITY);
    for (int i = tid; i < MEL_FPW * n_mel; i += MEL_THREADS) {
        const int f = i / n_mel, j = i % n_mel, fr = f0 + f;
        if (fr >= n_fft_frames) continue;
        const float* pw = dst + f * 800;
        double sum = 0.0;
        int k = 0;
        for (k = 0; k < 201 - 3; k += 4) {
            sum += pw[k + 0] * filt_t[(k + 0) * n_mel + j] + pw[k + 1] * filt_t[(k + 1) * n_mel + j] +
                   pw[k + 2] * filt_t[(k + 2) * n_mel + j] + pw[k + 3] * filt_t[(k + 3) * n_mel + j];
        }
        for (; k < 201; k++) sum += pw[k] * filt_t[k * n_mel + j];
        sum = log10(sum > 1e-10 ? sum : 1e-10);
        const float v = (float)sum;
        out[(size_t)j * nl + fr] = v;
        local_max = max(local_max, ordered_key(v));
    }
    atomicMax(&s_max, local_max);
    __syncthreads();
    if (tid == 0) atomicMax(&max_key[job], s_max);
}

// Normalise ((max-8) clamp, (x+4)/4 in double, exactly as log_mel_spectrogram) and extract the
// encoder window [seek, seek+3000) of each job into the conv1 input image: f16/bf16, time-major,
// with one zero frame on each side (conv padding) -> out[b][3002][n_mel]. Frames past n_len are 0
// (whisper_encode_internal zero-fills them); frames in [n_fft_frames, n_len) carry log10(1e-10).
template <typename T>
__global__ void mel_window_kernel(float* const* __restrict__ mel, const int* __restrict__ n_len,
                                  const int* __restrict__ n_samples, const int* __restrict__ max_key,
                                  const int* __restrict__ win_job, const int* __restrict__ win_seek,
                                  int n_mel, T* __restrict__ out) {
    const int b = blockIdx.y;
    const int job = win_job[b];
    const int seek = win_seek[b];
    const int nl = n_len[job];
    const int n_fft_frames = min((n_samples[job] + 200) / 160 + 1, nl);
    const int kmax = max_key[job];
    const float fmax = __int_as_float(kmax >= 0 ? kmax : (kmax ^ 0x7fffffff));
    const double mmax = (double)fmax - 8.0;
    const float empty = (float)log10(1e-10);
    const float* m = mel[job];
    T* o = out + (size_t)b * 3002 * n_mel;
    const int total = 3002 * n_mel;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int row = i / n_mel, j = i % n_mel;
        float v = 0.0f;
        const int fr = seek + row - 1;
        if (row > 0 && row < 3001 && fr < nl) {
            float raw = fr < n_fft_frames ? m[(size_t)j * nl + fr] : empty;
            if ((double)raw < mmax) raw = (float)mmax;
            v = (float)(((double)raw + 4.0) / 4.0);
        }
        o[i] = (T)v;
    }
}

// Full normalised mel of one job into [n_mel][n_len] f32 (whisper_pcm_to_mel API / tests).
__global__ void mel_normalize_kernel(const float* __restrict__ mel, int nl, int n_samples, const int* __restrict__ max_key,
                                     int n_mel, float* __restrict__ out) {
    const int n_fft_frames = min((n_samples + 200) / 160 + 1, nl);
    const int kmax = *max_key;
    const float fmax = __int_as_float(kmax >= 0 ? kmax : (kmax ^ 0x7fffffff));
    const double mmax = (double)fmax - 8.0;
    const float empty = (float)log10(1e-10);
    const long total = (long)n_mel * nl;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int fr = (int)(i % nl);
        float raw = fr < n_fft_frames ? mel[i] : empty;
        if ((double)raw < mmax) raw = (float)mmax;
        out[i] = (float)(((double)raw + 4.0) / 4.0);
    }
}

__global__ void mel_init_max_kernel(int* max_key, int n, const int* __restrict__ n_samples, const int* __restrict__ n_len) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int n_fft_frames = min((n_samples[i] + 200) / 160 + 1, n_len[i]);
        // frames past n_fft_frames hold log10(1e-10) and take part in the global max
        max_key[i] = n_fft_frames < n_len[i] ? ordered_key((float)log10(1e-10)) : ordered_key(-INFINITY);
    }
}

void launch_mel(const float* const* d_pcm, const int* d_n, const void* d_tab, const float* d_filt_t, int n_mel,
                float* const* d_mel, const int* d_nlen, int* d_max, int n_jobs, int max_frames, hipStream_t st) {
    mel_init_max_kernel<<<cdiv(n_jobs, 64), 64, 0, st>>>(d_max, n_jobs, d_n, d_nlen);
    dim3 grid(cdiv(max_frames, MEL_FPW), n_jobs);
    mel_kernel<<<grid, MEL_THREADS, 0, st>>>(d_pcm, d_n, (const MelTablesDev*)d_tab, d_filt_t, n_mel, d_mel, d_nlen, d_max);
}

void launch_mel_window(DType dt, float* const* d_mel, const int* d_nlen, const int* d_n, const int* d_max,
                       const int* d_win_job, const int* d_win_seek, int n_win, int n_mel, void* out, hipStream_t st) {
    dim3 grid(cdiv(3002 * n_mel, 256 * 8), n_win);
    if (dt == DType::F16)
        mel_window_kernel<half_t><<<grid, 256, 0, st>>>(d_mel, d_nlen, d_n, d_max, d_win_job, d_win_seek, n_mel, (half_t*)out);
    else
        mel_window_kernel<bf16_t><<<grid, 256, 0, st>>>(d_mel, d_nlen, d_n, d_max, d_win_job, d_win_seek, n_mel, (bf16_t*)out);
}

void launch_mel_normalize(const float* d_mel, int nl, int n_samples, const int* d_max, int n_mel, float* out, hipStream_t st) {
    mel_normalize_kernel<<<cdiv((long)n_mel * nl, 256 * 4), 256, 0, st>>>(d_mel, nl, n_samples, d_max, n_mel, out);
}

}  // namespace wm
