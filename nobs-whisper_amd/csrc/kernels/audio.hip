// Audio front-end on the GPU: the reference app's voice-activity chunking
// and its 16 kHz resampler (src-tauri/src/audio.rs), over a batch of clips already in HBM.
//
// 1. Silence boundaries (audio.rs:364-467 calculate_rms / estimate_noise_floor /
//    find_silence_boundaries). rms_windows_kernel: RMS of every 20 ms window, each window summed
//    by ONE thread in sample order (Rust's f32 `.sum()` is a sequential fold) with separately
//    rounded products and adds (this file is compiled with -ffp-contract=off), so every RMS is
//    bit-identical to the reference's and the threshold comparisons, hence the integer
//    boundaries, are exact. A workgroup stages its windows through LDS with coalesced loads (row
//    stride ws + 1 floats: the per-thread serial reads then fall in distinct banks).
//    silence_scan_kernel: one lane per clip runs the noise-floor percentile (first 25 windows)
//    and the boundary state machine over that clip's RMS row (<= 1500 windows per 30 s).
//    HBM-bound: 4 B per sample read once, 4 B per window written/read.
// 2. Resampler (audio.rs:509-563 resample_audio = rubato 0.15.0 FftFixedIn, chunk 1024, 2
//    sub-chunks [ext]). FftFixedIn is an overlap-add FFT filter: input blocks of fsi samples are
//    zero-padded to 2*fsi, multiplied in frequency by a windowed-sinc low-pass, the spectrum is
//    truncated to fso bins and inverse-transformed at 2*fso points; output block m = first half of
//    block m's transform + second half of block m-1's. That map is linear in the 2*fsi samples
//    x[(m-1)*fsi, (m+1)*fsi), so the host folds the whole FFT pipeline into one [2*fsi][fso]
//    operator (engine side: audio.cpp) and resample_kernel applies it: out[m][j] =
//    sum_t x[(m-1)*fsi + t] * W[t][j], an LDS-tiled f32 VALU product over rows that overlap by
//    fsi samples (no im2col copy). 48 kHz -> 16 kHz: fsi 513, fso 171, 2*1026*171 = 351 kFLOP per
//    output block, ~1 GFLOP per 30 s clip: VALU-bound (f32 FMA; the reference's FFT is f32 too).
#include "../common.h"
#include "../kernels.h"

namespace wm {

static constexpr int RMS_THREADS = 256;

// rms[c][w] for w < n_samples[c] / ws; wpg windows per workgroup
__global__ void __launch_bounds__(RMS_THREADS)
rms_windows_kernel(const float* const* __restrict__ pcm, const int* __restrict__ n_samples, int ws, int wpg,
                   float* __restrict__ rms, int rms_stride) {
    extern __shared__ float s[];  // [wpg][ws + 1]
    const int c = blockIdx.y;
    const int n = n_samples[c];
    const int n_win = n / ws;
    const int w0 = blockIdx.x * wpg;
    if (w0 >= n_win) return;
    const int nw = min(wpg, n_win - w0);
    const float* x = pcm[c] + (long)w0 * ws;
    const int tot = nw * ws;
    for (int i = threadIdx.x; i < tot; i += RMS_THREADS) {
        const int w = i / ws, k = i - w * ws;
        s[w * (ws + 1) + k] = x[i];
    }
    __syncthreads();
    if (threadIdx.x < nw) {
        const float* r = s + threadIdx.x * (ws + 1);
        float acc = 0.0f;
        for (int k = 0; k < ws; k++) acc = __fadd_rn(acc, __fmul_rn(r[k], r[k]));
        // f32 division and square root, correctly rounded as the reference's: through double (whose
        // division and sqrt are correctly rounded here) and one rounding back; double rounding is
        // innocuous for / and sqrt since 53 >= 2 * 24 + 2
        const float q = (float)((double)acc / (double)ws);
        rms[(long)c * rms_stride + w0 + threadIdx.x] = (float)sqrt((double)q);
    }
}

// audio.rs constants (SILENCE_THRESHOLD 0.01 ... NOISE_FLOOR_PERCENTILE 0.1), products as the
// reference's f32 consts evaluate them
struct VadConsts {
    float min_noise_floor;   // SILENCE_THRESHOLD * MIN_NOISE_FLOOR_FACTOR
    float min_threshold;     // SILENCE_THRESHOLD * MIN_THRESHOLD_FACTOR
    float silence_threshold; // SILENCE_THRESHOLD
};

__global__ void silence_scan_kernel(const float* __restrict__ rms, int rms_stride, const int* __restrict__ n_samples,
                                    int n_clips, int sample_rate, VadConsts k, int* __restrict__ counts,
                                    int* __restrict__ bounds, int cap, float* __restrict__ floor_out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_clips) return;
    const int n = n_samples[c];
    const int ws = sample_rate / 50;
    const int n_win = n / ws;
    const float* r = rms + (long)c * rms_stride;
    // estimate_noise_floor (audio.rs:373-397): 10th percentile of the first 25 window RMS values
    float v[25];
    const int nv = min(25, n_win);
    for (int i = 0; i < nv; i++) {
        const float x = r[i];
        int j = i;
        while (j > 0 && v[j - 1] > x) { v[j] = v[j - 1]; j--; }  // stable ascending insertion
        v[j] = x;
    }
    float nf = k.silence_threshold;
    if (nv > 0) nf = v[(int)__fmul_rn((float)nv, 0.1f)];
    nf = fmaxf(nf, k.min_noise_floor);
    const float thr = fmaxf(__fmul_rn(nf, 3.0f), k.min_threshold);
    if (floor_out) floor_out[c] = nf;
    // find_silence_boundaries (audio.rs:400-467)
    const long min_sil = (long)((unsigned)sample_rate * 700u / 1000u);
    const long min_chunk = (long)((unsigned)sample_rate * 1000u / 1000u);
    long sil_start = -1, last = 0;
    int cnt = 0;
    auto try_add = [&](long s0, long s1) {
        const long dur = s1 - s0;
        if (dur >= min_sil) {
            const long split = s0 + dur / 2;
            if (split - last >= min_chunk) {
                if (cnt < cap) bounds[(long)c * cap + cnt] = (int)split;
                cnt++;
                last = split;
            }
        }
    };
    for (int w = 0; w < n_win; w++) {
        const long pos = (long)w * ws;
        if (r[w] < thr) {
            if (sil_start < 0) sil_start = pos;
        } else {
            if (sil_start >= 0) try_add(sil_start, pos);
            sil_start = -1;
        }
    }
    if (sil_start >= 0) try_add(sil_start, n);
    counts[c] = cnt;
}

void launch_silence_boundaries(const float* const* pcm, const int* n_samples, int n_clips, int max_n, int sample_rate,
                               float* rms, int rms_stride, int* counts, int* bounds, int cap, float* floor_out,
                               hipStream_t st) {
    if (n_clips <= 0) return;
    const int ws = sample_rate / 50;
    if (ws <= 0) WM_FAIL("sample rate %d too low for 20 ms windows", sample_rate);
    const int max_win = max_n / ws;
    if (max_win > rms_stride) WM_FAIL("rms row %d < %d windows", rms_stride, max_win);
    if (max_win > 0) {
        const int wpg = std::max(1, std::min(64, (int)((120 * 1024) / ((ws + 1) * 4))));
        const size_t lds = (size_t)wpg * (ws + 1) * 4;
        if (lds > 160 * 1024) WM_FAIL("20 ms window of %d samples too large", ws);
        rms_windows_kernel<<<dim3((max_win + wpg - 1) / wpg, n_clips), RMS_THREADS, lds, st>>>(pcm, n_samples, ws, wpg,
                                                                                             rms, rms_stride);
    }
    const VadConsts k{0.01f * 0.3f, 0.01f * 0.5f, 0.01f};
    silence_scan_kernel<<<(n_clips + 63) / 64, 64, 0, st>>>(rms, rms_stride, n_samples, n_clips, sample_rate, k, counts,
                                                            bounds, cap, floor_out);
}

// ---- resampler -----------------------------------------------------------------------------------
static constexpr int RS_BM = 64, RS_BN = 64, RS_BK = 16, RS_THREADS = 256;

// out[c][m*fso + j] = sum_{t < 2 fsi} x_c[(m-1)*fsi + t] * W[t][j]  (x_c = 0 outside [0, n_in[c]))
// for m*fso + j < n_out[c]. W: [2*fsi][ldw] f32. grid: (row tiles * col tiles, clips); each thread
// a 4 x 4 register tile, K staged through LDS 16 at a time.
__global__ void __launch_bounds__(RS_THREADS)
resample_kernel(const float* const* __restrict__ in, const int* __restrict__ n_in, const float* __restrict__ W, int ldw,
                int fsi, int fso, float* const* __restrict__ out, const int* __restrict__ n_out, int col_tiles) {
    __shared__ float sa[RS_BK][RS_BM + 4];
    __shared__ float sb[RS_BK][RS_BN];
    const int c = blockIdx.y;
    const int no = n_out[c];
    const int rt = blockIdx.x / col_tiles, ct = blockIdx.x - rt * col_tiles;
    const int m0 = rt * RS_BM, j0 = ct * RS_BN;
    if ((long)m0 * fso >= no) return;
    const float* x = in[c];
    const long n = n_in[c];
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    float acc[4][4] = {};
    const int K = 2 * fsi;
    for (int k0 = 0; k0 < K; k0 += RS_BK) {
        // A tile: 64 rows x 16 k; rows overlap by fsi samples, so each row is a contiguous slice
        for (int i = tid; i < RS_BM * RS_BK; i += RS_THREADS) {
            const int r = i / RS_BK, kk = i - r * RS_BK;
            const long idx = (long)(m0 + r - 1) * fsi + k0 + kk;
            sa[kk][r] = (k0 + kk < K && idx >= 0 && idx < n) ? x[idx] : 0.0f;
        }
        for (int i = tid; i < RS_BK * RS_BN; i += RS_THREADS) {
            const int kk = i / RS_BN, jj = i - kk * RS_BN;
            sb[kk][jj] = (k0 + kk < K) ? W[(long)(k0 + kk) * ldw + j0 + jj] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < RS_BK; kk++) {
            float a[4], b[4];
#pragma unroll
            for (int u = 0; u < 4; u++) { a[u] = sa[kk][tr * 4 + u]; b[u] = sb[kk][tc * 4 + u]; }
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int v = 0; v < 4; v++) acc[u][v] = __builtin_fmaf(a[u], b[v], acc[u][v]);
        }
        __syncthreads();
    }
    float* o = out[c];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int m = m0 + tr * 4 + u;
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int j = j0 + tc * 4 + v;
            const long p = (long)m * fso + j;
            if (j < fso && p < no) o[p] = acc[u][v];
        }
    }
}

void launch_resample(const float* const* in, const int* n_in, int n_clips, int max_out, const float* W, int ldw, int fsi,
                     int fso, float* const* out, const int* n_out, hipStream_t st) {
    if (n_clips <= 0 || max_out <= 0) return;
    if (ldw % RS_BN || ldw < fso) WM_FAIL("resampler operator stride %d", ldw);
    const int rows = (max_out + fso - 1) / fso;
    const int col_tiles = ldw / RS_BN;
    const int row_tiles = (rows + RS_BM - 1) / RS_BM;
    resample_kernel<<<dim3(row_tiles * col_tiles, n_clips), RS_THREADS, 0, st>>>(in, n_in, W, ldw, fsi, fso, out, n_out,
                                                                                col_tiles);
}

}  // namespace wm
