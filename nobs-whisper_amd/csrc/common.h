// Shared definitions for the MI355X (gfx950) Whisper engine: error handling, element types,
// vector types for 16-byte loads and MFMA fragments.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace wm {

// Every failure of the engine (a HIP error such as out-of-memory, an unsupported shape) is thrown
// as wm::Error and turned into a non-zero return / NULL at the C ABI (capi.cpp), never abort():
// whisper-rs maps a non-zero whisper_full return to WhisperError (whisper.rs:127-129) and the app's
// streaming worker logs it and skips the chunk (state.rs:157-159).
struct Error : std::runtime_error {
    hipError_t hip;
    Error(const char* m, hipError_t h) : std::runtime_error(m), hip(h) {}
};
[[noreturn]] __attribute__((format(printf, 2, 3))) inline void fail_hip(hipError_t h, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fprintf(stderr, "whisper_mi355x: %s\n", buf);
    throw Error(buf, h);
}
#define WM_FAIL(...) ::wm::fail_hip(hipSuccess, __VA_ARGS__)

}  // namespace wm

#define WM_CHECK(x)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            (void)hipGetLastError(); /* clear a non-sticky error (out of memory) for the next call */ \
            ::wm::fail_hip(e_, "HIP error %s at %s:%d: %s", hipGetErrorName(e_), __FILE__, __LINE__, #x); \
        }                                                                                             \
    } while (0)

namespace wm {

// Compute element type of the weights and the GEMM-side activations.
//  F16  — the GGML file's own weight type; reproduces ggml's f16 roundings (parity mode).
//  BF16 — weights rounded f16->bf16 at load; same MFMA rate, wider exponent.
enum class DType : int { F16 = 0, BF16 = 1 };

typedef _Float16 half_t;
typedef __bf16 bf16_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct Frag;
template <> struct Frag<half_t> { typedef half8 type; };
template <> struct Frag<bf16_t> { typedef bfx8 type; };

__device__ __forceinline__ f32x4 mfma16x16x32(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x32(bfx8 a, bfx8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32x32x16(half8 a, half8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x32x16(bfx8 a, bfx8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ T to_t(float x) { return (T)x; }
template <typename T> __device__ __forceinline__ float from_t(T x) { return (float)x; }

// Block-wide (256-thread) LayerNorm of one row held in registers: thread t owns columns
// t + 256*k. ggml_norm arithmetic: double sums, float mean/variance, 1/sqrtf(var + 1e-5), then
// (v*scale)*w + b with every op separately rounded (explicit _rn intrinsics: no FMA contraction
// whatever the file's -ffp-contract). `sh` is >= 4 doubles of LDS.
__device__ __forceinline__ double block256_sum_d(double x, double* sh) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = x;
    __syncthreads();
    const double r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return r;
}
template <typename T, int NPT>
__device__ __forceinline__ void block256_layernorm(float (&v)[NPT], int D, const float* __restrict__ w,
                                                   const float* __restrict__ b, T* __restrict__ y, double* sh) {
#pragma clang fp contract(off)  // (v*scale)*w + b separately rounded, as ggml_norm (the __f*_rn forms alone get fused)
    const int tid = threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; k++)
        if (tid + 256 * k < D) s += (double)v[k];
    s = block256_sum_d(s, sh);
    const float mean = (float)(s / D);
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; k++)
        if (tid + 256 * k < D) {
            v[k] = __fsub_rn(v[k], mean);
            s2 += (double)__fmul_rn(v[k], v[k]);
        }
    s2 = block256_sum_d(s2, sh);
    const float variance = (float)(s2 / D);
    const float scale = 1.0f / sqrtf(variance + 1e-5f);
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int n = tid + 256 * k;
        if (n < D) y[n] = (T)((v[k] * scale) * w[n] + b[n]);  // plain ops: the pragma applies
    }
}

// host-side conversions (weights are converted once at load)
static inline float h2f(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f, mant = h & 0x3ffu, x;
    if (exp == 0) {
        if (mant == 0) x = sign;
        else {
            int e = -1;
            do { e++; mant <<= 1; } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 0x1f) x = sign | 0x7f800000u | (mant << 13);
    else x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    float f;
    __builtin_memcpy(&f, &x, 4);
    return f;
}
static inline uint16_t f2bf(float f) {  // round-to-nearest-even, NaN kept NaN
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace wm
