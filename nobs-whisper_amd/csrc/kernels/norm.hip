// LayerNorm (ggml_norm + ggml_mul + ggml_add) and decoder token/position embedding.
//
// LayerNorm follows ggml-cpu's arithmetic: mean and variance sums in double, mean/variance
// rounded to float, scale = 1/sqrtf(var + 1e-5), then (v*scale)*w + b as three separately rounded
// float ops (this file is compiled with -ffp-contract=off). Output is rounded to the GEMM input
// type, which is exactly the f16 conversion ggml applies to a matmul's src1.
// Roofline: HBM-bound, 4 B read + 2 B written per element; one wave per row.
#include "../common.h"
#include "../kernels.h"

namespace wm {

// One wave per row; the row is loaded into registers once (NPL = ceil(D/64) floats per lane, all
// loads issued before the first use) and reduced from registers.
template <typename T, int NPL>
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, const int* __restrict__ rows, int M, int D,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        T* __restrict__ y) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= M) return;
    const long r = rows ? rows[i] : i;
    const float* xr = x + r * D;
    float v[NPL];
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        v[e] = k < D ? xr[k] : 0.0f;
    }
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < NPL; e++) s += (double)v[e];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = (float)(s / D);
    double s2 = 0.0;
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        v[e] = v[e] - mean;
        if (k < D) s2 += (double)(v[e] * v[e]);
    }
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const float variance = (float)(s2 / D);
    const float scale = 1.0f / sqrtf(variance + 1e-5f);
    T* yr = y + (long)i * D;
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        if (k < D) {
            float t = v[e] * scale;
            t = t * w[k];
            yr[k] = (T)(t + b[k]);
        }
    }
}

// LayerNorm with the output quantized to fp8 e4m3 (OCP) per row for the fp8 encoder GEMMs:
// t = LN(x) * w + b in f32 (as layernorm_kernel, without the rounding to the MFMA type), then
// s[i] = max|t| / 448, q[i][k] = e4m3(t[k] / s[i]). One wave per row.
template <int NPL>
__global__ void __launch_bounds__(256) layernorm_fp8_kernel(const float* __restrict__ x, int M, int D,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            uint8_t* __restrict__ q, float* __restrict__ s) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= M) return;
    const float* xr = x + (long)i * D;
    float v[NPL];
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        v[e] = k < D ? xr[k] : 0.0f;
    }
    double s1 = 0.0;
#pragma unroll
    for (int e = 0; e < NPL; e++) s1 += (double)v[e];
    for (int o = 32; o > 0; o >>= 1) s1 += __shfl_xor(s1, o);
    const float mean = (float)(s1 / D);
    double s2 = 0.0;
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        v[e] = v[e] - mean;
        if (k < D) s2 += (double)(v[e] * v[e]);
    }
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const float variance = (float)(s2 / D);
    const float scale = 1.0f / sqrtf(variance + 1e-5f);
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        if (k < D) {
            v[e] = (v[e] * scale) * w[k] + b[k];
            amax = fmaxf(amax, fabsf(v[e]));
        }
    }
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float sc = amax > 0.f ? amax / 448.f : 1.f, inv = 1.f / sc;
    if (lane == 0) s[i] = sc;
    uint8_t* qr = q + (long)i * D;
#pragma unroll
    for (int e = 0; e < NPL; e++) {
        const int k = lane + 64 * e;
        if (k < D) {
            const float t = fminf(fmaxf(v[e] * inv, -448.f), 448.f);
            qr[k] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(t, t, 0, false) & 0xff);
        }
    }
}

// the same with 4 consecutive columns per lane (D % 256 == 0): 16-byte row reads, 4-byte
// coalesced fp8 stores (the strided form above stores single bytes)
template <int NV>
__global__ void __launch_bounds__(256) layernorm_fp8_v4_kernel(const float* __restrict__ x, int M, int D,
                                                               const float* __restrict__ w, const float* __restrict__ b,
                                                               uint8_t* __restrict__ q, float* __restrict__ s) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= M) return;
    const float4* xr = (const float4*)(x + (long)i * D);
    float4 v[NV];
    double s1 = 0.0;
#pragma unroll
    for (int e = 0; e < NV; e++) {
        v[e] = xr[lane + 64 * e];
        s1 += (double)v[e].x + (double)v[e].y + (double)v[e].z + (double)v[e].w;
    }
    for (int o = 32; o > 0; o >>= 1) s1 += __shfl_xor(s1, o);
    const float mean = (float)(s1 / D);
    double s2 = 0.0;
#pragma unroll
    for (int e = 0; e < NV; e++) {
        v[e].x -= mean; v[e].y -= mean; v[e].z -= mean; v[e].w -= mean;
        s2 += (double)(v[e].x * v[e].x) + (double)(v[e].y * v[e].y) + (double)(v[e].z * v[e].z) + (double)(v[e].w * v[e].w);
    }
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const float scale = 1.0f / sqrtf((float)(s2 / D) + 1e-5f);
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < NV; e++) {
        const int k = 4 * (lane + 64 * e);
        const float4 ww = *(const float4*)(w + k), bb = *(const float4*)(b + k);
        v[e].x = (v[e].x * scale) * ww.x + bb.x; v[e].y = (v[e].y * scale) * ww.y + bb.y;
        v[e].z = (v[e].z * scale) * ww.z + bb.z; v[e].w = (v[e].w * scale) * ww.w + bb.w;
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[e].x), fabsf(v[e].y)), fmaxf(fabsf(v[e].z), fabsf(v[e].w))));
    }
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float sc = amax > 0.f ? amax / 448.f : 1.f, inv = 1.f / sc;
    if (lane == 0) s[i] = sc;
    uint32_t* qr = (uint32_t*)(q + (long)i * D);
    auto c = [&](float t) { return fminf(fmaxf(t * inv, -448.f), 448.f); };
#pragma unroll
    for (int e = 0; e < NV; e++) {
        uint32_t u = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[e].x), c(v[e].y), 0, false);
        u = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[e].z), c(v[e].w), u, true);
        qr[lane + 64 * e] = u;
    }
}

void launch_layernorm_fp8(const float* x, int M, int D, const float* w, const float* b, void* q, float* s,
                          hipStream_t st) {
    if (M <= 0) return;
    if (D % 256 == 0 && D <= 2048) {
#define WM_LN8V(N)                                                                                          \
        if (D == 256 * N) {                                                                                 \
            layernorm_fp8_v4_kernel<N><<<cdiv(M, 4), 256, 0, st>>>(x, M, D, w, b, (uint8_t*)q, s);         \
            return;                                                                                         \
        }
        WM_LN8V(2) WM_LN8V(3) WM_LN8V(4) WM_LN8V(5) WM_LN8V(6) WM_LN8V(8)
#undef WM_LN8V
    }
#define WM_LN8(N)                                                                                           \
    if (D <= 64 * N) {                                                                                      \
        layernorm_fp8_kernel<N><<<cdiv(M, 4), 256, 0, st>>>(x, M, D, w, b, (uint8_t*)q, s);                 \
        return;                                                                                             \
    }
    WM_LN8(6) WM_LN8(8) WM_LN8(12) WM_LN8(16) WM_LN8(20) WM_LN8(24) WM_LN8(32)
#undef WM_LN8
    WM_FAIL("layernorm width %d > 2048", D);
}

// TE: the token-embedding table's type: the MFMA type, or f32 for a quantized GGML embedding that
// ggml_get_rows dequantizes to f32 (exact q*d (+m)) while the logits matmul sees it rounded to f16
template <typename TE>
__global__ void embed_kernel(const TE* __restrict__ te, const float* __restrict__ pe, const int* __restrict__ tok,
                             const int* __restrict__ pos, int D, float* __restrict__ x) {
    const int i = blockIdx.x;
    const long t = tok[i], p = pos[i];
    for (int k = threadIdx.x; k < D; k += blockDim.x) x[(long)i * D + k] = (float)te[t * D + k] + pe[p * D + k];
}

// decoder token + position embedding fused with the first layer's LayerNorm (one block per token)
template <typename T, int NPT, typename TE>
__global__ void __launch_bounds__(256) embed_ln_kernel(const TE* __restrict__ te, const float* __restrict__ pe,
                                                       const int* __restrict__ tok, const int* __restrict__ pos, int D,
                                                       float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ b, T* __restrict__ y) {
    __shared__ double sh[4];
    const int i = blockIdx.x;
    const long t = tok[i], p = pos[i];
    float v[NPT];
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int n = threadIdx.x + 256 * k;
        v[k] = 0.0f;
        if (n < D) {
            v[k] = (float)te[t * D + n] + pe[p * D + n];
            x[(long)i * D + n] = v[k];
        }
    }
    block256_layernorm<T, NPT>(v, D, w, b, y + (long)i * D, sh);
}

void launch_embed_ln(DType dt, const void* te, bool te_f32, const float* pe, const int* tok, const int* pos, int n, int D,
                     float* x, const float* w, const float* b, void* y, hipStream_t st) {
    if (n <= 0) return;
    if (D > 2048) WM_FAIL("embed LN width %d > 2048", D);
#define WM_ELN(T, NPT)                                                                                                    \
    if (te_f32) embed_ln_kernel<T, NPT, float><<<n, 256, 0, st>>>((const float*)te, pe, tok, pos, D, x, w, b, (T*)y);       \
    else embed_ln_kernel<T, NPT, T><<<n, 256, 0, st>>>((const T*)te, pe, tok, pos, D, x, w, b, (T*)y)
    if (D <= 1024) {
        if (dt == DType::F16) { WM_ELN(half_t, 4); } else { WM_ELN(bf16_t, 4); }
    } else {
        if (dt == DType::F16) { WM_ELN(half_t, 8); } else { WM_ELN(bf16_t, 8); }
    }
#undef WM_ELN
}

void launch_layernorm(DType dt, const float* x, const int* rows, int M, int D, const float* w, const float* b, void* y,
                      hipStream_t st) {
    if (M <= 0) return;
    const int npl = cdiv(D, 64);
#define WM_LN(N)                                                                                              \
    if (npl <= N) {                                                                                           \
        if (dt == DType::F16) layernorm_kernel<half_t, N><<<cdiv(M, 4), 256, 0, st>>>(x, rows, M, D, w, b, (half_t*)y); \
        else layernorm_kernel<bf16_t, N><<<cdiv(M, 4), 256, 0, st>>>(x, rows, M, D, w, b, (bf16_t*)y);     \
        return;                                                                                               \
    }
    WM_LN(1) WM_LN(2) WM_LN(4) WM_LN(6) WM_LN(8) WM_LN(12) WM_LN(16) WM_LN(20) WM_LN(24) WM_LN(32)
#undef WM_LN
    WM_FAIL("layernorm width %d > 2048", D);
}

void launch_embed(DType dt, const void* te, bool te_f32, const float* pe, const int* tok, const int* pos, int n, int D,
                  float* x, hipStream_t st) {
    if (n <= 0) return;
    if (te_f32) embed_kernel<float><<<n, 256, 0, st>>>((const float*)te, pe, tok, pos, D, x);
    else if (dt == DType::F16) embed_kernel<half_t><<<n, 256, 0, st>>>((const half_t*)te, pe, tok, pos, D, x);
    else embed_kernel<bf16_t><<<n, 256, 0, st>>>((const bf16_t*)te, pe, tok, pos, D, x);
}

}  // namespace wm
