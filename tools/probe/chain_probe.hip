// Probe: what one kernel of the decode chain costs inside a replayed hipGraph, by component.
// A graph holds a chain of NK dependent launches of one kernel kind; per-kernel time = replay time / NK.
// Kinds (grid / block as the decode-step GEMM at M = 128, N = K = 1280: 200 workgroups x 256 threads):
//   empty        : returns at once
//   empty_lds96  : returns at once, 96 KiB static LDS (one workgroup per CU)
//   dma48        : 48 KiB per workgroup by LDS-DMA (16-byte pieces), counted wait, no store
//   reg48        : 48 KiB per workgroup by global_load_dwordx4 into registers, no store
//   st32         : 32 KiB f32 per workgroup, plain 16-byte stores
//   st32wt       : the same, write-through (sc1)
//   dma48_st32   : dma48 then st32 (the split-K GEMM minus its MFMAs)
//   dma48_st32wt : dma48 then st32wt
//   red128       : the split-K reduce shape: 128 workgroups x 320 threads, each reads 10 x 5 KiB
//                  of f32 slabs and writes 5 KiB
//   gemv80       : 80 workgroups x 512 threads, 40 KiB of weights per workgroup into registers +
//                  16 x 1280 activations, 16 x 16 f32 outputs (the small-M GEMM's memory shape)
// Build: hipcc -O3 --offload-arch=gfx950 -o chain_probe chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct Args {
    const char* src;  // read buffer (hot: 64 MiB, rotated per launch)
    float* dst;       // write buffer
    long rot;         // byte offset of this launch's slice
};

__global__ void k_empty(Args) {}
__global__ void __launch_bounds__(256) k_empty_lds(Args a) {
    __shared__ u32x4 lds[96 * 64];
    if (a.rot < 0) lds[threadIdx.x] = (u32x4){1, 2, 3, 4};
    __syncthreads();
    if (a.rot < 0) a.dst[0] = (float)lds[threadIdx.x + 1].x;
}

template <bool STORE, bool WT, bool LOAD>
__global__ void __launch_bounds__(256) k_gemmlike(Args a) {
    __shared__ u32x4 lds[3 * 1024];  // 48 KiB
    const int tid = threadIdx.x, wave = tid >> 6;
    if (LOAD) {
        const char* src = a.src + a.rot + (long)blockIdx.x * 48 * 1024;
#pragma unroll
        for (int i = 0; i < 12; i++)
            __builtin_amdgcn_global_load_lds((const void*)(src + (long)(i * 256 + tid) * 16), (lds_ptr_t)&lds[i * 256 + wave * 64], 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (STORE) {
        float* o = a.dst + (long)blockIdx.x * 8 * 1024;
        const f32x4 v = LOAD ? __builtin_bit_cast(f32x4, lds[tid]) : (f32x4){1.f, 2.f, 3.f, 4.f};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            float* p = o + (i * 256 + tid) * 4;
            if (WT) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            else *(f32x4*)p = v;
        }
    } else if (LOAD) {
        if (a.rot < 0) a.dst[tid] = (float)lds[tid].x;
    }
}


// the decode GEMM's slab store pattern: acc[4][2] f32x4 of 16x16 MFMA tiles (lane holds rows
// 4*(lane>>4)+r of column lane&15), stored element by element into a [M=128][N=1280] f32 slab
template <bool WT, bool LOAD>
__global__ void __launch_bounds__(256) k_fragstore(Args a) {
    __shared__ u32x4 lds[3 * 1024];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    float val = 1.0f;
    if (LOAD) {
        const char* src = a.src + a.rot + (long)blockIdx.x * 48 * 1024;
#pragma unroll
        for (int i = 0; i < 12; i++)
            __builtin_amdgcn_global_load_lds((const void*)(src + (long)(i * 256 + tid) * 16), (lds_ptr_t)&lds[i * 256 + wave * 64], 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        val = (float)lds[tid].x;
    }
    const int n0 = (blockIdx.x % 20) * 64;
    float* slab = a.dst + (long)(blockIdx.x / 20) * 128 * 1280;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int n = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
                float* p = slab + (long)m * 1280 + n;
                if (WT) __hip_atomic_store(p, val + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else *p = val + r;
            }
        }
}

__global__ void __launch_bounds__(256) k_reg48(Args a) {
    const char* src = a.src + a.rot + (long)blockIdx.x * 48 * 1024;
    u32x4 r[12];
#pragma unroll
    for (int i = 0; i < 12; i++) r[i] = *(const u32x4*)(src + (long)(i * 256 + threadIdx.x) * 16);
    u32x4 x = r[0];
#pragma unroll
    for (int i = 1; i < 12; i++) x ^= r[i];
    if (x.x == 0x12345679u && a.rot < 0) a.dst[threadIdx.x] = 1.0f;
}

// split-K reduce shape: row m (one workgroup), 10 slabs of [128][1280] f32, 320 threads x float4
__global__ void __launch_bounds__(320) k_red(Args a) {
    const float* s = (const float*)(a.src + a.rot) + (long)blockIdx.x * 1280 + threadIdx.x * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < 10; z++) acc += *(const f32x4*)(s + (long)z * 128 * 1280);
    *(f32x4*)(a.dst + (long)blockIdx.x * 1280 + threadIdx.x * 4) = acc;
}

// small-M GEMM memory shape: 80 workgroups x 512 threads; per wave 5 x 16 B of weights and of
// activations per lane (in flight together), then a 16 x 16 output
__global__ void __launch_bounds__(512) k_gemv(Args a) {
    const int tid = threadIdx.x;
    const char* w = a.src + a.rot + (long)blockIdx.x * 40 * 1024;
    const char* x = a.src + (long)(tid & 63) * 16;  // activations: shared by every workgroup
    u32x4 r[10];
#pragma unroll
    for (int i = 0; i < 5; i++) r[i] = *(const u32x4*)(w + (long)(i * 512 + tid) * 16);
#pragma unroll
    for (int i = 0; i < 5; i++) r[5 + i] = *(const u32x4*)(x + (long)i * 8192);
    u32x4 v = r[0];
#pragma unroll
    for (int i = 1; i < 10; i++) v ^= r[i];
    __shared__ float red[512];
    red[tid] = (float)v.x;
    __syncthreads();
    if (tid < 256) a.dst[blockIdx.x * 256 + tid] = red[tid] + red[tid + 256];
}

int main(int argc, char** argv) {
    const int NK = argc > 1 ? atoi(argv[1]) : 200;
    const int REP = 20;
    char* src;
    float* dst;
    const long SRC = 512L << 20;  // rotate through 512 MiB so each launch reads cold-ish lines
    CK(hipMalloc(&src, SRC));
    CK(hipMalloc(&dst, 64L << 20));
    CK(hipMemset(src, 1, SRC));
    CK(hipMemset(dst, 0, 64L << 20));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Kind { const char* name; int grid, block; long bytes_per_launch; void (*launch)(int, int, Args, hipStream_t); };
    std::vector<Kind> kinds = {
        {"empty", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_empty<<<g, b, 0, s>>>(a); }},
        {"empty_lds96", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_empty_lds<<<g, b, 0, s>>>(a); }},
        {"dma48", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_gemmlike<false, false, true><<<g, b, 0, s>>>(a); }},
        {"reg48", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_reg48<<<g, b, 0, s>>>(a); }},
        {"st32", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_gemmlike<true, false, false><<<g, b, 0, s>>>(a); }},
        {"st32wt", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_gemmlike<true, true, false><<<g, b, 0, s>>>(a); }},
        {"dma48_st32", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_gemmlike<true, false, true><<<g, b, 0, s>>>(a); }},
        {"dma48_st32wt", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_gemmlike<true, true, true><<<g, b, 0, s>>>(a); }},
        {"frag32", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_fragstore<false, false><<<g, b, 0, s>>>(a); }},
        {"frag32wt", 200, 256, 0, [](int g, int b, Args a, hipStream_t s) { k_fragstore<true, false><<<g, b, 0, s>>>(a); }},
        {"dma48_frag32wt", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_fragstore<true, true><<<g, b, 0, s>>>(a); }},
        {"dma48_frag32", 200, 256, 200L * 48 * 1024, [](int g, int b, Args a, hipStream_t s) { k_fragstore<false, true><<<g, b, 0, s>>>(a); }},
        {"red128", 128, 320, 10L * 128 * 1280 * 4, [](int g, int b, Args a, hipStream_t s) { k_red<<<g, b, 0, s>>>(a); }},
        {"gemv80", 80, 512, 80L * 40 * 1024, [](int g, int b, Args a, hipStream_t s) { k_gemv<<<g, b, 0, s>>>(a); }},
    };
    for (const Kind& k : kinds) {
        for (int hot = 0; hot < 2; hot++) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            long off = 0;
            for (int i = 0; i < NK; i++) {
                Args a{src, dst, hot ? 0 : off};
                k.launch(k.grid, k.block, a, st);
                off += (k.bytes_per_launch + 4095) / 4096 * 4096;
                if (off + k.bytes_per_launch > SRC) off = 0;
            }
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, st));
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < REP; r++) CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / REP / NK;
            printf("%-14s grid %4d x %3d  %s  %6.2f us per kernel  (%.0f GB/s)\n", k.name, k.grid, k.block,
                   hot ? "hot " : "cold", us, k.bytes_per_launch / us / 1e3);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    return 0;
}
