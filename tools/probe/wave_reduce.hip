// Probe: the lane maps of the DPP controls the persistent step's reductions use (kernels/pdec_body.h),
// and of the gfx950 permlane swaps (which, called as below, did NOT return lane ^ 16 / lane ^ 32 values:
// the reductions read the row sums as scalars instead). Run on the GPU box; prints one line per control.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__device__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__global__ void k(const float* in, float* out) {
    const int l = threadIdx.x;
    float x = in[l];
    out[0 * 64 + l] = dppf<0xB1>(x);
    out[1 * 64 + l] = dppf<0x4E>(x);
    out[2 * 64 + l] = dppf<0x141>(x);
    out[3 * 64 + l] = dppf<0x140>(x);
    out[4 * 64 + l] = dppf<0x128>(x);
    // wave sum as the persistent step does it: row sums by DPP, row_bcast:15 / :31 into lane 63
    float w = x;
    w += dppf<0xB1>(w); w += dppf<0x4E>(w); w += dppf<0x141>(w); w += dppf<0x140>(w);
    w += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, w), 0x142, 0xA, 0xF, false));
    w += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, w), 0x143, 0xC, 0xF, false));
    out[9 * 64 + l] = w;
    unsigned y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(__builtin_bit_cast(unsigned, x)));
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), y, false, false);
    out[5 * 64 + l] = __builtin_bit_cast(float, r[0]);
    out[6 * 64 + l] = __builtin_bit_cast(float, r[1]);
    const auto q = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), y, false, false);
    out[7 * 64 + l] = __builtin_bit_cast(float, q[0]);
    out[8 * 64 + l] = __builtin_bit_cast(float, q[1]);
}
int main() {
    float h[64], o[10 * 64];
    for (int i = 0; i < 64; i++) h[i] = (float)i;
    float *din, *dout;
    hipMalloc(&din, 256); hipMalloc(&dout, sizeof(o));
    hipMemcpy(din, h, 256, hipMemcpyHostToDevice);
    k<<<1, 64>>>(din, dout);
    hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    const char* names[10] = {"quad xor1 0xB1", "quad xor2 0x4E", "half mirror 0x141", "row mirror 0x140", "row ror8 0x128",
                             "pl16 r0", "pl16 r1", "pl32 r0", "pl32 r1", "wave sum (l63=2016)"};
    for (int t = 0; t < 10; t++) {
        printf("%-18s", names[t]);
        for (int i = 0; i < 64; i++) printf(" %d", (int)o[t * 64 + i]);
        printf("\n");
    }
    return 0;
}
