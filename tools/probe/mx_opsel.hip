// Probe (GPU box): does the opsel_a operand of v_mfma_scale_f32_16x16x128_f8f6f4 select the byte of the
// scale VGPR? A = B = 1.0 (e4m3), scale_a of lane l = (95 + l) placed in byte `sel`, other bytes 127:
// with byte selection C = 32 * sum over the row's 4 scale lanes of 2^(l - 32) for every sel.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int SEL>
__global__ void probe(float* out) {
    const int lane = threadIdx.x;
    i32x8 a, b;
    for (int i = 0; i < 8; i++) { a[i] = 0x38383838; b[i] = 0x38383838; }
    unsigned sc = 0x7F7F7F7Fu;
    sc &= ~(0xFFu << (8 * SEL));
    sc |= (unsigned)(95 + lane) << (8 * SEL);
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, SEL, (int)sc, 0, 127);
    for (int r = 0; r < 4; r++) out[((lane >> 4) * 4 + r) * 16 + (lane & 15)] = c[r];
}
int main() {
    float* d; float h[256];
    (void)hipMalloc(&d, 256 * 4);
    probe<0><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost); printf("sel0 row0 %g row5 %g\n", h[0], h[5 * 16]);
    probe<1><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost); printf("sel1 row0 %g row5 %g\n", h[0], h[5 * 16]);
    probe<2><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost); printf("sel2 row0 %g row5 %g\n", h[0], h[5 * 16]);
    probe<3><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost); printf("sel3 row0 %g row5 %g\n", h[0], h[5 * 16]);
    // expected with byte selection: row r = 32 * (2^(r-32) + 2^(r-16) + 2^r + 2^(r+16))
    printf("expect row0 %g row5 %g\n", 32.0 * (ldexp(1, -32) + ldexp(1, -16) + 1 + ldexp(1, 16)),
           32.0 * (ldexp(1, -27) + ldexp(1, -11) + ldexp(1, 5) + ldexp(1, 21)));
    return 0;
}
