// Probe (GPU box): which A-operand scale lane multiplies each (lane, byte) of the A operand of
// v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3). For every (lane L, byte P): A = 1.0 at that byte only,
// B = 1.0 everywhere, scale_a of lane l = 2^(l - 32) (E8M0 95 + l), scale_b = 1: C[row][col] = 2^(lam - 32)
// in the row the byte belongs to, lam = the scale lane. Prints "L P row lam" lines.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
    const int lane = threadIdx.x;
    for (int L = 0; L < 64; L++)
        for (int P = 0; P < 32; P++) {
            i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b;
            for (int i = 0; i < 8; i++) b[i] = 0x38383838;
            if (lane == L) a[P >> 2] = 0x38 << (8 * (P & 3));
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
            c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 95 + lane, 0, 127);
            for (int r = 0; r < 4; r++) {
                const int row = (lane >> 4) * 4 + r, col = lane & 15;
                out[((L * 32 + P) * 16 + row) * 16 + col] = c[r];
            }
        }
}

int main() {
    float* d;
    const size_t n = 64 * 32 * 256;
    hipMalloc(&d, n * 4);
    probe<<<1, 64>>>(d);
    float* h = new float[n];
    hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    for (int L = 0; L < 64; L++)
        for (int P = 0; P < 32; P++) {
            int nz = 0, row = -1;
            float v = 0;
            for (int r = 0; r < 16; r++)
                for (int c = 0; c < 16; c++) {
                    const float x = h[((L * 32 + P) * 16 + r) * 16 + c];
                    if (x != 0.f) { nz++; row = r; v = x; }
                }
            printf("%d %d row=%d nz=%d lam=%g\n", L, P, row, nz, v != 0.f ? log2f(v) + 32 : -1.0f);
        }
    return 0;
}
