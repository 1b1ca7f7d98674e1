// Probe: does hipEventElapsedTime work on events recorded inside a captured hipGraph?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(float* x, int n) {
    float v = x[threadIdx.x];
    for (int i = 0; i < n; i++) v = v * 1.000001f + 0.5f;
    x[threadIdx.x] = v;
}
int main() {
    float* d;
    hipMalloc(&d, 1024 * 4);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t a, b, c2, d2;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventCreateWithFlags(&c2, 0); hipEventCreateWithFlags(&d2, 0);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    hipEventRecord(a, s);
    spin<<<1, 256, 0, s>>>(d, 1 << 20);
    hipEventRecord(b, s);
    hipStreamEndCapture(s, &g);
    hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    printf("instantiate %s\n", hipGetErrorString(e));
    for (int r = 0; r < 3; r++) {
        hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        float ms = -1;
        e = hipEventElapsedTime(&ms, a, b);
        printf("replay %d: elapsed err=%s ms=%f query a=%s b=%s\n", r, hipGetErrorString(e), ms,
               hipGetErrorString(hipEventQuery(a)), hipGetErrorString(hipEventQuery(b)));
    }
    // eager reference
    hipEventRecord(c2, s);
    spin<<<1, 256, 0, s>>>(d, 1 << 20);
    hipEventRecord(d2, s);
    hipStreamSynchronize(s);
    float ms = -1;
    e = hipEventElapsedTime(&ms, c2, d2);
    printf("eager: err=%s ms=%f\n", hipGetErrorString(e), ms);
    // graph with explicit event-record nodes
    hipGraph_t g2;
    hipGraphCreate(&g2, 0);
    hipGraphNode_t n1, n2, n3;
    hipGraphAddEventRecordNode(&n1, g2, nullptr, 0, c2);
    hipKernelNodeParams kp{};
    int iters = 1 << 20;
    void* args[] = {&d, &iters};
    kp.func = (void*)spin; kp.gridDim = dim3(1); kp.blockDim = dim3(256); kp.kernelParams = args;
    hipGraphAddKernelNode(&n2, g2, &n1, 1, &kp);
    hipGraphAddEventRecordNode(&n3, g2, &n2, 1, d2);
    hipGraphExec_t ge2;
    e = hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
    printf("instantiate2 %s\n", hipGetErrorString(e));
    hipGraphLaunch(ge2, s);
    hipStreamSynchronize(s);
    e = hipEventElapsedTime(&ms, c2, d2);
    printf("explicit nodes: err=%s ms=%f\n", hipGetErrorString(e), ms);
    return 0;
}
