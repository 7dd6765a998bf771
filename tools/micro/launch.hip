// Launch-overhead probe: K dependent tiny kernels, stream launches vs one captured hipGraph.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void k_tiny(int* p, int k) { if (threadIdx.x == 0 && blockIdx.x == 0) p[k & 1023] += 1; }
int main() {
    int* d; CK(hipMalloc(&d, 4096)); CK(hipMemset(d, 0, 4096));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int K = 64;
    for (int blocks : {1, 2048}) {
        for (int rep = 0; rep < 3; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 20; ++it) for (int k = 0; k < K; ++k) k_tiny<<<blocks, 256, 0, s>>>(d, k);
            CK(hipStreamSynchronize(s));
            auto t1 = std::chrono::steady_clock::now();
            printf("stream blocks=%d: %.2f us/kernel\n", blocks, std::chrono::duration<double, std::micro>(t1 - t0).count() / (20 * K));
        }
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int k = 0; k < K; ++k) k_tiny<<<blocks, 256, 0, s>>>(d, k);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 20; ++it) CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            auto t1 = std::chrono::steady_clock::now();
            printf("graph  blocks=%d: %.2f us/kernel\n", blocks, std::chrono::duration<double, std::micro>(t1 - t0).count() / (20 * K));
        }
    }
    return 0;
}
