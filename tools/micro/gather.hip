// FETCH_SIZE calibration for the access widths of the CD decide kernel:
// known byte counts, one kernel per pattern, each its own launch so a --pmc pass attributes
// counters per pattern.
//   k_stream16 : 16 B/lane coalesced streaming read of S bytes (the guide's calibrated case)
//   k_gather4  : G random 4-B gathers (one dword per lane, random index) over a table of T bytes
//   k_scatter4 : G random 4-B stores over a table of T bytes
//   k_gather4s : G random 4-B gathers, the 64 lanes of a wave inside one 256-B window
//                (the in-community half of a pull sweep after the storage ordering)
// Tables: 1 GiB (misses L2 and the 256 MiB Infinity Cache), 64 MiB (misses L2, resident in
// the Infinity Cache), 4 MiB (one XCD's L2).  Prints ns/launch and bytes; run it under
// `rocprofv3 --pmc FETCH_SIZE` (and TCC_EA0_RDREQ_sum / TCC_MISS_sum) to read the counters.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_stream16(const int4* __restrict__ p, int64_t n16, int* out) {
    int4 acc = make_int4(0, 0, 0, 0);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const int4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x7fffffff) out[0] = 1;   // keeps the loads
}

// 8 independent gathers per thread (the decide kernel keeps 4-8 in flight per lane)
__global__ void k_gather4(const int* __restrict__ t, uint32_t mask, int64_t g8, uint32_t salt, int* out) {
    int acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g8; i += (int64_t)gridDim.x * blockDim.x) {
        int v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = t[mix((uint32_t)(i * 8 + u) ^ salt) & mask];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
    if (acc == 0x7fffffff) out[0] = 1;
}

// a wave's 64 lanes gather inside one random 256-B window (64 dwords): 2 lines per wave load
__global__ void k_gather4s(const int* __restrict__ t, uint32_t mask, int64_t g8, uint32_t salt, int* out) {
    int acc = 0;
    const int lane = threadIdx.x & 63;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g8; i += (int64_t)gridDim.x * blockDim.x) {
        int v[8];
        const int64_t wv = i >> 6;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t base = (mix((uint32_t)(wv * 8 + u) ^ salt) & mask) & ~63u;
            v[u] = t[base + (mix(lane * 131 + u) & 63)];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
    if (acc == 0x7fffffff) out[0] = 1;
}

// G random 4-B stores (the push of a move into its neighbours' nlab entries)
__global__ void k_scatter4(int* __restrict__ t, uint32_t mask, int64_t g8, uint32_t salt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g8; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int u = 0; u < 8; ++u) t[mix((uint32_t)(i * 8 + u) ^ salt) & mask] = (int)i;
    }
}

int main() {
    const int64_t BIG = 1ll << 30;
    int* tab;
    int* out;
    CK(hipMalloc(&tab, BIG));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(tab, 1, BIG));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 256 * 8 * 4, tb = 256;
    auto timeit = [&](const char* name, double bytes_known, double gathers, auto launch) -> int {
        launch();   // warm
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %9.1f us  known_bytes %12.0f  gathers %12.0f  -> %7.1f GB/s known, %7.2f Ggather/s\n", name,
               1e3 * ms, bytes_known, gathers, bytes_known / (ms * 1e6), gathers / (ms * 1e6));
        return 0;
    };
    // streaming: 1 GiB
    if (timeit("stream16 1GiB", (double)BIG, 0, [&] { k_stream16<<<grid, tb>>>((const int4*)tab, BIG / 16, out); })) return 1;
    const int64_t G = 1ll << 26;   // 64M gathers (256 MB of dwords)
    struct T { const char* name; int64_t bytes; };
    T tabs[] = {{"gather4 1GiB", 1ll << 30}, {"gather4 64MiB", 64ll << 20}, {"gather4 4MiB", 4ll << 20}};
    for (auto& tt : tabs) {
        const uint32_t mask = (uint32_t)(tt.bytes / 4 - 1);
        if (timeit(tt.name, 4.0 * G, (double)G, [&] { k_gather4<<<grid, tb>>>(tab, mask, G / 8, 0x9e3779b9u, out); })) return 1;
    }
    T stabs[] = {{"gather4s(256B win) 1GiB", 1ll << 30}, {"gather4s(256B win) 64MiB", 64ll << 20}};
    for (auto& tt : stabs) {
        const uint32_t mask = (uint32_t)(tt.bytes / 4 - 1);
        if (timeit(tt.name, 4.0 * G, (double)G, [&] { k_gather4s<<<grid, tb>>>(tab, mask, G / 8, 0x85ebca6bu, out); })) return 1;
    }
    T wtabs[] = {{"scatter4 1GiB", 1ll << 30}, {"scatter4 64MiB", 64ll << 20}, {"scatter4 4MiB", 4ll << 20}};
    for (auto& tt : wtabs) {
        const uint32_t mask = (uint32_t)(tt.bytes / 4 - 1);
        if (timeit(tt.name, 4.0 * G, (double)G, [&] { k_scatter4<<<grid, tb>>>(tab, mask, G / 8, 0x27d4eb2fu); })) return 1;
    }
    CK(hipFree(tab));
    CK(hipFree(out));
    return 0;
}
