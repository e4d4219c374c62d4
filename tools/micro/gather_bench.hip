// Random 4-B gather throughput vs table size (L2-, MALL-, HBM-resident): the ceiling for the
// index probe. Each thread gathers G independent random entries (all loads in flight), XORs them
// and writes one word. usage: gather_bench [G]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int G>
__global__ void gather(const uint32_t* __restrict__ tab, uint64_t mask, uint32_t* __restrict__ out, uint64_t n, uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t x = (uint32_t)t * 2654435761u ^ seed;
    uint32_t v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint64_t idx = ((uint64_t)x * 0x9E3779B97F4A7C15ull >> 20) & mask;
        v[g] = tab[idx];
    }
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) a ^= v[g];
    out[t] = a;
}

int main() {
    const uint64_t n = 10'000'000;  // threads (reads); 6 gathers each = 60M
    uint32_t* out;
    CK(hipMalloc(&out, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint64_t mb : {2ull, 8ull, 32ull, 64ull, 128ull, 256ull, 512ull, 1024ull}) {
        const uint64_t words = mb << 18;  // power of two
        uint32_t* tab;
        CK(hipMalloc(&tab, words * 4));
        CK(hipMemset(tab, 1, words * 4));
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(gather<6>, dim3((n + 255) / 256), dim3(256), 0, 0, tab, words - 1, out, n, 77u + rep);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) best = ms < best ? ms : best;
        }
        printf("table %5llu MiB: %.3f ms for %llu gathers -> %.1f G gathers/s\n", (unsigned long long)mb, best,
               (unsigned long long)(n * 6), n * 6 / (best * 1e-3) / 1e9);
        CK(hipFree(tab));
    }
    return 0;
}
