// Random gather throughput vs table size (L2-, MALL-, HBM-resident) and entry width: the ceiling
// for the index probe. Each thread gathers G independent random entries (all loads in flight),
// XORs them and writes one word. Entry widths: 4 B (one dword) or W x 16 B (W uint4 loads of one
// aligned entry). usage: gather_bench [max_table_MiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t next_idx(uint32_t& x) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return x;
}

// W = 0: 4-B entries; W > 0: entries of W uint4
template <int G, int W>
__global__ void gather(const uint32_t* __restrict__ tab, uint64_t mask, uint32_t* __restrict__ out, uint64_t n, uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t x = (uint32_t)t * 2654435761u ^ seed;
    uint32_t a = 0;
    if (W == 0) {
        uint32_t v[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint64_t idx = ((uint64_t)next_idx(x) * 0x9E3779B97F4A7C15ull >> 20) & mask;
            v[g] = tab[idx];
        }
#pragma unroll
        for (int g = 0; g < G; ++g) a ^= v[g];
    } else {
        uint4 v[G][W > 0 ? W : 1];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint64_t idx = ((uint64_t)next_idx(x) * 0x9E3779B97F4A7C15ull >> 20) & mask;
            const uint4* e = reinterpret_cast<const uint4*>(tab) + idx * W;
#pragma unroll
            for (int w = 0; w < W; ++w) v[g][w] = e[w];
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int w = 0; w < W; ++w) a ^= v[g][w].x ^ v[g][w].y ^ v[g][w].z ^ v[g][w].w;
    }
    out[t] = a;
}

// cooperative: the C lanes of a group load one entry of C x 16 B together (lane c takes part c),
// so one instruction fetches 64 / C whole entries; each lane issues 6 x C loads, i.e. the same
// 6 entries per lane on average as the per-lane kernels
template <int C>
__global__ void gather_coop(const uint32_t* __restrict__ tab, uint64_t mask, uint32_t* __restrict__ out, uint64_t n,
                            uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t part = (uint32_t)t % C;
    uint32_t x = (uint32_t)(t / C) * 2654435761u ^ seed;
    uint4 v[6 * C];
#pragma unroll
    for (int g = 0; g < 6 * C; ++g) {
        const uint64_t idx = ((uint64_t)next_idx(x) * 0x9E3779B97F4A7C15ull >> 20) & mask;
        v[g] = reinterpret_cast<const uint4*>(tab)[idx * C + part];
    }
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < 6 * C; ++g) a ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
    out[t] = a;
}

template <int C>
int run_coop(uint64_t max_mb, uint32_t* out, uint64_t n, hipEvent_t a, hipEvent_t b, bool big = false) {
    const std::vector<uint64_t> sizes = big ? std::vector<uint64_t>{544, 1024, 8192, 16384, 28672}
                                            : std::vector<uint64_t>{256, 512, 1024, 2048, 8192};
    for (uint64_t mb : sizes) {
        if (mb > max_mb) break;
        const uint64_t bytes = mb << 20, entries = bytes / (16 * C);
        uint32_t* tab;
        CK(hipMalloc(&tab, bytes));
        CK(hipMemset(tab, 1, bytes));
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((gather_coop<C>), dim3((n + 255) / 256), dim3(256), 0, 0, tab, entries - 1, out, n, 77u + rep);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) best = ms < best ? ms : best;
        }
        printf("coop entry %2d B table %6llu MiB: %.3f ms for %llu gathers -> %.1f G gathers/s\n", 16 * C,
               (unsigned long long)mb, best, (unsigned long long)(n * 6), n * 6 / (best * 1e-3) / 1e9);
        fflush(stdout);
        CK(hipFree(tab));
    }
    return 0;
}

template <int W>
int run(uint64_t max_mb, uint32_t* out, uint64_t n, hipEvent_t a, hipEvent_t b) {
    const uint64_t esz = W == 0 ? 4 : 16 * W;
    for (uint64_t mb : {2ull, 32ull, 256ull, 1024ull, 2048ull, 4096ull, 8192ull, 16384ull}) {
        if (mb > max_mb) break;
        const uint64_t bytes = mb << 20, entries = bytes / esz;  // power of two
        uint32_t* tab;
        CK(hipMalloc(&tab, bytes));
        CK(hipMemset(tab, 1, bytes));
        float best = 1e9;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((gather<6, W>), dim3((n + 255) / 256), dim3(256), 0, 0, tab, entries - 1, out, n, 77u + rep);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) best = ms < best ? ms : best;
        }
        printf("entry %2llu B table %6llu MiB: %.3f ms for %llu gathers -> %.1f G gathers/s\n",
               (unsigned long long)esz, (unsigned long long)mb, best, (unsigned long long)(n * 6),
               n * 6 / (best * 1e-3) / 1e9);
        fflush(stdout);
        CK(hipFree(tab));
    }
    return 0;
}

int main(int argc, char** argv) {
    const uint64_t max_mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 16384;
    const uint64_t n = 10'000'000;  // threads (reads); 6 gathers each = 60M
    uint32_t* out;
    CK(hipMalloc(&out, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    if (argc > 2 && argv[2][0] == 'b') {  // 128-B entries (chained tables) up to 28 GiB: TLB reach
        if (run_coop<8>(max_mb, out, n, a, b, true) || run_coop<2>(max_mb, out, n, a, b, true)) return 1;
        return 0;
    }
    if (argc > 2) {  // coop only
        if (run_coop<2>(max_mb, out, n, a, b) || run_coop<4>(max_mb, out, n, a, b)) return 1;
        return 0;
    }
    if (run<0>(max_mb, out, n, a, b) || run<1>(max_mb, out, n, a, b) || run<2>(max_mb, out, n, a, b) ||
        run<4>(max_mb, out, n, a, b) || run_coop<2>(max_mb, out, n, a, b) || run_coop<4>(max_mb, out, n, a, b))
        return 1;
    return 0;
}
