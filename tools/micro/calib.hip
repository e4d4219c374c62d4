// Counter calibration on known byte counts (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE is
// calibrated only for wide streaming reads; other access widths must be calibrated in the
// kernel's own pattern). Each kernel runs twice (the second dispatch is the one to read):
//   k_stream_read  : 1 GiB read once, 16 B per lane, coalesced          -> FETCH per byte
//   k_stream_write : 1 GiB written once, 16 B per lane, coalesced       -> WRITE per byte
//   k_pair_gather  : 60M random 32-B entries from an 8 GiB table, a lane pair per entry (two
//                    16-B loads of one aligned entry: k_map1's access) -> FETCH / RDREQ per gather
//   k_pair_gather_mall : the same from a 128 MiB table (Infinity-Cache resident)
// usage: calib   (prints one line per kernel with its known byte / request counts)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                  \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_stream_read(const uint4* __restrict__ a, uint64_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;  // (never true for the fill below: keeps the loads)
}

__global__ void k_stream_write(uint4* __restrict__ a, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__device__ __forceinline__ uint32_t xs(uint32_t& x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

// lane pairs: lane 2q and 2q + 1 load halves of the same 32-B entry; 6 entries per pair
__global__ void k_pair_gather(const uint4* __restrict__ tab, uint64_t entries, uint32_t* __restrict__ out, uint64_t pairs,
                              uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * pairs) return;
    uint32_t x = (uint32_t)(t >> 1) * 2654435761u ^ seed;
    uint4 v[6];
#pragma unroll
    for (int g = 0; g < 6; ++g) {
        const uint64_t idx = ((uint64_t)xs(x) * 0x9E3779B97F4A7C15ull >> 20) % entries;
        v[g] = tab[idx * 2 + (t & 1)];
    }
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < 6; ++g) a ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
    out[t] = a;
}

int main() {
    const uint64_t sbytes = 1ull << 30;
    uint4* s;
    uint32_t* out;
    CK(hipMalloc(&s, sbytes));
    CK(hipMalloc(&out, 20'000'000ull * 4));
    CK(hipMemset(s, 1, sbytes));
    const uint64_t sn = sbytes / 16;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream_read, dim3(8192), dim3(256), 0, 0, s, sn, out);
        CK(hipDeviceSynchronize());
    }
    printf("k_stream_read: %llu bytes read (coalesced 16 B per lane)\n", (unsigned long long)sbytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream_write, dim3(8192), dim3(256), 0, 0, s, sn);
        CK(hipDeviceSynchronize());
    }
    printf("k_stream_write: %llu bytes written (coalesced 16 B per lane)\n", (unsigned long long)sbytes);
    CK(hipFree(s));
    const uint64_t pairs = 10'000'000;  // 60M entries per launch
    for (uint64_t mb : {8192ull, 128ull}) {
        uint4* tab;
        const uint64_t bytes = mb << 20;
        CK(hipMalloc(&tab, bytes));
        CK(hipMemset(tab, 1, bytes));
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k_pair_gather, dim3((2 * pairs + 255) / 256), dim3(256), 0, 0, tab, bytes / 32, out, pairs,
                               77u + rep);
            CK(hipDeviceSynchronize());
        }
        printf("k_pair_gather table %llu MiB: %llu random 32-B entries (%llu bytes)\n", (unsigned long long)mb,
               (unsigned long long)(pairs * 6), (unsigned long long)(pairs * 6 * 32));
        CK(hipFree(tab));
    }
    return 0;
}
