// VALU issue rate on gfx950 by instruction kind and waves per SIMD (development microbenchmark,
// DESIGN.md §5): each wave runs 8 independent chains of one instruction, 64 x 8 per iteration,
// timed with s_memtime (shader clock). Prints cycles per wave-instruction seen by one wave and
// the SIMD's throughput (wave-instructions per cycle) at 1, 2, 4 and 8 waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rate.hip -o tools/micro/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int KIND>
__global__ __launch_bounds__(512) void k_rate(uint64_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    const uint32_t b = seed * 0x9E3779B1u + threadIdx.x;
    float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)a3, f4 = (float)a4, f5 = (float)a5,
          f6 = (float)a6, f7 = (float)a7;
    const float fb = 1.0001f;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 64; ++u) {
            if (KIND == 0) {  // v_xor_b32
                asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n"
                             "v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 1) {  // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %8, 31\n v_alignbit_b32 %1, %1, %8, 31\n v_alignbit_b32 %2, %2, %8, 31\n"
                             "v_alignbit_b32 %3, %3, %8, 31\n v_alignbit_b32 %4, %4, %8, 31\n v_alignbit_b32 %5, %5, %8, 31\n"
                             "v_alignbit_b32 %6, %6, %8, 31\n v_alignbit_b32 %7, %7, %8, 31"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 2) {  // v_lshl_add_u32 (VOP3)
                asm volatile("v_lshl_add_u32 %0, %0, 3, %8\n v_lshl_add_u32 %1, %1, 3, %8\n v_lshl_add_u32 %2, %2, 3, %8\n"
                             "v_lshl_add_u32 %3, %3, 3, %8\n v_lshl_add_u32 %4, %4, 3, %8\n v_lshl_add_u32 %5, %5, 3, %8\n"
                             "v_lshl_add_u32 %6, %6, 3, %8\n v_lshl_add_u32 %7, %7, 3, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 3) {  // v_fma_f32 (reference: 2 cycles per wave-instruction)
                asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n"
                             "v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n"
                             "v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8"
                             : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(fb));
            } else if (KIND == 4) {  // v_add_u32 (VOP2)
                asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                             "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 5) {  // v_cndmask_b32 with vcc
                asm volatile("v_cmp_gt_u32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                             "v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                             "v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");
            } else if (KIND == 7) {  // v_cmp -> SGPR pair -> v_cndmask, 4 independent pairs
                asm volatile("v_cmp_gt_u32 s[20:21], %0, %8\n v_cmp_gt_u32 s[22:23], %1, %8\n v_cmp_gt_u32 s[24:25], %2, %8\n"
                             "v_cmp_gt_u32 s[26:27], %3, %8\n v_cndmask_b32 %4, %4, %8, s[20:21]\n v_cndmask_b32 %5, %5, %8, s[22:23]\n"
                             "v_cndmask_b32 %6, %6, %8, s[24:25]\n v_cndmask_b32 %7, %7, %8, s[26:27]"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)
                             : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
            } else if (KIND == 8) {  // v_sub_u32 clamp + v_min_u32 (a compare with no SGPR result)
                asm volatile("v_sub_u32 %0, %8, %0 clamp\n v_sub_u32 %1, %8, %1 clamp\n v_sub_u32 %2, %8, %2 clamp\n"
                             "v_sub_u32 %3, %8, %3 clamp\n v_min_u32 %4, %4, %0\n v_min_u32 %5, %5, %1\n"
                             "v_min_u32 %6, %6, %2\n v_min_u32 %7, %7, %3"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 9) {  // v_bitop3_b32 (gfx950: any 3-input bitwise function)
                asm volatile("v_bitop3_b32 %0, %0, %8, %1 bitop3:0x96\n v_bitop3_b32 %1, %1, %8, %2 bitop3:0x96\n"
                             "v_bitop3_b32 %2, %2, %8, %3 bitop3:0x96\n v_bitop3_b32 %3, %3, %8, %4 bitop3:0x96\n"
                             "v_bitop3_b32 %4, %4, %8, %5 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %6 bitop3:0x96\n"
                             "v_bitop3_b32 %6, %6, %8, %7 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %0 bitop3:0x96"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            } else if (KIND == 6) {  // v_pk_add_u16 (packed)
                asm volatile("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n"
                             "v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint32_t x = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = (t1 - t0) | ((uint64_t)(x & 1) << 63);
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const char* names[] = {"v_xor_b32", "v_alignbit_b32", "v_lshl_add_u32", "v_fma_f32", "v_add_u32", "v_cndmask_b32",
                           "v_pk_add_u16", "cmp->sgpr->cndmask", "sub clamp + min", "v_bitop3_b32"};
    uint64_t* d = nullptr;
    CK(hipMalloc(&d, sizeof(uint64_t) * ncu * 64));
    CK(hipMemset(d, 0, sizeof(uint64_t) * ncu * 64));
    const int iters = 200;
    for (int kind = 0; kind < 10; ++kind) {
        for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: one workgroup of 4 * wps waves per CU
            // (512-thread workgroups, wps / 2 of them per CU; wps 1: one of 256)
            const int threads = wps == 1 ? 256 : 512;
            const int grid = wps == 1 ? ncu : ncu * wps / 2;
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            auto launch = [&] {
                switch (kind) {
                case 0: hipLaunchKernelGGL(k_rate<0>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 1: hipLaunchKernelGGL(k_rate<1>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 2: hipLaunchKernelGGL(k_rate<2>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 3: hipLaunchKernelGGL(k_rate<3>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 4: hipLaunchKernelGGL(k_rate<4>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 5: hipLaunchKernelGGL(k_rate<5>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 6: hipLaunchKernelGGL(k_rate<6>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 7: hipLaunchKernelGGL(k_rate<7>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 8: hipLaunchKernelGGL(k_rate<8>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                case 9: hipLaunchKernelGGL(k_rate<9>, dim3(grid), dim3(threads), 0, 0, d, iters, 7u); break;
                }
            };
            launch();
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint64_t> h((size_t)grid * threads / 64);
            CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            double cyc = 0;
            for (auto v : h) cyc += (double)(v & ~(1ull << 63));
            cyc /= h.size();
            const double ninst = (double)iters * 64 * 8;
            // per wave: cycles per instruction; per SIMD: wps waves' instructions over the span
            std::printf("%-16s waves/SIMD %d: %.2f cyc per wave-instruction (one wave's view), SIMD %.3f "
                        "wave-instr/cyc, wall %.3f ms -> %.2f GHz-equivalent\n",
                        names[kind], wps, cyc / ninst, wps * ninst / cyc, ms, cyc / (ms * 1e-3) / 1e9);
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
        }
    }
    CK(hipFree(d));
    return 0;
}
