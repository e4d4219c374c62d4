// VALU throughput by instruction on gfx950 (development microbenchmark): each
// kernel runs 8 independent chains of one instruction form at 8 waves per SIMD; the SIMD's
// cycles per wave-instruction come from the wall time and the clock the caller passes (GRBM:
// rocprofv3 --pmc GRBM_GUI_ACTIVE over the same run). Prints one line per form.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/valu_mix.hip -o tools/micro/valu_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define R8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define OUTS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])

#define KERNEL(NAME, FORM)                                                                       \
    __global__ __launch_bounds__(512) void NAME(uint32_t* out, int iters, uint32_t seed) {       \
        uint32_t a[8];                                                                           \
        for (int i = 0; i < 8; ++i) a[i] = (seed + threadIdx.x) * (2 * i + 3);                   \
        const uint32_t b = seed * 0x9E3779B1u + threadIdx.x, c = b ^ 0x5555u;                    \
        asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cmp_gt_u32_e64 s[20:21], %1, %0" :: "v"(b), "v"(c) : "vcc", "s20", "s21"); \
        for (int it = 0; it < iters; ++it) {                                                     \
            _Pragma("unroll") for (int u = 0; u < 32; ++u) {                                     \
                asm volatile(FORM(0) FORM(1) FORM(2) FORM(3) FORM(4) FORM(5) FORM(6) FORM(7)      \
                             : OUTS : "v"(b), "v"(c) : "vcc", "s20", "s21");                     \
            }                                                                                    \
        }                                                                                        \
        uint32_t x = 0;                                                                          \
        for (int i = 0; i < 8; ++i) x ^= a[i];                                                   \
        if (x == 0x12345678u) out[threadIdx.x] = x;                                              \
    }

#define S(x) #x
#define F_XOR(i) "v_xor_b32 %" S(i) ", %" S(i) ", %8\n"
#define F_AND(i) "v_and_b32 %" S(i) ", %" S(i) ", %8\n"
#define F_LSHR(i) "v_lshrrev_b32 %" S(i) ", 3, %" S(i) "\n"
#define F_LSHL(i) "v_lshlrev_b32 %" S(i) ", 3, %" S(i) "\n"
#define F_MIN(i) "v_min_u32 %" S(i) ", %" S(i) ", %8\n"
#define F_SUB(i) "v_sub_u32 %" S(i) ", %8, %" S(i) "\n"
#define F_MOV(i) "v_mov_b32 %" S(i) ", %8\n"
#define F_ALIGNBIT(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %8, 31\n"
#define F_BFE(i) "v_bfe_u32 %" S(i) ", %" S(i) ", 3, 4\n"
#define F_PERM(i) "v_perm_b32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_ADD3(i) "v_add3_u32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_OR3(i) "v_or3_b32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_LSHLOR(i) "v_lshl_or_b32 %" S(i) ", %" S(i) ", 3, %8\n"
#define F_ANDOR(i) "v_and_or_b32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_BITOP3(i) "v_bitop3_b32 %" S(i) ", %" S(i) ", %8, %9 bitop3:0x96\n"
#define F_CMP32(i) "v_cmp_gt_u32 vcc, %" S(i) ", %8\n"
#define F_CMP64(i) "v_cmp_gt_u32_e64 s[20:21], %" S(i) ", %8\n"
#define F_CND32(i) "v_cndmask_b32 %" S(i) ", %" S(i) ", %8, vcc\n"
#define F_MAD24(i) "v_mad_u32_u24 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_MULLO(i) "v_mul_lo_u32 %" S(i) ", %" S(i) ", %8\n"
#define F_DOT4(i) "v_dot4_u32_u8 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_MED3(i) "v_med3_u32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_ADDE64(i) "v_add_u32_e64 %" S(i) ", %" S(i) ", %8\n"
#define F_XORE64(i) "v_xor_b32_e64 %" S(i) ", %" S(i) ", %8\n"
#define F_LSHRE64(i) "v_lshrrev_b32_e64 %" S(i) ", 3, %" S(i) "\n"
#define F_ADDC(i) "v_addc_co_u32 %" S(i) ", vcc, %" S(i) ", %8, vcc\n"
#define F_LSHLADD(i) "v_lshl_add_u32 %" S(i) ", %" S(i) ", 3, %8\n"
#define F_CNDE64V(i) "v_cndmask_b32_e64 %" S(i) ", %" S(i) ", %8, vcc\n"
#define F_CNDE64S(i) "v_cndmask_b32_e64 %" S(i) ", %" S(i) ", %8, s[20:21]\n"
#define F_MAX(i) "v_max_u32 %" S(i) ", %" S(i) ", %8\n"
#define F_ASHR(i) "v_ashrrev_i32 %" S(i) ", 3, %" S(i) "\n"
#define F_OR(i) "v_or_b32 %" S(i) ", %" S(i) ", %8\n"
#define F_NOT(i) "v_not_b32 %" S(i) ", %" S(i) "\n"
#define F_BFI(i) "v_bfi_b32 %" S(i) ", %" S(i) ", %8, %9\n"
#define F_ADDCO(i) "v_add_co_u32 %" S(i) ", vcc, %" S(i) ", %8\n"
#define F_MBCNT(i) "v_mbcnt_lo_u32_b32 %" S(i) ", %8, %" S(i) "\n"
#define F_LSHLREVE64(i) "v_lshlrev_b32_e64 %" S(i) ", 3, %" S(i) "\n"
#define F_MINE64(i) "v_min_u32_e64 %" S(i) ", %" S(i) ", %8\n"
#define F_ADDSAT(i) "v_add_u32_e64 %" S(i) ", %" S(i) ", %8 clamp\n"
#define F_SUBSAT(i) "v_sub_u32_e64 %" S(i) ", %" S(i) ", %8 clamp\n"
#define F_CMPNE64(i) "v_cmp_ne_u32_e64 s[20:21], %" S(i) ", %8\n"
#define F_CMPX(i) "v_cmp_eq_u32 vcc, %" S(i) ", %8\n v_cndmask_b32 %" S(i) ", %" S(i) ", %9, vcc\n"

KERNEL(k_xor, F_XOR)
KERNEL(k_and, F_AND)
KERNEL(k_lshr, F_LSHR)
KERNEL(k_lshl, F_LSHL)
KERNEL(k_min, F_MIN)
KERNEL(k_sub, F_SUB)
KERNEL(k_mov, F_MOV)
KERNEL(k_alignbit, F_ALIGNBIT)
KERNEL(k_bfe, F_BFE)
KERNEL(k_perm, F_PERM)
KERNEL(k_add3, F_ADD3)
KERNEL(k_or3, F_OR3)
KERNEL(k_lshlor, F_LSHLOR)
KERNEL(k_andor, F_ANDOR)
KERNEL(k_bitop3, F_BITOP3)
KERNEL(k_cmp32, F_CMP32)
KERNEL(k_cmp64, F_CMP64)
KERNEL(k_cnd32, F_CND32)
KERNEL(k_mad24, F_MAD24)
KERNEL(k_mullo, F_MULLO)
KERNEL(k_dot4, F_DOT4)
KERNEL(k_med3, F_MED3)
KERNEL(k_adde64, F_ADDE64)
KERNEL(k_xore64, F_XORE64)
KERNEL(k_lshre64, F_LSHRE64)
KERNEL(k_addc, F_ADDC)
KERNEL(k_lshladd, F_LSHLADD)
KERNEL(k_cnde64v, F_CNDE64V)
KERNEL(k_cnde64s, F_CNDE64S)
KERNEL(k_max, F_MAX)
KERNEL(k_ashr, F_ASHR)
KERNEL(k_or, F_OR)
KERNEL(k_not, F_NOT)
KERNEL(k_bfi, F_BFI)
KERNEL(k_addco, F_ADDCO)
KERNEL(k_mbcnt, F_MBCNT)
KERNEL(k_lshle64, F_LSHLREVE64)
KERNEL(k_mine64, F_MINE64)
KERNEL(k_addsat, F_ADDSAT)
KERNEL(k_subsat, F_SUBSAT)
KERNEL(k_cmpne64, F_CMPNE64)
KERNEL(k_cmpx, F_CMPX)

int main(int argc, char** argv) {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const double ghz = argc > 1 ? std::atof(argv[1]) : 2.1;
    uint32_t* d = nullptr;
    CK(hipMalloc(&d, 4096));
    const int iters = 100;
    struct K { const char* name; void (*f)(uint32_t*, int, uint32_t); };
    const K ks[] = {{"v_xor_b32", k_xor}, {"v_and_b32", k_and}, {"v_lshrrev_b32", k_lshr}, {"v_lshlrev_b32", k_lshl},
                    {"v_min_u32", k_min}, {"v_sub_u32", k_sub}, {"v_mov_b32", k_mov}, {"v_alignbit_b32", k_alignbit},
                    {"v_bfe_u32", k_bfe}, {"v_perm_b32", k_perm}, {"v_add3_u32", k_add3}, {"v_or3_b32", k_or3},
                    {"v_lshl_or_b32", k_lshlor}, {"v_and_or_b32", k_andor}, {"v_bitop3_b32", k_bitop3},
                    {"v_cmp_gt_u32 (vcc)", k_cmp32}, {"v_cmp_gt_u32_e64 (sgpr)", k_cmp64}, {"v_cndmask_b32 (vcc)", k_cnd32},
                    {"v_mad_u32_u24", k_mad24}, {"v_mul_lo_u32", k_mullo}, {"v_dot4_u32_u8", k_dot4}, {"v_med3_u32", k_med3},
                    {"v_add_u32_e64", k_adde64}, {"v_xor_b32_e64", k_xore64}, {"v_lshrrev_b32_e64", k_lshre64},
                    {"v_addc_co_u32 (vcc chain)", k_addc}, {"v_lshl_add_u32", k_lshladd},
                    {"v_cndmask_b32_e64 vcc", k_cnde64v}, {"v_cndmask_b32_e64 s[20:21]", k_cnde64s}, {"v_max_u32", k_max},
                    {"v_ashrrev_i32", k_ashr}, {"v_or_b32", k_or}, {"v_not_b32", k_not}, {"v_bfi_b32", k_bfi},
                    {"v_add_co_u32 (vcc out)", k_addco}, {"v_mbcnt_lo_u32_b32", k_mbcnt}, {"v_lshlrev_b32_e64", k_lshle64},
                    {"v_min_u32_e64", k_mine64}, {"v_add_u32 clamp", k_addsat}, {"v_sub_u32 clamp", k_subsat},
                    {"v_cmp_ne_u32_e64 (sgpr)", k_cmpne64}, {"cmp vcc + cndmask vcc (pair)", k_cmpx}};
    // 8 waves per SIMD: 4 workgroups of 512 threads per CU
    const int grid = ncu * 4, threads = 512;
    for (const K& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(threads), 0, 0, d, iters, 7u);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(threads), 0, 0, d, iters, 7u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double inst_per_simd = 8.0 * iters * 32 * 8;  // waves x iterations x unroll x forms
        std::printf("%-28s %.3f ms  %.2f cycles per wave-instruction per SIMD at %.2f GHz\n", k.name, ms,
                    ms * 1e-3 * ghz * 1e9 / inst_per_simd, ghz);
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
    }
    CK(hipFree(d));
    return 0;
}
