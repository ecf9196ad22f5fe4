// Issue cost of selects and 32-bit ops on gfx950 (SIMD-cycles per wave64
// instruction), completing op_rates2: op_rates2's v_cndmask_b32 stream read
// an uninitialised VCC and measured 22.9 cycles; these variants set the mask
// first, use an SGPR-pair mask, interleave with f64 work, and compare the
// alternatives (v_bfi_b32, v_and_or_b32, 32-bit ALU).
// hipcc --offload-arch=gfx950 -O3 tools/probes/op_rates3.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R16(s) s s s s s s s s s s s s s s s s
#define KERNEL(NAME, PRE, BODY, ...)                                                   \
    __global__ __launch_bounds__(256) void NAME(double* out, int iters, double x)       \
    {                                                                                   \
        double a = x + threadIdx.x, b = a * 0.5, c = a + 1.0;                           \
        unsigned ua = threadIdx.x, ub = ua * 3u, uc = ua ^ 0x5555u;                     \
        asm volatile(PRE : __VA_ARGS__);                                                \
        for (int i = 0; i < iters; ++i) { asm volatile(BODY : __VA_ARGS__); }          \
        if (a + b + c + ua + ub + uc == 1.2345) out[0] = a;                            \
    }
#define OPS "+v"(a), "+v"(b), "+v"(c), "+v"(ua), "+v"(ub), "+v"(uc)

KERNEL(k_cnd_vcc_set, "v_cmp_lt_u32 vcc, %3, %4\n", R16("v_cndmask_b32 %3, %3, %4, vcc\n"), OPS : : "vcc")
KERNEL(k_cnd_vcc_indep, "v_cmp_lt_u32 vcc, %3, %4\n", R16("v_cndmask_b32 %5, %4, %3, vcc\n"), OPS : : "vcc")
KERNEL(k_cnd_sgpr, "v_cmp_lt_u32_e64 s[0:1], %3, %4\n", R16("v_cndmask_b32_e64 %3, %3, %4, s[0:1]\n"), OPS : : "s0", "s1")
KERNEL(k_cnd_uninit, "", R16("v_cndmask_b32 %3, %3, %4, vcc\n"), OPS : : "vcc")
KERNEL(k_bfi, "", R16("v_bfi_b32 %3, %5, %3, %4\n"), OPS)
KERNEL(k_andor, "", R16("v_and_or_b32 %3, %3, %5, %4\n"), OPS)
KERNEL(k_mov32, "", R16("v_mov_b32 %3, %4\n"), OPS)
KERNEL(k_or32, "", R16("v_or_b32 %3, %3, %4\n"), OPS)
KERNEL(k_xor32, "", R16("v_xor_b32 %3, %3, %4\n"), OPS)
KERNEL(k_lsh32, "", R16("v_lshlrev_b32 %3, 3, %4\n"), OPS)
KERNEL(k_mullo, "", R16("v_mul_lo_u32 %3, %3, %4\n"), OPS)
KERNEL(k_mulhi, "", R16("v_mul_hi_u32 %3, %3, %4\n"), OPS)
KERNEL(k_cvti, "", R16("v_cvt_i32_f64 %3, %0\n"), OPS)
KERNEL(k_fmamix, "v_cmp_lt_u32 vcc, %3, %4\n", R16("v_fma_f64 %0, %1, %2, %0\nv_cndmask_b32 %3, %3, %4, vcc\n"), OPS : : "vcc")
KERNEL(k_fmacmp, "", R16("v_fma_f64 %0, %1, %2, %0\nv_cmp_lt_f64 vcc, %1, %2\n"), OPS : : "vcc")
KERNEL(k_cmpcnd, "", R16("v_cmp_lt_f64 vcc, %1, %2\nv_cndmask_b32 %3, %3, %4, vcc\n"), OPS : : "vcc")
KERNEL(k_addf64, "", R16("v_add_f64 %0, %1, %2\n"), OPS)
KERNEL(k_fmaf64, "", R16("v_fma_f64 %0, %1, %2, %0\n"), OPS)

typedef void (*KF)(double*, int, double);
int main()
{
    double* d;
    (void)hipMalloc(&d, 8);
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    struct { const char* n; KF f; int per; } ks[] = {
        {"v_cndmask_b32 vcc (set, dep)", k_cnd_vcc_set, 16}, {"v_cndmask_b32 vcc (set, indep)", k_cnd_vcc_indep, 16},
        {"v_cndmask_b32_e64 s[0:1]", k_cnd_sgpr, 16}, {"v_cndmask_b32 vcc (uninit)", k_cnd_uninit, 16},
        {"v_bfi_b32", k_bfi, 16}, {"v_and_or_b32", k_andor, 16}, {"v_mov_b32", k_mov32, 16},
        {"v_or_b32", k_or32, 16}, {"v_xor_b32", k_xor32, 16}, {"v_lshlrev_b32", k_lsh32, 16},
        {"v_mul_lo_u32", k_mullo, 16}, {"v_mul_hi_u32", k_mulhi, 16}, {"v_cvt_i32_f64", k_cvti, 16},
        {"fma_f64 + cndmask pair", k_fmamix, 32}, {"fma_f64 + cmp_f64 pair", k_fmacmp, 32},
        {"cmp_f64(vcc) + cndmask pair", k_cmpcnd, 32}, {"v_add_f64", k_addf64, 16}, {"v_fma_f64", k_fmaf64, 16}};
    const int iters = 4000;
    for (int wps : {4, 8}) {
        for (auto& k : ks) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            hipLaunchKernelGGL(k.f, ncu * wps, 256, 0, 0, d, iters, 1.5);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, ncu * wps, 256, 0, 0, d, iters, 1.5);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double winstr = (double)wps * iters * k.per;
            printf("waves/SIMD %d  %-32s %.2f SIMD-cycles/instr (at 2.4 GHz)\n", wps, k.n, ms * 1e-3 * 2.4e9 / winstr);
        }
    }
    return 0;
}
