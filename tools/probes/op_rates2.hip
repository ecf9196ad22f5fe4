// Issue cost (SIMD-cycles per wave64 instruction, 4 and 8 waves per SIMD) of
// single gfx950 VALU instructions, from inline-asm streams of 16 independent
// copies per loop iteration.  Informs the f64 -> f32 candidate-pass choices
// (DESIGN.md).  hipcc --offload-arch=gfx950 -O3 tools/probes/op_rates2.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R16(s) s s s s s s s s s s s s s s s s
#define KERNEL(NAME, BODY, ...)                                                   \
    __global__ __launch_bounds__(256) void NAME(double* out, int iters, double x)  \
    {                                                                              \
        double a = x + threadIdx.x, b = a * 0.5, c = a + 1.0;                      \
        float fa = (float)a, fb = (float)b, fc = (float)c;                         \
        unsigned ua = threadIdx.x, ub = ua * 3u;                                   \
        for (int i = 0; i < iters; ++i) { asm volatile(BODY : __VA_ARGS__); }             \
        if (a + b + c + fa + fb + fc + ua + ub == 1.2345) out[0] = a;             \
    }

KERNEL(k_fma64, R16("v_fma_f64 %0, %1, %2, %0\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_mul64, R16("v_mul_f64 %0, %1, %2\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_cmp64, R16("v_cmp_lt_f64 vcc, %0, %1\n"), "+v"(a), "+v"(b), "+v"(c) : : "vcc")
KERNEL(k_cmp64e, R16("v_cmp_lt_f64_e64 s[0:1], %0, %1\n"), "+v"(a), "+v"(b), "+v"(c) : : "s0", "s1")
KERNEL(k_cmpcls64, R16("v_cmp_class_f64 vcc, %0, %3\n"), "+v"(a), "+v"(b), "+v"(c) : "v"(ua) : "vcc")
KERNEL(k_max64, R16("v_max_f64 %0, %1, %2\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_rsq64, R16("v_rsq_f64 %0, %1\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_sqrt64, R16("v_sqrt_f64 %0, %1\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_cvt6432, R16("v_cvt_f32_f64 %0, %1\n"), "+v"(fa), "+v"(b), "+v"(c))
KERNEL(k_cvt3264, R16("v_cvt_f64_f32 %0, %1\n"), "+v"(a), "+v"(fb), "+v"(c))
KERNEL(k_fma32, R16("v_fma_f32 %0, %1, %2, %0\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_pkfma32, R16("v_pk_fma_f32 %0, %1, %2, %0\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_cmp32, R16("v_cmp_lt_f32 vcc, %0, %1\n"), "+v"(fa), "+v"(fb), "+v"(fc) : : "vcc")
KERNEL(k_min32, R16("v_min_f32 %0, %1, %2\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_min332, R16("v_min3_f32 %0, %1, %2, %0\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_rsq32, R16("v_rsq_f32 %0, %1\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_rcp32, R16("v_rcp_f32 %0, %1\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_sqrt32, R16("v_sqrt_f32 %0, %1\n"), "+v"(fa), "+v"(fb), "+v"(fc))
KERNEL(k_cnd, R16("v_cndmask_b32 %0, %0, %1, vcc\n"), "+v"(ua), "+v"(ub), "+v"(fc) : : "vcc")
KERNEL(k_add32, R16("v_add_u32 %0, %0, %1\n"), "+v"(ua), "+v"(ub), "+v"(fc))
KERNEL(k_cmpu32, R16("v_cmp_lt_u32 vcc, %0, %1\n"), "+v"(ua), "+v"(ub), "+v"(fc) : : "vcc")
KERNEL(k_mov64, R16("v_mov_b64 %0, %1\n"), "+v"(a), "+v"(b), "+v"(c))
KERNEL(k_madu64, R16("v_mad_u64_u32 %0, s[0:1], %1, %2, %0\n"), "+v"(a), "+v"(ua), "+v"(ub) : : "s0", "s1")
KERNEL(k_ldexp, R16("v_ldexp_f64 %0, %1, %3\n"), "+v"(a), "+v"(b), "+v"(c) : "v"(ua))
KERNEL(k_mix, R16("v_fma_f64 %0, %1, %2, %0\nv_fma_f32 %3, %4, %5, %3\n"), "+v"(a), "+v"(b), "+v"(c), "+v"(fa), "+v"(fb), "+v"(fc))

typedef void (*KF)(double*, int, double);
int main()
{
    double* d;
    (void)hipMalloc(&d, 8);
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    struct { const char* n; KF f; int per; } ks[] = {
        {"v_fma_f64", k_fma64, 16}, {"v_mul_f64", k_mul64, 16}, {"v_cmp_lt_f64 (vcc)", k_cmp64, 16},
        {"v_cmp_lt_f64_e64", k_cmp64e, 16}, {"v_cmp_class_f64", k_cmpcls64, 16}, {"v_max_f64", k_max64, 16},
        {"v_rsq_f64", k_rsq64, 16}, {"v_sqrt_f64", k_sqrt64, 16}, {"v_cvt_f32_f64", k_cvt6432, 16},
        {"v_cvt_f64_f32", k_cvt3264, 16}, {"v_fma_f32", k_fma32, 16}, {"v_pk_fma_f32", k_pkfma32, 16},
        {"v_cmp_lt_f32", k_cmp32, 16}, {"v_min_f32", k_min32, 16}, {"v_min3_f32", k_min332, 16},
        {"v_rsq_f32", k_rsq32, 16}, {"v_rcp_f32", k_rcp32, 16}, {"v_sqrt_f32", k_sqrt32, 16},
        {"v_cndmask_b32", k_cnd, 16}, {"v_add_u32", k_add32, 16}, {"v_cmp_lt_u32", k_cmpu32, 16},
        {"v_mov_b64", k_mov64, 16}, {"v_mad_u64_u32", k_madu64, 16}, {"v_ldexp_f64", k_ldexp, 16},
        {"fma_f64+fma_f32 pair", k_mix, 32}};
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
            printf("waves/SIMD %d  %-22s %.2f SIMD-cycles/instr (at 2.4 GHz)\n", wps, k.n, ms * 1e-3 * 2.4e9 / winstr);
        }
    }
    return 0;
}
