// Issue cost of single VALU ops on gfx950 with several waves per SIMD:
// SIMD-cycles per wave64 instruction for f64 fma/add/cmp+cndmask, f32
// fma, v_rsq/rcp (f32, f64), int add.  Informs which parts of the render
// kernel pay to move from f64 to f32.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/probes/op_rates.hip -o tools/probes/op_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH 8
template <int OP>
__global__ __launch_bounds__(256) void k(double* out, int iters, double seed)
{
    double a[CH];
    float f[CH];
    unsigned u[CH];
    for (int j = 0; j < CH; ++j) {
        a[j] = seed + threadIdx.x * 1e-7 + j;
        f[j] = (float)a[j];
        u[j] = threadIdx.x + j;
    }
    const double m = 0.999999, c = 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                if (OP == 0) a[j] = __builtin_fma(a[j], m, c);
                if (OP == 1) f[j] = __builtin_fmaf(f[j], 0.999999f, 1e-9f);
                if (OP == 2) a[j] = a[j] + c;
                if (OP == 3) a[j] = __builtin_amdgcn_rsq(a[j]);
                if (OP == 4) f[j] = __builtin_amdgcn_rsqf(f[j]);
                if (OP == 5) u[j] = u[j] * 0x9E3779B9u + 7u;
                if (OP == 6) a[j] = a[j] > c ? a[j] * m : a[j];       // cmp + mul + 2 cndmask
                if (OP == 7) a[j] = __builtin_amdgcn_rcp(a[j]);
                if (OP == 8) f[j] = __builtin_fminf(f[j], 0.5f) + 1e-9f;
                if (OP == 9) a[j] = __builtin_fmin(a[j], 2.0) + c;
            }
    }
    double s = 0;
    for (int j = 0; j < CH; ++j) s += a[j] + f[j] + u[j];
    if (s == 12345.678) out[0] = s;
}

int main()
{
    double* d;
    hipMalloc(&d, 8);
    const char* names[] = {"v_fma_f64", "v_fma_f32", "v_add_f64", "v_rsq_f64", "v_rsq_f32", "v_mul_lo_u32+add",
                           "cmp_f64+mul+cnd", "v_rcp_f64", "v_min_f32+add", "v_min_f64+add"};
    int dev;
    hipGetDevice(&dev);
    int ncu;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 2000;
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = ncu * wps;       // 256-thread blocks: 4 waves = 1 per SIMD per block
        for (int op = 0; op < 10; ++op) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            auto launch = [&]() {
                switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 1: hipLaunchKernelGGL(k<1>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 2: hipLaunchKernelGGL(k<2>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 3: hipLaunchKernelGGL(k<3>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 4: hipLaunchKernelGGL(k<4>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 5: hipLaunchKernelGGL(k<5>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 6: hipLaunchKernelGGL(k<6>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 7: hipLaunchKernelGGL(k<7>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 8: hipLaunchKernelGGL(k<8>, blocks, 256, 0, 0, d, iters, 1.0); break;
                case 9: hipLaunchKernelGGL(k<9>, blocks, 256, 0, 0, d, iters, 1.0); break;
                }
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per SIMD: waves per SIMD x iters x 64 ops
            const double winstr = (double)wps * iters * 8 * CH;
            const double cyc = ms * 1e-3 * 2.4e9;
            printf("waves/SIMD %d  %-18s %.2f SIMD-cycles per wave-instruction\n", wps, names[op], cyc / winstr);
        }
    }
    return 0;
}
