// Does gfx950's f64 matrix pipe run beside f64 VALU work?  Waves of one
// kernel run either a stream of independent v_fma_f64 (VALU) or a stream of
// independent v_mfma_f64_16x16x4_f64 (matrix pipe); the mixed launch runs
// both kinds side by side on every SIMD (even waves VALU, odd waves MFMA).
// If the mixed time is close to max(VALU alone, MFMA alone) the pipes
// overlap and an f64 GEMM-shaped part of the candidate pass could move to
// the matrix pipe; if it is close to the sum they share one datapath.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_overlap.hip -o tools/probes/mfma_f64_overlap
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

#define R8(s) s s s s s s s s

__device__ __forceinline__ void valu_body(double& a, double& b, double& c, double& e, int iters)
{
    for (int i = 0; i < iters; ++i) {
        // 32 independent-ish f64 FMAs per iteration (4 chains x 8)
        asm volatile(R8("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n")
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(e) : "v"(0.999), "v"(1e-3));
    }
}

__device__ __forceinline__ void mfma_body(d4& x0, d4& x1, d4& x2, d4& x3, double p, double q, int iters)
{
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(p, q, x0, 0, 0, 0);
            x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(p, q, x1, 0, 0, 0);
            x2 = __builtin_amdgcn_mfma_f64_16x16x4f64(p, q, x2, 0, 0, 0);
            x3 = __builtin_amdgcn_mfma_f64_16x16x4f64(p, q, x3, 0, 0, 0);
        }
    }
}

// mode 0: every wave VALU; 1: every wave MFMA; 2: even waves VALU, odd MFMA
__global__ __launch_bounds__(512) void probe(double* out, int mode, int iv, int im)
{
    const int w = threadIdx.x >> 6;
    double a = threadIdx.x * 1e-3, b = a + 1, c = a + 2, e = a + 3;
    d4 x0 = {a, b, c, e}, x1 = x0, x2 = x0, x3 = x0;
    const bool do_valu = mode == 0 || (mode == 2 && (w & 1) == 0);
    const bool do_mfma = mode == 1 || (mode == 2 && (w & 1) == 1);
    if (do_valu) valu_body(a, b, c, e, iv);
    if (do_mfma) mfma_body(x0, x1, x2, x3, a, b, im);
    const double s = a + b + c + e + x0.x + x1.y + x2.z + x3.w;
    if (s == 1.2345) out[0] = s;
}

int main()
{
    double* d;
    (void)hipMalloc(&d, 8);
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int iv = 20000, im = 2500;      // per wave: 640000 VALU fma, 20000 MFMA
    for (int blocks_per_cu : {1, 2, 4}) { // 512-thread blocks: 2, 4 or 8 waves per SIMD
        float t[3];
        for (int mode = 0; mode < 3; ++mode) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            hipLaunchKernelGGL(probe, ncu * blocks_per_cu, 512, 0, 0, d, mode, iv, im);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(probe, ncu * blocks_per_cu, 512, 0, 0, d, mode, iv, im);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&t[mode], e0, e1);
        }
        const int wps = 2 * blocks_per_cu;
        // per SIMD: mode 0 runs wps VALU waves, mode 1 wps MFMA waves, mode 2 wps/2 of each
        const double cyc = 2.4e6;   // SIMD cycles per ms at 2.4 GHz
        printf("waves/SIMD %d: VALU-only %.3f ms (%.2f cyc/fma64), MFMA-only %.3f ms (%.1f cyc/mfma), "
               "mixed (half each) %.3f ms; half+half if serial: %.3f, if overlapped: %.3f\n",
               wps, t[0], t[0] * cyc / (wps * iv * 32.0), t[1], t[1] * cyc / (wps * im * 8.0), t[2],
               0.5 * (t[0] + t[1]), 0.5 * (t[0] > t[1] ? t[0] : t[1]));
    }
    return 0;
}
