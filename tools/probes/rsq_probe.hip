// Probe: relative error of v_rsq_f64 and of one Newton step, over many inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
__global__ void k(unsigned long long seed, int n, double* maxe0, double* maxe1, double* maxe2) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    double m0 = 0, m1 = 0, m2 = 0;
    unsigned long long s = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
    for (int it = 0; it < n; ++it) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        // exponents in [-600, 600], random mantissa
        double x = ldexp(1.0 + (double)(s >> 11) * 0x1p-53, (int)((s >> 3) % 1200) - 600);
        double r0 = __builtin_amdgcn_rsq(x);
        double r1 = r0 * (1.5 - 0.5 * x * r0 * r0);
        double sq = sqrt(x);
        double sa = x * r1;
        double e0 = fabs(r0 * sq - 1.0);
        double e1 = fabs(sa - sq) / sq;
        const double tt = x * r0;                                   // kernel form (rt_kernels.hip)
        const double sb = fma(tt * 0.5, fma(-tt, r0, 1.0), tt);
        double e2 = fabs(sb - sq) / sq;
        m0 = fmax(m0, e0); m1 = fmax(m1, e1); m2 = fmax(m2, e2);
    }
    maxe0[i] = m0; maxe1[i] = m1; maxe2[i] = m2;
}
int main() {
    const int T = 256 * 1024, N = 4096;
    double *a, *b, *c; hipMalloc(&a, T * 8); hipMalloc(&b, T * 8); hipMalloc(&c, T * 8);
    hipLaunchKernelGGL(k, dim3(T / 256), dim3(256), 0, 0, 12345ull, N, a, b, c);
    double *ha = new double[T], *hb = new double[T], *hc = new double[T];
    hipMemcpy(ha, a, T * 8, hipMemcpyDeviceToHost); hipMemcpy(hb, b, T * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hc, c, T * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0, m2 = 0;
    for (int i = 0; i < T; ++i) { m0 = fmax(m0, ha[i]); m1 = fmax(m1, hb[i]); m2 = fmax(m2, hc[i]); }
    printf("samples %lld  max rel err rsq %.3e (2^%.1f)  after 1 Newton + mul %.3e (2^%.1f)  fma form %.3e (2^%.1f)\n",
           (long long)T * N, m0, log2(m0), m1, log2(m1), m2, log2(m2));
    return 0;
}
