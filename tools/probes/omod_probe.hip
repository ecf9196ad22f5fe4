// Does the VOP3 output modifier (div:2 / mul:2) apply to v_rsq_f64 / v_mul_f64
// on gfx950 with the MODE.IEEE bit set (the compute default), and with it clear?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(const double* x, double* out, int ieee_off)
{
    if (ieee_off) asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 9, 1), 0");
    const double v = x[threadIdx.x];
    double r, m;
    asm volatile("v_rsq_f64 %0, %1 div:2" : "=v"(r) : "v"(v));
    asm volatile("v_mul_f64 %0, %1, %2 mul:2" : "=v"(m) : "v"(v), "v"(v));
    out[3 * threadIdx.x + 0] = r;
    out[3 * threadIdx.x + 1] = __builtin_amdgcn_rsq(v);
    out[3 * threadIdx.x + 2] = m;
}
int main()
{
    const int n = 4;
    double hx[n] = {4.0, 2.0, 0.25, 1e10}, *dx, *dout, ho[3 * n];
    hipMalloc(&dx, sizeof hx);
    hipMalloc(&dout, sizeof ho);
    hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
    for (int off = 0; off < 2; ++off) {
        probe<<<1, n>>>(dx, dout, off);
        hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
        for (int i = 0; i < n; ++i)
            printf("ieee_off=%d x=%g rsq_div2=%.17g rsq=%.17g (ratio %.17g) mul2(x*x)=%.17g x*x=%.17g\n", off, hx[i],
                   ho[3 * i], ho[3 * i + 1], ho[3 * i] / ho[3 * i + 1], ho[3 * i + 2], hx[i] * hx[i]);
    }
    return 0;
}
