"""sqrt_rcp_near1 / div_core0 (rt_device_math.h), the sampler's normalize
without v_rsq_f64, checked on the CPU against IEEE sqrt and division.

The functions' own source text is cut out of the header and compiled with
gcc (-ffp-contract=off; fma is the correctly rounded C fma, as v_fma_f64), so
the check runs the code the kernel runs.  This test covers every double
within 2^-30 of 1 (where sqrt(x) is closest to rounding midpoints), a strided
sweep of the whole domain [1 - 2^-18, 1 + 2^-18] and, for every tested x, a
pseudo-random numerator through div_core0 (plus +-0).  tools/check_near1.sh
runs all 5.2e10 doubles of the domain (about 4 minutes on 8 cores)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "tipe-raytracer_amd", "csrc", "rt_device_math.h")


def extract(src, name):
    m = re.search(r"__device__ __forceinline__ (?:void|double) " + name + r"\(.*?\n\}\n", src, re.S)
    assert m, name
    return m.group(0).replace("__device__ __forceinline__", "static inline").replace("double& ", "double* ")


CHECK_C = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
%(funcs)s
static inline double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint64_t ubits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
/* numerator in [-2, 2] from the bits of x (splitmix64) */
static inline double numer(uint64_t u) {
    u += 0x9E3779B97F4A7C15ull; u = (u ^ (u >> 30)) * 0xBF58476D1CE4E5B9ull;
    u = (u ^ (u >> 27)) * 0x94D049BB133111EBull; u ^= u >> 31;
    return ((double)(u >> 11) * 0x1p-53) * 4.0 - 2.0;
}
int main(int argc, char** argv) {
    const double lo = atof(argv[1]), hi = atof(argv[2]);
    const uint64_t stride = strtoull(argv[3], 0, 10);
    long bad_sqrt = 0, bad_div = 0, n = 0;
    for (uint64_t u = ubits(lo); u <= ubits(hi); u += stride) {
        const double x = bits(u);
        double L, rc;
        sqrt_rcp_near1(x, &L, &rc);
        const double Lw = sqrt(x);
        if (L != Lw && bad_sqrt++ < 4) printf("sqrt x=%%a got %%a want %%a\n", x, L, Lw);
        const double a = numer(u);
        const double q = div_core0(a, L, rc), qw = a / L;
        if (memcmp(&q, &qw, 8) != 0 && bad_div++ < 4) printf("div a=%%a L=%%a got %%a want %%a\n", a, L, q, qw);
        if (n == 0) {                                      /* signed zeros keep their sign */
            const double z0 = div_core0(0.0, L, rc), z1 = div_core0(-0.0, L, rc);
            if (signbit(z0) || !signbit(z1) || z0 != 0.0 || z1 != 0.0) ++bad_div;
        }
        ++n;
    }
    printf("n %%ld bad_sqrt %%ld bad_div %%ld\n", n, bad_sqrt, bad_div);
    return 0;
}
"""


def build(tmp_path):
    src = open(HDR).read()
    # the function bodies use references (double& L): rewrite the two
    # assignments through pointers for C
    near1 = extract(src, "sqrt_rcp_near1").replace("\n    L = ", "\n    *L = ").replace("\n    rc = ", "\n    *rc = ")
    near1 = re.sub(r"fma\(-L, y", "fma(-*L, y", near1)
    funcs = near1 + extract(src, "div_core0")
    c = tmp_path / "near1.c"
    c.write_text(CHECK_C % {"funcs": funcs})
    exe = tmp_path / "near1"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    return exe


def run(exe, lo, hi, stride):
    out = subprocess.run([str(exe), repr(lo), repr(hi), str(stride)], capture_output=True, text=True,
                         check=True).stdout
    last = out.strip().splitlines()[-1].split()
    n, bs, bd = int(last[1]), int(last[3]), int(last[5])
    assert bs == 0 and bd == 0, out
    return n


def test_near1_exhaustive_around_one(tmp_path):
    exe = build(tmp_path)
    n = run(exe, 1.0 - 2.0 ** -30, 1.0 + 2.0 ** -30, 1)
    assert n == 2 ** 23 + 2 ** 22 + 1


def test_near1_strided_whole_domain(tmp_path):
    exe = build(tmp_path)
    n = run(exe, 1.0 - 2.0 ** -18, 1.0 + 2.0 ** -18, 1009)
    assert n > 5 * 10 ** 7
