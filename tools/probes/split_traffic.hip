// What a kernel-level wavefront split of C4's path kernel
// would pay before doing any work: the path state and the walk queue moved
// through memory every round.  Two kernels per round, as the split needs:
//   path:  every path slot reads and writes its state (SW fp64 words, SoA,
//          coalesced) and appends a 64-byte ray for the walk_pct % of slots
//          whose cast goes to the walk kernel;
//   walk:  reads the appended rays and writes a 16-byte hit per ray.
// No arithmetic: the time per round is a lower bound on the split's overhead
// (state traffic + the two kernel boundaries per round).  Swept over the slot
// count n (256 Ki: state resident in the 256 MB MALL; 2 Mi: enough walk rays
// to fill 8 waves/SIMD when every cast walks), the state size (21 words =
// 168 B, the smallest bit-exact C4 path state: o, d, cd, inc, rc, top_n2 and
// 16 B of counters / draw-cache / task words; 12 words: a lower bound that
// drops cd and packs the rest) and the walk fraction (21 %: casts that go
// below the root; 100 %: the walk kernel also does the root visit).
// Prints one JSON line per point with the C4 frame total for its measured
// casts (BENCH r04 configs.C4: 8.752 casts/sample, 1200x900x2000 samples).
// hipcc --offload-arch=gfx950 -O3 -o tools/probes/split_traffic tools/probes/split_traffic.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int SW>
__global__ __launch_bounds__(256) void path_kernel(double* __restrict__ st, double4* __restrict__ q,
                                                   unsigned* __restrict__ qn, int n, unsigned walk_pct)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double v[SW];
#pragma unroll
    for (int k = 0; k < SW; ++k) v[k] = st[(size_t)k * n + i];
    double s = 0;
#pragma unroll
    for (int k = 0; k < SW; ++k) s += v[k];
#pragma unroll
    for (int k = 0; k < SW; ++k) st[(size_t)k * n + i] = v[k] + 1.0;
    const bool walk = ((unsigned)i * 2654435761u) % 100u < walk_pct;
    const unsigned long long m = __ballot(walk);                          // one atomic per wave
    const int lane = threadIdx.x & 63, lead = __ffsll((long long)m) - 1;
    unsigned base = 0;
    if (m && lane == lead) base = atomicAdd(qn, (unsigned)__popcll(m));
    base = __shfl(base, lead < 0 ? 0 : lead, 64);
    if (walk) {
        const unsigned slot = base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
        q[2 * (size_t)slot] = make_double4(s, v[0], v[1], v[2]);
        q[2 * (size_t)slot + 1] = make_double4(v[3], v[4], v[5], (double)i);
    }
}

__global__ __launch_bounds__(256) void walk_kernel(const double4* __restrict__ q, const unsigned* __restrict__ qn,
                                                   double2* __restrict__ hits)
{
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i >= *qn) return;
    const double4 a = q[2 * (size_t)i], b = q[2 * (size_t)i + 1];
    hits[i] = make_double2(a.x + b.x, a.y + b.w);
}

template <int SW>
static void point(int n, unsigned walk_pct, double* st, double4* q, double2* hits, unsigned* qn, hipEvent_t e0,
                  hipEvent_t e1)
{
    const double casts_per_frame = 8.752 * 1200.0 * 900.0 * 2000.0;
    const int rounds = 200;
    float ms = 0;
    for (int pass = 0; pass < 2; ++pass) {               // pass 0 warms up
        (void)hipEventRecord(e0);
        for (int r = 0; r < rounds; ++r) {
            (void)hipMemsetAsync(qn, 0, sizeof(unsigned));
            hipLaunchKernelGGL(path_kernel<SW>, dim3(n / 256), dim3(256), 0, 0, st, q, qn, n, walk_pct);
            hipLaunchKernelGGL(walk_kernel, dim3(n / 256), dim3(256), 0, 0, q, qn, hits);
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double us = ms * 1e3 / rounds;
    const double bytes = (double)n * (2.0 * SW * 8) + n * walk_pct / 100.0 * (64.0 * 2 + 16.0 * 2);
    const double frame_s = casts_per_frame / n * us * 1e-6;
    printf("{\"path_slots\": %d, \"state_bytes\": %d, \"walk_pct\": %u, \"us_per_round\": %.2f, "
           "\"bytes_per_round\": %.0f, \"GBps\": %.0f, \"rounds_per_C4_frame\": %.0f, \"C4_frame_overhead_s\": %.3f}\n",
           n, SW * 8, walk_pct, us, bytes, bytes / (us * 1e-6) / 1e9, casts_per_frame / n, frame_s);
    fflush(stdout);
}

int main()
{
    const int nmax = 1 << 21;
    double* st;
    double4* q;
    double2* hits;
    unsigned* qn;
    if (hipMalloc(&st, (size_t)21 * nmax * sizeof(double)) != hipSuccess ||
        hipMalloc(&q, (size_t)2 * nmax * sizeof(double4)) != hipSuccess ||
        hipMalloc(&hits, (size_t)nmax * sizeof(double2)) != hipSuccess || hipMalloc(&qn, sizeof(unsigned)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    (void)hipMemset(st, 0, (size_t)21 * nmax * sizeof(double));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int n = 1 << 18; n <= nmax; n <<= 1)
        for (unsigned w : {21u, 100u}) {
            point<21>(n, w, st, q, hits, qn, e0, e1);
            point<12>(n, w, st, q, hits, qn, e0, e1);
        }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
