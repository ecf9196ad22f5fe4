// What a kernel-level wavefront split of C4's path kernel
// would pay before doing any work: the path state and the walk queue moved
// through HBM every round.  Two kernels per round, as the split needs:
//   path:  every path slot reads and writes its state (STATE bytes, SoA,
//          coalesced) and appends a 64-byte ray for the WALK_FRAC of slots
//          whose cast enters the tree;
//   walk:  reads the appended rays and writes a 16-byte hit per ray.
// No arithmetic: the time per round is a lower bound on the split's overhead.
// Prints the per-round time and the C4 frame total for the measured casts.
// hipcc --offload-arch=gfx950 -O3 tools/probes/split_traffic.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int STATE_WORDS = 20;         // 160 B of fp64 path state per slot (o, d, inc, rc, best, ...)

__global__ __launch_bounds__(256) void path_kernel(double* __restrict__ st, double4* __restrict__ q,
                                                   unsigned* __restrict__ qn, int n, unsigned walk_mod)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double v[STATE_WORDS];
#pragma unroll
    for (int k = 0; k < STATE_WORDS; ++k) v[k] = st[(size_t)k * n + i];
    double s = 0;
#pragma unroll
    for (int k = 0; k < STATE_WORDS; ++k) s += v[k];
#pragma unroll
    for (int k = 0; k < STATE_WORDS; ++k) st[(size_t)k * n + i] = v[k] + 1.0;
    const bool walk = ((unsigned)i * 2654435761u) % 100u < walk_mod;   // ~WALK_FRAC of the slots
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

int main()
{
    const int n = 1 << 20;                  // path slots in flight (4 per lane of a 256-CU grid)
    const unsigned walk_pct = 21;           // C4: 21 % of casts go below the root
    const double casts_per_frame = 8.752 * 1200.0 * 900.0 * 2000.0;   // BENCH_r03 C4 casts/sample x samples
    double* st;
    double4* q;
    double2* hits;
    unsigned* qn;
    (void)hipMalloc(&st, (size_t)STATE_WORDS * n * sizeof(double));
    (void)hipMalloc(&q, (size_t)2 * n * sizeof(double4));
    (void)hipMalloc(&hits, (size_t)n * sizeof(double2));
    (void)hipMalloc(&qn, sizeof(unsigned));
    (void)hipMemset(st, 0, (size_t)STATE_WORDS * n * sizeof(double));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int rounds = 200;
    for (int pass = 0; pass < 2; ++pass) {
        (void)hipEventRecord(e0);
        for (int r = 0; r < rounds; ++r) {
            (void)hipMemsetAsync(qn, 0, sizeof(unsigned));
            hipLaunchKernelGGL(path_kernel, dim3(n / 256), dim3(256), 0, 0, st, q, qn, n, walk_pct);
            hipLaunchKernelGGL(walk_kernel, dim3(n / 256), dim3(256), 0, 0, q, qn, hits);
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (pass == 0) continue;            // warm-up pass
        const double us = ms * 1e3 / rounds;
        const double bytes = (double)n * (2.0 * STATE_WORDS * 8) + n * walk_pct / 100.0 * (64.0 * 2 + 16.0);
        const double frame_s = casts_per_frame / n * us * 1e-6;
        printf("{\"path_slots\": %d, \"state_bytes\": %d, \"walk_frac\": %.2f, \"us_per_round\": %.2f, "
               "\"GBps\": %.0f, \"rounds_per_C4_frame\": %.0f, \"C4_frame_overhead_s\": %.3f}\n",
               n, STATE_WORDS * 8, walk_pct / 100.0, us, bytes / (us * 1e-6) / 1e9, casts_per_frame / n, frame_s);
    }
    return 0;
}
