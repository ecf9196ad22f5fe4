/*
 * oracle/ref_tracer_stream.h — TEST INFRASTRUCTURE (container only).
 *
 * Included by oracle/build_ref_tracer.sh's `philox` variant after the system
 * headers and BEFORE the reference's headers: the reference's two external
 * dependencies on the render path are swapped for the GPU's stream spec
 * (rt.h RT_RNG_PHILOX) by object-like macros, so the
 * reference's own code (main.c:22-284 and the leaf headers, compiled
 * verbatim) draws exactly what librt_hip.so draws:
 *
 *   rand()            rtutility.h:192-193,230 -> ref_stream_rand(): word
 *                     (n & 3) of Philox4x32-10(counter {n >> 2, 0, pixel,
 *                     sample}, key = seed) >> 1, n = draws so far in the sample
 *   acos              rtutility.h:196         -> pm_acos
 *   sinf, cosf        rtutility.h:198-200     -> pm_sinf, pm_cosf
 *   pow               main.c:109              -> pm_pow
 *
 * sqrt / sqrtf / fmod are correctly rounded in libm and on the device alike,
 * and tan (camera.h:25) only runs in init_camera on the host.  The driver
 * (ref_trace_rows_philox) sets ref_ps.pixel / .sample / .n before each sample.
 */
#ifndef REF_TRACER_STREAM_H
#define REF_TRACER_STREAM_H

#include <stdint.h>

#include "pm_math.h"
#include "../include/rt/rt.h"

static struct {
    uint64_t seed;
    uint32_t pixel, sample, n;
    uint32_t block[4];
} ref_ps;

static inline int ref_stream_rand(void)
{
    if ((ref_ps.n & 3u) == 0u) {
        const uint32_t ctr[4] = {ref_ps.n >> 2, 0u, ref_ps.pixel, ref_ps.sample};
        const uint32_t key[2] = {(uint32_t)ref_ps.seed, (uint32_t)(ref_ps.seed >> 32)};
        pm_philox4x32_10(ctr, key, ref_ps.block);
    }
    const uint32_t w = ref_ps.block[ref_ps.n & 3u];
    ref_ps.n++;
    return (int)(w >> 1);
}

#define rand() ref_stream_rand()
#define acos pm_acos
#define sinf pm_sinf
#define cosf pm_cosf
#define pow pm_pow

#endif
