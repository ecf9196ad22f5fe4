#!/usr/bin/env bash
# oracle/build_ref_tracer.sh — TEST INFRASTRUCTURE (container only).
#
# Compiles the reference's own render composition — main.c:22-284 (ThreadData,
# closest_hit, ambient_occlusion, tracer, fill_canva) and denoiser.h:11-29
# (col_alb_norm, can_create, add_col_alb_norm) — VERBATIM from where they lie
# under $REFROOT, with the reference's leaf headers in main.c's include order,
# into oracle/_ref/libref_tracer.so.  See ref_tracer_harness.c for the layout
# of the translation unit.
#
# * Nothing is stubbed.  main.c:9 (<OpenImageDenoise/oidn.h>), main()
#   (main.c:286-498) and denoiser() (denoiser.h:31-91) are outside the ranges;
#   the render path calls none of them.
# * Each range's sha256 must equal the value in oracle/ref_tracer.sha256, else
#   the build refuses (a different reference revision needs a new review).
# * The TU is streamed to gcc on stdin: no copy of the reference text is
#   written anywhere.  #line directives keep diagnostics pointing at the
#   reference's own files and lines.
# * Flags: the reference Makefile's (gcc -O3; Makefile:2) + -fPIC -shared.
set -euo pipefail

HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REFROOT="${REFROOT:-/root/reference}"
CC="${CC:-gcc}"
OUT="$HERE/_ref/libref_tracer.so"
VARIANT="${1:-glibc}"            # glibc (the reference as shipped) | philox (the GPU's stream spec)
if [ "$VARIANT" = philox ]; then
    OUT="$HERE/_ref/libref_tracer_philox.so"
fi

if [ ! -f "$REFROOT/main.c" ] || [ ! -f "$REFROOT/denoiser.h" ]; then
    echo "build_ref_tracer: $REFROOT absent, skipping" >&2
    exit 0
fi

range() {  # file first last
    sed -n "${2},${3}p" "$REFROOT/$1"
}

check() {  # file first last
    local want got
    want="$(awk -v k="$1:$2-$3" '$2 == k { print $1 }' "$HERE/ref_tracer.sha256")"
    got="$(range "$1" "$2" "$3" | sha256sum | cut -d' ' -f1)"
    if [ -z "$want" ] || [ "$want" != "$got" ]; then
        echo "build_ref_tracer: $1:$2-$3 sha256 $got does not match the pinned '$want'; refusing" >&2
        exit 1
    fi
}

check denoiser.h 11 29
check main.c 22 284

mkdir -p "$HERE/_ref"
{
    printf '#include <stdio.h>\n#include <math.h>\n#include <stdbool.h>\n#include <stdlib.h>\n'
    printf '#include <time.h>\n#include <sys/time.h>\n#include <pthread.h>\n#include <string.h>\n'
    if [ "$VARIANT" = philox ]; then
        # rand() -> rt.h's RT_RNG_PHILOX draw; acos/sinf/cosf/pow -> pm_math.h
        printf '#define REF_STREAM_PHILOX 1\n#include "ref_tracer_stream.h"\n'
    fi
    printf '#include "vec3.h"\n#include "ray.h"\n#include "hitinfo.h"\n#include "sphere.h"\n'
    printf '#include "rtutility.h"\n#include "camera.h"\n'
    printf '#line 11 "%s/denoiser.h"\n' "$REFROOT"
    range denoiser.h 11 29
    printf '#include "mesh.h"\n#include "texture.h"\n#include "pile.h"\n'
    printf '#line 22 "%s/main.c"\n' "$REFROOT"
    range main.c 22 284
    printf '#line 1 "%s/ref_tracer_harness.c"\n#include "ref_tracer_harness.c"\n' "$HERE"
} | "$CC" -O3 -fPIC -shared -w -fvisibility=hidden -Wl,-Bsymbolic -I"$REFROOT" -I"$HERE" -x c - \
        -o "$OUT" -lm -lpthread
echo "build_ref_tracer: built $OUT"
