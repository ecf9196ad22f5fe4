"""Regenerate tests/golden/gpu_reference.json FROM THE REFERENCE (container only).

Renders every case of tests/composition_cases.PHILOX_CASES through the
reference's own render composition (main.c:22-284 + denoiser.h:11-29
compiled verbatim) built with the GPU's stream spec in place of glibc rand()
and libm's acos/sinf/cosf/pow (oracle/_ref/libref_tracer_philox.so,
oracle/ref_tracer_stream.h), summing each pixel's samples in the case's
spp_chunks slices.  Records per plane the sha256 of its float64 bytes
(composition_cases.plane_sha: NaN and -0.0 canonical) and the mean.

tests/test_gpu_reference.py then checks librt_hip.so against these hashes
on the GPU box (no oracle in between), and the oracle's PHILOX mode against
them on the CPU.
Usage:  python tests/golden/make_gpu_reference_fixtures.py [case ...]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: E402,F401  (sys.path)
import composition_cases as cc  # noqa: E402

OUT = os.path.join(HERE, "gpu_reference.json")


def main(names):
    try:
        with open(OUT) as f:
            doc = json.load(f)
    except FileNotFoundError:
        doc = {}
    doc["_about"] = ("Outputs of the reference's own main.c:22-284 + denoiser.h:11-29 (compiled verbatim, "
                     "sha256-pinned ranges, oracle/build_ref_tracer.sh philox) with rt.h's RT_RNG_PHILOX stream "
                     "for rand() and pm_math.h's acos/sinf/cosf/pow (oracle/ref_tracer_stream.h), per-pixel "
                     "sums in rt_chunk_bound slices.  Scenes: tests/composition_cases.PHILOX_CASES.  Hash: "
                     "composition_cases.plane_sha.  Generator: tests/golden/make_gpu_reference_fixtures.py.")
    cases = doc.setdefault("cases", {})
    for c in cc.PHILOX_CASES:
        if names and c.name not in names:
            continue
        t = time.time()
        bundle, p = c.scene()
        ref = cc.reference_planes_philox(bundle, p)
        assert ref is not None, "oracle/_ref/libref_tracer_philox.so unavailable (needs /root/reference)"
        cases[c.name] = {"what": c.what, "W": p.largeur_image, "H": p.hauteur_image, "spp": p.nbRayonParPixel,
                         "bounces": p.nbRebondMax, "useAO": int(p.useAO), "AO_intensity": float(p.AO_intensity).hex(),
                         "compat_int_truncation": int(p.compat_int_truncation), "spp_chunks": int(p.spp_chunks),
                         "seed": int(p.seed),
                         "planes": {k: {"sha256": cc.plane_sha(v), "mean": float(v.mean()).hex()}
                                    for k, v in ref.items()}}
        print("%-16s %4dx%-4d spp %3d chunks %3d  %.1fs" % (c.name, p.largeur_image, p.hauteur_image,
                                                         p.nbRayonParPixel, p.spp_chunks, time.time() - t), flush=True)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
