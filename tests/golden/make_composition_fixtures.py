"""Regenerate tests/golden/composition.json FROM THE REFERENCE (container only).

Renders every case of tests/composition_cases.py through the reference's own
render composition — main.c:22-284 + denoiser.h:11-29 compiled verbatim into
oracle/_ref/libref_tracer.so by oracle/build_ref_tracer.sh — in the
reference's stream mode (glibc rand() after srand(1), libm, one thread) and
records, per output plane, the sha256 of its float64 bytes ((H, W, 3),
C order, little endian) plus the plane's mean as float.hex.  For the
config-1 case it also records the md5 of the P3 file main.c:457-465 writes.

Nothing here uses the oracle: the fixture is the reference's output only.
Usage:  python tests/golden/make_composition_fixtures.py [case ...]
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: E402,F401  (sys.path)
import composition_cases as cc  # noqa: E402
import helpers  # noqa: E402

OUT = os.path.join(HERE, "composition.json")


def plane_record(a):
    return {"sha256": hashlib.sha256(a.astype("<f8").tobytes()).hexdigest(), "mean": float(a.mean()).hex()}


def main(names):
    try:
        with open(OUT) as f:
            doc = json.load(f)
    except FileNotFoundError:
        doc = {}
    doc["_about"] = ("Outputs of the reference's own main.c:22-284 + denoiser.h:11-29 (compiled verbatim, "
                     "oracle/build_ref_tracer.sh; sha256 of the ranges in oracle/ref_tracer.sha256), glibc "
                     "rand() after srand(1), one thread.  Scenes: tests/composition_cases.py.  Generator: "
                     "tests/golden/make_composition_fixtures.py.")
    cases = doc.setdefault("cases", {})
    for c in cc.CASES:
        if names and c.name not in names:
            continue
        t = time.time()
        ref = cc.reference_planes(c)
        assert ref is not None, "oracle/_ref/libref_tracer.so unavailable (needs /root/reference)"
        _, p = c.scene()
        rec = {"what": c.what, "driver": c.driver, "W": p.largeur_image, "H": p.hauteur_image,
               "spp": p.nbRayonParPixel, "bounces": p.nbRebondMax, "useAO": int(p.useAO),
               "AO_intensity": float(p.AO_intensity).hex(), "compat_int_truncation": int(p.compat_int_truncation),
               "planes": {k: plane_record(v) for k, v in ref.items()}}
        if c.name == "c1_full":
            rec["ppm_md5"] = helpers.ppm_md5(ref["canva"])
        cases[c.name] = rec
        print("%-16s %-10s %4dx%-4d spp %4d  %.1fs" % (c.name, c.driver, p.largeur_image, p.hauteur_image,
                                                    p.nbRayonParPixel, time.time() - t), flush=True)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
