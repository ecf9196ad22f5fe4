"""The oracle's COMPOSITION pinned to the reference's own code.

oracle/build_ref_tracer.sh compiles main.c:22-284 (closest_hit,
ambient_occlusion, tracer, fill_canva) and denoiser.h:11-29 verbatim from
/root/reference, sha256-checked, with the reference's leaf headers and no
stub; tests/golden/make_composition_fixtures.py recorded its outputs in
tests/golden/composition.json.  Here the oracle (oracle/rt_oracle.c, GLIBC
stream mode: glibc rand() after srand(1), libm, one thread) must reproduce
every plane of every case bit for bit:

* README box (config 1 in full, + AO at int 2 and at 2.5),
* translucent spheres (refraction + IOR stack enter/exit),
* alpha-hole spheres + AO (alpha_depth bookkeeping),
* the C3 pyramid (texture + refraction, with and without AO),
* mineways (alpha-hole texels),
* the C4 tree + AO (int-truncated 2 via ThreadData, and 2.5),
* 12 enclosed random scenes (aperture, focus, AO, textured meshes with the
  texture.h:71-87 material overrides).

With /root/reference present the live tests also render fresh random
scenes through the compiled reference and the oracle side by side.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import composition_cases as cc
import oracle_ffi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "composition.json")
with open(GOLDEN) as f:
    FIX = json.load(f)["cases"]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).astype("<f8").tobytes()).hexdigest()


def _params(cases):
    return [pytest.param(c.name, marks=pytest.mark.slow) if c.slow else c.name for c in cases]


def test_fixture_covers_every_case():
    assert sorted(FIX) == sorted(c.name for c in cc.CASES)
    assert FIX["c1_full"]["ppm_md5"] == "930550ea86f4b2de4ac3a92726beb976"   # SURVEY.md §6, now reproduced
    for name, rec in FIX.items():
        assert set(rec["planes"]) == set(cc.PLANES), name


@pytest.mark.parametrize("name", _params(cc.CASES))
def test_oracle_matches_reference_composition(name):
    c = cc.BY_NAME[name]
    rec = FIX[name]
    out = cc.oracle_planes(c)
    _, p = c.scene()
    assert (p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax) == \
        (rec["W"], rec["H"], rec["spp"], rec["bounces"])
    assert float(p.AO_intensity).hex() == rec["AO_intensity"] and int(p.useAO) == rec["useAO"]
    for k in cc.PLANES:
        assert _sha(out[k]) == rec["planes"][k]["sha256"], \
            "%s/%s: oracle mean %s vs reference %s" % (name, k, float(out[k].mean()).hex(), rec["planes"][k]["mean"])
    if "ppm_md5" in rec:
        import helpers
        assert helpers.ppm_md5(out["canva"]) == rec["ppm_md5"]


def _ref_or_skip():
    lib = oracle_ffi.ref_tracer()
    if lib is None:
        pytest.skip("oracle/_ref/libref_tracer.so needs /root/reference (container only)")
    return lib


def test_ref_tracer_recipe_pins_the_ranges():
    """The build refuses a reference whose ranges changed; check the pinned
    hashes against the tree that is here."""
    _ref_or_skip()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "oracle", "ref_tracer.sha256")) as f:
        pins = dict(reversed(line.split()) for line in f if line.strip())
    for key, want in pins.items():
        fname, rng = key.split(":")
        a, b = (int(x) for x in rng.split("-"))
        with open(os.path.join("/root/reference", fname), "rb") as f:
            lines = f.read().split(b"\n")
        text = b"\n".join(lines[a - 1:b]) + b"\n"
        assert hashlib.sha256(text).hexdigest() == want, key


@pytest.mark.parametrize("seed", range(300, 316))
def test_live_reference_vs_oracle_random(seed):
    """Fresh random scenes (not in the fixture) through the compiled
    reference and the oracle, all four planes bit for bit."""
    _ref_or_skip()
    c = cc.Case("live_%d" % seed, cc._random(seed), 0, 0, 0, 0)
    ref = cc.reference_planes(c)
    out = cc.oracle_planes(c)
    for k in cc.PLANES:
        assert ref[k].tobytes() == out[k].tobytes(), k


@pytest.mark.parametrize("name", ["cornell_ao_int2", "hole_spheres", "pyramid_ao_int2"])
def test_live_reference_fill_canva_vs_oracle(name):
    """The reference's fill_canva itself (ThreadData, one pthread) against the
    oracle, live; reference_planes also asserts trace_rows == fill_canva."""
    _ref_or_skip()
    c = cc.BY_NAME[name]
    ref = cc.reference_planes(c)
    out = cc.oracle_planes(c)
    for k in cc.PLANES:
        assert ref[k].tobytes() == out[k].tobytes(), k
