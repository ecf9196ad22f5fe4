"""librt_hip.so against the REFERENCE's own code, with no oracle in between.

tests/golden/gpu_reference.json holds the frames of main.c:22-284 +
denoiser.h:11-29 compiled verbatim (sha256-pinned ranges) with the GPU's
stream spec in place of the reference's two external dependencies -- glibc
rand() -> rt.h's RT_RNG_PHILOX draws, libm acos/sinf/cosf/pow -> the portable
pm_math.h functions the kernel implements (oracle/ref_tracer_stream.h) -- and
each pixel's samples summed in the case's spp_chunks slices.  The reference's
tracer, closest_hit, ambient_occlusion, hit tests, texturing, IOR stack and
shading are its own compiled code; only the random numbers and four
transcendentals are the kernel's.

* -m gpu: the kernel's canva / albedo / normal / radiance hash to the
  reference's, bit for bit (NaN payloads and zero signs canonical), over the
  C2 / C3 / C4 scenes on the queue and fixed-grid kernels, translucent and
  alpha-hole spheres, mineways' alpha texels and 16 random scenes;
* CPU: the oracle's PHILOX mode reproduces the same hashes, and with
  /root/reference present the compiled reference and the oracle agree on
  fresh random scenes too.
"""
import json
import os

import numpy as np
import pytest

import composition_cases as cc
import helpers
import oracle_ffi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gpu_reference.json")
with open(GOLDEN) as f:
    FIX = json.load(f)["cases"]

NAMES = [c.name for c in cc.PHILOX_CASES]


def _check(name, planes):
    rec = FIX[name]
    for k in cc.PLANES:
        got = cc.plane_sha(planes[k])
        assert got == rec["planes"][k]["sha256"], \
            "%s/%s: mean %s vs the reference's %s" % (name, k, float(np.nanmean(planes[k])).hex(),
                                                      rec["planes"][k]["mean"])


def _scene(name):
    bundle, p = cc.PHILOX_BY_NAME[name].scene()
    rec = FIX[name]
    assert (p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax, p.spp_chunks, p.seed) == \
        (rec["W"], rec["H"], rec["spp"], rec["bounces"], rec["spp_chunks"], rec["seed"])
    return bundle, p


def test_fixture_covers_every_case():
    assert sorted(FIX) == sorted(NAMES)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_reference_code(name):
    from test_gpu_parity import gpu_render
    bundle, p = _scene(name)
    canva, alb, nrm, rad = gpu_render(bundle, p)
    _check(name, dict(canva=canva, albedo=alb, normal=nrm, radiance=rad))
    want = cc.PHILOX_BY_NAME[name].kernel
    if want is not None:
        import tipe_rt
        assert tipe_rt.last_render_kernel() == want


@pytest.mark.parametrize("name", NAMES)
def test_oracle_philox_matches_reference_code(name):
    bundle, p = _scene(name)
    _check(name, helpers.oracle_render(bundle, p))


@pytest.mark.parametrize("seed", range(600, 612))
def test_live_reference_philox_vs_oracle(seed):
    if oracle_ffi.ref_tracer_philox() is None:
        pytest.skip("oracle/_ref/libref_tracer_philox.so needs /root/reference (container only)")
    bundle, p = cc._random(seed)()
    ref = cc.reference_planes_philox(bundle, p)
    out = helpers.oracle_render(bundle, p)
    for k in cc.PLANES:
        assert cc.plane_sha(ref[k]) == cc.plane_sha(out[k]), k
