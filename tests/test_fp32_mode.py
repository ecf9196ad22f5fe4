"""rt_params.precision = RT_PREC_FP32 (rt.h): the integrator in binary32.

This mode is NOT bit-exact.  It makes the same Philox draws in the same order
as the fp64 path, so most paths follow the fp64 path up to float rounding, and
a path diverges only where a float decision (hit/miss, nearest surface,
refraction draw against alpha) comes out differently.  The bar here is the
fp64 image from the bit-exact kernel, which the parity suite pins to the
oracle.  Measured (r02): image means and per-pixel MAE agree within 1e-3
(sky scene; 0 to 5e-5 elsewhere), >= 99.5 % of canva values identical, none
more than 16 levels apart except 0.02 % on the sky scene.  The tolerances:
  * per-channel image means of pre-gamma radiance within REL_MEAN (relative);
  * per-pixel mean absolute radiance difference within REL_MAE of the mean;
  * at most CANVA_FRAC of the 8-bit canva values more than CANVA_LEVELS apart.
The fp64 oracle refuses precision FP32 (it restates fp64 only).
"""
import ctypes as C

import numpy as np
import pytest

import helpers
import tipe_rt
from tipe_rt import types as T

REL_MEAN = 0.005
REL_MAE = 0.005
CANVA_LEVELS = 16
CANVA_FRAC = 0.002


def test_precision_validation_without_device():
    L = tipe_rt.lib()
    sc = T.Scene()
    p = T.Params()
    L.rt_params_init(C.byref(p))
    assert p.precision == T.RT_PREC_FP64
    p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax = 8, 6, 1, 5
    buf = (C.c_double * (8 * 6 * 3))()
    p.precision = 7
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EINVAL
    p.precision, p.semantics = T.RT_PREC_FP32, T.RT_SEM_CUDA
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EUNSUPPORTED


def test_oracle_refuses_fp32():
    p = helpers.params(8, 6, 1, 2)
    p.precision = T.RT_PREC_FP32
    with pytest.raises(AssertionError):
        helpers.oracle_render(helpers.cornell(), p)


def _gpu_render(bundle, p):
    from test_gpu_parity import gpu_render
    return gpu_render(bundle, p)


def _mineways():
    tris, qm, mats, tw, th, nm = tipe_rt.scenes.load_mesh_fixture("mineways")
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0] = P.e[0] * 0.1 - 0.2
            P.e[1] = P.e[1] * 0.1 - 1.0
            P.e[2] = P.e[2] * 0.1 - 2.5
    return helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), (tris, qm, mats, tw, th, nm))


CASES = {
    "cornell": lambda: (helpers.cornell(), helpers.params(96, 72, 64, 6, chunks=4)),
    "cornell_ao": lambda: (helpers.cornell(), helpers.params(64, 48, 32, 6, use_ao=True)),
    "pyramid": lambda: (helpers.pyramid_scene(), helpers.params(64, 48, 32, 6)),
    "mineways": lambda: (_mineways(), helpers.params(48, 36, 16, 6)),
    "tree_ao": lambda: (helpers.tree_scene(), helpers.params(48, 36, 16, 8, use_ao=True)),
    "sky": lambda: (helpers.sky_scene(), helpers.params(48, 36, 16, 5, sky_mode=1)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_fp32_close_to_fp64(name):
    bundle, p = CASES[name]()
    c64, _, _, r64 = _gpu_render(bundle, p)
    p.precision = T.RT_PREC_FP32
    c32, a32, n32, r32 = _gpu_render(bundle, p)
    for b in (c32, a32, n32, r32):
        assert (b != -1.0).any(), "fp32 kernel wrote nothing"
    assert (np.isfinite(r32) == np.isfinite(r64)).all(), "fp32 produced NaN/inf where fp64 did not (or vice versa)"
    r64, r32 = np.nan_to_num(r64), np.nan_to_num(r32)
    m64 = r64.reshape(-1, 3).mean(0)
    m32 = r32.reshape(-1, 3).mean(0)
    mae = np.abs(r32 - r64).reshape(-1, 3).mean(0)
    far = float((np.abs(c32 - c64) > CANVA_LEVELS).mean())
    scale = np.maximum(m64, 1e-3)
    print("fp32 %s: rel mean %s, rel mae %s, canva far %.5f, identical canva %.4f" %
          (name, np.round(np.abs(m32 - m64) / scale, 5), np.round(mae / scale, 5), far, float((c32 == c64).mean())))
    assert (np.abs(m32 - m64) <= REL_MEAN * scale).all()
    assert (mae <= REL_MAE * scale).all()
    assert far <= CANVA_FRAC


# north_star's gate: "within 1e-4 per-channel RMSE" of main.c's image on
# identical seeds.  Here: per-channel RMSE over the full C2 / C3 frame of the
# pre-gamma radiance (sum / S) and of canva / 255, FP32 kernel against the
# ORACLE's fp64 image.  Measured r03 (16 / 8 spp): see DESIGN.md §4d -- the
# FP32 mode does NOT meet 1e-4 (a path whose float decision differs from fp64
# diverges completely, so the error is Monte-Carlo noise of the diverged
# samples, ~sigma * sqrt(f / S)).  The assertion bounds it at RMSE_FP32_MAX,
# so a regression shows; the fp64 default is bit-exact (RMSE 0).
RMSE_FP32_MAX = 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C2", "C3"])
def test_fp32_rmse_vs_oracle(name):
    import os
    bundle, p = {"C2": lambda: (helpers.cornell(), helpers.params(1200, 900, 16, 6, chunks=4)),
                 "C3": lambda: (helpers.pyramid_scene(), helpers.params(1200, 900, 8, 6, chunks=4))}[name]()
    ref = helpers.oracle_render(bundle, p, nthreads=max(1, min(16, os.cpu_count() or 1)))
    p.precision = T.RT_PREC_FP32
    c32, _, _, r32 = _gpu_render(bundle, p)
    assert (np.isfinite(r32) == np.isfinite(ref["radiance"])).all()
    rad = helpers.rmse_per_channel(r32, ref["radiance"])
    can = helpers.rmse_per_channel(c32 / 255.0, ref["canva"] / 255.0)
    print("fp32 %s vs oracle fp64: radiance RMSE %s, canva/255 RMSE %s (north_star gate 1e-4)" %
          (name, np.array2string(rad, precision=6), np.array2string(can, precision=6)))
    assert (rad <= RMSE_FP32_MAX).all() and (can <= RMSE_FP32_MAX).all()


def test_fill_precision_setter_round_trip():
    L = tipe_rt.lib()
    assert L.rt_set_fill_precision(T.RT_PREC_FP32) == T.RT_PREC_FP64
    assert L.rt_set_fill_precision(5) == T.RT_PREC_FP32          # invalid selects FP64
    assert L.rt_set_fill_precision(T.RT_PREC_FP64) == T.RT_PREC_FP64


@pytest.mark.gpu
def test_fill_canva_fp32_close_to_fp64():
    """main.c's drop-in (rt_fill_canva, 3 pthreads over row bands) with
    rt_set_fill_precision(RT_PREC_FP32), against the same drop-in in FP64."""
    import threading
    from tipe_rt.types import ThreadData, Sphere
    bundle = helpers.cornell()
    W, H, S, B = 48, 36, 16, 5
    p = helpers.params(W, H, S, B)
    L = tipe_rt.lib()

    def fill():
        canva = np.zeros((H, W, 3))
        tds = []
        for hi, lo in [(35, 24), (23, 12), (11, 0)]:
            td = ThreadData()
            td.start_row, td.end_row = hi, lo
            td.canva = C.cast(canva.ctypes.data, C.POINTER(tipe_rt.Vec3))
            td.cam = p.cam
            td.largeur_image, td.hauteur_image = W, H
            td.nbRayonParPixel, td.nbRebondMax = S, B
            td.total_pixels = W * H
            td.sphere_list = C.cast(bundle.spheres, C.POINTER(Sphere))
            td.nbSpheres = len(bundle.spheres)
            td.focus_distance = 3
            tds.append(td)
        res = []
        ths = [threading.Thread(target=lambda t=t: res.append(L.rt_fill_canva(C.byref(t)))) for t in tds]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(r is None for r in res), L.rt_last_error()
        return canva

    c64 = fill()
    prev = L.rt_set_fill_precision(T.RT_PREC_FP32)
    try:
        c32 = fill()
    finally:
        L.rt_set_fill_precision(prev)
    assert c64.max() > 0
    assert float((np.abs(c32 - c64) > CANVA_LEVELS).mean()) <= CANVA_FRAC
    assert abs(c32.mean() - c64.mean()) <= REL_MEAN * c64.mean()
