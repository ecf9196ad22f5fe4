"""rt_params.precision (rt.h): FP64 is the only renderable value.

RT_PREC_FP32, an experimental binary32 integrator of rounds 2-4, was removed
in r05: its per-channel RMSE against the FP64 frames (1.1-3.4e-4, measured
in r03-r04) was above north_star's 1e-4.  The value stays reserved and is
refused loudly; the drop-in's precision setter always selects FP64.
"""
import ctypes as C

import tipe_rt
from tipe_rt import types as T


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
    p.precision = T.RT_PREC_FP32
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EUNSUPPORTED
    assert b"removed" in L.rt_last_error()


def test_oracle_refuses_fp32():
    import helpers
    import oracle_ffi
    bundle = helpers.cornell()
    p = helpers.params(8, 6, 1, 5)
    p.precision = T.RT_PREC_FP32
    canva = (C.c_double * (8 * 6 * 3))()
    assert oracle_ffi.oracle().oracle_render_rows(C.byref(bundle.scene), C.byref(p), 5, 0, 1, 1, canva,
                                                  None, None, None, None) == T.RT_EINVAL


def test_fill_precision_setter_refuses_fp32():
    """asking the drop-in for FP32 is an error, not a silent FP64."""
    L = tipe_rt.lib()
    assert L.rt_set_fill_precision(T.RT_PREC_FP32) == T.RT_EUNSUPPORTED
    assert b"removed" in L.rt_last_error()
    assert L.rt_set_fill_precision(9) == T.RT_EINVAL
    assert L.rt_set_fill_precision(T.RT_PREC_FP64) == T.RT_PREC_FP64
