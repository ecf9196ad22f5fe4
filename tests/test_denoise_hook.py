"""Denoiser boundary: the hook with denoiser()'s signature
(denoiser.h:31) that rt_render_rows runs on a finished frame (main.c:455),
and the OIDN "RT" buffer formats either side of it (denoiser.h:44-60,
80-84).  Host conversions and hook plumbing run without a GPU; the device
pack and the end-to-end call are gpu-marked."""
import ctypes as C

import numpy as np
import pytest

import helpers
import tipe_rt


def reference_pack(canva, albedo, normal):
    """denoiser.h:44-60: (float)canva / 255.0f, (float)albedo, (float)normal."""
    return (canva.astype(np.float32) / np.float32(255.0), albedo.astype(np.float32), normal.astype(np.float32))


def reference_unpack(color3):
    """denoiser.h:80-84: canva = (int)(f * 255.0f), stored in a double."""
    return np.trunc(color3.astype(np.float32) * np.float32(255.0)).astype(np.int64).astype(np.float64)


def frames(H=7, W=9, seed=0):
    rng = np.random.default_rng(seed)
    canva = rng.integers(0, 256, (H, W, 3)).astype(np.float64)
    albedo = rng.uniform(0, 1, (H, W, 3))
    normal = rng.uniform(-1, 1, (H, W, 3))
    return canva, albedo, normal


def test_pack_matches_denoiser_h():
    canva, albedo, normal = frames()
    got = tipe_rt.denoise_pack(canva, albedo, normal)
    for g, w in zip(got, reference_pack(canva, albedo, normal)):
        assert (g.view(np.uint32) == w.view(np.uint32)).all()


def test_unpack_matches_denoiser_h_including_edges():
    rng = np.random.default_rng(1)
    c3 = rng.uniform(-0.1, 1.1, (5, 6, 3)).astype(np.float32)
    c3[0, 0] = [1.0, 0.0, np.float32(254.999) / np.float32(255.0)]
    assert (tipe_rt.denoise_unpack(c3) == reference_unpack(c3)).all()


def test_round_trip_of_an_identity_denoiser_keeps_the_image():
    canva, albedo, normal = frames(seed=2)
    c3, _, _ = tipe_rt.denoise_pack(canva, albedo, normal)
    back = tipe_rt.denoise_unpack(c3)
    assert np.abs(back - canva).max() <= 1.0     # (int) truncation of x/255*255


def test_hook_install_and_clear():
    seen = []
    tipe_rt.set_denoise_hook(lambda *a: seen.append(a))
    try:
        assert tipe_rt.lib().rt_get_denoise_hook()
    finally:
        tipe_rt.set_denoise_hook(None)
    assert not tipe_rt.lib().rt_get_denoise_hook()


@pytest.mark.gpu
def test_render_rows_calls_the_hook_on_the_full_frame():
    bundle = helpers.cornell()
    W, H = 24, 18
    p = helpers.params(W, H, 2, 4)
    calls = []

    def hook(w, h, canva_p, cam, alb_p, nrm_p):
        n = w * h * 3
        get = lambda ptr: np.ctypeslib.as_array((C.c_double * n).from_address(ptr)).copy().reshape(h, w, 3)  # noqa
        calls.append((w, h, get(canva_p), cam.origin.tolist(), get(alb_p), get(nrm_p)))

    canva, alb, nrm = (np.zeros((H, W, 3)) for _ in range(3))
    tipe_rt.set_denoise_hook(hook)
    try:
        tipe_rt.check(tipe_rt.lib().rt_render_rows(C.byref(bundle.scene), C.byref(p), H - 1, 0, canva.ctypes.data,
                                                   alb.ctypes.data, nrm.ctypes.data))
        # a band does not trigger it (fill_canva threads never call denoiser)
        tipe_rt.check(tipe_rt.lib().rt_render_rows(C.byref(bundle.scene), C.byref(p), 9, 0, canva.ctypes.data,
                                                   alb.ctypes.data, nrm.ctypes.data))
    finally:
        tipe_rt.set_denoise_hook(None)
    assert len(calls) == 1
    w, h, c, origin, a, n = calls[0]
    assert (w, h) == (W, H) and origin == p.cam.origin.tolist()
    assert (c == canva).all() and (a == alb).all() and (n == nrm).all()


@pytest.mark.gpu
def test_device_pack_matches_host_pack():
    import torch
    canva, albedo, normal = frames(H=33, W=41, seed=3)
    dev = torch.device("cuda:0")
    planes = [torch.from_numpy(x).to(dev) for x in (canva, albedo, normal)]
    outs = [torch.zeros((33, 41, 3), dtype=torch.float32, device=dev) for _ in range(3)]
    fr = tipe_rt.types.Frame()
    fr.canva, fr.albedo, fr.normal = (t.data_ptr() for t in planes)
    tipe_rt.check(tipe_rt.lib().rt_denoise_pack_async(41, 33, C.byref(fr), outs[0].data_ptr(), outs[1].data_ptr(),
                                                      outs[2].data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    for g, w in zip(outs, reference_pack(canva, albedo, normal)):
        assert (g.cpu().numpy().view(np.uint32) == w.view(np.uint32)).all()
