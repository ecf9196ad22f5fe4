"""Device-resident multi-device frames and process exit.

rt_render_gather_async renders the cyclic row tiles of a frame on every
device slot of rt_init's list, gathers the slots' planes onto the first
device with peer copies (xGMI between distinct GPUs) and un-permutes them
with the assemble kernel -- the device-destination replacement of
main_cuda.cu:280-339.  The one-GPU box runs several slots on GPU 0 (the
peer copy is then a device-local copy); the images must equal the oracle's
bit for bit, since the Philox stream is keyed by the global pixel.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import helpers
import tipe_rt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _slots(n):
    lib = tipe_rt.lib()
    tipe_rt.check(lib.rt_init(n, (C.c_int * n)(*([0] * n))))
    return lib


@pytest.mark.parametrize("slots,tile_rows,chunks", [(2, 1, 4), (3, 4, 1), (2, 2, 1)])
def test_render_gather_slots_bitexact(slots, tile_rows, chunks):
    import torch
    lib = _slots(slots)
    try:
        bundle = helpers.pyramid_scene()
        W, H = 52, 41
        p = helpers.params(W, H, 8, 6, chunks=chunks)
        ref = helpers.oracle_render(bundle, p)
        planes = torch.full((4, H, W, 3), -2.0, dtype=torch.float64, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        tipe_rt.render_gather_async(bundle.scene, p, tile_rows, *[planes[k].data_ptr() for k in range(4)], stream=st)
        torch.cuda.synchronize()
        got = planes.cpu().numpy()
        for k, name in enumerate(("canva", "albedo", "normal", "radiance")):
            assert (got[k] == ref[name]).all(), name
    finally:
        lib.rt_shutdown()
        tipe_rt.check(lib.rt_init(0, None))


def test_render_gather_canva_only_and_repeat():
    """Only the requested planes travel; a second call reuses the cached
    scene and pooled streams and gives the same frame."""
    import torch
    lib = _slots(2)
    try:
        bundle = helpers.cornell()
        W, H = 64, 48
        p = helpers.params(W, H, 6, 5, chunks=3)
        ref = helpers.oracle_render(bundle, p)
        st = torch.cuda.current_stream().cuda_stream
        outs = []
        for _ in range(2):
            c = torch.full((H, W, 3), -1.0, dtype=torch.float64, device="cuda:0")
            tipe_rt.render_gather_async(bundle.scene, p, 1, c.data_ptr(), stream=st)
            outs.append(c)
        torch.cuda.synchronize()
        for c in outs:
            assert (c.cpu().numpy() == ref["canva"]).all()
    finally:
        lib.rt_shutdown()
        tipe_rt.check(lib.rt_init(0, None))


def test_gather_async_explicit_locals():
    """rt_gather_async on slot frames the caller rendered itself."""
    import torch
    bundle = helpers.cornell()
    W, H, k, world = 40, 30, 3, 3
    p = helpers.params(W, H, 4, 5)
    ref = helpers.oracle_render(bundle, p)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    st = torch.cuda.current_stream().cuda_stream
    per_rank = tipe_rt.cyclic_tiling(H, k, 0, world).n_tiles * k
    locs = [torch.zeros((per_rank, W, 3), dtype=torch.float64, device="cuda:0") for _ in range(world)]
    for r in range(world):
        tipe_rt.render_async(ds, p, tipe_rt.cyclic_tiling(H, k, r, world), locs[r].data_ptr(), stream=st)
    full = torch.full((H, W, 3), -1.0, dtype=torch.float64, device="cuda:0")
    tipe_rt.gather_async([0] * world, [t.data_ptr() for t in locs], k, per_rank, W, H, 0, full.data_ptr(), st)
    torch.cuda.synchronize()
    ds.close()
    assert (full.cpu().numpy() == ref["canva"]).all()


def test_gather_rejects_short_geometry():
    lib = tipe_rt.lib()
    devs = (C.c_int * 2)(0, 0)
    locs = (C.c_void_p * 2)(None, None)
    assert lib.rt_gather_async(2, devs, locs, 4, 4, 10, 30, 0, None, None) == tipe_rt.RT_EINVAL
    dummy = (C.c_double * 3)()
    # 2 ranks x 1 tile of 4 rows < ceil(30 / 4) tiles
    assert lib.rt_gather_async(2, devs, locs, 4, 4, 10, 30, 0, C.cast(dummy, C.c_void_p), None) == tipe_rt.RT_EINVAL


def test_demo_exits_cleanly_without_shutdown(tmp_path):
    """rt_demo is main.c's flow in C: one rt_render_rows (which fills the
    scene cache and the stream pool) and exit WITHOUT rt_shutdown, as main.c's
    drop-in never calls it.  The process must exit 0 (no device frees from
    static destructors after the HIP runtime is gone) and write the oracle's
    image."""
    exe = os.path.join(ROOT, "tipe-raytracer_amd", "rt_demo")
    out = tmp_path / "demo.ppm"
    r = subprocess.run([exe, "-w", "64", "-s", "4", "-b", "5", "-o", str(out)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    W, H = 64, 48
    p = helpers.params(W, H, 4, 5, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
    ref = helpers.oracle_render(helpers.cornell(), p)
    assert out.read_text().split() == helpers.ppm_text(ref["canva"]).split()
