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
import sys

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


@pytest.mark.parametrize("slots,tile_rows,chunks,scene", [(2, 1, 4, "pyramid"), (3, 4, 1, "pyramid"),
                                                          (2, 2, 1, "pyramid"), (2, 1, 4, "tree"),
                                                          (3, 1, 32, "tree")])
def test_render_gather_slots_bitexact(slots, tile_rows, chunks, scene):
    """tree: the C4 scene (1320-triangle BVH + AO 2.5, 8 bounces) through the
    BVH queue kernel on cyclic 1-row tiles and the gather -- C4's own
    multi-GPU layout (BASELINE config 4)."""
    import torch
    lib = _slots(slots)
    try:
        W, H = 52, 41
        if scene == "tree":
            bundle = helpers.tree_scene()
            p = helpers.params(W, H, 8 if chunks < 32 else 32, 8, use_ao=True, ao=2.5, chunks=chunks)
        else:
            bundle = helpers.pyramid_scene()
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


def test_rt_init_rejects_invisible_device_and_keeps_list():
    """rt_init with a device id that is not visible returns RT_EINVAL and
    leaves the previous device list in force (nothing half-committed)."""
    lib = tipe_rt.lib()
    n = lib.rt_device_count()
    assert n >= 1
    tipe_rt.check(lib.rt_init(1, (C.c_int * 1)(0)))
    try:
        for bad in ([0, n], [-1], [n + 7, 0]):
            assert lib.rt_init(len(bad), (C.c_int * len(bad))(*bad)) == tipe_rt.RT_EINVAL
            assert b"not visible" in lib.rt_last_error()
        bundle = helpers.cornell()
        p = helpers.params(16, 12, 2, 4)
        canva, _, _ = tipe_rt.render_rows(bundle.scene, p)       # still device 0 alone
        assert (canva == helpers.oracle_render(bundle, p)["canva"]).all()
    finally:
        tipe_rt.check(lib.rt_init(0, None))


def test_peer_access_query():
    lib = tipe_rt.lib()
    n = lib.rt_device_count()
    assert lib.rt_peer_access(0, 0) == 1
    assert lib.rt_peer_access(0, n) == tipe_rt.RT_EINVAL
    assert lib.rt_peer_access(-1, 0) == tipe_rt.RT_EINVAL


def _device_count():
    try:
        return tipe_rt.lib().rt_device_count()
    except Exception:
        return 0


@pytest.mark.parametrize("peer_env", ["1", "0"])
def test_render_gather_distinct_devices_bitexact(peer_env):
    """Slots on distinct GPUs: peer enable (or, with RT_PEER_ACCESS=0, the
    runtime's staged copies), cross-device event waits and xGMI copies.
    Needs >= 2 GPUs, so it is skipped on the builder's one-GPU box; run in a
    subprocess so the environment switch applies from the library's first
    peer call."""
    if _device_count() < 2:
        pytest.skip("needs >= 2 visible GPUs (the distinct-device path has not run on the builder's box)")
    code = r'''
import ctypes as C, sys
sys.path[:0] = %r
import torch, helpers, tipe_rt
lib = tipe_rt.lib()
tipe_rt.check(lib.rt_init(2, (C.c_int * 2)(0, 1)))
bundle = helpers.pyramid_scene()
W, H = 52, 41
p = helpers.params(W, H, 8, 6, chunks=4)
ref = helpers.oracle_render(bundle, p)
planes = torch.full((4, H, W, 3), -2.0, dtype=torch.float64, device="cuda:0")
tipe_rt.render_gather_async(bundle.scene, p, 1, *[planes[k].data_ptr() for k in range(4)],
                            stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
got = planes.cpu().numpy()
ok = all((got[k] == ref[n]).all() for k, n in enumerate(("canva", "albedo", "normal", "radiance")))
st = lib.rt_peer_access(0, 1)
print("RESULT", int(ok), st)
''' % ([os.path.join(ROOT, "tests"), os.path.join(ROOT, "tipe-raytracer_amd")],)
    env = dict(os.environ, RT_PEER_ACCESS=peer_env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1].split()
    assert res[1] == "1"
    if peer_env == "0":
        assert res[2] == "0"
