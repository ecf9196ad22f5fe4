"""Device-resident multi-device frames and process exit.

rt_render_gather_async renders the cyclic row tiles of a frame on every
device slot of rt_init's list, gathers the slots' planes onto the first
device and un-permutes them with the assemble kernel -- the
device-destination replacement of main.c:404-453 / main_cuda.cu:280-339.
The gather is an RCCL ncclGather over one communicator per device
(rt_params.gather = RT_GATHER_RCCL, the default) or, on request, peer copies
(RT_GATHER_PEER).  RCCL has one rank per GPU, so the one-GPU box runs the
RCCL path as a 1-rank communicator and several slots on GPU 0 through the
peer path (the copy is then device-local); the images must equal the
oracle's bit for bit, since the Philox stream is keyed by the global pixel.
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


PEER = tipe_rt.types.RT_GATHER_PEER
RCCL = tipe_rt.types.RT_GATHER_RCCL


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
        p.gather = PEER                    # slots on one GPU: peer copies (RCCL has one rank per GPU)
        ref = helpers.oracle_render(bundle, p)
        planes = torch.full((4, H, W, 3), -2.0, dtype=torch.float64, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        tipe_rt.render_gather_async(bundle.scene, p, tile_rows, *[planes[k].data_ptr() for k in range(4)], stream=st)
        torch.cuda.synchronize()
        got = planes.cpu().numpy()
        for k, name in enumerate(("canva", "albedo", "normal", "radiance")):
            assert (got[k] == ref[name]).all(), name
        assert tipe_rt.last_gather_transport().startswith("peer:")
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
        p.gather = PEER
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


@pytest.mark.parametrize("scene,planes_wanted", [("pyramid", 4), ("tree", 4), ("cornell", 1)])
def test_rccl_gather_one_device_bitexact(scene, planes_wanted):
    """RT_GATHER_RCCL (the default) through the whole path on the one-GPU box:
    rt_init(1, {0}) -> a 1-rank RCCL communicator (ncclCommInitAll), the
    slot's planes gathered to rank 0 by ncclGather and assembled; bit for
    bit vs the oracle, twice (the communicator is reused)."""
    import torch
    lib = tipe_rt.lib()
    tipe_rt.check(lib.rt_init(1, (C.c_int * 1)(0)))
    try:
        W, H = 52, 41
        if scene == "tree":
            bundle = helpers.tree_scene()
            p = helpers.params(W, H, 8, 8, use_ao=True, ao=2.5, chunks=4)
        elif scene == "pyramid":
            bundle = helpers.pyramid_scene()
            p = helpers.params(W, H, 8, 6, chunks=32)
        else:
            bundle = helpers.cornell()
            p = helpers.params(W, H, 6, 5, chunks=3)
        assert p.gather == RCCL
        ref = helpers.oracle_render(bundle, p)
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            planes = torch.full((4, H, W, 3), -2.0, dtype=torch.float64, device="cuda:0")
            ptrs = [planes[k].data_ptr() if k < planes_wanted else None for k in range(4)]
            tipe_rt.render_gather_async(bundle.scene, p, 1, *ptrs, stream=st)
            torch.cuda.synchronize()
            got = planes.cpu().numpy()
            for k, name in enumerate(("canva", "albedo", "normal", "radiance")[:planes_wanted]):
                assert (got[k] == ref[name]).all(), name
            assert tipe_rt.last_gather_transport().startswith("rccl: ncclGather"), tipe_rt.last_gather_transport()
    finally:
        lib.rt_shutdown()
        tipe_rt.check(lib.rt_init(0, None))


def test_rccl_gather_refuses_a_repeated_device():
    """No silent fallback: RCCL has one rank per GPU, so a device list that
    names a GPU twice is RT_EUNSUPPORTED under RT_GATHER_RCCL."""
    import torch
    lib = _slots(2)
    try:
        bundle = helpers.cornell()
        p = helpers.params(16, 12, 2, 4)
        c = torch.zeros((12, 16, 3), dtype=torch.float64, device="cuda:0")
        fr = tipe_rt.Frame(c.data_ptr(), None, None, None)
        assert lib.rt_render_gather_async(C.byref(bundle.scene), C.byref(p), 1, C.byref(fr), None) == \
            tipe_rt.RT_EUNSUPPORTED
        assert b"RT_GATHER_PEER" in lib.rt_last_error()
        p.gather = 7
        assert lib.rt_render_gather_async(C.byref(bundle.scene), C.byref(p), 1, C.byref(fr), None) == tipe_rt.RT_EINVAL
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


@pytest.mark.parametrize("peer_env,gather", [("1", 1), ("0", 1), ("1", 0)])
def test_render_gather_distinct_devices_bitexact(peer_env, gather):
    """Slots on distinct GPUs: RCCL (gather 0: a 2-rank communicator and
    ncclGather over xGMI) or peer copies (gather 1: peer enable or, with
    RT_PEER_ACCESS=0, the runtime's staged copies), cross-device event waits.
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
p.gather = %d
ref = helpers.oracle_render(bundle, p)
planes = torch.full((4, H, W, 3), -2.0, dtype=torch.float64, device="cuda:0")
tipe_rt.render_gather_async(bundle.scene, p, 1, *[planes[k].data_ptr() for k in range(4)],
                            stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
got = planes.cpu().numpy()
ok = all((got[k] == ref[n]).all() for k, n in enumerate(("canva", "albedo", "normal", "radiance")))
st = lib.rt_peer_access(0, 1)
print("TRANSPORT", tipe_rt.last_gather_transport())
print("RESULT", int(ok), st)
''' % ([os.path.join(ROOT, "tests"), os.path.join(ROOT, "tipe-raytracer_amd")], gather)
    env = dict(os.environ, RT_PEER_ACCESS=peer_env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1].split()
    assert res[1] == "1"
    tr = [ln for ln in r.stdout.splitlines() if ln.startswith("TRANSPORT")][-1]
    assert ("rccl: ncclGather" if gather == 0 else "peer:") in tr
    if peer_env == "0" and gather == 1:
        assert res[2] == "0"
