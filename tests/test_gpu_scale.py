"""GPU parity at the scale the benchmark runs, and the host-buffer drop-ins.

The headline number (bench.py) comes from render_kernel_q, the persistent
task-queue kernel: a 1200x900 frame with spp_chunks = 32 is 34.6 M
(chunk, pixel) tasks over ~262 k resident lanes, so every lane runs ~130
tasks, re-grabs batches under contention and hands its LDS sums over between
tasks.  These tests run that kernel at those sizes (reduced spp only) and on
grids shrunk to a few blocks (hundreds of tasks per lane), bit-exact against
the CPU oracle (oracle_render_rows, same Philox stream and slice grouping),
plus rt_render_rows / rt_fill_canva (main.c:402-453 drop-ins) with the
scene cache, the automatic chunking and several device slots.
"""
import ctypes as C
import os
import threading

import numpy as np
import pytest

import helpers
import tipe_rt
from tipe_rt.types import ThreadData, Sphere
from test_gpu_parity import check_parity, gpu_render, assert_same

pytestmark = pytest.mark.gpu

# The box's CPU share (16 cores per GPU); os.cpu_count() reports the whole host.
ORACLE_THREADS = max(1, min(16, os.cpu_count() or 1))


# ---- the benchmarked kernel at full frame size --------------------------------
def test_queue_kernel_c2_full_frame():
    """C2 exactly as bench.py renders it (README box, 1200x900, 6 bounces,
    spp_chunks 32) at 64 spp: 34.6 M tasks of 2 samples each."""
    check_parity(helpers.cornell(), helpers.params(1200, 900, 64, 6, chunks=32), nthreads=ORACLE_THREADS)


def test_queue_kernel_c3_full_frame():
    """C3 (spheres + textured, refracting pyramid) full frame, 32 spp in 16 chunks."""
    ref = check_parity(helpers.pyramid_scene(), helpers.params(1200, 900, 32, 6, chunks=16),
                       nthreads=ORACLE_THREADS)
    assert ref["canva"].max() > 0


def test_queue_kernel_c5_4k_frame():
    """C5's 3840x2880 frame (pyramid scene) with spp_chunks 4 at 4 spp:
    44 M tasks, task indices beyond 2^25, pixel indices beyond 2^23."""
    bundle = helpers.pyramid_scene()
    p = helpers.params(3840, 2880, 4, 6, chunks=4)
    ref = helpers.oracle_render(bundle, p, nthreads=ORACLE_THREADS)
    canva, alb, nrm, rad = gpu_render(bundle, p)
    assert_same(canva, ref["canva"], "canva")
    assert_same(rad, ref["radiance"], "radiance")
    assert_same(alb, ref["albedo"], "albedo")
    assert_same(nrm, ref["normal"], "normal")


def test_bvh_kernel_c4_band():
    """C4 (tree, AO 2.5 -> 2, 8 bounces) on a full-width 64-row band of the
    1200x900 frame through the BVH kernel (the oracle scans every triangle)."""
    bundle = helpers.tree_scene()
    p = helpers.params(1200, 900, 2, 8, use_ao=True)
    ref = helpers.oracle_render(bundle, p, row_hi=463, row_lo=400, nthreads=ORACLE_THREADS)
    import torch
    rows = 64
    bufs = [torch.full((rows, 1200, 3), -1.0, dtype=torch.float64, device="cuda:0") for _ in range(4)]
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    tipe_rt.render_async(ds, p, tipe_rt.band_tiling(400, 463), *[b.data_ptr() for b in bufs],
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    got = [b.cpu().numpy() for b in bufs]
    for k, name in enumerate(("canva", "albedo", "normal", "radiance")):
        assert_same(got[k], ref[name][400:464], name)


def test_bvh_queue_kernel_c4_band():
    """C4 (tree, AO 2.5 -> 2, 8 bounces) on a full-width 64-row band with
    spp_chunks 4: the BVH task-queue kernel (resumable walks) at frame width."""
    bundle = helpers.tree_scene()
    p = helpers.params(1200, 900, 4, 8, use_ao=True, chunks=4)
    ref = helpers.oracle_render(bundle, p, row_hi=463, row_lo=400, nthreads=ORACLE_THREADS)
    import torch
    rows = 64
    bufs = [torch.full((rows, 1200, 3), -1.0, dtype=torch.float64, device="cuda:0") for _ in range(4)]
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    tipe_rt.render_async(ds, p, tipe_rt.band_tiling(400, 463), *[b.data_ptr() for b in bufs],
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    got = [b.cpu().numpy() for b in bufs]
    for k, name in enumerate(("canva", "albedo", "normal", "radiance")):
        assert_same(got[k], ref[name][400:464], name)


def test_bvh_queue_kernel_c4_full_frame():
    """C4 at its own size: the full 1200x900 frame of the tree scene (1320
    triangles, AO 2.5 -> 2, 8 bounces) through the BVH task-queue kernel with
    resumable walks, 2 spp in 2 chunks (2.2 M tasks), every plane bit-exact
    against the oracle (which scans all 1320 triangles per cast)."""
    ref = check_parity(helpers.tree_scene(), helpers.params(1200, 900, 2, 8, use_ao=True, chunks=2),
                       nthreads=ORACLE_THREADS)
    assert ref["canva"].max() > 0


# ---- many tasks per lane: the queue kernel on a few blocks -------------------
@pytest.mark.parametrize("blocks,case", [(1, "cornell"), (3, "cornell"), (2, "cornell_ao"), (1, "pyramid"),
                                         (5, "aperture"), (2, "tree_ao"), (1, "sweep")])
def test_queue_kernel_tiny_grid(blocks, case, monkeypatch):
    """RT_QUEUE_BLOCKS (read on every launch) shrinks the persistent grid to
    a few blocks: every lane runs hundreds of tasks, so batch re-grabs, the
    partial-batch hand-out, the owner's flush of the previous task's sums and
    the camera-ray prefetch reset between tasks all run many times."""
    monkeypatch.setenv("RT_QUEUE_BLOCKS", str(blocks))
    bundle, p = {
        "cornell": lambda: (helpers.cornell(), helpers.params(96, 72, 24, 6, chunks=8)),
        "cornell_ao": lambda: (helpers.cornell(), helpers.params(64, 48, 12, 6, use_ao=True, ao=2.5, compat=0,
                                                                chunks=4)),
        "pyramid": lambda: (helpers.pyramid_scene(), helpers.params(64, 48, 12, 6, chunks=6)),
        "aperture": lambda: (helpers.cornell(), helpers.params(40, 30, 12, 5, aperture=(0.3, 0.2), compat=0,
                                                              focus=2.5, chunks=3)),
        "tree_ao": lambda: (helpers.tree_scene(), helpers.params(40, 30, 8, 8, use_ao=True, chunks=4)),
        "sweep": lambda: (helpers.SceneBundle(*tipe_rt.scenes.synthetic_cornell(10, 100)),
                          helpers.params(64, 48, 12, 6, chunks=6)),
    }[case]()
    check_parity(bundle, p)


# ---- host-buffer drop-ins -----------------------------------------------------
def test_render_rows_auto_chunks_reaches_queue_kernel():
    """rt_params_init's default spp_chunks is RT_SPP_CHUNKS_AUTO (P = min(32,
    S)): rt_render_rows then runs the task-queue kernel, and the oracle
    resolves AUTO to the same slice grouping."""
    p0 = tipe_rt.Params()
    tipe_rt.lib().rt_params_init(C.byref(p0))
    assert p0.spp_chunks == tipe_rt.RT_SPP_CHUNKS_AUTO
    bundle = helpers.cornell()
    p = helpers.params(64, 48, 40, 6, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
    ref = helpers.oracle_render(bundle, p)
    canva, alb, nrm = tipe_rt.render_rows(bundle.scene, p)
    assert (canva == ref["canva"]).all() and (alb == ref["albedo"]).all() and (nrm == ref["normal"]).all()
    # AUTO at 40 spp is 32 slices: not the strict running sum
    strict = helpers.oracle_render(bundle, helpers.params(64, 48, 40, 6, chunks=1))
    assert not (strict["radiance"] == ref["radiance"]).all()


def test_render_rows_scene_cache_tracks_content():
    """Repeated calls reuse the uploaded scene; changing the caller's array
    in place changes the image exactly as a fresh upload would."""
    lib = tipe_rt.lib()
    lib.rt_scene_cache_clear()
    spheres = tipe_rt.scenes.cornell_spheres()
    bundle = helpers.SceneBundle(spheres)
    p = helpers.params(40, 30, 6, 5, chunks=3)
    a = tipe_rt.render_rows(bundle.scene, p)[0]
    b = tipe_rt.render_rows(bundle.scene, p)[0]
    assert (a == b).all()
    assert (a == helpers.oracle_render(bundle, p)["canva"]).all()
    spheres[9].center.e[0] = 0.1                       # same pointer, new contents (mirror sphere moved)
    c = tipe_rt.render_rows(bundle.scene, p)[0]
    assert (c == helpers.oracle_render(bundle, p)["canva"]).all()
    assert not (c == a).all()
    assert lib.rt_scene_cache_clear() >= 2


@pytest.mark.parametrize("planes", ["all", "canva_only"])
def test_render_rows_two_device_slots(planes):
    """rt_init(2, {0, 0}): rt_render_rows deals cyclic 1-row tiles over two
    device slots (here both on GPU 0), copies each slot's planes back
    asynchronously and scatters the rows; only the requested planes."""
    lib = tipe_rt.lib()
    devs = (C.c_int * 2)(0, 0)
    tipe_rt.check(lib.rt_init(2, devs))
    try:
        bundle = helpers.pyramid_scene()
        W, H = 50, 37
        for chunks in (1, 4):
            p = helpers.params(W, H, 8, 6, chunks=chunks)
            ref = helpers.oracle_render(bundle, p)
            canva = np.full((H, W, 3), -3.0)
            alb = np.full((H, W, 3), -3.0) if planes == "all" else None
            nrm = np.full((H, W, 3), -3.0) if planes == "all" else None
            tipe_rt.check(lib.rt_render_rows(C.byref(bundle.scene), C.byref(p), H - 2, 3, canva.ctypes.data,
                                             alb.ctypes.data if alb is not None else None,
                                             nrm.ctypes.data if nrm is not None else None))
            assert (canva[3:H - 1] == ref["canva"][3:H - 1]).all()
            assert (canva[:3] == -3.0).all() and (canva[H - 1:] == -3.0).all()
            if planes == "all":
                assert (alb[3:H - 1] == ref["albedo"][3:H - 1]).all()
                assert (nrm[3:H - 1] == ref["normal"][3:H - 1]).all()
    finally:
        lib.rt_shutdown()
        tipe_rt.check(lib.rt_init(0, None))


@pytest.mark.parametrize("ndev", [1, 2])
def test_render_rows_large_band_threaded_scatter(ndev):
    """Planes of >= 4 MB are scattered into the caller's arrays on several
    host threads as each plane's D2H copy lands (rt_render_rows step 3):
    a 1024-wide band of 686 rows on one slot, and cyclic 1-row tiles over two
    slots, bit-exact against the oracle, rows outside the band untouched."""
    lib = tipe_rt.lib()
    devs = (C.c_int * 2)(0, 0)
    tipe_rt.check(lib.rt_init(ndev, devs))
    try:
        bundle = helpers.cornell()
        W, H, lo, hi = 1024, 700, 5, 690
        p = helpers.params(W, H, 2, 4, chunks=2)
        ref = helpers.oracle_render(bundle, p, row_hi=hi, row_lo=lo, nthreads=ORACLE_THREADS)
        planes = [np.full((H, W, 3), -5.0) for _ in range(3)]
        tipe_rt.check(lib.rt_render_rows(C.byref(bundle.scene), C.byref(p), hi, lo,
                                         *[a.ctypes.data for a in planes]))
        for a, key in zip(planes, ("canva", "albedo", "normal")):
            assert (a[lo:hi + 1] == ref[key][lo:hi + 1]).all(), key
            assert (a[:lo] == -5.0).all() and (a[hi + 1:] == -5.0).all(), key
    finally:
        lib.rt_shutdown()
        tipe_rt.check(lib.rt_init(0, None))


def test_fill_canva_twelve_threads_auto_chunks():
    """main.c's flow: NUM_THREADS = 12 pthreads call the drop-in on their
    row bands (main.c:407-449: H / 12 rows each, the last one takes the
    remainder) with the default RT_SPP_CHUNKS_AUTO grouping; the assembled
    frame equals the oracle's frame for that grouping."""
    lib = tipe_rt.lib()
    assert lib.rt_set_fill_spp_chunks(tipe_rt.RT_SPP_CHUNKS_AUTO) == tipe_rt.RT_SPP_CHUNKS_AUTO
    bundle = helpers.cornell()
    W, H, S, B, NT = 120, 90, 40, 6, 12
    p = helpers.params(W, H, S, B, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO, compat=0)
    ref = helpers.oracle_render(bundle, p)
    canva, alb, nrm = (np.zeros((H, W, 3)) for _ in range(3))
    rows = H // NT
    tds = []
    for t in range(NT):
        hi = H - 1 - t * rows
        lo = hi - rows + 1 if t < NT - 1 else 0
        td = ThreadData()
        td.start_row, td.end_row = hi, lo
        td.canva = C.cast(canva.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.albedo_tab = C.cast(alb.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.normal_tab = C.cast(nrm.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.cam = p.cam
        td.largeur_image, td.hauteur_image = W, H
        td.nbRayonParPixel, td.nbRebondMax = S, B
        td.total_pixels = W * H
        td.sphere_list = C.cast(bundle.spheres, C.POINTER(Sphere))
        td.nbSpheres = len(bundle.spheres)
        td.focus_distance = 3
        tds.append(td)
    res = []
    ths = [threading.Thread(target=lambda t=t: res.append(lib.rt_fill_canva(C.byref(t)))) for t in tds]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert all(r is None for r in res), lib.rt_last_error()
    assert (canva == ref["canva"]).all() and (alb == ref["albedo"]).all() and (nrm == ref["normal"]).all()
    # strict fill_canva order on request
    prev = lib.rt_set_fill_spp_chunks(1)
    try:
        assert prev == tipe_rt.RT_SPP_CHUNKS_AUTO
        td = tds[0]
        lib.rt_fill_canva(C.byref(td))
        strict = helpers.oracle_render(bundle, helpers.params(W, H, S, B, chunks=1, compat=0))
        lo, hi = td.end_row, td.start_row
        assert (canva[lo:hi + 1] == strict["canva"][lo:hi + 1]).all()
        assert (alb[lo:hi + 1] == strict["albedo"][lo:hi + 1]).all()
    finally:
        lib.rt_set_fill_spp_chunks(tipe_rt.RT_SPP_CHUNKS_AUTO)
