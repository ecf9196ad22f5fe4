"""GPU parity: librt_hip.so (through the C-ABI) vs the CPU oracle in
RT_RNG_PHILOX mode on identical seeded inputs.

The kernel performs the reference's IEEE operations in the same order as the
oracle, so the bar is BIT-EXACT equality of canva (8-bit resolve), albedo,
normal and pre-gamma radiance.  north_star's tolerance (per-channel RMSE
<= 1e-4 on float accumulation) is asserted as well, as the outer bound.
"""
import ctypes as C
import threading

import numpy as np
import pytest

import helpers
import oracle_ffi
import tipe_rt
from tipe_rt.types import ThreadData, Sphere, Triangle, Material

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4   # north_star: per-channel RMSE on identical seeds


def gpu_render(bundle, p, tiling=None, radiance=True):
    """Device path: rt_scene_upload + rt_render_async into torch buffers."""
    import torch
    W, H = p.largeur_image, p.hauteur_image
    if tiling is None:
        tiling = tipe_rt.band_tiling(0, H - 1)
    rows = tiling.n_tiles * tiling.tile_rows
    dev = torch.device("cuda:0")
    bufs = [torch.full((rows, W, 3), -1.0, dtype=torch.float64, device=dev) for _ in range(4)]
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    stream = torch.cuda.current_stream().cuda_stream
    tipe_rt.render_async(ds, p, tiling, bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(),
                         bufs[3].data_ptr() if radiance else None, stream)
    torch.cuda.synchronize()
    ds.close()
    return [b.cpu().numpy() for b in bufs]


def gpu_counts(bundle, p):
    """rt_count_async over the whole frame: the RT_NCOUNTERS event totals."""
    import torch
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    d = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, p.hauteur_image - 1), d.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    return [int(x) for x in d.cpu()]


def assert_stack_bound_holds(bundle, p):
    """Every BVH push of the frame's walks stays inside the LDS stack of the
    kernel that renders the tree (rt.h RT_CNT_BVH_STACK_OVER == 0), i.e.
    the host's stack bound (rt_bvh.cpp) covers the kernel's push rule."""
    c = gpu_counts(bundle, p)
    assert c[tipe_rt.types.RT_CNT_BVH_STACK_OVER] == 0, c
    return c


def assert_same(gpu, ref, what):
    """Bit-for-bit equal values; NaN must sit at the same places (payloads
    may differ: x86 and gfx950 produce different default NaNs)."""
    assert gpu.shape == ref.shape, what
    diff = np.argwhere((gpu != ref) & ~(np.isnan(gpu) & np.isnan(ref)))
    if len(diff):
        j, i, c = diff[0]
        raise AssertionError("%s: %d mismatching values; first at row %d col %d ch %d: gpu %r oracle %r" %
                             (what, len(diff), j, i, c, gpu[j, i, c], ref[j, i, c]))


def check_parity(bundle, p, nthreads=1):
    ref = helpers.oracle_render(bundle, p, nthreads=nthreads)
    canva, alb, nrm, rad = gpu_render(bundle, p)
    fin = ~np.isnan(ref["radiance"])               # NaN radiance: the reference's own (e.g. AO 0)
    assert (np.isnan(rad) == ~fin).all()
    assert (helpers.rmse_per_channel(np.where(fin, rad, 0), np.where(fin, ref["radiance"], 0)) <= RMSE_TOL).all()
    assert (helpers.rmse_per_channel(canva / 255.0, ref["canva"] / 255.0) <= RMSE_TOL).all()
    assert_same(canva, ref["canva"], "canva")
    assert_same(rad, ref["radiance"], "radiance")
    assert_same(alb, ref["albedo"], "albedo")
    assert_same(nrm, ref["normal"], "normal")
    return ref


# ---- device primitives ------------------------------------------------------
def test_device_math_bitexact():
    o = oracle_ffi.oracle()
    rng = np.random.default_rng(7)
    n = 4096
    k = rng.integers(0, 2 ** 31, n)
    edge = [-1.0, -0.5, 0.5, 0.0, 1e-20, -1e-300, 1 - 2.0 ** -53, -1 + 2.0 ** -53, 0.5 - 2.0 ** -54,
            -0.5 + 2.0 ** -54, 2.0 ** -31, -(2.0 ** -31), 0.9999999999, -0.9999999999]
    xs = np.concatenate([2.0 * (k / 2147483648.0) - 1.0, rng.uniform(-1, 1, n), edge])
    got = tipe_rt.selftest_math(0, xs, len(xs))
    want = np.array([o.oracle_pm_acos(x) for x in xs])
    assert (got.view(np.uint64) == want.view(np.uint64)).all()
    fs = np.concatenate([rng.uniform(0, 2 * np.pi, n), rng.uniform(0, np.pi, n), [0.0, np.pi / 2, 1e-30]])
    fs = fs.astype(np.float32).astype(np.float64)
    got = tipe_rt.selftest_math(1, fs, len(fs))
    assert (got == np.array([o.oracle_pm_sinf(x) for x in fs])).all()
    got = tipe_rt.selftest_math(2, fs, len(fs))
    assert (got == np.array([o.oracle_pm_cosf(x) for x in fs])).all()
    xy = np.stack([1.0 + rng.uniform(-1e-15, 1e-15, n), rng.choice([2.0, 2.5, 3.0, 8.0, 0.5], n)], 1).ravel()
    got = tipe_rt.selftest_math(3, xy, n)
    want = np.array([o.oracle_pm_pow(xy[2 * i], xy[2 * i + 1]) for i in range(n)])
    assert (got.view(np.uint64) == want.view(np.uint64)).all()
    xs = rng.uniform(0, 1e6, n) * rng.choice([1e-300, 1e-10, 1.0, 1e300], n)
    assert (tipe_rt.selftest_math(4, xs, n).view(np.uint64) == np.sqrt(xs).view(np.uint64)).all()
    ab = rng.uniform(-10, 10, 2 * n)
    assert (tipe_rt.selftest_math(5, ab, n) == ab[0::2] / ab[1::2]).all()
    fs = rng.uniform(0, 1e4, n).astype(np.float32)
    assert (tipe_rt.selftest_math(6, fs.astype(np.float64), n) == np.sqrt(fs).astype(np.float64)).all()


def test_device_pow_special_and_wide_inputs():
    """pm_pow's device form (one straight-line log/exp with the special cases
    selected afterwards, rt_device_math.h) against oracle/pm_math.h's branchy
    pm_pow: zeros, negatives, infinities, NaN, subnormals, exp's overflow and
    underflow limits, and wide random x, for the AO intensities a scene can
    set (fractional, integer, negative, huge, infinite, NaN)."""
    o = oracle_ffi.oracle()
    rng = np.random.default_rng(23)
    inf, nan = np.inf, np.nan
    xs_edge = [0.0, -0.0, -1.0, -2.5, inf, -inf, nan, 5e-324, 1e-310, 2.0 ** -1022, 2.0 ** -1022 * (1 - 2.0 ** -52),
               1.0, 1 + 2.0 ** -52, 1 - 2.0 ** -53, 0.5, 2.0, 1e300, 1e-300, 1.7976931348623157e308]
    ys_edge = [2.5, -2.5, 0.5, 0.1, 3.0, -3.0, 100.5, -100.5, 1e10, -1e10, inf, -inf, nan, 0.0, 64.0, 65.0, 1e-300]
    n = 4096
    xr = np.concatenate([rng.uniform(0, 4, n), 10.0 ** rng.uniform(-320, 308, n), 1 + rng.uniform(-1e-12, 1e-12, n)])
    yr = rng.choice([2.5, 0.7, -1.3, 7.25, 300.5], len(xr))
    x = np.concatenate([np.repeat(xs_edge, len(ys_edge)), xr])
    y = np.concatenate([np.tile(ys_edge, len(xs_edge)), yr])
    got = tipe_rt.selftest_math(3, np.stack([x, y], 1).ravel(), len(x))
    want = np.array([o.oracle_pm_pow(a, b) for a, b in zip(x, y)])
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), list(zip(x[~same], y[~same], got[~same], want[~same]))[:6]


def _oracle_pow_n(x, y):
    o = oracle_ffi.oracle()
    xy = np.ascontiguousarray(np.stack([x, y], 1).ravel())
    out = np.empty(len(x))
    o.oracle_pm_pow_n(xy.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double)), len(x))
    return out


@pytest.mark.parametrize("y", [2.5, 0.5, 0.1, 1.75, 7.3, 100.5, 999.9, -2.5, 1e-300, 4e6, 1e9])
def test_device_pow_near1_dense(y):
    """pm_pow where ambient_occlusion calls it (main.c:109-111: distance / t
    of the AO hit, 1 up to the rounding of the hit point) against
    oracle/pm_math.h's pm_pow: every x within 2^15 ulps of 1 on both sides
    and a random spread out to 2^-26, for AO intensities from 1e-300 to 1e9."""
    rng = np.random.default_rng(int(abs(y) * 1000) % 2**31)
    k = np.arange(-2 ** 15, 2 ** 15 + 1, dtype=np.float64)
    lim = 2.0 ** -26
    x = np.concatenate([1.0 + k[k >= 0] * 2.0 ** -52, 1.0 + k[k < 0] * 2.0 ** -53,
                        1.0 + rng.uniform(-lim, lim, 1 << 17), 1.0 + rng.uniform(-(2.0 ** -40), 2.0 ** -40, 1 << 15),
                        1.0 + np.array([lim, -lim, lim + 2.0 ** -52, -lim - 2.0 ** -53, 2 * lim, 1e-3, -1e-3])])
    ys = np.full(len(x), y)
    got = tipe_rt.selftest_math(3, np.stack([x, ys], 1).ravel(), len(x))
    want = _oracle_pow_n(x, ys)
    same = got.view(np.uint64) == want.view(np.uint64)
    assert same.all(), list(zip(x[~same], got[~same], want[~same]))[:6]


def test_device_normalize_fast_path_is_ieee():
    """normalize() skips the sqrt/division range fixups on in-range lanes and
    shares 1/|a| (rt_kernels.hip); it must equal a / sqrt(a.a) in IEEE f64
    for every input, including the lanes routed to the generic path."""
    rng = np.random.default_rng(11)
    n = 1 << 18
    v = rng.normal(size=(n, 3)) * rng.choice([1e-300, 1e-200, 1e-9, 1.0, 1e3, 1e200, 1e300], (n, 1))
    v[: n // 16, rng.integers(0, 3)] = 0.0                      # zero components
    v[n // 16: n // 8, 1] *= 1e-290                             # one tiny component
    v[n // 8: n // 8 + 64] = [[-0.0, 1.0, 0.0]]
    v[n // 8 + 64: n // 8 + 128] = rng.normal(size=(64, 3)) * 2.0 ** -380
    got = tipe_rt.selftest_math(8, v.ravel(), n).reshape(n, 3)
    with np.errstate(all="ignore"):
        L = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
        want = v / L[:, None]
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), v[~same.all(1)][:4]


def test_device_normalize_stress():
    """normalize()'s fast path (sqrt_rcp_core: 1/|a| refined from the sqrt
    sequence's rsq, then div_core) and its seeded forms equal IEEE
    a / sqrt(a.a) bit for bit on 2^32 pseudo-random vectors: directions, n + dir
    sums, scales 2^-450..2^450 (normalize), the sampler's float-built unit
    vectors (normalize_unit, series seed) and sphere hit offsets hp - C
    (normalize_sph, radius seed), a quarter each of the last two."""
    fast, bad = tipe_rt.verify_normalize(seed=20261016, n=1 << 32)
    assert bad == 0
    assert fast > (1 << 31)


def test_sampler_phi_fast_path_exhaustive():
    """The fast phi path (phi_sincosf_fast) gives the full path's floats for
    every one of the 2^31 rand() values, and falls back rarely."""
    fb, bad = tipe_rt.verify_sampler_phi(0, 1 << 31)
    assert bad == 0
    assert fb < (1 << 31) // 2000


def test_device_atan2_matches_oracle():
    o = oracle_ffi.oracle()
    rng = np.random.default_rng(21)
    n = 20000
    yx = np.stack([np.concatenate([rng.uniform(-1, 1, n - 12), [0.0, -0.0, 0.0, -0.0, 1, -1, np.inf, 1, 1,
                                                                  np.inf, -np.inf, 1e-300]]),
                   np.concatenate([rng.uniform(-1, 1, n - 12), [1.0, 1.0, -1.0, -1.0, 0, 0, 1, np.inf, -np.inf,
                                                                  np.inf, -np.inf, -1e300]])], 1)
    got = tipe_rt.selftest_math(9, yx.ravel(), n)
    want = np.array([o.oracle_pm_atan2(y, x) for y, x in yx])
    assert (got.view(np.uint64) == want.view(np.uint64)).all()


def test_sky_mode_last_sphere():
    """main.c:64-71's commented-out sky branch (RT_SKY_LAST_SPHERE): the last
    sphere shows sphere_uvmapping's texel as emission."""
    bundle = helpers.sky_scene()
    ref = check_parity(bundle, helpers.params(48, 36, 6, 5, sky_mode=1))
    off = check_parity(bundle, helpers.params(48, 36, 6, 5, sky_mode=0))
    assert not (ref["canva"] == off["canva"]).all()     # the sky changes the image


def test_device_philox_matches_oracle():
    o = oracle_ffi.oracle()
    rng = np.random.default_rng(3)
    n = 512
    q = rng.integers(0, 2 ** 32, (n, 6), dtype=np.uint64)
    got = tipe_rt.selftest_math(7, q.astype(np.float64).ravel(), n).astype(np.uint64).reshape(n, 4)
    for i in range(n):
        ctr = (C.c_uint * 4)(*[int(x) for x in q[i, :4]])
        key = (C.c_uint * 2)(*[int(x) for x in q[i, 4:]])
        out = (C.c_uint * 4)()
        o.oracle_philox(ctr, key, out)
        assert list(out) == [int(x) for x in got[i]]


# ---- full renders -------------------------------------------------------------
def test_cornell_spheres_bitexact():
    check_parity(helpers.cornell(), helpers.params(64, 48, 16, 5))


def test_cornell_spp_chunks_bitexact():
    # spp_chunks = 4: fixed slice sums, combined in slice order (rt.h)
    check_parity(helpers.cornell(), helpers.params(40, 30, 10, 6, chunks=4))


def test_spp_chunks_row_bands(monkeypatch):
    """A partial-sum budget smaller than the frame splits the launch into
    16-row bands reusing one buffer (rt_api.cpp launch_on_stream): same image."""
    monkeypatch.setenv("RT_PARTIAL_BUDGET", str(16 * 37 * 4 * 72))     # 16 rows of 37 px x 4 chunks
    check_parity(helpers.cornell(), helpers.params(37, 53, 8, 5, chunks=4))


@pytest.mark.parametrize("case", ["cornell", "cornell_ao", "pyramid", "sky", "bands", "one_sample_chunks", "aperture",
                                  "neg_zero_origin"])
def test_task_queue_kernel_bitexact(case, monkeypatch):
    """spp_chunks > 1 without a BVH runs render_kernel_q: persistent lanes
    take (chunk, pixel) tasks from a counter in whatever order the waves get
    to them; the chunk partials, summed in chunk order, equal the oracle's."""
    bundle, p = {
        "cornell": lambda: (helpers.cornell(), helpers.params(96, 72, 24, 6, chunks=8)),
        "cornell_ao": lambda: (helpers.cornell(), helpers.params(64, 48, 12, 6, use_ao=True, ao=2.5, compat=0,
                                                                chunks=4)),
        "pyramid": lambda: (helpers.pyramid_scene(), helpers.params(64, 48, 12, 6, chunks=6)),
        "sky": lambda: (helpers.sky_scene(), helpers.params(48, 36, 9, 5, sky_mode=1, chunks=3)),
        "bands": lambda: (helpers.cornell(), helpers.params(37, 53, 8, 5, chunks=4)),
        "one_sample_chunks": lambda: (helpers.cornell(), helpers.params(33, 25, 5, 6, chunks=5)),
        # aperture: rays leave from co + (dx, dy, 0), one camera ray kept ahead (not two)
        "aperture": lambda: (helpers.cornell(), helpers.params(40, 30, 12, 5, aperture=(0.3, 0.2), compat=0,
                                                              focus=2.5, chunks=3)),
        # a -0 camera coordinate: co + (+0) would be +0, so also one ray ahead
        "neg_zero_origin": lambda: (helpers.cornell(), helpers.params(
            40, 30, 12, 5, chunks=3, cam=tipe_rt.init_camera((-0.0, 0.3, 0.5), (0.0, -0.5, -3.0), (0, 1, 0),
                                                             70.0, 4.0 / 3.0))),
    }[case]()
    if case == "bands":
        monkeypatch.setenv("RT_PARTIAL_BUDGET", str(16 * 37 * 4 * 72))
    check_parity(bundle, p)


@pytest.mark.parametrize("B,W,H,S,P", [(0, 16, 12, 4, 2), (1, 16, 12, 6, 3), (2, 1, 1, 8, 4), (6, 1, 7, 5, 5),
                                        (6, 9, 1, 4, 4)])
def test_task_queue_kernel_edges(B, W, H, S, P):
    """Queue kernel edge cases: no bounce (tracer's zero path, no camera-ray
    prefetch), one bounce, 1-pixel / 1-column / 1-row frames (main.c:265
    divides by W-1 = 0), one sample per chunk."""
    check_parity(helpers.cornell(), helpers.params(W, H, S, B, chunks=P))


@pytest.mark.parametrize("ns,nt", [(32, 0), (128, 0), (32, 100), (10, 1000), (128, 1000)])
def test_synthetic_sweep_scenes_bitexact(ns, nt):
    """The roofline-sweep scenes (tools/roofline_sweep.py):
    up to 128 spheres (the candidate pass over 64 scalar-loaded pairs) and
    1000 random triangles (BVH), with the queue kernel (chunks) and without."""
    sph, mesh = tipe_rt.scenes.synthetic_cornell(ns, nt)
    bundle = helpers.SceneBundle(sph, mesh)
    check_parity(bundle, helpers.params(32, 24, 4, 6, chunks=2))
    check_parity(bundle, helpers.params(24, 18, 3, 5, use_ao=True, ao=2.5, compat=0))


def test_task_queue_kernel_cyclic_tiles():
    """The queue kernel on a rank's cyclic row tiles (multi-GPU layout)."""
    import torch
    bundle = helpers.cornell()
    W, H, k, world = 40, 30, 2, 3
    p = helpers.params(W, H, 8, 5, chunks=4)
    ref = helpers.oracle_render(bundle, p)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    stream = torch.cuda.current_stream().cuda_stream
    per_rank = tipe_rt.cyclic_tiling(H, k, 0, world).n_tiles
    gathered = torch.zeros((world, per_rank * k, W, 3), dtype=torch.float64, device="cuda:0")
    for r in range(world):
        t = tipe_rt.cyclic_tiling(H, k, r, world)
        tipe_rt.render_async(ds, p, t, gathered[r].data_ptr(), stream=stream)
    full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    tipe_rt.assemble_async(gathered.data_ptr(), world, k, per_rank * k, W, H, full.data_ptr(), stream)
    torch.cuda.synchronize()
    ds.close()
    assert (full.cpu().numpy() == ref["canva"]).all()


def test_spp_chunks_only_move_the_last_bits():
    bundle = helpers.cornell()
    a = helpers.oracle_render(bundle, helpers.params(24, 18, 16, 6))
    b = gpu_render(bundle, helpers.params(24, 18, 16, 6, chunks=8))
    assert (helpers.rmse_per_channel(b[3], a["radiance"]) <= 1e-12).all()


def test_cornell_six_bounces_odd_size():
    check_parity(helpers.cornell(), helpers.params(37, 29, 9, 6, seed=77))


def test_cornell_ao_compat_int():
    # AO_intensity 2.5 -> 2 (ThreadData int, main.c:43)
    check_parity(helpers.cornell(), helpers.params(48, 36, 8, 8, use_ao=True, ao=2.5))


def test_cornell_ao_fractional_intensity():
    check_parity(helpers.cornell(), helpers.params(32, 24, 8, 6, use_ao=True, ao=2.5, compat=0))


def test_depth_of_field_aperture():
    check_parity(helpers.cornell(), helpers.params(40, 30, 8, 5, aperture=(0.3, 0.2), compat=0, focus=2.5))


def test_pyramid_texture_refraction():
    ref = check_parity(helpers.pyramid_scene(), helpers.params(64, 48, 16, 6))
    cnt = helpers.oracle_render(helpers.pyramid_scene(), helpers.params(16, 12, 4, 6), counters=True)["counters"]
    assert cnt[tipe_rt.types.RT_CNT_REFRACT] > 0 and cnt[tipe_rt.types.RT_CNT_TEX_HITS] > 0
    assert ref["canva"].max() > 0


def test_mineways_alpha_holes():
    tris, qm, mats, tw, th, nm = tipe_rt.scenes.load_mesh_fixture("mineways")
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0] = P.e[0] * 0.1 - 0.2
            P.e[1] = P.e[1] * 0.1 - 1.0
            P.e[2] = P.e[2] * 0.1 - 2.5
    bundle = helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), (tris, qm, mats, tw, th, nm))
    check_parity(bundle, helpers.params(40, 30, 4, 6))


def _zero_uv(tris):
    for t in tris:
        for uv in (t.uvA, t.uvB, t.uvC):
            uv.u = uv.v = 0.0


@pytest.mark.parametrize("neg,chunks", [(False, 1), (False, 4), (True, 4)])
def test_uvless_pyramid_constant_texel(neg, chunks):
    """Every uv 0 (the texel of each hit is (0, 0) of its material:
    TriTex::tex0, the kernel's constant-texel path) on the brute-force
    kernel with the 16x16 refraction texture; -0.0 uvs as well."""
    bundle = helpers.pyramid_scene()
    tris = bundle.mesh[0]
    _zero_uv(tris)
    if neg:
        for t in tris:
            t.uvB.u = -0.0
            t.uvC.v = -0.0
    bundle = helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), bundle.mesh)
    check_parity(bundle, helpers.params(48, 36, 8, 6, chunks=chunks))


@pytest.mark.parametrize("chunks", [1, 4])
def test_uvless_mineways_bvh_constant_texel(chunks):
    """The constant-texel path on the BVH queue kernel with 11 16x16
    textures, alpha holes and refraction (mineways, every uv 0)."""
    tris, qm, mats, tw, th, nm = tipe_rt.scenes.load_mesh_fixture("mineways")
    _zero_uv(tris)
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0] = P.e[0] * 0.1 - 0.2
            P.e[1] = P.e[1] * 0.1 - 1.0
            P.e[2] = P.e[2] * 0.1 - 2.5
    bundle = helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), (tris, qm, mats, tw, th, nm))
    check_parity(bundle, helpers.params(40, 30, 4, 6, use_ao=True, chunks=chunks))


def _textured_quad(tw, th, u0, v0, su, sv, seed):
    """Two triangles filling the view at z = -2 (front-facing), uv from
    (u0, v0) over (su, sv) (several repeats, negative too), and a tw x th
    table of random opaque texels."""
    from tipe_rt.scenes import material
    rng = np.random.default_rng(seed)
    P = [(-1.5, -1.5, -2.0), (1.5, -1.5, -2.0), (1.5, 1.5, -2.0), (-1.5, 1.5, -2.0)]
    UVs = [(u0, v0), (u0 + su, v0), (u0 + su, v0 + sv), (u0, v0 + sv)]
    tris = (Triangle * 2)()
    for t, (a, b, c) in zip(tris, [(0, 1, 2), (0, 2, 3)]):
        for name, i in (("A", a), ("B", b), ("C", c)):
            getattr(t, name).e[:] = P[i]
            uv = getattr(t, "uv" + name)
            uv.u, uv.v = UVs[i]
        t.mat = material((0.5, 0.5, 0.5))
    qm = (C.c_int * 2)(0, 0)
    mats = (Material * (tw * th))()
    for k in range(tw * th):
        mats[k] = material(tuple(rng.uniform(0.05, 0.95, 3)))
    return tris, qm, mats, tw, th, 1


@pytest.mark.parametrize("tw,th,u0,v0,su,sv,chunks", [(16, 16, -1.3, -0.6, 3.7, 2.9, 1), (16, 16, 0.25, 0.5, 7.0, 5.0, 4),
                                                      (5, 3, -2.1, 0.3, 4.4, 3.3, 4)])
def test_textured_quad_texel_boundaries(tw, th, u0, v0, su, sv, chunks):
    """Thousands of texture hits at and near texel boundaries and integer uv
    wraps (uv spans several repeats, negatives included, 0.25-aligned
    corners): tri_texel's affine fast path and its exact fallback against the
    oracle's exact barycentric path, bit for bit."""
    bundle = helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), _textured_quad(tw, th, u0, v0, su, sv, 7))
    check_parity(bundle, helpers.params(96, 72, 4, 6, chunks=chunks))


def test_tree_ao_c4_scene():
    """C4 scene: README spheres + 1tree_tri.obj (1320 tris,
    Kd-flat materials, leaves = material 1 -> emitter override), AO on with
    the int-truncated intensity, 8 bounces."""
    ref = check_parity(helpers.tree_scene(), helpers.params(32, 24, 4, 8, use_ao=True))
    assert ref["canva"].max() > 0


def test_tree_brute_force_path_matches():
    """Same C4 scene through the every-triangle scan (RT_ACCEL_NONE): the
    triangle arrays stay in BVH leaf order, so this also checks the
    (dst, caller index) tie-break of the unordered scan."""
    check_parity(helpers.tree_scene(), helpers.params(24, 18, 3, 8, use_ao=True, accel=1))


def duplicate_mesh_scene(n=150, seed=5):
    """Random triangles, each present twice (second copy later in the list)
    with a different flat material: every hit on a pair is an exact dst tie
    the reference resolves to the first copy (strict < in list order)."""
    from tipe_rt.types import Triangle, Material, Vec3
    rng = np.random.default_rng(seed)
    base = []
    for _ in range(n):
        c = rng.uniform([-1.5, -1.5, -3.6], [1.5, 1.5, -1.0])
        e = rng.normal(size=(2, 3)) * 0.35
        base.append((c, c + e[0], c + e[1]))
    order = rng.permutation(2 * n)               # caller list: copies interleaved in random order
    tris = (Triangle * (2 * n))()
    qm = (C.c_int * (2 * n))()
    first_seen = set()
    for slot, k in enumerate(order):
        A, B, Cc = base[k % n]
        tris[slot].A, tris[slot].B, tris[slot].C = Vec3(*A), Vec3(*B), Vec3(*Cc)
        qm[slot] = 0 if (k % n) not in first_seen else 2
        first_seen.add(k % n)
    mats = (Material * 3)()
    cols = [(0.9, 0.2, 0.1), (0.5, 0.5, 0.5), (0.1, 0.3, 0.9)]
    for m in range(3):
        mats[m] = tipe_rt.scenes.material(cols[m], (0, 0, 0), 0.0, 0.0, 1.0, 0.0)
    return helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), (tris, qm, mats, 1, 1, 3))


def test_bvh_tie_break_on_duplicate_triangles():
    bundle = duplicate_mesh_scene()
    check_parity(bundle, helpers.params(40, 30, 4, 6))
    check_parity(bundle, helpers.params(24, 18, 2, 6, accel=1))


@pytest.mark.parametrize("case", ["tree_ao", "tree", "duplicates", "grazing", "sweep", "sky_tree"])
def test_bvh_task_queue_kernel_bitexact(case):
    """spp_chunks > 1 with a BVH runs render_kernel_q<.., BVH>: the sphere
    pass, then at most RT_QB_STEPS node visits per lane and round, the walk
    resuming next round while the lane's other work waits.  Exact ties
    (duplicate triangles), grazing rays over a fine grid (deep stacks), AO
    casts and the sky sphere through it, bit-exact vs the oracle."""
    bundle, p = {
        "tree_ao": lambda: (helpers.tree_scene(), helpers.params(40, 30, 8, 8, use_ao=True, chunks=4)),
        "tree": lambda: (helpers.tree_scene(), helpers.params(40, 30, 6, 6, chunks=3)),
        "duplicates": lambda: (duplicate_mesh_scene(), helpers.params(40, 30, 6, 6, chunks=3)),
        "grazing": lambda: (grazing_grid_scene(), helpers.params(40, 30, 4, 6, chunks=2)),
        "sweep": lambda: (helpers.SceneBundle(*tipe_rt.scenes.synthetic_cornell(10, 100)),
                          helpers.params(48, 36, 8, 6, chunks=4)),
        "sky_tree": lambda: (helpers.sky_tree_scene(), helpers.params(32, 24, 6, 5, sky_mode=1, use_ao=True,
                                                                       chunks=3)),
    }[case]()
    check_parity(bundle, p)


def grazing_grid_scene(n=40, seed=11):
    """A fine n x n quad grid (2 n^2 triangles) just above the README box's
    floor, with a small random height on every vertex, seen from a low
    camera: grazing rays cross many boxes, so the cooperative traversal's
    per-wave LIFO and the lanes' own stacks both fill (rt_kernels.hip
    samples_coop)."""
    from tipe_rt.types import Triangle, Material, Vec3, UV
    rng = np.random.default_rng(seed)
    xs = np.linspace(-1.0, 1.0, n + 1)
    zs = np.linspace(-3.5, -0.8, n + 1)
    hgt = -0.95 + rng.uniform(0.0, 0.01, size=(n + 1, n + 1))
    tris = (Triangle * (2 * n * n))()
    qm = (C.c_int * (2 * n * n))()
    t = 0
    for i in range(n):
        for j in range(n):
            p00 = (xs[i], hgt[i, j], zs[j])
            p10 = (xs[i + 1], hgt[i + 1, j], zs[j])
            p01 = (xs[i], hgt[i, j + 1], zs[j + 1])
            p11 = (xs[i + 1], hgt[i + 1, j + 1], zs[j + 1])
            # counter-clockwise seen from above: N = AB x AC points up
            for (a, b, c) in ((p00, p01, p10), (p10, p01, p11)):
                tris[t].A, tris[t].B, tris[t].C = Vec3(*a), Vec3(*b), Vec3(*c)
                tris[t].uvA = tris[t].uvB = tris[t].uvC = UV(0.5, 0.5)
                qm[t] = (i + j) % 2
                t += 1
    mats = (Material * 2)()
    # near-mirrors: reflected grazing rays stay grazing
    mats[0] = tipe_rt.scenes.material((0.8, 0.8, 0.7), (0, 0, 0), 0.0, 0.97)
    mats[1] = tipe_rt.scenes.material((0.2, 0.4, 0.8), (0, 0, 0), 0.0, 0.9)
    return helpers.SceneBundle(tipe_rt.scenes.cornell_spheres(), (tris, qm, mats, 1, 1, 2))


def test_bvh_grazing_grid_deep_traversal():
    bundle = grazing_grid_scene()
    cam = tipe_rt.init_camera((0.0, -0.9, -0.6), (0.0, -0.935, -3.0), (0, 1, 0), 40.0, 4.0 / 3.0)
    check_parity(bundle, helpers.params(32, 24, 4, 6, cam=cam))
    check_parity(bundle, helpers.params(24, 18, 2, 5, cam=cam, use_ao=True, ao=2.0))
    import torch
    p = helpers.params(32, 24, 4, 6, cam=cam)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, 23), d_cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    c = d_cnt.cpu().numpy()
    T = tipe_rt.types
    print("grazing grid: node visits / cast", c[T.RT_CNT_BVH_NODES] / c[T.RT_CNT_CASTS],
          "triangle tests / cast", c[T.RT_CNT_BVH_TRI_TESTS] / c[T.RT_CNT_CASTS])
    # 2.4 node visits per cast of any kind here (sphere-only casts included)
    assert c[T.RT_CNT_BVH_NODES] > 2 * c[T.RT_CNT_CASTS]


def adversarial_sphere_scene():
    """Sphere pairs the candidate pass cannot separate (spheres_closest):
    an exact duplicate (equal t: the reference keeps the first), a sphere
    1e-12 larger than its neighbour, spheres touching each other and the
    floor, a tiny sphere and a huge far one.  Each must fall back to the
    exact scan or be resolved exactly."""
    m = tipe_rt.scenes.material
    extra = [
        ((0.3, 0.2, -2.5), 0.3, m((1, 0, 0))),
        ((0.3, 0.2, -2.5), 0.3, m((0, 1, 0), refl=0.5)),                 # duplicate: first wins
        ((-0.4, 0.1, -2.0), 0.25, m((0, 0, 1))),
        ((-0.4, 0.1, -2.0), 0.25 + 1e-12, m((1, 1, 0))),                  # 1e-12 apart
        ((0.0, -0.5, -1.8), 0.5, m((0.9, 0.9, 0.9), refl=0.9)),          # touches the floor (y = -1)
        ((0.5, -0.5, -1.8), 0.5, m((0.2, 0.8, 0.5))),        # touches the previous one
        ((0.05, 0.3, -1.2), 1e-4, m((1, 1, 1), (1, 1, 1), 3.0)),         # tiny emitter
        ((0.0, 0.0, -2e4), 1e4, m((0.5, 0.5, 0.5))),                     # huge, far
    ]
    return helpers.cornell(extra)


def _stress_rays(spheres, n, seed):
    """Rays that stress the candidate pass's bound: origins on sphere surfaces
    (as a bounce leaves them), directions near tangent at 1e-3..1e-12, rays
    aimed at silhouettes (disc ~ 0), unnormalised directions, far origins."""
    rng = np.random.default_rng(seed)
    C_ = np.array([[s.center.e[0], s.center.e[1], s.center.e[2]] for s in spheres])
    R_ = np.array([s.radius for s in spheres])

    def unit(v):
        return v / np.linalg.norm(v, axis=-1, keepdims=True)
    m = n // 5
    k = rng.integers(0, len(R_), m)
    # 1. surface origins, random and near-tangent directions
    nrm = unit(rng.normal(size=(m, 3)))
    o1 = C_[k] + R_[k, None] * nrm
    tan = unit(np.cross(nrm, rng.normal(size=(m, 3))))
    eps = rng.choice([0.0, 1e-3, 1e-6, 1e-9, 1e-12], m)[:, None] * rng.choice([-1.0, 1.0], (m, 1))
    d1 = np.where(rng.random((m, 1)) < 0.5, unit(rng.normal(size=(m, 3))), tan + eps * nrm)
    # 2. silhouette rays from random box points
    o2 = rng.uniform([-1, -1, -4], [1, 1, 0.5], (m, 3))
    k2 = rng.integers(0, len(R_), m)
    w = C_[k2] - o2
    perp = unit(np.cross(w, rng.normal(size=(m, 3))))
    d2 = (C_[k2] + R_[k2, None] * perp * (1 + rng.choice([0, 1e-9, -1e-9, 1e-14], m)[:, None])) - o2
    # 3. random rays, 4. unnormalised, 5. far origins
    o3 = rng.uniform([-1, -1, -4], [1, 1, 0.5], (m, 3))
    d3 = unit(rng.normal(size=(m, 3)))
    d4 = unit(rng.normal(size=(m, 3))) * 10.0 ** rng.uniform(-3, 3, (m, 1))
    o5 = unit(rng.normal(size=(m, 3))) * rng.uniform(10, 2000, (m, 1))
    d5 = unit(rng.uniform(-1, 1, (m, 3)) - o5)
    o = np.concatenate([o1, o2, o3, o3, o5])
    d = np.concatenate([d1, d2, d3, d4, d5])
    return np.concatenate([o, d], axis=1)


@pytest.mark.parametrize("which", ["cornell", "adversarial"])
def test_sphere_candidate_pass_stress(which):
    """5M stress rays: the candidate pass (with its exact fallback) returns the
    exact scan's winner and distance bit for bit on every ray."""
    bundle = helpers.cornell() if which == "cornell" else adversarial_sphere_scene()
    rays = _stress_rays(bundle.spheres, 5_000_000, 7 if which == "cornell" else 8)
    fb, bad = tipe_rt.verify_sphere_pass(bundle.scene, rays)
    assert bad == 0
    assert fb < len(rays) // 2


def test_sphere_candidate_pass_adversarial():
    import torch
    bundle = adversarial_sphere_scene()
    check_parity(bundle, helpers.params(48, 36, 8, 6))
    check_parity(bundle, helpers.params(32, 24, 4, 6, use_ao=True, ao=2.5, compat=0))
    p = helpers.params(48, 36, 4, 6)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, 35), d_cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    assert d_cnt[tipe_rt.types.RT_CNT_EXACT_RESCANS].item() > 0      # the fallback scan ran


@pytest.mark.parametrize("W,H", [(1, 1), (1, 5), (5, 1), (2, 2), (17, 3)])
def test_degenerate_frames(W, H):
    """largeur_image or hauteur_image of 1 makes main.c:265 divide by zero
    (u or v = +-inf / nan); the kernel must follow the same IEEE path."""
    check_parity(helpers.cornell(), helpers.params(W, H, 3, 5))


def test_c5_4k_frame_pyramid_one_spp():
    """C5's 3840x2880 frame (pyramid scene) at 1 spp: 11.06M
    pixels, pixel indices beyond 2^23, every row of a 4K framebuffer."""
    bundle = helpers.pyramid_scene()
    p = helpers.params(3840, 2880, 1, 6)
    ref = helpers.oracle_render(bundle, p, nthreads=16)
    canva, alb, nrm, rad = gpu_render(bundle, p)
    assert_same(canva, ref["canva"], "canva")
    assert_same(rad, ref["radiance"], "radiance")
    assert_same(alb, ref["albedo"], "albedo")
    assert_same(nrm, ref["normal"], "normal")


def test_counters_match_oracle():
    import torch
    bundle = helpers.pyramid_scene()
    p = helpers.params(32, 24, 8, 6, use_ao=True)
    ref = helpers.oracle_render(bundle, p, counters=True)["counters"]
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    with tipe_rt.reference_counts():
        tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, 23), d_cnt.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    got = d_cnt.cpu().numpy().astype(np.uint64)
    ds.close()
    k = tipe_rt.types.RT_CNT_EXACT_RESCANS           # GPU-only diagnostic
    assert list(got[:k]) == list(ref[:k]), dict(zip(tipe_rt.COUNTER_NAMES, zip(got, ref)))
    assert got[k] <= got[tipe_rt.types.RT_CNT_CASTS] // 1000   # candidate pass almost never ambiguous


def _counts(bundle, p, rows):
    import torch
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, rows - 1), d_cnt.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    return d_cnt.cpu().numpy()


@pytest.mark.parametrize("scene,ao", [("cornell", False), ("cornell", True), ("pyramid", True), ("tree", True)])
def test_zero_throughput_exit(scene, ao):
    """Paths end once rayColor == 0 (rt_set_zero_throughput_exit): frames are
    bit-identical with the exit on and off and to the oracle (which never
    exits), and the exit only removes casts."""
    bundle = {"cornell": helpers.cornell, "pyramid": helpers.pyramid_scene, "tree": helpers.tree_scene}[scene]()
    p = helpers.params(32, 24, 8, 6, use_ao=ao, ao=2.5, compat=0)
    check_parity(bundle, p)
    on = gpu_render(bundle, p)
    with tipe_rt.reference_counts():
        off = gpu_render(bundle, p)
        ref_cnt = _counts(bundle, p, 24)
    for a, b in zip(on, off):
        assert_same(a, b, "exit on vs off")
    cnt = _counts(bundle, p, 24)
    T = tipe_rt.types
    assert cnt[T.RT_CNT_SAMPLES] == ref_cnt[T.RT_CNT_SAMPLES]
    assert cnt[T.RT_CNT_CASTS] < ref_cnt[T.RT_CNT_CASTS]
    print(scene, "ao" if ao else "", "casts per sample", ref_cnt[T.RT_CNT_CASTS] / ref_cnt[0], "->",
          cnt[T.RT_CNT_CASTS] / cnt[0])


def test_zero_throughput_exit_gated_off():
    """A material beyond the exit's bound (emission strength 1e200 > 2^100:
    the host cannot rule out em overflowing to inf, and inf * 0 is NaN) or
    AO_intensity outside (0, 1000] turns the exit off: the counts are then
    the reference's."""
    spheres = tipe_rt.scenes.cornell_spheres()
    spheres[3].mat.emissionStrength = 1e200
    bundle = helpers.SceneBundle(spheres)
    p = helpers.params(16, 12, 4, 6)
    check_parity(bundle, p)
    ref = helpers.oracle_render(bundle, p, counters=True)["counters"]
    cnt = _counts(bundle, p, 12)
    assert cnt[tipe_rt.types.RT_CNT_CASTS] == ref[tipe_rt.types.RT_CNT_CASTS]
    bundle = helpers.cornell()
    p = helpers.params(16, 12, 4, 6, use_ao=True, ao=2000.0, compat=0)
    check_parity(bundle, p)
    ref = helpers.oracle_render(bundle, p, counters=True)["counters"]
    cnt = _counts(bundle, p, 12)
    assert cnt[tipe_rt.types.RT_CNT_CASTS] == ref[tipe_rt.types.RT_CNT_CASTS]


# ---- boundary behaviour --------------------------------------------------------
def test_render_rows_host_api_band():
    bundle = helpers.cornell()
    p = helpers.params(48, 36, 4, 5)
    ref = helpers.oracle_render(bundle, p)
    canva = np.full((36, 48, 3), -7.0)
    alb = np.full((36, 48, 3), -7.0)
    nrm = np.full((36, 48, 3), -7.0)
    tipe_rt.check(tipe_rt.lib().rt_render_rows(C.byref(bundle.scene), C.byref(p), 20, 9, canva.ctypes.data,
                                               alb.ctypes.data, nrm.ctypes.data))
    assert (canva[9:21] == ref["canva"][9:21]).all()
    assert (alb[9:21] == ref["albedo"][9:21]).all() and (nrm[9:21] == ref["normal"][9:21]).all()
    untouched = np.ones(36, bool)
    untouched[9:21] = False
    assert (canva[untouched] == -7.0).all()       # only the named rows are written


def test_cyclic_tiles_assemble_to_full_frame():
    import torch
    bundle = helpers.cornell()
    W, H, k, world = 40, 30, 4, 3
    p = helpers.params(W, H, 4, 5)
    ref = helpers.oracle_render(bundle, p)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    stream = torch.cuda.current_stream().cuda_stream
    per_rank = tipe_rt.cyclic_tiling(H, k, 0, world).n_tiles
    gathered = torch.zeros((world, per_rank * k, W, 3), dtype=torch.float64, device="cuda:0")
    for r in range(world):
        t = tipe_rt.cyclic_tiling(H, k, r, world)
        tipe_rt.render_async(ds, p, t, gathered[r].data_ptr(), stream=stream)
    full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    tipe_rt.assemble_async(gathered.data_ptr(), world, k, per_rank * k, W, H, full.data_ptr(), stream)
    torch.cuda.synchronize()
    ds.close()
    assert (full.cpu().numpy() == ref["canva"]).all()


def test_fill_canva_pthread_dropin():
    """rt_fill_canva takes main.c's ThreadData; 4 threads on disjoint bands."""
    bundle = helpers.cornell()
    W, H = 40, 30
    p = helpers.params(W, H, 4, 5)
    ref = helpers.oracle_render(bundle, p)
    canva, alb, nrm = (np.zeros((H, W, 3)) for _ in range(3))
    tds = []
    bands = [(29, 22), (21, 15), (14, 8), (7, 0)]
    for hi, lo in bands:
        td = ThreadData()
        td.start_row, td.end_row = hi, lo
        td.canva = C.cast(canva.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.albedo_tab = C.cast(alb.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.normal_tab = C.cast(nrm.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.cam = p.cam
        td.largeur_image, td.hauteur_image = W, H
        td.nbRayonParPixel, td.nbRebondMax = 4, 5
        td.total_pixels = W * H
        td.sphere_list = C.cast(bundle.spheres, C.POINTER(Sphere))
        td.nbSpheres = len(bundle.spheres)
        td.focus_distance = 3
        tds.append(td)
    res = []
    ths = [threading.Thread(target=lambda t=t: res.append(tipe_rt.lib().rt_fill_canva(C.byref(t)))) for t in tds]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert all(r is None for r in res), tipe_rt.lib().rt_last_error()
    assert (canva == ref["canva"]).all() and (alb == ref["albedo"]).all() and (nrm == ref["normal"]).all()


def test_invalid_arguments_fail_loudly():
    bundle = helpers.cornell()
    p = helpers.params(8, 6, 0, 5)
    canva = np.zeros((6, 8, 3))
    rc = tipe_rt.lib().rt_render_rows(C.byref(bundle.scene), C.byref(p), 5, 0, canva.ctypes.data, None, None)
    assert rc == tipe_rt.RT_EINVAL and b"nbRayonParPixel" in tipe_rt.lib().rt_last_error()
    p = helpers.params(8, 6, 1, 5, rng=tipe_rt.RT_RNG_GLIBC)
    rc = tipe_rt.lib().rt_render_rows(C.byref(bundle.scene), C.byref(p), 5, 0, canva.ctypes.data, None, None)
    assert rc == tipe_rt.RT_EUNSUPPORTED


@pytest.mark.parametrize("tw,th", [(16, 16), (3, 1), (64, 5), (1, 1)])
def test_texel_map_fast_path_stress(tw, th):
    """rt_verify_texel_map: the affine uv fast path (rt_api.cpp tri_uv_affine
    + tri_texel_affine) against the reference's barycentric operations on
    random triangles (scales 1e-3..1e2, far from the origin, skinny ones),
    random and grid-aligned uvs (boundaries through structured points, uv
    repeats, negatives), and points in and around each triangle (barycentric
    coordinates on a 1/16 grid and random ones, off the plane by up to the
    triangle's size): no point may get another texel, and the fast path must
    decide almost every point."""
    from tipe_rt.scenes import material
    rng = np.random.default_rng(1000 + tw * 7 + th)
    total_fast = total = 0
    for scene_i in range(12):
        nt = 32
        tris = (Triangle * nt)()
        A = np.zeros((nt, 3)); B = np.zeros((nt, 3)); Cc = np.zeros((nt, 3))
        for k in range(nt):
            s = 10.0 ** rng.uniform(-3, 2)
            c = rng.uniform(-1, 1, 3) * (s * 10.0 ** rng.uniform(0, 3))
            a, b, cc = c + rng.normal(size=3) * s, c + rng.normal(size=3) * s, c + rng.normal(size=3) * s
            if k % 8 == 7:                                   # skinny: C near the segment AB
                cc = a + (b - a) * rng.uniform(0.2, 0.8) + rng.normal(size=3) * s * 1e-3
            A[k], B[k], Cc[k] = a, b, cc
            for name, v in (("A", a), ("B", b), ("C", cc)):
                getattr(tris[k], name).e[:] = tuple(v)
            if k % 2:                                        # grid-aligned uvs: multiples of 1/tw, 1/th
                uvs = [(rng.integers(-2 * tw, 3 * tw) / tw, rng.integers(-2 * th, 3 * th) / th) for _ in range(3)]
            else:
                uvs = [tuple(rng.uniform(-3, 6, 2)) for _ in range(3)]
            for name, (u, v) in zip(("uvA", "uvB", "uvC"), uvs):
                getattr(tris[k], name).u, getattr(tris[k], name).v = u, v
            tris[k].mat = material((0.5, 0.5, 0.5))
        qm = (C.c_int * nt)(*([0] * nt))
        mats = (Material * (tw * th))()
        for i in range(tw * th):
            mats[i] = material((0.5, 0.5, 0.5))
        scene = tipe_rt.make_scene(tipe_rt.scenes.cornell_spheres(), tris, qm, mats, tw, th, 1)
        m = 1 << 16
        tri = rng.integers(0, nt, m)
        grid = rng.integers(-3, 20, (m, 2)) / 16.0
        rnd = rng.uniform(-0.2, 1.2, (m, 2))
        bc = np.where((np.arange(m) % 2 == 0)[:, None], grid, rnd)
        b0, b1 = bc[:, 0], bc[:, 1]
        b2 = 1.0 - b0 - b1
        P = b0[:, None] * A[tri] + b1[:, None] * B[tri] + b2[:, None] * Cc[tri]
        N = np.cross(B[tri] - A[tri], Cc[tri] - A[tri])
        nl = np.linalg.norm(N, axis=1)[:, None]
        size = np.max(np.abs(np.stack([B[tri] - A[tri], Cc[tri] - A[tri]])), axis=(0, 2))[:, None]
        off = np.where((np.arange(m) % 3 == 0)[:, None], 0.0, rng.uniform(-1, 1, (m, 1)) * size)
        P = P + off * N / np.where(nl > 0, nl, 1.0)
        fast, bad = tipe_rt.verify_texel_map(scene, P, tri)
        assert bad == 0, (scene_i, fast, bad)
        total_fast += fast
        total += m
    print("texel map fast path: %d of %d points" % (total_fast, total))
    assert total_fast >= 0.5 * total, (total_fast, total)
