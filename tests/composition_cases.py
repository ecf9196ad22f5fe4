"""Scenes that pin the oracle's COMPOSITION (tracer / closest_hit /
ambient_occlusion / fill_canva, main.c:52-284) against the reference's own
code compiled here (oracle/_ref/libref_tracer.so, oracle/build_ref_tracer.sh).

TEST INFRASTRUCTURE.  Every case renders in the reference's own stream mode:
glibc rand() reseeded with srand(1), libm, one thread, running per-pixel sums
(spp_chunks 1).  Each case names the reference driver that produced its
fixture:

  fill_canva  the reference's fill_canva itself in one pthread (main.c:446),
              fed a struct ThreadData (int focus / aperture / AO, main.c:42-43)
  trace_rows  the same loop nest around the reference's tracer with a double
              AO intensity (tracer's own parameter type, main.c:118) and the
              pre-quantisation radiance plane

The oracle renders the same case through oracle_render_rows in RT_RNG_GLIBC
mode; `compat` selects ThreadData's integer truncation (rt.h
compat_int_truncation).
"""
import ctypes as C

import numpy as np

import helpers
import oracle_ffi
from tipe_rt import scenes
from tipe_rt.types import RT_RNG_GLIBC

PLANES = ("canva", "albedo", "normal", "radiance")


class Case:
    def __init__(self, name, build, W, H, spp, bounces, use_ao=False, ao=0.0, driver="trace_rows",
                 slow=False, what="", cam=None):
        self.name, self.build, self.W, self.H = name, build, W, H
        self.spp, self.bounces, self.use_ao, self.ao = spp, bounces, use_ao, ao
        self.driver, self.slow, self.what, self.cam = driver, slow, what, cam

    def scene(self):
        """-> (bundle, params) for the oracle in GLIBC mode."""
        b = self.build()
        if isinstance(b, tuple):                 # random scene: (bundle, params)
            bundle, p = b
            p.rng = RT_RNG_GLIBC
            p.spp_chunks = 1
            return bundle, p
        p = helpers.params(self.W, self.H, self.spp, self.bounces, use_ao=self.use_ao, ao=self.ao,
                           rng=RT_RNG_GLIBC, compat=1 if self.driver == "fill_canva" else 0,
                           cam=None if self.cam is None else helpers.camera_of(self.cam))
        return b, p


def _random(seed, bounce_hi=9):
    """tests/test_gpu_fuzz.random_scene(seed) inside a black, opaque sphere of
    radius 1e4 (appended last).  Without it a primary miss leaves the
    reference's albedo/normal undefined: closest_hit (main.c:54-56) never sets
    HitInfo.mat / .normal on a miss and tracer (main.c:137-140) reads them, so
    the reference adds stale stack values (seen on seeds 6 and 11), where the
    build defines 0.  Secondary misses (main.c:236-238) stay
    covered by the README-box cases (the box is open towards +z)."""
    def build():
        from test_gpu_fuzz import random_scene     # noqa: WPS433 (shared generator)
        from tipe_rt.types import Sphere, Vec3
        bundle, p = random_scene(seed, bounce_hi=bounce_hi)
        n = len(bundle.spheres)
        sph = (Sphere * (n + 1))()
        for k in range(n):
            sph[k] = bundle.spheres[k]
        sph[n].center = Vec3(0.0, 0.0, 0.0)
        sph[n].radius = 1e4
        sph[n].mat = scenes.material((0, 0, 0), (0, 0, 0), 0.0, 0.0, 1.0, 1.0)
        return helpers.SceneBundle(sph, bundle.mesh), p
    return build


def _glass():
    """README box with every sphere translucent (alpha 0.5, IOR 1.5): the
    IOR stack's enter/exit pairs (pile.h, main.c:169-181) on closed spheres."""
    return helpers.SceneBundle(scenes.cornell_spheres(alpha=0.5, material_index=1.5))


def _holes():
    """README box plus alpha-hole spheres (alpha 0, main.c:200-206) in front of
    lit ones: the alpha_depth / is_alpha albedo bookkeeping (main.c:137-150)."""
    hole = scenes.material((0.8, 0.8, 0.8), (0, 0, 0), 0.0, 0.0, 0.0, 1.0)
    return helpers.SceneBundle(scenes.cornell_spheres(extra=[((0.0, -0.3, -1.6), 0.45, hole),
                                                              ((-0.4, 0.6, -1.0), 0.3, hole)]))


CASES = [
    Case("c1_full", helpers.cornell, 400, 300, 100, 5, driver="fill_canva", slow=True,
         what="BASELINE config 1 itself: README box, 400x300, 100 spp, 5 bounces"),
    Case("cornell_ao_int2", helpers.cornell, 64, 48, 16, 6, use_ao=True, ao=2.0, driver="fill_canva",
         what="README box + AO, ThreadData's int AO_intensity 2"),
    Case("cornell_ao_2p5", helpers.cornell, 64, 48, 16, 6, use_ao=True, ao=2.5,
         what="README box + AO 2.5 as a double (pow(x, 2.5), 1.5*AO emission)"),
    Case("glass_spheres", _glass, 64, 48, 16, 6,
         what="all spheres translucent: refraction + IOR stack enter/exit"),
    Case("hole_spheres", _holes, 64, 48, 16, 6, use_ao=True, ao=2.0, driver="fill_canva",
         what="alpha-hole spheres + AO: alpha_depth albedo bookkeeping"),
    Case("pyramid", helpers.pyramid_scene, 64, 48, 16, 6,
         what="C3: pyramid mesh, 16x16 water texture, alpha 0.706 refraction"),
    Case("pyramid_ao_int2", helpers.pyramid_scene, 64, 48, 16, 6, use_ao=True, ao=2.0, driver="fill_canva",
         what="C3 scene + AO through fill_canva"),
    Case("mineways", helpers.mineways_scene, 64, 48, 16, 6,
         what="mineways_tri.obj: 11 textures incl. alpha-hole leaves"),
    Case("tree_ao_int2", helpers.tree_scene, 64, 48, 16, 8, use_ao=True, ao=2.5, driver="fill_canva",
         what="C4: 1320-triangle tree + AO 2.5 truncated to 2 by ThreadData (main.c:43), 8 bounces"),
    Case("tree_ao_2p5", helpers.tree_scene, 48, 36, 8, 8, use_ao=True, ao=2.5,
         what="C4 scene with AO 2.5 kept as a double"),
] + [Case("random_%d" % s, _random(s), 0, 0, 0, 0,
          what="tests/test_gpu_fuzz.random_scene(%d) (aperture, focus, AO, textures, mesh)" % s)
     for s in range(12)] + [
    # r06: main.c's own default depth nbRebondMax 20 (main.c:310) and 10 (the
    # nature render, RTX_nature_..._9RB: nbRebondMax - 1 = 9, main.c:328), and
    # main()'s coordinate regime (camera main.c:300-301, sky sphere 1e5 main.c:346)
    Case("glass_b20", _glass, 64, 48, 16, 20,
         what="translucent spheres at main.c's default 20 bounces: deep IOR enter/exit chains"),
    Case("holes_ao_b20", _holes, 64, 48, 16, 20, use_ao=True, ao=2.0, driver="fill_canva",
         what="alpha-hole spheres + AO (int 2), 20 bounces"),
    Case("mineways_b10", helpers.mineways_scene, 64, 48, 16, 10, what="mineways alpha texels, 10 bounces"),
    Case("mineways_b20", helpers.mineways_scene, 48, 36, 16, 20, what="mineways alpha texels, 20 bounces"),
    Case("tree_ao_b10", helpers.tree_scene, 48, 36, 8, 10, use_ao=True, ao=2.5, driver="fill_canva",
         what="C4 tree + AO 2.5 -> int 2 through fill_canva, 10 bounces"),
    Case("tree_ao_2p5_b20", helpers.tree_scene, 40, 30, 8, 20, use_ao=True, ao=2.5,
         what="C4 tree + AO 2.5 (double), 20 bounces"),
    Case("nature_b10", helpers.nature_scene, 48, 36, 8, 10, cam=scenes.NATURE_CAMERA,
         what="RTX_MAP/nature (5812 tris, 31 textures with alpha, texture.h overrides) + main.c:345-346 "
              "sun and sky, 10 bounces (the reference render's own depth)"),
    Case("nature_ao_b20", helpers.nature_scene, 32, 24, 4, 20, use_ao=True, ao=2.5, cam=scenes.NATURE_CAMERA,
         what="nature + AO 2.5 at main.c's default 20 bounces"),
    Case("main_regime_b20", helpers.main_regime_scene, 64, 40, 8, 20, cam=scenes.MAIN_CAMERA,
         what="main()'s defaults: pyramide_eau mesh at +-1813, camera main.c:300-301 (vfov 30.2, 16:10), "
              "sun + radius-1e5 sky (main.c:345-346), 20 bounces"),
    Case("main_regime_ao_b20", helpers.main_regime_scene, 48, 30, 8, 20, use_ao=True, ao=2.5,
         cam=scenes.MAIN_CAMERA, what="main()'s regime + AO 2.5 (main.c:316-317 values), 20 bounces"),
] + [Case("random_deep_%d" % s, _random(s, bounce_hi=25), 0, 0, 0, 0,
          what="tests/test_gpu_fuzz.random_scene(%d, bounce_hi=25): 0-24 bounces" % s)
     for s in (704, 705, 707, 708, 709, 712, 714, 717)]   # seeds drawing >= 12 bounces

BY_NAME = {c.name: c for c in CASES}


def oracle_planes(case):
    bundle, p = case.scene()
    out = helpers.oracle_render(bundle, p)
    return out


def reference_planes(case):
    """Render the case through the reference's own compiled composition.
    Returns None when oracle/_ref/libref_tracer.so is unavailable.

    fill_canva cases run the reference's fill_canva AND the trace_rows loop
    (same truncated ints) and require the two to agree bit for bit on canva,
    albedo and normal — the check that trace_rows is fill_canva's loop nest;
    the radiance plane then comes from trace_rows."""
    lib = oracle_ffi.ref_tracer()
    if lib is None:
        return None
    bundle, p = case.scene()
    sc = bundle.scene
    W, H, S, B = p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax
    out = {k: np.zeros((H, W, 3)) for k in PLANES}
    cam = p.cam
    geo = (sc.sphere_list, sc.nbSpheres, sc.triangle_list, sc.nbTriangles, sc.mat_list,
           sc.tex_width, sc.tex_height, sc.quelMatPourTri, C.byref(cam), W, H, S, B)
    f, ox, oy, ao = p.focus_distance, p.ouverture_x, p.ouverture_y, p.AO_intensity
    if p.compat_int_truncation:                 # what oracle_render_rows does with ThreadData's ints
        f, ox, oy, ao = float(int(f)), float(int(ox)), float(int(oy)), float(int(ao))
    lib.ref_tracer_srand(1)
    rc = lib.ref_trace_rows(*geo, f, ox, oy, int(p.useAO), ao, H - 1, 0,
                            out["canva"].ctypes.data, out["albedo"].ctypes.data, out["normal"].ctypes.data,
                            out["radiance"].ctypes.data)
    assert rc == 0, rc
    if case.driver == "fill_canva":
        assert p.compat_int_truncation
        fc = {k: np.zeros((H, W, 3)) for k in PLANES[:3]}
        lib.ref_tracer_srand(1)
        rc = lib.ref_fill_canva(*geo, int(p.focus_distance), int(p.ouverture_x), int(p.ouverture_y),
                                int(p.useAO), int(p.AO_intensity), H - 1, 0,
                                fc["canva"].ctypes.data, fc["albedo"].ctypes.data, fc["normal"].ctypes.data)
        assert rc == 0, rc
        for k in fc:
            assert fc[k].tobytes() == out[k].tobytes(), "trace_rows != the reference's fill_canva on " + k
    return out


def reference_planes_philox(bundle, p):
    """The reference's own composition with the GPU's stream spec (RT_RNG_PHILOX
    draws keyed by (seed, pixel, sample); portable acos/sinf/cosf/pow) and
    p.spp_chunks' slice grouping: what librt_hip.so must produce bit for bit.
    None when oracle/_ref/libref_tracer_philox.so is unavailable."""
    lib = oracle_ffi.ref_tracer_philox()
    if lib is None:
        return None
    sc = bundle.scene
    W, H, S, B = p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax
    out = {k: np.zeros((H, W, 3)) for k in PLANES}
    cam = p.cam
    f, ox, oy, ao = p.focus_distance, p.ouverture_x, p.ouverture_y, p.AO_intensity
    if p.compat_int_truncation:
        f, ox, oy, ao = float(int(f)), float(int(ox)), float(int(oy)), float(int(ao))
    rc = lib.ref_trace_rows_philox(sc.sphere_list, sc.nbSpheres, sc.triangle_list, sc.nbTriangles, sc.mat_list,
                                   sc.tex_width, sc.tex_height, sc.quelMatPourTri, C.byref(cam), W, H, S, B,
                                   f, ox, oy, int(p.useAO), ao, p.seed, p.spp_chunks, H - 1, 0,
                                   *[out[k].ctypes.data for k in PLANES])
    assert rc == 0, rc
    return out


# ---- the GPU's stream spec: cases for tests/golden/gpu_reference.json ------
class PhiloxCase:
    """A scene + RT_RNG_PHILOX params; `chunks` picks the kernel family the
    GPU takes (1: fixed grid; > 1: the persistent queue kernel)."""

    def __init__(self, name, build, W=64, H=48, spp=16, bounces=6, use_ao=False, ao=0.0, compat=1, chunks=32,
                 seed=1010, what="", cam=None, kernel=None):
        self.name, self.build, self.W, self.H, self.spp, self.bounces = name, build, W, H, spp, bounces
        self.use_ao, self.ao, self.compat, self.chunks, self.seed, self.what = use_ao, ao, compat, chunks, seed, what
        self.cam, self.kernel = cam, kernel      # kernel: rt_last_render_kernel() the GPU must take

    def scene(self):
        b = self.build()
        if isinstance(b, tuple):                 # random scene: its own params, Philox stream
            return b
        p = helpers.params(self.W, self.H, self.spp, self.bounces, use_ao=self.use_ao, ao=self.ao,
                           seed=self.seed, compat=self.compat, chunks=self.chunks,
                           cam=None if self.cam is None else helpers.camera_of(self.cam))
        return b, p


def _random_philox(seed, bounce_hi=9):
    return _random(seed, bounce_hi)


PHILOX_CASES = [
    PhiloxCase("c2_queue", helpers.cornell, what="C2 scene, spp_chunks AUTO (queue kernel, QB -2)"),
    PhiloxCase("c2_fixed_grid", helpers.cornell, chunks=1, what="C2 scene, fill_canva's order (fixed grid)"),
    PhiloxCase("c2_ao_2p5", helpers.cornell, use_ao=True, ao=2.5, compat=0, chunks=4,
               what="README box + AO 2.5 (double), queue kernel"),
    PhiloxCase("glass_spheres", _glass, chunks=4, what="translucent spheres (QB -1)"),
    PhiloxCase("hole_spheres_ao", _holes, use_ao=True, ao=2.0, chunks=3, what="alpha-hole spheres + AO"),
    PhiloxCase("c3_pyramid", helpers.pyramid_scene, what="C3 scene, queue kernel (QB 0)"),
    PhiloxCase("c3_pyramid_fixed", helpers.pyramid_scene, chunks=1, what="C3 scene, fixed grid"),
    PhiloxCase("mineways", helpers.mineways_scene, chunks=4, what="alpha-hole texels, BVH queue kernel (QB 3)"),
    PhiloxCase("c4_tree_ao", helpers.tree_scene, W=48, H=36, spp=8, bounces=8, use_ao=True, ao=2.5,
               chunks=4, what="C4 scene (AO 2.5 -> 2, ThreadData's int), deep-tree opaque kernel"),
    PhiloxCase("c4_tree_ao_2p5", helpers.tree_scene, W=40, H=30, spp=8, bounces=8, use_ao=True, ao=2.5,
               compat=0, chunks=1, what="C4 scene with AO 2.5 as a double, fixed-grid BVH kernel"),
] + [PhiloxCase("random_%d" % s, _random_philox(s), what="enclosed tests/test_gpu_fuzz.random_scene(%d)" % s)
     for s in range(100, 116)] + [
    # r06: 10 / 20 bounces (main.c:310), the nature scene, main()'s coordinate regime
    PhiloxCase("glass_b20", _glass, bounces=20, chunks=4, what="translucent spheres, 20 bounces (QB -1)"),
    PhiloxCase("glass_b20_fixed", _glass, W=48, H=36, bounces=20, chunks=1,
               what="translucent spheres, 20 bounces, fixed grid"),
    PhiloxCase("holes_ao_b20", _holes, bounces=20, use_ao=True, ao=2.0, chunks=3,
               what="alpha-hole spheres + AO, 20 bounces"),
    PhiloxCase("mineways_b10", helpers.mineways_scene, bounces=10, chunks=4, what="mineways, 10 bounces (QB 3)"),
    PhiloxCase("mineways_b20", helpers.mineways_scene, W=48, H=36, bounces=20, chunks=32,
               what="mineways, 20 bounces, spp_chunks 32"),
    PhiloxCase("c4_tree_ao_b10", helpers.tree_scene, W=48, H=36, spp=8, bounces=10, use_ao=True, ao=2.5,
               chunks=4, what="C4 tree + AO (int 2), 10 bounces, deep-tree opaque kernel"),
    PhiloxCase("c4_tree_ao_b20", helpers.tree_scene, W=40, H=30, spp=8, bounces=20, use_ao=True, ao=2.5,
               compat=0, chunks=8, kernel="render_kernel_q<QB=3,OP>", what="C4 tree + AO 2.5 (double), 20 bounces, deep-tree opaque kernel"),
    PhiloxCase("nature_b10", helpers.nature_scene, W=48, H=36, spp=8, bounces=10, chunks=4,
               cam=scenes.NATURE_CAMERA, kernel="render_kernel_q<QB=3>",
               what="RTX_MAP/nature, 10 bounces: non-opaque deep-tree kernel (QB 3)"),
    PhiloxCase("nature_b10_fixed", helpers.nature_scene, W=40, H=30, spp=4, bounces=10, chunks=1,
               cam=scenes.NATURE_CAMERA, kernel="render_kernel<BVH>",
               what="RTX_MAP/nature, 10 bounces, fixed-grid BVH kernel"),
    PhiloxCase("nature_ao_b20", helpers.nature_scene, W=32, H=24, spp=8, bounces=20, use_ao=True, ao=2.5,
               compat=0, chunks=8, cam=scenes.NATURE_CAMERA, kernel="render_kernel_q<QB=3>",
               what="nature + AO 2.5, 20 bounces"),
    PhiloxCase("main_regime_b20", helpers.main_regime_scene, W=64, H=40, spp=8, bounces=20, chunks=4,
               cam=scenes.MAIN_CAMERA, kernel="render_kernel<BVH>",
               what="main()'s camera / mesh scale / radius-1e5 sky, 20 bounces (34 triangles of up to ~4000 "
                    "units: no binary16 nodes, sky hit points beyond R_b, so the fixed-grid BVH kernel)"),
    PhiloxCase("main_regime_ao_b20", helpers.main_regime_scene, W=48, H=30, spp=8, bounces=20, use_ao=True,
               ao=2.5, compat=0, chunks=3, cam=scenes.MAIN_CAMERA, what="main()'s regime + AO 2.5, 20 bounces"),
    PhiloxCase("main_regime_fixed", helpers.main_regime_scene, W=48, H=30, spp=4, bounces=20, chunks=1,
               cam=scenes.MAIN_CAMERA, what="main()'s regime, 20 bounces, fixed grid"),
] + [PhiloxCase("random_deep_%d" % s, _random_philox(s, bounce_hi=25),
                what="enclosed tests/test_gpu_fuzz.random_scene(%d, bounce_hi=25)" % s)
     for s in (722, 724, 726, 728, 730, 731, 732, 735)]   # seeds drawing >= 12 bounces

PHILOX_BY_NAME = {c.name: c for c in PHILOX_CASES}


def plane_sha(a):
    """sha256 of a plane's float64 bytes with NaN and -0.0 made canonical
    (payloads and zero signs are not compared: gfx950 and x86 make
    different default NaNs, and the parity suite compares with ==)."""
    import hashlib
    a = np.ascontiguousarray(a, dtype="<f8").copy()
    a[np.isnan(a)] = np.nan
    a[a == 0] = 0.0
    return hashlib.sha256(a.tobytes()).hexdigest()
