"""Randomised scenes, GPU vs oracle bit for bit (RT_RNG_PHILOX).

Each seed builds a scene the hand-written tests do not: random spheres
(some enclosing the camera, translucent ones with 1e-4 <= alpha <= 0.99,
alpha holes, emitters, mirrors), optionally a random textured mesh with
the reference's hard-coded material overrides (texture.h:71-87, indices
1/3/4), random camera, aperture, focus, AO on/off, spp_chunks, and more
than 32 triangles on odd seeds so the BVH path runs.  Sizes stay small
so the oracle finishes in about a second per scene."""
import ctypes as C

import numpy as np
import pytest

import helpers
import tipe_rt
from tipe_rt import scenes
from tipe_rt.types import Sphere, Triangle, Material, Vec3, UV
from test_gpu_parity import check_parity, assert_stack_bound_holds

pytestmark = pytest.mark.gpu


def _zero_some(rng, c, zeros):
    """With zeros, each colour channel is exactly 0 with probability 0.35,
    so rayColor reaches (0, 0, 0) and the zero-throughput exit runs."""
    if not zeros:
        return c
    return tuple(0.0 if rng.random() < 0.35 else float(x) for x in c)


def random_scene(seed, zeros=False, chunks=None, nt_range=None, spp=None, opaque=False, mesh_p=0.7,
                 bounce_hi=25, far=False):
    """bounce_hi: nbRebondMax is drawn from [0, bounce_hi), covering main.c's
    own default of 20 (main.c:310); the scenes pinned by reference fixtures
    (tests/composition_cases._random) keep the r05 draw, bounce_hi 9.
    far: the scene moved into main()'s coordinate regime (below).
    opaque: only opaque materials (no glass or hole spheres, texels at
    alpha 1, no material index 3 or 4), the scenes the queue kernel's
    opaque instantiations take (QB -2, the deep-tree OPQ kernel);
    mesh_p: probability of a mesh when nt_range is None."""
    rng = np.random.default_rng(seed)
    ns = int(rng.integers(1, 14))
    sph = (Sphere * ns)()
    for k in range(ns):
        kind = rng.choice(["diffuse", "mirror", "light", "big"] if opaque
                          else ["diffuse", "mirror", "glass", "hole", "light", "big"])
        c = rng.uniform([-2, -2, -6], [2, 2, -1])
        r = rng.uniform(0.2, 1.2)
        diff = _zero_some(rng, tuple(rng.uniform(0, 1, 3)), zeros)
        em, es, refl, alpha, ior = (0, 0, 0), 0.0, 0.0, 1.0, 1.0
        if kind == "mirror":
            refl = float(rng.uniform(0.5, 1.0))
        elif kind == "glass":
            alpha, ior = float(rng.uniform(0.05, 0.99)), float(rng.uniform(1.0, 2.0))
        elif kind == "hole":
            alpha = 0.0
        elif kind == "light":
            em, es = tuple(rng.uniform(0.2, 1, 3)), float(rng.uniform(0.5, 5))
        elif kind == "big":                               # encloses the camera
            c, r = rng.uniform(-0.5, 0.5, 3), float(rng.uniform(20, 600))
        sph[k].center = Vec3(*c)
        sph[k].radius = r
        sph[k].mat = scenes.material(diff, em, es, refl, alpha, ior)
    mesh = None
    if nt_range is not None or rng.random() < mesh_p:
        nt = int(rng.integers(40, 120)) if seed % 2 else int(rng.integers(1, 20))
        if nt_range is not None:
            nt = int(rng.integers(*nt_range))
        tris = (Triangle * nt)()
        nm, tw, th = 5, int(rng.integers(1, 5)), int(rng.integers(1, 5))
        qm = (C.c_int * nt)(*[int(x) for x in (rng.choice([0, 1, 2], nt) if opaque else rng.integers(0, nm, nt))])
        for k in range(nt):
            A = rng.uniform([-2, -2, -5], [2, 2, -1.5])
            e = rng.normal(size=(2, 3)) * 0.5
            tris[k].A, tris[k].B, tris[k].C = Vec3(*A), Vec3(*(A + e[0])), Vec3(*(A + e[1]))
            tris[k].uvA, tris[k].uvB, tris[k].uvC = (UV(*rng.uniform(-2, 2, 2)) for _ in range(3))
        mats = (Material * (nm * tw * th))()
        for k in range(nm * tw * th):
            mats[k] = scenes.material(_zero_some(rng, tuple(rng.uniform(0, 1, 3)), zeros), (0, 0, 0), 0.0, 0.0,
                                      1.0 if opaque else float(rng.choice([0.0, 0.5, 1.0, 0.7])), 0.0)
        mesh = (tris, qm, mats, tw, th, nm)
    cam_o, cam_t = rng.uniform(-0.5, 0.5, 3), rng.uniform([-1, -1, -4], [1, 1, -2])
    vfov = float(rng.uniform(40, 100))
    W, H = int(rng.integers(8, 33)), int(rng.integers(6, 25))
    spp_b = (int(rng.integers(1, 6)), int(rng.integers(0, bounce_hi)))
    use_ao, ao, rseed = bool(rng.random() < 0.4), float(rng.uniform(0.5, 3.5)), int(rng.integers(0, 2 ** 40))
    aperture, focus = tuple(rng.choice([0.0, 0.0, 1.0, 2.0], 2)), float(rng.uniform(1, 5))
    compat, chunks_d = int(rng.integers(0, 2)), int(rng.choice([1, 1, 2, 3]))
    if far:
        # main()'s coordinate regime (camera at |o| ~ 1000, main.c:300-301;
        # sky sphere of radius 1e5, main.c:346): the whole scene scaled by s
        # and moved by T, then enclosed by an emissive radius-1e5 sky
        s, T = float(rng.uniform(50, 2000)), rng.uniform(-1000, 1000, 3)
        for k in range(ns):
            sph[k].center = Vec3(*(T + s * np.array(sph[k].center.tolist())))
            sph[k].radius = s * sph[k].radius
        if mesh is not None:
            for t in mesh[0]:
                t.A, t.B, t.C = (Vec3(*(T + s * np.array(P.tolist()))) for P in (t.A, t.B, t.C))
        cam_o, cam_t = T + s * cam_o, T + s * cam_t
        focus *= s
        sky = (Sphere * (ns + 1))()
        for k in range(ns):
            sky[k] = sph[k]
        sky[ns].center, sky[ns].radius = Vec3(0.0, 0.0, 0.0), 1e5
        sky[ns].mat = scenes.material((0, 0, 0), scenes.SKY, 1.0, 0.0, 1.0, 1.0)
        sph = sky
    bundle = helpers.SceneBundle(sph, mesh)
    cam = tipe_rt.init_camera(tuple(cam_o), tuple(cam_t), (0, 1, 0), vfov, 4.0 / 3.0)
    p = helpers.params(W, H, *spp_b, use_ao=use_ao, ao=ao, seed=rseed, cam=cam, aperture=aperture, focus=focus,
                       compat=compat, chunks=chunks_d)
    if chunks is not None:
        p.spp_chunks = chunks
        p.nbRayonParPixel = max(p.nbRayonParPixel, chunks)
    if spp is not None:
        p.nbRayonParPixel = spp
    return bundle, p


@pytest.mark.parametrize("seed", range(64))
def test_random_scene_bitexact(seed):
    bundle, p = random_scene(seed)
    check_parity(bundle, p)


@pytest.mark.parametrize("seed", range(800, 840))
def test_random_far_scene_bitexact(seed):
    """main()'s coordinate regime: every random scene scaled by 50-2000 and
    moved by up to 1000 units, inside a radius-1e5 emissive sky sphere
    (main.c:300-301, 346), so the candidate pass's interval bound
    (Hs = (|o| + L) sqrt(a)) and the BVH padding run at |o|, L ~ 1e3-1e5;
    0-24 bounces; spp_chunks 1-3; bit for bit vs the oracle.  Odd seeds run
    with the zero-throughput exit off, so paths go on after a sky hit and
    BVH walks start at |o| ~ 1e5 (per-ray margins, rt_kernels.hip ray32)."""
    bundle, p = random_scene(seed, far=True)
    if seed % 2:
        with tipe_rt.reference_counts():
            check_parity(bundle, p)
    else:
        check_parity(bundle, p)


@pytest.mark.parametrize("seed", range(200, 248))
def test_random_scene_zero_throughput_queue_bitexact(seed):
    """Random scenes whose colours have exact-zero channels (paths end at
    zero throughput), rendered with spp_chunks 2-4 (the queue kernel for
    sphere/brute-force scenes, the BVH kernel on odd seeds), bit for bit
    against the oracle, which never ends a path early."""
    bundle, p = random_scene(seed, zeros=True, chunks=2 + seed % 3)
    check_parity(bundle, p)


@pytest.mark.parametrize("seed", range(100, 124))
def test_random_scene_cuda_semantics_bitexact(seed):
    """rt.h RT_SEM_CUDA on random scenes: each triangle takes its first texel
    as its own material (scenes.with_cuda_materials), sky off."""
    bundle, p = random_scene(seed)
    if bundle.mesh is not None:
        scenes.with_cuda_materials(bundle.mesh)
    p.semantics = tipe_rt.types.RT_SEM_CUDA
    check_parity(bundle, p)


@pytest.mark.parametrize("seed", range(300, 324))
def test_random_bvh_scene_queue_tiny_grid_bitexact(seed, monkeypatch):
    """Random 100-400 triangle meshes (BVH) with random spheres, through the
    BVH task-queue kernel (resumable walks, rt_kernels.hip render_kernel_q<..,
    QB>) on a 1-3 block grid, so every lane runs many tasks and walks span
    rounds across task switches; 5-6 sample slices at 40-48 spp use the
    tapered slice bounds (rt_chunk_bound).  Bit for bit vs the oracle."""
    monkeypatch.setenv("RT_QUEUE_BLOCKS", str(1 + seed % 3))
    bundle, p = random_scene(seed, zeros=bool(seed % 2), chunks=5 + seed % 2, nt_range=(100, 400),
                             spp=40 + 8 * (seed % 2))
    p.largeur_image, p.hauteur_image = min(p.largeur_image, 20), min(p.hauteur_image, 15)
    check_parity(bundle, p)
    assert_stack_bound_holds(bundle, p)


@pytest.mark.parametrize("seed", range(400, 432))
def test_random_opaque_sphere_scene_queue_bitexact(seed):
    """Opaque sphere-only random scenes (r04's QB -2 queue instantiation: no
    triangle, hole or refraction code) at spp_chunks 2-5, zero-throughput
    colours on odd seeds; the kernel taken is checked, bit for bit vs the
    oracle."""
    bundle, p = random_scene(seed, zeros=bool(seed % 2), chunks=2 + seed % 4, opaque=True, mesh_p=0.0)
    check_parity(bundle, p)
    assert tipe_rt.last_render_kernel() == "render_kernel_q<QB=-2>"


@pytest.mark.parametrize("seed", range(500, 516))
def test_random_opaque_bvh_scene_queue_bitexact(seed, monkeypatch):
    """Opaque random 100-400 triangle scenes through the BVH queue kernel
    (the deep-tree OPQ instantiation where the tree is deep) on a 1-3 block
    grid, bit for bit vs the oracle."""
    monkeypatch.setenv("RT_QUEUE_BLOCKS", str(1 + seed % 3))
    bundle, p = random_scene(seed, zeros=bool(seed % 2), chunks=5 + seed % 2, nt_range=(100, 400),
                             spp=40 + 8 * (seed % 2), opaque=True)
    p.largeur_image, p.hauteur_image = min(p.largeur_image, 20), min(p.hauteur_image, 15)
    check_parity(bundle, p)
    assert_stack_bound_holds(bundle, p)
    # deep trees take the OPQ kernel; shallow ones QB 4; a camera outside the
    # scene bound the brute-force scan (QB 0); an over-deep tree the fixed grid
    assert tipe_rt.last_render_kernel() in ("render_kernel_q<QB=3,OP>", "render_kernel_q<QB=3>", "render_kernel_q<QB=4>",
                                            "render_kernel_q<QB=0>", "render_kernel<BVH>")
