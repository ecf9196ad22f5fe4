"""Shared scene builders and oracle/product drivers for the tests."""
import ctypes as C
import hashlib

import numpy as np

import oracle_ffi
import tipe_rt
from tipe_rt import scenes
from tipe_rt.types import Vec3, Scene, Params, RT_RNG_PHILOX, RT_RNG_GLIBC, RT_NCOUNTERS


def readme_camera_oracle():
    cam = scenes.README_CAMERA
    return oracle_ffi.oracle().oracle_init_camera(Vec3(*cam["origin"]), Vec3(*cam["target"]), Vec3(*cam["up"]),
                                                  cam["vfov"], cam["ratio"])


class SceneBundle:
    """Keeps the ctypes arrays alive next to the rt_scene that points at them."""

    def __init__(self, spheres=None, mesh=None, sky=None):
        self.spheres = spheres
        self.mesh = mesh
        self.sky = sky
        if mesh is not None:
            tris, qm, mats, tw, th, nm = mesh
            self.scene = tipe_rt.make_scene(spheres, tris, qm, mats, tw, th, nm, sky=sky)
        else:
            self.scene = tipe_rt.make_scene(spheres, sky=sky)


def cornell(extra=()):
    return SceneBundle(scenes.cornell_spheres(extra=extra))


def pyramid_scene(move=scenes.PYRAMID_MOVE):
    return SceneBundle(scenes.cornell_spheres(), scenes.moved(scenes.load_mesh_fixture("pyramide"), move))


def sky_scene(w=16, h=8, seed=3):
    """README spheres + an enclosing emissive sky sphere (the last sphere,
    main.c:64-71) with a w x h equirect texel table of random colours."""
    import ctypes as C
    from tipe_rt.types import Sphere, Material, Vec3
    base = scenes.cornell_spheres()
    sph = (Sphere * (len(base) + 1))()
    for k in range(len(base)):
        sph[k] = base[k]
    sph[len(base)].center = Vec3(0.0, 0.0, 0.0)
    sph[len(base)].radius = 2000.0
    sph[len(base)].mat = scenes.material((0.5, 0.5, 0.5), (1, 1, 1), 1.2, 0.0, 1.0, 1.0)
    rng = np.random.default_rng(seed)
    tex = (Material * (w * h))()
    for k in range(w * h):
        tex[k] = scenes.material(tuple(rng.uniform(0, 1, 3)), (0, 0, 0), 0.0, 0.0, 1.0, 0.0)
    return SceneBundle(sph, None, sky=(tex, w, h))


def sky_tree_scene():
    """The sky scene's spheres and texels with the C4 tree mesh (BVH + sky)."""
    sk = sky_scene()
    return SceneBundle(sk.spheres, scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE), sky=sk.sky)


def mineways_scene():
    """mineways_tri.obj (606 triangles, 11 textures incl. alpha leaves) scaled
    into the README box (as test_gpu_parity.test_mineways_alpha_holes)."""
    tris, qm, mats, tw, th, nm = scenes.load_mesh_fixture("mineways")
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0] = P.e[0] * 0.1 - 0.2
            P.e[1] = P.e[1] * 0.1 - 1.0
            P.e[2] = P.e[2] * 0.1 - 2.5
    return SceneBundle(scenes.cornell_spheres(), (tris, qm, mats, tw, th, nm))


def tree_scene(move=scenes.TREE_MOVE):
    """C4: README spheres + 1tree_tri.obj (1320 tris, Kd-flat materials)."""
    return SceneBundle(scenes.cornell_spheres(), scenes.moved(scenes.load_tree_fixture(), move))


def camera_of(spec):
    """scenes.*_CAMERA dict -> the oracle's init_camera (camera.h:21-40)."""
    return oracle_ffi.oracle().oracle_init_camera(Vec3(*spec["origin"]), Vec3(*spec["target"]), Vec3(*spec["up"]),
                                                  spec["vfov"], spec["ratio"])


def nature_scene():
    """RTX_MAP/nature (5812 textured triangles with alpha holes) lit by
    main.c:345-346's sun and sky sphere; camera scenes.NATURE_CAMERA."""
    return SceneBundle(scenes.main_spheres(), scenes.nature_mesh())


def main_regime_scene():
    """main()'s own coordinate regime: its default mesh pyramide_eau/scene.obj
    (+-1813 units, materials 1/3/4 = texture.h:71-87's light / glass / water
    overrides) under main.c:345-346's sun and radius-1e5 sky sphere; camera
    scenes.MAIN_CAMERA (main.c:298-302)."""
    return SceneBundle(scenes.main_spheres(), scenes.pyramide_eau_mesh())


def params(W, H, spp, bounces, use_ao=False, ao=2.5, rng=RT_RNG_PHILOX, seed=1010, compat=1, cam=None,
           aperture=(0.0, 0.0), focus=3.0, chunks=1, accel=0, sky_mode=0, semantics=0):
    if cam is None:
        cam = readme_camera_oracle()
    return tipe_rt.make_params(W, H, spp, bounces, cam, focus=focus, aperture=aperture, use_ao=use_ao, ao=ao,
                               seed=seed, rng=rng, compat=compat, chunks=chunks, accel=accel, sky_mode=sky_mode,
                               semantics=semantics)


def oracle_render(bundle, p, row_hi=None, row_lo=0, nthreads=1, counters=False):
    W, H = p.largeur_image, p.hauteur_image
    if row_hi is None:
        row_hi = H - 1
    canva, alb, nrm, rad = (np.zeros((H, W, 3)) for _ in range(4))
    cnt = oracle_ffi.counters() if counters else None
    rc = oracle_ffi.oracle().oracle_render_rows(C.byref(bundle.scene), C.byref(p), row_hi, row_lo, nthreads, 1,
                                                canva.ctypes.data, alb.ctypes.data, nrm.ctypes.data,
                                                rad.ctypes.data, cnt)
    assert rc == 0, rc
    out = dict(canva=canva, albedo=alb, normal=nrm, radiance=rad)
    if counters:
        out["counters"] = np.array(list(cnt), dtype=np.uint64)
    return out


def ppm_text(canva):
    """The P3 file main.c:457-465 writes (rows top to bottom: j = H-1 .. 0)."""
    H, W, _ = canva.shape
    lines = ["P3\n%d %d\n255\n" % (W, H)]
    for j in range(H - 1, -1, -1):
        row = canva[j].astype(np.int64)
        lines.extend("%d %d %d\n" % (r, g, b) for r, g, b in row)
    return "".join(lines)


def ppm_md5(canva):
    return hashlib.md5(ppm_text(canva).encode()).hexdigest()


def rmse_per_channel(a, b):
    d = (np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64)).reshape(-1, 3)
    return np.sqrt((d * d).mean(axis=0))
