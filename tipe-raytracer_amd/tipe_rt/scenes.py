"""Benchmark / parity scenes, as the reference's own data.

The Cornell box is README.md:46-59's `sphere_list` (the 4-field material
initialisers of main_cuda.cu's material), extended with alpha = 1.0 and
materialIndex = 1.0 so it is visible to main.c's 6-field material
(hitinfo.h:6-13; with alpha = 0 every non-emitter would be an alpha hole,
main.c:200-206).  Camera: README.md:14-22.  See SURVEY.md §8 "Config
resolution".
"""
import json
import os
import ctypes as C

from .types import Vec3, Material, Sphere, Triangle, UV, Camera

RED, GREEN, BLUE = (1, 0, 0), (0, 1, 0), (0, 0, 1)
WHITE, BLACK, SKY = (1, 1, 1), (0, 0, 0), (0.784, 0.965, 1)

# (center, radius, diffuse, emission, emissionStrength, reflectionStrength)
README_SPHERES = [
    ((-501, 0, 0), 500, GREEN, BLACK, 0.0, 0.96),
    ((0, -501, 0), 500, WHITE, BLACK, 0.0, 0.0),
    ((501, 0, 0), 500, RED, BLACK, 0.0, 0.96),
    ((-0.5, 1.4, -1.2), 0.5, BLACK, (1.0, 0.6, 0.2), 4.0, 0.0),     # orange
    ((0.5, 1.4, -2.2), 0.5, BLACK, (0.7, 0.2, 1.0), 4.0, 0.0),      # violet
    ((0.6, -1.4, -1.0), 0.5, BLACK, (0.55, 0.863, 1.0), 2.5, 0.0),  # light blue
    ((-0.5, -1.4, -3.1), 0.5, BLACK, (0.431, 1.0, 0.596), 2.5, 0.0),  # light green
    ((0, 0, -504), 500, WHITE, BLACK, 0.0, 0.0),
    ((0, 501, 0), 500, WHITE, BLACK, 0.0, 0.0),
    ((0.4, -0.5, -3.3), 0.5, SKY, BLACK, 0.0, 0.99),
]

README_CAMERA = dict(origin=(0.34, 0.3, 0.5), target=(0.0, -0.5, -3.0), up=(0, 1, 0),
                     vfov=70.0, ratio=4.0 / 3.0, focus=3.0, aperture=(0.0, 0.0))


def material(diffuse, emission=BLACK, es=0.0, refl=0.0, alpha=1.0, ior=1.0):
    m = Material()
    m.diffuseColor = Vec3(*diffuse)
    m.emissionColor = Vec3(*emission)
    m.emissionStrength, m.reflectionStrength = es, refl
    m.alpha, m.materialIndex = alpha, ior
    return m


def cornell_spheres(alpha=1.0, material_index=1.0, extra=()):
    """README 10-sphere box; `extra` appends (center, r, Material) tuples."""
    rows = list(README_SPHERES)
    arr = (Sphere * (len(rows) + len(extra)))()
    for k, (c, r, d, e, es, rf) in enumerate(rows):
        arr[k].center = Vec3(*c)
        arr[k].radius = r
        arr[k].mat = material(d, e, es, rf, alpha, material_index)
    for k, (c, r, m) in enumerate(extra):
        arr[len(rows) + k].center = Vec3(*c)
        arr[len(rows) + k].radius = r
        arr[len(rows) + k].mat = m
    return arr


def image_height(width, ratio=4.0 / 3.0):
    """main.c:295: hauteur_image = (int)(largeur_image / ratio)."""
    return int(width / ratio)


_GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "tests", "golden")


def load_mesh_fixture(name):
    """Load a mesh fixture (triangles, per-triangle material, texel table)
    written by tests/golden/make_fixtures.py from the reference loaders.
    Returns (triangles, quelMatPourTri, mat_list, tw, th, n_materials)."""
    with open(os.path.join(_GOLDEN, "scenes", name + ".json")) as f:
        d = json.load(f)
    if "tri" in d:          # compact rows (tests/golden/make_scene_fixtures.py)
        tris = d["tri"]
        arr = (Triangle * len(tris))()
        for k, t in enumerate(tris):
            arr[k].A, arr[k].B, arr[k].C = Vec3(*t[0:3]), Vec3(*t[3:6]), Vec3(*t[6:9])
            arr[k].uvA, arr[k].uvB, arr[k].uvC = UV(*t[9:11]), UV(*t[11:13]), UV(*t[13:15])
            arr[k].mat = material(SKY, BLACK, 0.0, 0.0, 0.0, 0.0)   # mesh.h:206
    else:
        tris = d["triangles"]
        arr = (Triangle * len(tris))()
        for k, t in enumerate(tris):
            arr[k].A, arr[k].B, arr[k].C = Vec3(*t["A"]), Vec3(*t["B"]), Vec3(*t["C"])
            arr[k].uvA, arr[k].uvB, arr[k].uvC = UV(*t["uvA"]), UV(*t["uvB"]), UV(*t["uvC"])
            arr[k].mat = material(SKY, BLACK, 0.0, 0.0, 0.0, 0.0)   # mesh.h:206
    qm = (C.c_int * len(tris))(*d["quelMatPourTri"])
    tex = d["texels"]
    mats = (Material * len(tex))()
    for k, (r, g, b, a) in enumerate(tex):
        # texture.h:233-246: diffuse = P3/maxval, alpha = first channel/maxval,
        # emissionStrength = 0; emissionColor/reflectionStrength/materialIndex
        # are never written by the reference loader (read as 0).
        mats[k] = material((r, g, b), BLACK, 0.0, 0.0, a, 0.0)
    return arr, qm, mats, d["tex_width"], d["tex_height"], d["n_materials"]


# Scene placements (SURVEY.md §8 "Config resolution").
PYRAMID_MOVE = (-0.6, -1.0, -2.0)    # C3/C5: probe-verified on the floor
TREE_MOVE = (0.3, -1.01, -2.1)       # C4: the CUDA loader's displacement, triangle.hu:87


def moved(mesh, delta):
    """move_mesh (mesh.h:220-234): add delta to every vertex, in place."""
    tris = mesh[0]
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0] += delta[0]
            P.e[1] += delta[1]
            P.e[2] += delta[2]
    return mesh


def load_tree_fixture():
    """tests/golden/scenes/tree.json (tests/golden/make_tree_fixture.py):
    1tree_tri.obj through librt_host.so, Kd-flat 1x1 texels with
    reflectionStrength = Ns/100.  Same tuple as load_mesh_fixture."""
    with open(os.path.join(_GOLDEN, "scenes", "tree.json")) as f:
        d = json.load(f)
    tris = d["triangles"]
    arr = (Triangle * len(tris))()
    for k, t in enumerate(tris):
        arr[k].A, arr[k].B, arr[k].C = Vec3(*t[0:3]), Vec3(*t[3:6]), Vec3(*t[6:9])
        arr[k].mat = material(SKY, BLACK, 0.0, 0.0, 0.0, 0.0)
    qm = (C.c_int * len(tris))(*d["quelMatPourTri"])
    mats = (Material * len(d["texels"]))()
    for k, (r, g, b, a, refl) in enumerate(d["texels"]):
        mats[k] = material((r, g, b), BLACK, 0.0, refl, a, 0.0)
    return arr, qm, mats, d["tex_width"], d["tex_height"], d["n_materials"]


# main()'s own settings (main.c:293-346): its camera at the +-1813 scale of
# its default mesh model3D/pyramide_eau/scene.obj, and the two last entries
# of its sphere list -- the sun (main.c:345) and the sky sphere of radius
# 1e5 (main.c:346, "derniere sphère = ciel").
MAIN_CAMERA = dict(origin=(237.6461, 144.496, -962.8788), target=(-176.9382, 141.5864, 651.8203), up=(0, 1, 0),
                   vfov=30.2, ratio=16.0 / 10.0)
MAIN_SUN = ((0.5145, 2.7877, -1.1792), 0.1, BLACK, WHITE, 70.0, 0.0)
MAIN_SKY = ((0.0, 0.0, 0.0), 100000.0, BLACK, SKY, 1.0, 0.0)
# RTX_MAP/nature (the reference's RTX_nature_1000RAYS_9RB render): a camera
# low in the valley looking across the pond, as the scene's screenshot
# (model3D/RTX_MAP/nature/screen/); chosen here, the reference's own is not
# recorded.  The mesh is used where the loader leaves it (move_mesh(0, 0, 0),
# main.c:366).
NATURE_CAMERA = dict(origin=(1.0, 0.6, 1.3), target=(-0.6, 0.75, -0.9), up=(0, 1, 0), vfov=60.0, ratio=4.0 / 3.0)


def main_spheres():
    """main.c:345-346: sun + sky sphere (radius 1e5), the sky last."""
    arr = (Sphere * 2)()
    for k, (c, r, d, e, es, rf) in enumerate((MAIN_SUN, MAIN_SKY)):
        arr[k].center = Vec3(*c)
        arr[k].radius = r
        arr[k].mat = material(d, e, es, rf, 1.0, 1.0)
    return arr


def nature_mesh():
    """model3D/RTX_MAP/nature/mineways_doubleface_tri.obj through the
    reference loader (tests/golden/scenes/nature.json): 5812 triangles, 31
    16x16 textures with alpha."""
    return load_mesh_fixture("nature")


def pyramide_eau_mesh():
    """main()'s default mesh (main.c:320) through the reference loader,
    synthetic texels (its PPMs are missing blobs)."""
    return load_mesh_fixture("pyramide_eau")


def pyramid_mesh():
    """C3/C5 mesh: pyramide_tri.obj (reference loader output) at PYRAMID_MOVE."""
    return moved(load_mesh_fixture("pyramide"), PYRAMID_MOVE)


def tree_mesh():
    """C4 mesh: 1tree_tri.obj (1320 tris) at TREE_MOVE."""
    return moved(load_tree_fixture(), TREE_MOVE)


def with_cuda_materials(mesh):
    """rt.h RT_SEM_CUDA: each triangle's own material = the first texel of
    its material (the Kd-flat texel of a Kd-only MTL, as main_cuda.cu's
    per-mesh {Kd, black, 0, Ns/100}), in place."""
    tris, qm, mats, tw, th, nm = mesh
    for k in range(len(tris)):
        tris[k].mat = mats[qm[k] * tw * th]
    return mesh


def synthetic_cornell(n_spheres=10, n_tris=0, seed=7):
    """SURVEY.md §8(d)'s roofline-sweep scenes: the README box with
    n_spheres - 10 extra small spheres (70 % diffuse, 15 % mirror, 15 %
    emitters) and n_tris small random triangles inside the box, textured by
    one 2x2 material table (material 0: no texture.h overrides).  Returns
    (spheres, mesh) with mesh = (triangles, quelMatPourTri, mat_list, tw,
    th, n_materials) or None; deterministic in seed."""
    import numpy as np
    rng = np.random.default_rng(seed)
    extra = []
    for _ in range(max(0, n_spheres - len(README_SPHERES))):
        c = (rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9), rng.uniform(-3.5, -1.0))
        r = rng.uniform(0.04, 0.12)
        kind = rng.uniform()
        col = tuple(rng.uniform(0.1, 1.0, 3))
        if kind < 0.70:
            m = material(col)
        elif kind < 0.85:
            m = material(col, BLACK, 0.0, 0.9)
        else:
            m = material(BLACK, col, rng.uniform(2.0, 4.0))
        extra.append((c, r, m))
    spheres = cornell_spheres(extra=extra)
    if n_tris <= 0:
        return spheres, None
    tris = (Triangle * n_tris)()
    qm = (C.c_int * n_tris)()
    for k in range(n_tris):
        ctr = np.array([rng.uniform(-0.9, 0.9), rng.uniform(-0.95, 0.9), rng.uniform(-3.5, -1.0)])
        e1, e2 = rng.normal(size=3), rng.normal(size=3)
        s = rng.uniform(0.05, 0.15)
        A, B, Cv = ctr, ctr + s * e1 / np.linalg.norm(e1), ctr + s * e2 / np.linalg.norm(e2)
        tris[k].A, tris[k].B, tris[k].C = Vec3(*A), Vec3(*B), Vec3(*Cv)
        tris[k].uvA, tris[k].uvB, tris[k].uvC = (UV(*rng.uniform(0, 1, 2)) for _ in range(3))
        qm[k] = 0
    mats = (Material * 4)()
    for i in range(4):
        mats[i] = material(tuple(rng.uniform(0.2, 0.9, 3)))
    return spheres, (tris, qm, mats, 2, 2, 1)
