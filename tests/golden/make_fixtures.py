"""Regenerate tests/golden fixtures FROM THE REFERENCE (container only).

Runs the reference's own leaf code (oracle/_ref/libref_leaf.so, compiled
from /root/reference's headers by oracle/Makefile) and writes its outputs:

  scenes/pyramide.json   list_of_mesh + create_mat_list_mtl on
                         model3D/pyramide/pyramide_tri.obj (5 tris, 16x16
                         water texture with alpha 180/255)
  scenes/mineways.json   the same on mcworld_tiltedtex_water/mineways_tri.obj
                         (606 tris, 11 textures incl. alpha holes)
  kat_leaf.json          seeded random inputs -> reference outputs of
                         hit_sphere, hit_triangle, tri_uvmapping,
                         refracted_vec, reflected_vec, vec3_lerp,
                         write_color_canva, rgb_to_hsl, hsl_to_rgb,
                         init_camera, get_ray, pile.h sequences, rand(),
                         randomDouble, random_dir_no_norm

Doubles are stored as float.hex() strings (bit-exact round trip).
Usage:  python tests/golden/make_fixtures.py
"""
import ctypes as C
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: E402,F401  (sys.path)
import oracle_ffi  # noqa: E402
from tipe_rt.types import Vec3, Ray, Material, Triangle, Camera, UV  # noqa: E402

REF = "/root/reference"


def hx(x):
    return float(x).hex()


def v(x):
    return [hx(x.e[0]), hx(x.e[1]), hx(x.e[2])]


def load_ref_mesh(lib, obj, mtl):
    n_tri, n_mat = C.c_int(), C.c_int()
    qm = C.POINTER(C.c_int)()
    tris = lib.ref_list_of_mesh(obj.encode(), mtl.encode(), C.byref(n_tri), C.byref(n_mat), C.byref(qm))
    tw, th = C.c_int(), C.c_int()
    mats = lib.ref_load_textures(obj.encode(), mtl.encode(), C.byref(tw), C.byref(th))
    assert tris and mats, "reference loader failed on %s" % obj
    out = {
        "source": os.path.relpath(obj, REF),
        "tex_width": tw.value, "tex_height": th.value, "n_materials": n_mat.value,
        "triangles": [], "quelMatPourTri": [qm[i] for i in range(n_tri.value)], "texels": [],
    }
    for i in range(n_tri.value):
        t = tris[i]
        out["triangles"].append({"A": t.A.tolist(), "B": t.B.tolist(), "C": t.C.tolist(),
                                 "uvA": [t.uvA.u, t.uvA.v], "uvB": [t.uvB.u, t.uvB.v],
                                 "uvC": [t.uvC.u, t.uvC.v]})
    for k in range(n_mat.value * tw.value * th.value):
        m = mats[k]
        out["texels"].append([m.diffuseColor.e[0], m.diffuseColor.e[1], m.diffuseColor.e[2], m.alpha])
    lib.ref_free(C.cast(tris, C.c_void_p))
    lib.ref_free(C.cast(mats, C.c_void_p))
    lib.ref_free(C.cast(qm, C.c_void_p))
    return out


def rv(rng, lo=-2.0, hi=2.0):
    return Vec3(rng.uniform(lo, hi), rng.uniform(lo, hi), rng.uniform(lo, hi))


def unit(rng):
    while True:
        x = rv(rng, -1, 1)
        n = sum(c * c for c in x.tolist()) ** 0.5
        if n > 1e-3:
            return Vec3(*(c / n for c in x.tolist()))


def make_kat(lib, mesh):
    rng = random.Random(20241015)
    kat = {}
    # hit_sphere
    rows = []
    for _ in range(200):
        c = rv(rng)
        r = rng.choice([0.3, 0.5, 1.0, 500.0])
        if r == 500.0:
            c = Vec3(*(x * 250 for x in c.tolist()))
        ray = Ray(rv(rng), unit(rng))
        h = oracle_ffi.OracleHit()
        lib.ref_hit_sphere(C.byref(c), r, C.byref(ray), C.byref(h))
        rows.append({"c": v(c), "r": hx(r), "o": v(ray.origin), "d": v(ray.dir),
                     "hit": h.didHit, "dst": hx(h.dst), "p": v(h.hitPoint), "n": v(h.normal)})
    kat["hit_sphere"] = rows
    # hit_triangle (random + mesh triangles)
    rows = []
    for k in range(200):
        t = Triangle()
        t.A, t.B, t.C = rv(rng), rv(rng), rv(rng)
        ray = Ray(rv(rng, -3, 3), unit(rng))
        if k % 2:   # aim at the triangle
            tgt = [(a + b + c) / 3 for a, b, c in zip(t.A.tolist(), t.B.tolist(), t.C.tolist())]
            d = [x - o for x, o in zip(tgt, ray.origin.tolist())]
            n = sum(x * x for x in d) ** 0.5
            ray.dir = Vec3(*(x / n for x in d))
        h = oracle_ffi.OracleHit()
        lib.ref_hit_triangle(C.byref(t), C.byref(ray), C.byref(h))
        rows.append({"A": v(t.A), "B": v(t.B), "C": v(t.C), "o": v(ray.origin), "d": v(ray.dir),
                     "hit": h.didHit, "dst": hx(h.dst), "p": v(h.hitPoint), "n": v(h.normal)})
    kat["hit_triangle"] = rows
    # tri_uvmapping on the mineways mesh: hits at random barycentric points
    tris, qm, texels, tw, th, nm = mesh
    mats = (Material * len(texels))()
    for i, (r_, g_, b_, a_) in enumerate(texels):
        mats[i].diffuseColor = Vec3(r_, g_, b_)
        mats[i].alpha = a_
    qarr = (C.c_int * len(qm))(*qm)
    rows = []
    for _ in range(150):
        i = rng.randrange(len(tris))
        td = tris[i]
        t = Triangle()
        t.A, t.B, t.C = Vec3(*td["A"]), Vec3(*td["B"]), Vec3(*td["C"])
        t.uvA, t.uvB, t.uvC = UV(*td["uvA"]), UV(*td["uvB"]), UV(*td["uvC"])
        a, b = rng.random(), rng.random()
        if a + b > 1:
            a, b = 1 - a, 1 - b
        P = [x + a * (y - x) + b * (z - x) for x, y, z in zip(t.A.tolist(), t.B.tolist(), t.C.tolist())]
        ab = [y - x for x, y in zip(t.A.tolist(), t.B.tolist())]
        ac = [z - x for x, z in zip(t.A.tolist(), t.C.tolist())]
        nv = [ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]]
        nn = sum(x * x for x in nv) ** 0.5
        h = oracle_ffi.OracleHit()
        h.didHit = 1
        h.hitPoint = Vec3(*P)
        h.normal = Vec3(*(x / nn for x in nv))
        out = Material()
        lib.ref_tri_uvmapping(C.byref(t), C.byref(h), mats, tw, th, i, qarr, C.byref(out))
        rows.append({"tri": i, "p": v(h.hitPoint), "n": v(h.normal),
                     "diffuse": v(out.diffuseColor), "emission": v(out.emissionColor),
                     "es": hx(out.emissionStrength), "rs": hx(out.reflectionStrength),
                     "alpha": hx(out.alpha), "ior": hx(out.materialIndex)})
    kat["tri_uvmapping_mineways"] = rows
    # refracted / reflected / lerp
    rows = []
    for _ in range(150):
        d, n = unit(rng), unit(rng)
        n1, n2 = rng.choice([1.0, 1.33, 1.5, 0.0]), rng.choice([1.0, 1.33, 1.5, 2.4])
        o1, o2, o3 = Vec3(), Vec3(), Vec3()
        t = rng.random()
        lib.ref_refracted_vec(C.byref(d), C.byref(n), n1, n2, C.byref(o1))
        lib.ref_reflected_vec(C.byref(d), C.byref(n), C.byref(o2))
        lib.ref_vec3_lerp(C.byref(d), C.byref(n), t, C.byref(o3))
        rows.append({"d": v(d), "n": v(n), "n1": hx(n1), "n2": hx(n2), "t": hx(t),
                     "refr": v(o1), "refl": v(o2), "lerp": v(o3)})
    kat["optics"] = rows
    # colour
    rows = []
    for k in range(150):
        c = Vec3(*(rng.choice([0.0, 0.2, 0.5, 1.0, rng.random()]) for _ in range(3)))
        spp = rng.choice([1, 16, 100, 1000])
        s = Vec3(*(rng.random() * spp * rng.choice([0.5, 1.0, 3.0]) for _ in range(3)))
        o1, o2, o3 = Vec3(), Vec3(), Vec3()
        lib.ref_write_color_canva(C.byref(s), spp, C.byref(o1))
        lib.ref_rgb_to_hsl(C.byref(c), C.byref(o2))
        lib.ref_hsl_to_rgb(C.byref(o2), C.byref(o3))
        rows.append({"sum": v(s), "spp": spp, "canva": v(o1), "rgb": v(c), "hsl": v(o2), "back": v(o3)})
    kat["colour"] = rows
    # camera + get_ray
    rows = []
    for k in range(20):
        if k == 0:
            o, tg, vfov, ratio = Vec3(0.34, 0.3, 0.5), Vec3(0.0, -0.5, -3.0), 70.0, 4.0 / 3.0
        else:
            o, tg, vfov, ratio = rv(rng), rv(rng), rng.uniform(20, 100), rng.choice([4 / 3, 16 / 10, 1.0])
        up = Vec3(0, 1, 0)
        cam = Camera()
        lib.ref_init_camera(C.byref(o), C.byref(tg), C.byref(up), vfov, ratio, C.byref(cam))
        rays = []
        for _ in range(6):
            u, w = rng.random(), rng.random()
            dx, dy = rng.uniform(-0.5, 0.5) * rng.choice([0, 1, 2]), rng.uniform(-0.5, 0.5) * rng.choice([0, 1])
            focus = rng.choice([1.0, 3.0])
            ray = Ray()
            lib.ref_get_ray(u, w, C.byref(cam), focus, dx, dy, C.byref(ray))
            rays.append({"u": hx(u), "v": hx(w), "focus": hx(focus), "dx": hx(dx), "dy": hx(dy),
                         "o": v(ray.origin), "d": v(ray.dir)})
        rows.append({"origin": v(o), "target": v(tg), "vfov": hx(vfov), "ratio": hx(ratio),
                     "horizontal": v(cam.horizontal), "vertical": v(cam.vertical),
                     "corner": v(cam.coin_bas_gauche), "rays": rays})
    kat["camera"] = rows
    # pile.h sequences
    rows = []
    for _ in range(100):
        n = rng.randrange(1, 12)
        ops = [rng.choice([1.0, 1.33, 1.5, 0.0, 2.4]) for _ in range(n)]
        ex = [rng.randrange(2) for _ in range(n)]
        a, b = (C.c_double * n)(), (C.c_double * n)()
        lib.ref_pile_sequence((C.c_double * n)(*ops), (C.c_int * n)(*ex), n, a, b)
        rows.append({"ops": [hx(x) for x in ops], "exit": ex, "n1": [hx(x) for x in a], "n2": [hx(x) for x in b]})
    kat["pile"] = rows
    # glibc stream through the reference's own helpers (seed 1 = unseeded)
    lib.ref_srand(1)
    kat["rand_seed1"] = [lib.ref_rand() for _ in range(8)]
    lib.ref_srand(1)
    kat["randomDouble_seed1"] = [hx(lib.ref_randomDouble(-0.5, 0.5)) for _ in range(8)]
    lib.ref_srand(7)
    dirs = []
    for _ in range(64):
        o = Vec3()
        lib.ref_random_dir_no_norm(C.byref(o))
        dirs.append(v(o))
    kat["random_dir_no_norm_seed7"] = dirs
    # sphere_uvmapping (texture.h:92-112, the sky mapping): texel k's diffuse
    # red channel holds k, so the output names the index the reference picked.
    # The table is padded so that the reference's unchecked index stays in
    # memory; rows whose index falls outside w*h (its UB) are dropped.
    srng = random.Random(2024)
    rows = []
    for w, h in ((8, 4), (64, 32), (7, 5)):
        n = w * h
        mats = (Material * (n + 4 * w + 8))()
        for k in range(len(mats)):
            mats[k].diffuseColor = Vec3(float(k), 0.0, 0.0)
        for _ in range(120):
            c = Vec3(*(srng.uniform(-3, 3) for _ in range(3)))
            radius = srng.choice([0.5, 1.0, 500.0, srng.uniform(0.1, 50)])
            dv = [srng.gauss(0, 1) for _ in range(3)]
            nv = sum(x * x for x in dv) ** 0.5
            p = Vec3(*(ci + radius * x / nv for ci, x in zip(c.tolist(), dv)))
            out = Material()
            lib.ref_sphere_uvmapping(C.byref(c), C.c_double(radius), C.byref(p), mats, w, h, C.byref(out))
            k = int(out.diffuseColor.e[0])
            if 0 <= k < n:
                rows.append({"c": v(c), "r": hx(radius), "p": v(p), "w": w, "h": h, "index": k})
    kat["sphere_uvmapping"] = rows
    return kat


def main():
    lib = oracle_ffi.ref()
    assert lib is not None, "needs /root/reference and oracle/_ref (run make -C oracle)"
    os.makedirs(os.path.join(HERE, "scenes"), exist_ok=True)
    pyr = load_ref_mesh(lib, REF + "/model3D/pyramide/pyramide_tri.obj", REF + "/model3D/pyramide/pyramide_tri.mtl")
    mw = load_ref_mesh(lib, REF + "/model3D/mcworld_tiltedtex_water/mineways_tri.obj",
                       REF + "/model3D/mcworld_tiltedtex_water/mineways_tri.mtl")
    for name, d in (("pyramide", pyr), ("mineways", mw)):
        with open(os.path.join(HERE, "scenes", name + ".json"), "w") as f:
            json.dump(d, f, separators=(",", ":"))
    kat = make_kat(lib, (mw["triangles"], mw["quelMatPourTri"], mw["texels"], mw["tex_width"],
                         mw["tex_height"], mw["n_materials"]))
    with open(os.path.join(HERE, "kat_leaf.json"), "w") as f:
        json.dump(kat, f, separators=(",", ":"))
    print("wrote pyramide (%d tris), mineways (%d tris), kat_leaf" % (len(pyr["triangles"]), len(mw["triangles"])))


if __name__ == "__main__":
    main()
