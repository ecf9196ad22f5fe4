"""Write the large-scene inputs FROM THE REFERENCE'S LOADER (container only).

  scenes/nature.json        model3D/RTX_MAP/nature/mineways_doubleface_tri.obj
                            (+ .mtl and its 16x16 PPM textures with alpha
                            PPMs): the scene of the reference's own
                            RTX_nature_1000RAYS_9RB render
                            (.MISSING_LARGE_BLOBS:8; name rule main.c:328).
                            5812 triangles, 31 materials, `f v/vt/vn` faces.
                            list_of_mesh + create_mat_list_mtl (mesh.h:110-218,
                            texture.h:145-354) through oracle/_ref/libref_leaf.so.
  scenes/pyramide_eau.json  main()'s own default mesh, model3D/pyramide_eau/
                            scene.obj (main.c:320-321; 34 triangles at the
                            +-1813 scale of main()'s camera, main.c:300-301).
                            GEOMETRY ONLY from the reference loader: its PPM
                            textures are listed in /root/reference/
                            .MISSING_LARGE_BLOBS, so create_mat_list_mtl cannot
                            run; the texel table is synthetic (16x16 per
                            material, seeded, alpha 1 -- the texture.h:71-87
                            overrides for materials 1/3/4 still apply, and they
                            were written for this very scene: lumiere, vitre,
                            eau).

Compact rows: "tri" = [Ax, Ay, Az, Bx, ..., Cz, uAu, uAv, uBu, uBv, uCu, uCv]
per triangle (JSON numbers: shortest repr, exact double round trip).
Usage:  python tests/golden/make_scene_fixtures.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: E402,F401  (sys.path)
import oracle_ffi  # noqa: E402

REF = "/root/reference"


def _tri_rows(tris, n):
    rows = []
    for i in range(n):
        t = tris[i]
        rows.append([float(c) for P in (t.A, t.B, t.C) for c in P.tolist()] +
                    [t.uvA.u, t.uvA.v, t.uvB.u, t.uvB.v, t.uvC.u, t.uvC.v])
    return rows


def load_geometry(lib, obj, mtl):
    n_tri, n_mat = C.c_int(), C.c_int()
    qm = C.POINTER(C.c_int)()
    tris = lib.ref_list_of_mesh(obj.encode(), mtl.encode(), C.byref(n_tri), C.byref(n_mat), C.byref(qm))
    assert tris, "reference loader failed on %s" % obj
    out = {"source": os.path.relpath(obj, REF), "n_materials": n_mat.value,
           "quelMatPourTri": [qm[i] for i in range(n_tri.value)], "tri": _tri_rows(tris, n_tri.value)}
    lib.ref_free(C.cast(tris, C.c_void_p))
    lib.ref_free(C.cast(qm, C.c_void_p))
    return out


def nature(lib):
    d = REF + "/model3D/RTX_MAP/nature/"
    out = load_geometry(lib, d + "mineways_doubleface_tri.obj", d + "mineways_doubleface_tri.mtl")
    tw, th = C.c_int(), C.c_int()
    mats = lib.ref_load_textures((d + "mineways_doubleface_tri.obj").encode(),
                                 (d + "mineways_doubleface_tri.mtl").encode(), C.byref(tw), C.byref(th))
    assert mats
    out["tex_width"], out["tex_height"] = tw.value, th.value
    out["texels"] = []
    for k in range(out["n_materials"] * tw.value * th.value):
        m = mats[k]
        out["texels"].append([m.diffuseColor.e[0], m.diffuseColor.e[1], m.diffuseColor.e[2], m.alpha])
    lib.ref_free(C.cast(mats, C.c_void_p))
    return out


def pyramide_eau(lib):
    d = REF + "/model3D/pyramide_eau/"
    out = load_geometry(lib, d + "scene.obj", d + "scene.mtl")
    out["texels_note"] = ("synthetic: the scene's PPM textures are missing from the reference checkout "
                          "(.MISSING_LARGE_BLOBS); seeded 16x16 colours, alpha 1")
    rng = np.random.default_rng(20261018)
    tw = th = 16
    out["tex_width"], out["tex_height"] = tw, th
    out["texels"] = [[float(x) for x in rng.uniform(0.15, 0.95, 3)] + [1.0]
                     for _ in range(out["n_materials"] * tw * th)]
    return out


def main():
    lib = oracle_ffi.ref()
    assert lib is not None, "needs /root/reference and oracle/_ref (run make -C oracle)"
    for name, fn in (("nature", nature), ("pyramide_eau", pyramide_eau)):
        d = fn(lib)
        with open(os.path.join(HERE, "scenes", name + ".json"), "w") as f:
            json.dump(d, f, separators=(",", ":"))
        print("%s: %d triangles, %d materials, %dx%d texels" % (name, len(d["tri"]), d["n_materials"],
                                                               d["tex_width"], d["tex_height"]))


if __name__ == "__main__":
    main()
