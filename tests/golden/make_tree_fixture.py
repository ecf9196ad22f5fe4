"""Write tests/golden/scenes/tree.json: model3D/1tree_tri.obj (1320 tris,
`f v//vn` faces, Kd-only MTL) as loaded by OUR host library
(librt_host.so, Kd-flat texels, reflectionStrength = Ns/100).

The reference loader segfaults on this file, so unlike
pyramide.json / mineways.json this fixture is not a reference output: it is
the C4 scene input, checked against the OBJ/MTL text in
tests/test_host_lib.py::test_loader_reads_tree_the_reference_loader_crashes_on.
Container only (reads /root/reference/model3D).  Doubles as JSON numbers
(shortest repr, exact round trip).
Usage:  python tests/golden/make_tree_fixture.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: E402,F401  (sys.path)
from tipe_rt import host_io  # noqa: E402

SRC = "/root/reference/model3D"


def main():
    rc, m, (mats, tw, th) = host_io.load(os.path.join(SRC, "1tree_tri.obj"), os.path.join(SRC, "1tree_tri.mtl"))
    assert rc == 0, rc
    hx = float                       # JSON repr round-trips doubles exactly
    out = {"source": "model3D/1tree_tri.obj (+1tree_tri.mtl), librt_host.so kd_fallback=1",
           "tex_width": tw, "tex_height": th, "n_materials": m.nbMaterials,
           "triangles": [], "quelMatPourTri": [m.quelMatPourTri[i] for i in range(m.nbTriangles)], "texels": []}
    for i in range(m.nbTriangles):
        t = m.triangles[i]
        assert t.uvA.u == t.uvA.v == t.uvB.u == t.uvB.v == t.uvC.u == t.uvC.v == 0.0
        out["triangles"].append([hx(c) for P in (t.A, t.B, t.C) for c in P.tolist()])
    for k in range(m.nbMaterials * tw * th):
        q = mats[k]
        out["texels"].append([hx(c) for c in q.diffuseColor.tolist()] + [hx(q.alpha), hx(q.reflectionStrength)])
    host_io.free(m, mats)
    with open(os.path.join(HERE, "scenes", "tree.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
