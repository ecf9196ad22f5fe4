"""C host library (librt_host.so): camera, OBJ/MTL/PPM IO.

Reference-loader parity uses tests/golden/scenes/*.json, which hold the
reference's own list_of_mesh + create_mat_list_mtl output
(tests/golden/make_fixtures.py); the OBJ inputs are read from
/root/reference/model3D when present (container), otherwise those tests
skip.  Synthetic OBJ/PPM files cover the cases the reference loader
crashes on (SURVEY.md §7 "Loader gaps")."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import tipe_rt
from tipe_rt.types import Vec3, Triangle, Material, Camera

REF = "/root/reference/model3D"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


from tipe_rt.host_io import Mesh, lib as host, load  # noqa: E402  (the ctypes mirror under test)


def test_init_camera_matches_survey_kat():
    cam = tipe_rt.init_camera((0.34, 0.3, 0.5), (0.0, -0.5, -3.0), (0, 1, 0), 70.0, 4.0 / 3.0)
    assert cam.horizontal.tolist() == [1.8584717400487587, 0.0, -0.18053725474759372]
    assert cam.coin_bas_gauche.tolist() == [-0.66849622616424687, -0.60459405382114229, -0.22564680347778088]


def test_init_camera_matches_reference_fixture():
    with open(os.path.join(GOLDEN, "kat_leaf.json")) as f:
        rows = json.load(f)["camera"]
    fx = float.fromhex
    for row in rows:
        cam = tipe_rt.init_camera([fx(x) for x in row["origin"]], [fx(x) for x in row["target"]], (0, 1, 0),
                                  fx(row["vfov"]), fx(row["ratio"]))
        assert cam.vertical.tolist() == [fx(x) for x in row["vertical"]]
        assert cam.coin_bas_gauche.tolist() == [fx(x) for x in row["corner"]]


def fixture_equal(m, tex, name):
    with open(os.path.join(GOLDEN, "scenes", name + ".json")) as f:
        d = json.load(f)
    mats, tw, th = tex
    assert m.nbTriangles == len(d["triangles"]) and m.nbMaterials == d["n_materials"]
    assert (tw, th) == (d["tex_width"], d["tex_height"])
    for k, t in enumerate(d["triangles"]):
        tr = m.triangles[k]
        assert tr.A.tolist() == t["A"] and tr.B.tolist() == t["B"] and tr.C.tolist() == t["C"]
        assert [tr.uvA.u, tr.uvA.v, tr.uvB.u, tr.uvB.v, tr.uvC.u, tr.uvC.v] == t["uvA"] + t["uvB"] + t["uvC"]
    assert [m.quelMatPourTri[k] for k in range(m.nbTriangles)] == d["quelMatPourTri"]
    for k, (r, g, b, a) in enumerate(d["texels"]):
        mt = mats[k]
        assert mt.diffuseColor.tolist() == [r, g, b] and mt.alpha == a and mt.emissionStrength == 0.0


@pytest.mark.skipif(not os.path.exists(REF), reason="reference assets absent")
@pytest.mark.parametrize("obj,mtl,name", [
    ("pyramide/pyramide_tri.obj", "pyramide/pyramide_tri.mtl", "pyramide"),
    ("mcworld_tiltedtex_water/mineways_tri.obj", "mcworld_tiltedtex_water/mineways_tri.mtl", "mineways"),
])
def test_loader_matches_reference_loader(obj, mtl, name):
    rc, m, tex = load(os.path.join(REF, obj), os.path.join(REF, mtl), mode=0, kd_fallback=0)
    assert rc == 0
    fixture_equal(m, tex, name)
    host().rt_host_free(C.cast(tex[0], C.c_void_p))
    host().rt_host_free_mesh(C.byref(m))


@pytest.mark.skipif(not os.path.exists(REF), reason="reference assets absent")
def test_loader_reads_tree_the_reference_loader_crashes_on():
    """1tree_tri.obj: `f v//vn` faces and Kd-only MTL (reference segfaults,
    SURVEY.md §8c).  Kd-flat texels, reflectionStrength = Ns/100."""
    rc, m, tex = load(os.path.join(REF, "1tree_tri.obj"), os.path.join(REF, "1tree_tri.mtl"))
    assert rc == 0 and m.nbTriangles == 1320 and m.nbMaterials == 2
    mats, tw, th = tex
    assert (tw, th) == (1, 1)
    assert mats[0].diffuseColor.tolist() == [0.213409, 0.099387, 0.035471]
    assert mats[1].diffuseColor.tolist() == [0.041648, 0.236554, 0.025988]
    assert mats[0].reflectionStrength == float(np.float32(np.float32(20.0) / np.float32(100.0)))
    assert mats[0].alpha == 1.0


def write(path, text):
    with open(path, "w", newline="") as f:
        f.write(text)


def test_loader_faces_quads_crlf_and_errors(tmp_path):
    d = tmp_path
    write(d / "t.mtl", "newmtl a\r\nKd 0.5 0.25 1\r\nNs 50\r\nnewmtl b\r\nmap_Kd ./tex.png\r\n")
    write(d / "tex.ppm", "P3\n2 2\n255\n255 0 0  0 255 0\n0 0 255  255 255 255\n")
    write(d / "tex_alpha.ppm", "P3\n2 2\n255\n255 255 255 0 0 0\n128 128 128 255 255 255\n")
    obj = ("v 0 0 0\r\nv 1 0 0\r\nv 1 1 0\r\nv 0 1 0\r\nvt 0 0\r\nvt 1 0\r\nvt 1 1\r\nvt 0 1\r\n"
           "usemtl a\r\nf 1//1 2//1 3//1\r\nf 1 3 4\r\nusemtl b\r\nf 1/1/1 2/2/1 3/3/1 4/4/1\r\nf -4/-4 -2/-2 -1/-1\r\n")
    write(d / "t.obj", obj)
    rc, m, tex = load(str(d / "t.obj"), str(d / "t.mtl"), mode=0)        # compat: quad -> first 3
    assert rc == 0 and m.nbTriangles == 4 and m.nbMaterials == 2
    assert [m.quelMatPourTri[k] for k in range(4)] == [0, 0, 1, 1]
    assert m.triangles[2].C.tolist() == [1.0, 1.0, 0.0]
    assert m.triangles[3].uvC.u == 0.0 and m.triangles[3].uvC.v == 1.0   # relative indices
    mats, tw, th = tex
    assert (tw, th) == (2, 2)
    assert mats[0].diffuseColor.tolist() == [0.5, 0.25, 1.0] and mats[0].reflectionStrength == 0.5
    # material b: rows bottom-up (texture.h:227-229): file row 0 -> table row 1
    assert mats[4 + 2].diffuseColor.tolist() == [1.0, 0.0, 0.0]
    assert mats[4 + 0].diffuseColor.tolist() == [0.0, 0.0, 1.0]
    assert mats[4 + 0].alpha == 128 / 255
    rc, m2, _ = load(str(d / "t.obj"), str(d / "t.mtl"), mode=1)        # fan
    assert rc == 0 and m2.nbTriangles == 5
    write(d / "bad.obj", "v 0 0 0\nf 1 2 3\n")
    assert load(str(d / "bad.obj"), None)[0] == tipe_rt.RT_EINVAL      # face before usemtl / bad index
    assert load(str(d / "missing.obj"), None)[0] == tipe_rt.RT_EINVAL
    rc, m3, _ = load(str(d / "t.obj"), str(d / "t.mtl"), kd_fallback=0)
    assert rc == tipe_rt.RT_EINVAL                                      # Kd-only without fallback


def test_ppm_write_read_roundtrip(tmp_path):
    H = host()
    W_, H_ = 5, 3
    canva = np.zeros((H_, W_, 3))
    canva[..., 0] = np.arange(W_)[None, :] * 50
    canva[..., 1] = np.arange(H_)[:, None] * 100
    path = str(tmp_path / "o.ppm").encode()
    assert H.rt_host_write_ppm(path, canva.ctypes.data, W_, H_) == 0
    txt = open(path.decode()).read().split("\n")
    assert txt[:3] == ["P3", "5 3", "255"]
    assert txt[3] == "0 200 0"                      # first line = top row (j = H-1), main.c:460
    w, h, mv = C.c_int(), C.c_int(), C.c_int()
    vals = C.POINTER(C.c_int)()
    assert H.rt_host_read_ppm(path, C.byref(w), C.byref(h), C.byref(mv), C.byref(vals)) == 0
    got = np.array([vals[i] for i in range(w.value * h.value * 3)]).reshape(h.value, w.value, 3)
    assert (got[::-1] == canva.astype(int)).all()
    H.rt_host_free(vals)
