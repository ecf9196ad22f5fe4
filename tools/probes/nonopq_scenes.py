"""Kernel rates of non-opaque BVH scenes on the deep-tree queue kernel
(render_kernel_q<QB=3>): RTX_MAP/nature, mineways in the README box, and
the C4 tree with material index 4 on every 7th triangle (texture.h:77-81's
water override makes it non-opaque).  Usage: python tools/probes/nonopq_scenes.py [spp]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import tipe_rt
from tipe_rt import scenes
from tipe_rt.types import Material
SPP = int(sys.argv[1]) if len(sys.argv) > 1 else 128
W, H = 1200, 900


def cam_of(spec):
    return tipe_rt.init_camera(**{k: spec[k] for k in ("origin", "target", "up", "vfov", "ratio")})


def mineways():
    tris, qm, mats, tw, th, nm = scenes.load_mesh_fixture("mineways")
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0], P.e[1], P.e[2] = P.e[0] * 0.1 - 0.2, P.e[1] * 0.1 - 1.0, P.e[2] * 0.1 - 2.5
    return scenes.cornell_spheres(), (tris, qm, mats, tw, th, nm), scenes.README_CAMERA, 6, False


def tree_water():
    tris, qm, mats, tw, th, nm = scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE)
    mats2 = (Material * (5 * tw * th))()
    for k in range(5 * tw * th):
        mats2[k] = mats[k] if k < nm * tw * th else mats[0]
    for k in range(0, len(tris), 7):
        qm[k] = 4
    return scenes.cornell_spheres(), (tris, qm, mats2, tw, th, 5), scenes.README_CAMERA, 8, True


def nature():
    return scenes.main_spheres(), scenes.nature_mesh(), scenes.NATURE_CAMERA, 10, False


st = torch.cuda.current_stream()
for name, fn in (("nature", nature), ("mineways", mineways), ("tree_water_ao", tree_water)):
    sph, mesh, camspec, bounces, ao = fn()
    ds = tipe_rt.DeviceScene(tipe_rt.make_scene(sph, *mesh), 0)
    p = tipe_rt.make_params(W, H, SPP, bounces, cam_of(camspec), use_ao=ao, ao=2.5, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
    out = torch.empty((3, H, W, 3), dtype=torch.float64, device="cuda:0")
    t = tipe_rt.band_tiling(0, H - 1)
    f = lambda: tipe_rt.render_async(ds, p, t, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, st.cuda_stream)
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); f(); f(); e1.record(st); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 2
    print(json.dumps({"scene": name, "kernel": tipe_rt.last_render_kernel(), "spp": SPP,
                      "msamples_per_s": round(W * H * SPP / ms / 1e3, 1)}), flush=True)
    ds.close()
