"""Nature scene: BVH node visits and kernel rate against the scene radius R
that pads the tree (rt_bvh.cpp): main.c:346's sky sphere of radius 1e5 sets
R = 1e5; smaller sky radii give the same image up to where the sky is hit.
Usage: python tools/probes/nature_radius.py"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch
import tipe_rt
from tipe_rt import scenes
W, H, SPP = 1200, 900, 64
cam = tipe_rt.init_camera(**{k: scenes.NATURE_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
st = torch.cuda.current_stream()
for r_sky in (1e5, 1e3, 20.0):
    sph = scenes.main_spheres()
    sph[1].radius = r_sky
    tris, qm, mats, tw, th, nm = scenes.nature_mesh()
    ds = tipe_rt.DeviceScene(tipe_rt.make_scene(sph, tris, qm, mats, tw, th, nm), 0)
    p = tipe_rt.make_params(W, H, SPP, 10, cam, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
    out = torch.empty((3, H, W, 3), dtype=torch.float64, device="cuda:0")
    t = tipe_rt.band_tiling(0, H - 1)
    f = lambda: tipe_rt.render_async(ds, p, t, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, st.cuda_stream)
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); f(); f(); e1.record(st); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 2
    k = tipe_rt.last_render_kernel()
    pc = tipe_rt.make_params(W, H, 4, 10, cam)
    d = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, pc, t, d.data_ptr(), st.cuda_stream); torch.cuda.synchronize()
    c = [int(x) for x in d.cpu()]
    ds.close()
    print(json.dumps({"r_sky": r_sky, "kernel": k, "msamples_per_s": round(W * H * SPP / ms / 1e3, 1),
                      "per_sample": {n: round(c[i] / c[0], 3) for i, n in enumerate(tipe_rt.COUNTER_NAMES) if c[i]}}), flush=True)
