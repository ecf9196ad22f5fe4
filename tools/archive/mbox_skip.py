"""Fraction of brute-force casts whose wave skips the triangle scan (rt.h
RT_CNT_MBOX_SKIP, RT_MESH_BOX pre-test) on C3 / C5, from rt_count_async at a
few spp.  Usage: python tools/mbox_skip.py
Needs the library of commit 8bc63d2 (the RT_MESH_BOX experiment, measured
C3 -3.1 % / C5 -2.9 % and removed again; profiles/r05_mbox/)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: E402
import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

T = tipe_rt.types
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
sc = tipe_rt.make_scene(scenes.cornell_spheres(), *scenes.pyramid_mesh())
ds = tipe_rt.DeviceScene(sc, 0)
for name, (w, h) in {"C3": (1200, 900), "C5": (3840, 2880)}.items():
    p = tipe_rt.make_params(w, h, 4, 6, cam, focus=3.0, seed=1010)
    d = torch.zeros(T.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
    tipe_rt.count_async(ds, p, tipe_rt.band_tiling(0, h - 1), d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = [int(x) for x in d.cpu()]
    print(json.dumps({"config": name, "casts": c[T.RT_CNT_CASTS], "mbox_skip": c[T.RT_CNT_MBOX_SKIP],
                      "skip_frac": round(c[T.RT_CNT_MBOX_SKIP] / max(c[T.RT_CNT_CASTS], 1), 4),
                      "note": "rt_count_async's fixed-grid waves (8x8 pixel tiles), 4 spp"}))
ds.close()
