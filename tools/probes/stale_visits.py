"""Diagnostic (RT_DIAG_STALE=2 build): the queue kernel's node visits and the
visits to nodes whose entry distance already exceeds the cull distance (the
stack entry went stale after a closer hit), per scene, from RT_QUEUE_TRACE.
    bash tools/build_variants.sh stale "-DRT_DIAG_STALE=2"
    RT_HIP_LIB=tools/variants/stale.so python tools/probes/stale_visits.py [spp]"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: E402
import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402
from phase_clock import scene_of  # noqa: E402
SPP = int(sys.argv[1]) if len(sys.argv) > 1 else 32
for kind in ("c4", "nature", "sweep"):
    path = os.path.join(ROOT, "gpurun_out", "stale_%s.bin" % kind)
    if os.path.exists(path):
        os.remove(path)
    sc, bounces, ao = scene_of(kind)
    spec = scenes.NATURE_CAMERA if kind == "nature" else scenes.README_CAMERA
    cam = tipe_rt.init_camera(**{k: spec[k] for k in ("origin", "target", "up", "vfov", "ratio")})
    p = tipe_rt.make_params(1200, 900, SPP, bounces, cam, focus=3.0, seed=1010, chunks=32, use_ao=ao, ao=2.5)
    ds = tipe_rt.DeviceScene(sc, 0)
    out = torch.empty((3, 900, 1200, 3), dtype=torch.float64, device="cuda:0")
    os.environ["RT_QUEUE_TRACE"] = path
    tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, 899), out[0].data_ptr(), out[1].data_ptr(),
                         out[2].data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del os.environ["RT_QUEUE_TRACE"]
    d = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    v, st = int(d[:, 2].sum()), int(d[:, 3].sum())
    n = 1200 * 900 * SPP
    print(json.dumps({"scene": kind, "kernel": tipe_rt.last_render_kernel(), "visits_per_sample": v / n,
                      "stale_per_sample": st / n, "stale_frac": st / max(v, 1)}), flush=True)
