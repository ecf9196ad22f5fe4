"""PCIe-inclusive rate of the host-buffer drop-in (rt_render_rows on C2):
scene upload + render + D2H of canva/albedo/normal into host arrays."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: F401  (share torch's HIP runtime)
import tipe_rt
from tipe_rt import scenes
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
scene = tipe_rt.make_scene(scenes.cornell_spheres())
p = tipe_rt.make_params(1200, 900, 1000, 6, cam, focus=3.0, chunks=8)
tipe_rt.render_rows(scene, p)                       # warm-up (code object load, pools)
t = time.perf_counter()
n = 2
for _ in range(n):
    canva, alb, nrm = tipe_rt.render_rows(scene, p)
dt = (time.perf_counter() - t) / n
print(json.dumps({"path": "rt_render_rows (host buffers, PCIe-inclusive)", "ms_per_frame": round(dt * 1e3, 2),
                  "msamples_per_s": round(1200 * 900 * 1000 / dt / 1e6, 1), "canva_mean": float(canva.mean())}))
