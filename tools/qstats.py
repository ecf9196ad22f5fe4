"""Round census of render_kernel_q (diagnostic build -DRT_QSTATS=1).

    RT_HIP_LIB=tools/variants/qstats.so python tools/qstats.py [spp] [scene]

Renders one C2-shaped frame with RT_QUEUE_TRACE and reports, per wave:
rounds, lane utilisation of the cast+resolve pass, camera-ray events and
their lane utilisation, lanes waiting (SM_CAM) or done during casts."""
import os
import sys
import json
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: E402
import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 250
kind = sys.argv[2] if len(sys.argv) > 2 else "c2"
path = os.path.join(ROOT, "gpurun_out", "qstats.bin")
if os.path.exists(path):
    os.remove(path)
os.environ["RT_QUEUE_TRACE"] = path
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
sph = scenes.cornell_spheres()
bounces, ao = 6, False
if kind == "c2":
    sc = tipe_rt.make_scene(sph)
elif kind == "c4":
    sc = tipe_rt.make_scene(sph, *scenes.tree_mesh())
    bounces, ao = 8, True
elif kind == "sweep":
    sph, mesh = scenes.synthetic_cornell(10, 100)
    sc = tipe_rt.make_scene(sph, *mesh)
else:
    sc = tipe_rt.make_scene(sph, *scenes.pyramid_mesh())
p = tipe_rt.make_params(1200, 900, spp, bounces, cam, focus=3.0, seed=1010, chunks=32, use_ao=ao, ao=2.5)
ds = tipe_rt.DeviceScene(sc, 0)
out = torch.empty((3, 900, 1200, 3), dtype=torch.float64, device="cuda:0")
tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, 899), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                     None, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
del os.environ["RT_QUEUE_TRACE"]
d = np.fromfile(path, dtype=np.uint64).reshape(-1, 18)
w = d[::64]                                  # lane 0 of each wave holds the wave census
q = w[:, 4:18].astype(np.float64)
tot = q.sum(0)
rounds, cast_l, bounce_l, cam_l, task_r, task_l = tot[:6]
t = tot[8:13]  # (slot 13: the sphere pass of BVH scenes, split from slot 8)
res = {"spp": spp, "scene": kind, "waves": int(len(w)), "rounds_per_wave": rounds / len(w),
       "cast_lane_util": cast_l / (64 * rounds), "bounce_lanes_per_round": bounce_l / rounds,
       "camera_lanes_per_round": cam_l / rounds, "task_rounds_frac": task_r / rounds,
       "tasks_per_task_round": task_l / max(task_r, 1),
       "time_share": {k: round(v / t.sum(), 4) for k, v in zip(("cast", "resolve_hit", "tasks", "next_ray",
                                                                 "finish"), t)},
       "trav_steps_per_round": tot[6] / rounds, "trav_lane_util": tot[7] / max(64 * tot[6], 1),
       "sphere_pass_share": tot[13] / (t.sum() + tot[13]),
       "samples": 1200 * 900 * spp, "casts_per_sample": cast_l / (1200 * 900 * spp)}
print(json.dumps(res))
