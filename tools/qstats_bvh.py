"""Census of the BVH kernel's samples_coop (diagnostic build -DRT_QSTATS=1).

    RT_HIP_LIB=tools/qstats.so python tools/qstats_bvh.py [spp] [c4|sweep]
"""
import os
import sys
import json
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: E402
import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 8
kind = sys.argv[2] if len(sys.argv) > 2 else "c4"
path = os.path.join(ROOT, "gpurun_out", "qstats_bvh.bin")
if os.path.exists(path):
    os.remove(path)
os.environ["RT_QUEUE_TRACE"] = path
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
if kind == "c4":
    sph = scenes.cornell_spheres()
    sc = tipe_rt.make_scene(sph, *scenes.tree_mesh())
    p = tipe_rt.make_params(1200, 900, spp, 8, cam, focus=3.0, use_ao=True, ao=2.5, seed=1010, chunks=8)
else:
    sph, mesh = scenes.synthetic_cornell(10, 100)
    sc = tipe_rt.make_scene(sph, *mesh)
    p = tipe_rt.make_params(1200, 900, spp, 6, cam, focus=3.0, seed=1010, chunks=8)
ds = tipe_rt.DeviceScene(sc, 0)
out = torch.empty((3, 900, 1200, 3), dtype=torch.float64, device="cuda:0")
tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, 899), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                     None, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
del os.environ["RT_QUEUE_TRACE"]
q = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).sum(0).astype(np.float64)
rounds, phases, iters, task_l, parked_l, res_l, start_l, cast_l, t_rs, t_cast, t_coop = q[:11]
tt = t_rs + t_cast + t_coop
S = 1200 * 900 * spp
print(json.dumps({"scene": kind, "spp": spp, "rounds_per_sample_x64": rounds * 64 / S,
                  "resolve_util": res_l / (64 * rounds), "start_util": start_l / (64 * rounds),
                  "cast_util": cast_l / (64 * rounds), "coop_phases_per_round": phases / rounds,
                  "parked_per_phase": parked_l / max(phases, 1), "coop_iters_per_phase": iters / max(phases, 1),
                  "coop_lane_util": task_l / (64 * max(iters, 1)),
                  "time_share": {"resolve_start": t_rs / tt, "cast_root": t_cast / tt, "coop": t_coop / tt},
                  "casts_per_sample": cast_l / S}))
